/*
 * gk_addon.c — N-API binding of the MI355X simplex core (include/glpk_mi355x.h)
 * for the JavaScript host (Cyame/glpk.js).  Every function is a thin,
 * synchronous marshal of typed arrays to one C-ABI call; a GK_EABI return is
 * rethrown as a JS Error carrying gk_last_error() (the reference's xerror
 * text).  See js/gk_core.js for the JS side and INTEGRATION.md for wiring.
 *
 *   create(device)                 -> ctx       gk_ctx_create
 *   deviceCount(), abiVersion(), lastError()
 *   bfdCreate(ctx)                 -> bfd       gk_bfd_create (finalizer: gk_bfd_destroy)
 *   bfdSetParm(bfd, parm)                       gk_bfd_set_parm      (glpbfd.js:31)
 *   bfdFactorizeCsc(bfd, m, ptr, ind, val) -> int  gk_bfd_factorize_csc (glpbfd.js:47)
 *   bfdFtran(bfd, x), bfdBtran(bfd, x)          gk_bfd_ftran/btran   (glpbfd.js:148/159)
 *   bfdUpdate(bfd, j, len, ind, idx, val) -> int gk_bfd_update       (glpbfd.js:170)
 *   bfdGetCount(bfd), bfdValid(bfd)             (glpbfd.js:225)
 *   spx(ctx, bfd, lp, smcp, dual)  -> int       gk_spx_primal/dual (glpspx01.js:1 / glpspx02.js:1)
 *   stats(bfd)                     -> object    gk_bfd_last_stats
 *   nppCreate/nppLoad/nppSimplex/nppInteger/nppBuildSize/nppBuild/
 *   nppPostprocess/nppUnloadSol/nppUnloadMip   gk_npp_* (glpnpp01.js .. 05.js)
 */
#define NAPI_VERSION 6
#include <node_api.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <unistd.h>
#include "../include/glpk_mi355x.h"

#define CHECK(call)                                                                 \
    do {                                                                            \
        if ((call) != napi_ok) {                                                    \
            napi_throw_error(env, NULL, "gk_addon: N-API call failed: " #call);     \
            return NULL;                                                            \
        }                                                                           \
    } while (0)
/* the same in a helper returning int (0: an exception is pending) */
#define CHECK0(call)                                                                \
    do {                                                                            \
        if ((call) != napi_ok) {                                                    \
            napi_throw_error(env, NULL, "gk_addon: N-API call failed: " #call);     \
            return 0;                                                               \
        }                                                                           \
    } while (0)

static napi_value throw_gk(napi_env env, const char *what)
{
    char msg[1024];
    snprintf(msg, sizeof msg, "%s: %s", what, gk_last_error());
    napi_throw_error(env, NULL, msg);
    return NULL;
}

static napi_value mk_int(napi_env env, long long v)
{
    napi_value r;
    napi_create_double(env, (double)v, &r);
    return r;
}

static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value *argv)
{
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < want) {
        napi_throw_type_error(env, NULL, "gk_addon: wrong number of arguments");
        return 0;
    }
    return 1;
}

static void *get_ext(napi_env env, napi_value v)
{
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok) return NULL;
    return p;
}

/* typed array data pointer (any element type); NULL for null/undefined */
static void *ta(napi_env env, napi_value v)
{
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_null || t == napi_undefined) return NULL;
    bool is = false;
    napi_is_typedarray(env, v, &is);
    if (!is) return NULL;
    napi_typedarray_type type;
    size_t len, off;
    void *data;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &len, &data, &ab, &off) != napi_ok) return NULL;
    return data;
}

/* the same with its element count */
static void *ta_len(napi_env env, napi_value v, size_t *len)
{
    bool is = false;
    *len = 0;
    if (napi_is_typedarray(env, v, &is) != napi_ok || !is) return NULL;
    napi_typedarray_type type;
    size_t off;
    void *data;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, len, &data, &ab, &off) != napi_ok) return NULL;
    return data;
}

static napi_value prop(napi_env env, napi_value obj, const char *name)
{
    napi_value v;
    if (napi_get_named_property(env, obj, name, &v) != napi_ok) return NULL;
    return v;
}

static double dprop(napi_env env, napi_value obj, const char *name, double def)
{
    napi_value v = prop(env, obj, name);
    double d;
    if (!v || napi_get_value_double(env, v, &d) != napi_ok) return def;
    return d;
}

static void *tprop(napi_env env, napi_value obj, const char *name)
{
    napi_value v = prop(env, obj, name);
    return v ? ta(env, v) : NULL;
}

static void set_num(napi_env env, napi_value obj, const char *name, double v)
{
    napi_value x;
    napi_create_double(env, v, &x);
    napi_set_named_property(env, obj, name, x);
}

/* ---------------------------------------------------------------- context */
/* set by the environment cleanup hook: at teardown the handles are left to
 * the process exit (the HIP runtime may already be shutting down, and the
 * order in which the remaining externals are finalized is not defined) */
static int g_teardown = 0;

static void npp_free_all(void);

static void teardown_hook(void *arg)
{
    (void)arg;
    g_teardown = 1;
    npp_free_all();                 /* the preprocessor workspaces are host memory only */
}

static void ctx_fin(napi_env env, void *data, void *hint)
{
    (void)env; (void)hint;
    if (!g_teardown) gk_ctx_destroy((gk_ctx *)data);
}

static napi_value js_create(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    int dev = 0;
    CHECK(napi_get_value_int32(env, argv[0], &dev));
    gk_ctx *c = gk_ctx_create(dev);
    if (!c) {
        char what[64];
        snprintf(what, sizeof what, "gk_ctx_create(%d)", dev);
        return throw_gk(env, what);
    }
    napi_value r;
    CHECK(napi_create_external(env, c, ctx_fin, NULL, &r));
    return r;
}

static napi_value js_device_count(napi_env env, napi_callback_info info)
{
    (void)info;
    return mk_int(env, gk_device_count());
}

static napi_value js_abi_version(napi_env env, napi_callback_info info)
{
    (void)info;
    return mk_int(env, gk_abi_version());
}

static napi_value js_last_error(napi_env env, napi_callback_info info)
{
    (void)info;
    napi_value r;
    napi_create_string_utf8(env, gk_last_error(), NAPI_AUTO_LENGTH, &r);
    return r;
}

/* -------------------------------------------------------------------- bfd */
static void bfd_fin(napi_env env, void *data, void *hint)
{
    (void)env; (void)hint;
    if (!g_teardown) gk_bfd_destroy((gk_bfd *)data);
}

static napi_value js_bfd_create(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    gk_ctx *c = (gk_ctx *)get_ext(env, argv[0]);
    gk_bfd *b = gk_bfd_create(c);
    if (!b) return throw_gk(env, "bfd_create_it");
    napi_value r;
    CHECK(napi_create_external(env, b, bfd_fin, NULL, &r));
    return r;
}

static napi_value js_bfd_set_parm(napi_env env, napi_callback_info info)
{
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[0]);
    gk_bfcp p;
    p.type = (int)dprop(env, argv[1], "type", 1);
    p.lu_size = (int)dprop(env, argv[1], "lu_size", 0);
    p.piv_tol = dprop(env, argv[1], "piv_tol", 0.10);
    p.piv_lim = (int)dprop(env, argv[1], "piv_lim", 4);
    p.suhl = (int)dprop(env, argv[1], "suhl", 1);
    p.eps_tol = dprop(env, argv[1], "eps_tol", 1e-15);
    p.max_gro = dprop(env, argv[1], "max_gro", 1e10);
    p.nfs_max = (int)dprop(env, argv[1], "nfs_max", 100);
    p.upd_tol = dprop(env, argv[1], "upd_tol", 1e-6);
    p.nrs_max = (int)dprop(env, argv[1], "nrs_max", 100);
    p.rs_size = (int)dprop(env, argv[1], "rs_size", 0);
    if (gk_bfd_set_parm(b, &p) != 0) napi_throw_error(env, NULL, gk_last_error());
    return NULL;
}

/* bfdResetParm(bfd): glp_get_bfcp's defaults with the engine's re-inversion
 * interval (copy_bfcp of a problem without lp.bfcp, glpapi12.js:127-131) */
static napi_value js_bfd_reset_parm(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[0]);
    if (gk_bfd_reset_parm(b) != 0) napi_throw_error(env, NULL, gk_last_error());
    return NULL;
}

static napi_value js_bfd_factorize_csc(napi_env env, napi_callback_info info)
{
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return NULL;
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[0]);
    int m = 0;
    CHECK(napi_get_value_int32(env, argv[1], &m));
    const int *ptr = (const int *)ta(env, argv[2]);
    const int *ind = (const int *)ta(env, argv[3]);
    const double *val = (const double *)ta(env, argv[4]);
    if (!ptr || !ind || !val) {
        napi_throw_type_error(env, NULL, "bfdFactorizeCsc: ptr/ind must be Int32Array, val Float64Array");
        return NULL;
    }
    int ret = gk_bfd_factorize_csc(b, m, ptr, ind, val);
    if (ret == GK_EABI) return throw_gk(env, "bfd_factorize");
    return mk_int(env, ret);
}

static napi_value solve(napi_env env, napi_callback_info info, int tr)
{
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[0]);
    double *x = (double *)ta(env, argv[1]);
    if (!x) {
        napi_throw_type_error(env, NULL, "bfd_ftran/btran: x must be a Float64Array");
        return NULL;
    }
    if (!gk_bfd_valid(b)) {
        napi_throw_error(env, NULL, tr ? "bfd_btran: factorization is not valid" : "bfd_ftran: factorization is not valid");
        return NULL;
    }
    if (tr) gk_bfd_btran(b, x);
    else gk_bfd_ftran(b, x);
    return NULL;
}

static napi_value js_bfd_ftran(napi_env env, napi_callback_info info) { return solve(env, info, 0); }
static napi_value js_bfd_btran(napi_env env, napi_callback_info info) { return solve(env, info, 1); }

static napi_value js_bfd_update(napi_env env, napi_callback_info info)
{
    napi_value argv[6];
    if (!get_args(env, info, 6, argv)) return NULL;
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[0]);
    int j, len, idx;
    CHECK(napi_get_value_int32(env, argv[1], &j));
    CHECK(napi_get_value_int32(env, argv[2], &len));
    CHECK(napi_get_value_int32(env, argv[4], &idx));
    const int *ind = (const int *)ta(env, argv[3]);
    const double *val = (const double *)ta(env, argv[5]);
    int ret = gk_bfd_update(b, j, len, ind, idx, val);
    if (ret == GK_EABI) return throw_gk(env, "bfd_update_it");
    return mk_int(env, ret);
}

static napi_value js_bfd_get_count(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    int r = gk_bfd_get_count((gk_bfd *)get_ext(env, argv[0]));
    if (r == GK_EABI) return throw_gk(env, "bfd_get_count");
    return mk_int(env, r);
}

static napi_value js_bfd_valid(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    return mk_int(env, gk_bfd_valid((gk_bfd *)get_ext(env, argv[0])));
}

/* -------------------------------------------------------------------- spx */
/* the gk_lp arrays of the marshalled problem object L (js/gk_core.js) */
static int fill_lp(napi_env env, napi_value L, gk_lp *out)
{
    gk_lp lp;
    memset(&lp, 0, sizeof lp);
    lp.m = (int)dprop(env, L, "m", 0);
    lp.n = (int)dprop(env, L, "n", 0);
    lp.nnz = (int)dprop(env, L, "nnz", 0);
    lp.dir = (int)dprop(env, L, "dir", 1);
    lp.c0 = dprop(env, L, "c0", 0.0);
    lp.row_type = (const signed char *)tprop(env, L, "row_type");
    lp.row_lb = (const double *)tprop(env, L, "row_lb");
    lp.row_ub = (const double *)tprop(env, L, "row_ub");
    lp.rii = (const double *)tprop(env, L, "rii");
    lp.col_type = (const signed char *)tprop(env, L, "col_type");
    lp.col_lb = (const double *)tprop(env, L, "col_lb");
    lp.col_ub = (const double *)tprop(env, L, "col_ub");
    lp.col_coef = (const double *)tprop(env, L, "col_coef");
    lp.sjj = (const double *)tprop(env, L, "sjj");
    lp.A_ptr = (const int *)tprop(env, L, "A_ptr");
    lp.A_ind = (const int *)tprop(env, L, "A_ind");
    lp.A_val = (const double *)tprop(env, L, "A_val");
    lp.a_version = (unsigned long long)dprop(env, L, "a_version", 0);
    lp.b_version = (unsigned long long)dprop(env, L, "b_version", 0);
    lp.head = (int *)tprop(env, L, "head");
    lp.row_stat = (signed char *)tprop(env, L, "row_stat");
    lp.col_stat = (signed char *)tprop(env, L, "col_stat");
    lp.row_bind = (int *)tprop(env, L, "row_bind");
    lp.col_bind = (int *)tprop(env, L, "col_bind");
    lp.row_prim = (double *)tprop(env, L, "row_prim");
    lp.row_dual = (double *)tprop(env, L, "row_dual");
    lp.col_prim = (double *)tprop(env, L, "col_prim");
    lp.col_dual = (double *)tprop(env, L, "col_dual");
    lp.it_cnt = (int)dprop(env, L, "it_cnt", 0);
    if (!lp.row_type || !lp.row_lb || !lp.row_ub || !lp.rii || !lp.col_type || !lp.col_lb || !lp.col_ub ||
        !lp.col_coef || !lp.sjj || !lp.A_ptr || !lp.A_ind || !lp.A_val || !lp.head || !lp.row_stat ||
        !lp.col_stat || !lp.row_prim || !lp.row_dual || !lp.col_prim || !lp.col_dual) {
        napi_throw_type_error(env, NULL, "gk_addon: lp arrays missing or not typed arrays");
        return 0;
    }
    *out = lp;
    return 1;
}

/* the reports of one gk_spx_* call (gk_bfd_set_report), handed to JS as
 * L.reports = [[kind, code, it_cnt, phase, obj, infeas, aux], ...] */
typedef struct {
    int kind, code, it_cnt, phase, aux;
    double obj, infeas;
} rpt_rec;
typedef struct {
    rpt_rec *v;
    size_t n, cap;
} rpt_buf;

static void rpt_collect(void *ud, int kind, int code, int it_cnt, int phase, double obj, double infeas, int aux)
{
    rpt_buf *b = (rpt_buf *)ud;
    if (b->n == b->cap) {
        size_t cap = b->cap ? 2 * b->cap : 64;
        rpt_rec *v = (rpt_rec *)realloc(b->v, cap * sizeof(rpt_rec));
        if (!v) return;
        b->v = v;
        b->cap = cap;
    }
    rpt_rec r = {kind, code, it_cnt, phase, aux, obj, infeas};
    b->v[b->n++] = r;
}

/* L.reports = the collected records (frees them) */
static int set_reports(napi_env env, napi_value L, rpt_buf *rb)
{
    napi_value arr;
    CHECK0(napi_create_array_with_length(env, rb->n, &arr));
    for (size_t k = 0; k < rb->n; k++) {
        const rpt_rec *r = &rb->v[k];
        const double f[7] = {r->kind, r->code, r->it_cnt, r->phase, r->obj, r->infeas, r->aux};
        napi_value e, x;
        CHECK0(napi_create_array_with_length(env, 7, &e));
        for (uint32_t t = 0; t < 7; t++) {
            CHECK0(napi_create_double(env, f[t], &x));
            CHECK0(napi_set_element(env, e, t, x));
        }
        CHECK0(napi_set_element(env, arr, (uint32_t)k, e));
    }
    CHECK0(napi_set_named_property(env, L, "reports", arr));
    free(rb->v);
    rb->v = NULL;
    rb->n = rb->cap = 0;
    return 1;
}

static napi_value js_spx(napi_env env, napi_callback_info info)
{
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return NULL;
    gk_ctx *c = (gk_ctx *)get_ext(env, argv[0]);
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[1]);
    napi_value L = argv[2], S = argv[3];
    bool dual = false;
    CHECK(napi_get_value_bool(env, argv[4], &dual));
    gk_lp lp;
    if (!fill_lp(env, L, &lp)) return NULL;
    gk_smcp p;
    p.msg_lev = (int)dprop(env, S, "msg_lev", 3);
    p.meth = (int)dprop(env, S, "meth", 1);
    p.pricing = (int)dprop(env, S, "pricing", 0x22);
    p.r_test = (int)dprop(env, S, "r_test", 0x22);
    p.tol_bnd = dprop(env, S, "tol_bnd", 1e-7);
    p.tol_dj = dprop(env, S, "tol_dj", 1e-7);
    p.tol_piv = dprop(env, S, "tol_piv", 1e-10);
    p.obj_ll = dprop(env, S, "obj_ll", -1.7976931348623157e308);
    p.obj_ul = dprop(env, S, "obj_ul", +1.7976931348623157e308);
    p.it_lim = (int)dprop(env, S, "it_lim", 2147483647.0);
    p.tm_lim = (int)dprop(env, S, "tm_lim", 2147483647.0);
    p.out_frq = (int)dprop(env, S, "out_frq", 500);
    p.out_dly = (int)dprop(env, S, "out_dly", 0);
    p.presolve = (int)dprop(env, S, "presolve", 0);
    rpt_buf rb = {NULL, 0, 0};
    gk_bfd_set_report(b, rpt_collect, &rb);
    int ret = dual ? gk_spx_dual(c, &lp, b, &p) : gk_spx_primal(c, &lp, b, &p);
    gk_bfd_set_report(b, NULL, NULL);
    if (!set_reports(env, L, &rb)) return NULL;
    if (ret == GK_EABI) return throw_gk(env, dual ? "spx_dual" : "spx_primal");
    set_num(env, L, "it_cnt", lp.it_cnt);
    set_num(env, L, "pbs_stat", lp.pbs_stat);
    set_num(env, L, "dbs_stat", lp.dbs_stat);
    set_num(env, L, "some", lp.some);
    set_num(env, L, "obj_val", lp.obj_val);
    set_num(env, L, "valid", lp.valid);
    return mk_int(env, ret);
}

/* ------------------------------------------------------------- collective */
static void comm_fin(napi_env env, void *data, void *hint)
{
    (void)env; (void)hint;
    if (!g_teardown) gk_comm_destroy((gk_comm *)data);
}

/* commCreate(ctx, rank, size, addr, backend): the library's collective for
 * the sharded branch and bound (gk_comm_create); ctx may be null (TCP) */
static napi_value js_comm_create(napi_env env, napi_callback_info info)
{
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return NULL;
    napi_valuetype t;
    CHECK(napi_typeof(env, argv[0], &t));
    gk_ctx *c = (t == napi_external) ? (gk_ctx *)get_ext(env, argv[0]) : NULL;
    int rank = 0, size = 1, backend = 0;
    CHECK(napi_get_value_int32(env, argv[1], &rank));
    CHECK(napi_get_value_int32(env, argv[2], &size));
    CHECK(napi_get_value_int32(env, argv[4], &backend));
    char addr[256];
    size_t len = 0;
    CHECK(napi_get_value_string_utf8(env, argv[3], addr, sizeof addr, &len));
    gk_comm *m = gk_comm_create(c, rank, size, addr, backend);
    if (!m) return throw_gk(env, "gk_comm_create");
    napi_value r;
    CHECK(napi_create_external(env, m, comm_fin, NULL, &r));
    return r;
}

static napi_value js_comm_backend(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    return mk_int(env, gk_comm_backend((gk_comm *)get_ext(env, argv[0])));
}

/* commOption(comm, opt, value): gk_comm_set_option */
static napi_value js_comm_option(napi_env env, napi_callback_info info)
{
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    int opt = 0, v = 0;
    CHECK(napi_get_value_int32(env, argv[1], &opt));
    CHECK(napi_get_value_int32(env, argv[2], &v));
    return mk_int(env, gk_comm_set_option((gk_comm *)get_ext(env, argv[0]), opt, v));
}

/* bfdSetComm(bfd, comm | null): column-sharded pricing of the dual simplex
 * on this factor (gk_bfd_set_comm) */
static napi_value js_bfd_set_comm(napi_env env, napi_callback_info info)
{
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    napi_valuetype t;
    CHECK(napi_typeof(env, argv[1], &t));
    gk_comm *comm = (t == napi_external) ? (gk_comm *)get_ext(env, argv[1]) : NULL;
    if (gk_bfd_set_comm((gk_bfd *)get_ext(env, argv[0]), comm) != 0) return throw_gk(env, "gk_bfd_set_comm");
    return mk_int(env, 0);
}

/* -------------------------------------------------------------- ios_driver */
/* ios(ctx, L, iocp): L = the marshalled root problem (solved to optimality,
 * pbs_stat/dbs_stat/obj_val set) plus col_kind (Int8Array [1..n]) and the
 * outputs row_mipx / col_mipx (Float64Array); sets L.mip_stat, L.mip_obj,
 * L.lp_solves; returns the ios_driver code (0 or GLP_ETMLIM) */
static napi_value js_ios(napi_env env, napi_callback_info info)
{
    /* ios(ctx, L, iocp[, comm]): with a communicator of more than one rank
     * the search is sharded over the ranks (gk_ios_driver_comm) */
    napi_value argv[4];
    size_t argc = 4;
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 3) {
        napi_throw_type_error(env, NULL, "ios: (ctx, L, iocp[, comm]) expected");
        return NULL;
    }
    gk_comm *comm = NULL;
    if (argc >= 4) {
        napi_valuetype t;
        CHECK(napi_typeof(env, argv[3], &t));
        if (t == napi_external) comm = (gk_comm *)get_ext(env, argv[3]);
    }
    gk_ctx *c = (gk_ctx *)get_ext(env, argv[0]);
    napi_value L = argv[1], I = argv[2];
    gk_mip mip;
    memset(&mip, 0, sizeof mip);
    if (!fill_lp(env, L, &mip.lp)) return NULL;
    mip.lp.pbs_stat = (int)dprop(env, L, "pbs_stat", 0);
    mip.lp.dbs_stat = (int)dprop(env, L, "dbs_stat", 0);
    mip.lp.obj_val = dprop(env, L, "obj_val", 0.0);
    mip.col_kind = (const signed char *)tprop(env, L, "col_kind");
    mip.row_mipx = (double *)tprop(env, L, "row_mipx");
    mip.col_mipx = (double *)tprop(env, L, "col_mipx");
    if (!mip.col_kind || !mip.row_mipx || !mip.col_mipx) {
        napi_throw_type_error(env, NULL, "ios: col_kind / row_mipx / col_mipx missing or not typed arrays");
        return NULL;
    }
    gk_iocp p;
    p.msg_lev = (int)dprop(env, I, "msg_lev", 3);
    p.br_tech = (int)dprop(env, I, "br_tech", 4);
    p.bt_tech = (int)dprop(env, I, "bt_tech", 4);
    p.tol_int = dprop(env, I, "tol_int", 1e-5);
    p.tol_obj = dprop(env, I, "tol_obj", 1e-7);
    p.tm_lim = (int)dprop(env, I, "tm_lim", 2147483647.0);
    p.out_frq = (int)dprop(env, I, "out_frq", 5000);
    p.out_dly = (int)dprop(env, I, "out_dly", 10000);
    p.pp_tech = (int)dprop(env, I, "pp_tech", 2);
    p.mip_gap = dprop(env, I, "mip_gap", 0.0);
    p.presolve = (int)dprop(env, I, "presolve", 0);
    rpt_buf rb = {NULL, 0, 0};
    gk_ios_set_report(c, rpt_collect, &rb);         /* show_progress lines (glpios03.js:2-48) */
    int ret = comm ? gk_ios_driver_comm(c, &mip, &p, comm) : gk_ios_driver(c, &mip, &p);
    gk_ios_set_report(c, NULL, NULL);
    if (!set_reports(env, L, &rb)) return NULL;
    if (ret == GK_EABI) return throw_gk(env, "ios_driver");
    set_num(env, L, "mip_stat", mip.mip_stat);
    set_num(env, L, "mip_obj", mip.mip_obj);
    set_num(env, L, "lp_solves", (double)mip.lp_solves);
    return mk_int(env, ret);
}

static napi_value js_stats(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    gk_spx_stats st;
    memset(&st, 0, sizeof st);
    gk_bfd_last_stats((gk_bfd *)get_ext(env, argv[0]), &st);
    napi_value o;
    CHECK(napi_create_object(env, &o));
    set_num(env, o, "pivots", (double)st.pivots);
    set_num(env, o, "reinversions", (double)st.reinversions);
    set_num(env, o, "batches", (double)st.batches);
    set_num(env, o, "seconds_total", st.seconds_total);
    set_num(env, o, "bytes_pivots", st.bytes_pivots);
    set_num(env, o, "panel_hits", (double)st.panel_hits);
    set_num(env, o, "panel_refills", (double)st.panel_refills);
    set_num(env, o, "factor_sparse", (double)st.factor_sparse);
    set_num(env, o, "seconds_lu", st.seconds_lu);
    set_num(env, o, "shard_exchanges", (double)st.shard_exchanges);
    return o;
}

/* scale(ctx, m, n, ptr, ind, val, flags, rii, sjj, report) -> 0 | 1 (bad flags) */
static napi_value js_scale(napi_env env, napi_callback_info info)
{
    napi_value argv[10];
    if (!get_args(env, info, 10, argv)) return NULL;
    gk_ctx *c = (gk_ctx *)get_ext(env, argv[0]);
    int m = 0, n = 0, flags = 0;
    CHECK(napi_get_value_int32(env, argv[1], &m));
    CHECK(napi_get_value_int32(env, argv[2], &n));
    CHECK(napi_get_value_int32(env, argv[6], &flags));
    const int *ptr = (const int *)ta(env, argv[3]);
    const int *ind = (const int *)ta(env, argv[4]);
    const double *val = (const double *)ta(env, argv[5]);
    double *rii = (double *)ta(env, argv[7]), *sjj = (double *)ta(env, argv[8]), *rep = (double *)ta(env, argv[9]);
    if (!c || !ptr || !ind || !val || !rii || !sjj || !rep) {
        napi_throw_type_error(env, NULL, "scale: ptr/ind Int32Array, val/rii/sjj/report Float64Array");
        return NULL;
    }
    int ret = gk_scale_prob(c, m, n, ptr, ind, val, flags, rii, sjj, rep);
    if (ret == GK_EABI) return throw_gk(env, "scale_prob");
    return mk_int(env, ret);
}

/* advBasis(m, n, row_type, row_lb, row_ub, col_type, col_lb, col_ub, ptr, ind,
 *           row_stat, col_stat) -> size of the triangular part; types and
 * statuses Int8Array [1..], bounds Float64Array [1..], ptr / ind Int32Array
 * (1-based positions, list order).  Host code: no context. */
static napi_value js_adv_basis(napi_env env, napi_callback_info info)
{
    napi_value argv[12];
    if (!get_args(env, info, 12, argv)) return NULL;
    gk_lp L;
    memset(&L, 0, sizeof L);
    CHECK(napi_get_value_int32(env, argv[0], &L.m));
    CHECK(napi_get_value_int32(env, argv[1], &L.n));
    L.row_type = (const signed char *)ta(env, argv[2]);
    L.row_lb = (const double *)ta(env, argv[3]);
    L.row_ub = (const double *)ta(env, argv[4]);
    L.col_type = (const signed char *)ta(env, argv[5]);
    L.col_lb = (const double *)ta(env, argv[6]);
    L.col_ub = (const double *)ta(env, argv[7]);
    L.A_ptr = (const int *)ta(env, argv[8]);
    L.A_ind = (const int *)ta(env, argv[9]);
    L.row_stat = (signed char *)ta(env, argv[10]);
    L.col_stat = (signed char *)ta(env, argv[11]);
    if (!L.row_type || !L.row_lb || !L.row_ub || !L.col_type || !L.col_lb || !L.col_ub || !L.A_ptr || !L.A_ind ||
        !L.row_stat || !L.col_stat) {
        napi_throw_type_error(env, NULL, "advBasis: typed arrays expected");
        return NULL;
    }
    int ret = gk_adv_basis(&L);
    if (ret == GK_EABI) return throw_gk(env, "adv_basis");
    return mk_int(env, ret);
}

// evalTabRows(bfd, L, ks Int32Array, out Float64Array (nk * (m + n)), flags):
// gk_bfd_eval_tab_rows (glp_eval_tab_row for a batch, glpapi12.js:401)
static napi_value js_eval_tab_rows(napi_env env, napi_callback_info info)
{
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return NULL;
    gk_bfd *b = (gk_bfd *)get_ext(env, argv[0]);
    gk_lp lp;
    if (!fill_lp(env, argv[1], &lp)) return NULL;
    size_t nk = 0, nout = 0;
    const int *ks = (const int *)ta_len(env, argv[2], &nk);
    double *out = (double *)ta_len(env, argv[3], &nout);
    int flags = 0;
    CHECK(napi_get_value_int32(env, argv[4], &flags));
    if (!ks || !out || nout < nk * (size_t)(lp.m + lp.n)) {
        napi_throw_type_error(env, NULL, "evalTabRows: Int32Array ks and Float64Array nk * (m + n) expected");
        return NULL;
    }
    if (gk_bfd_eval_tab_rows(b, &lp, (int)nk, ks, out, flags) == GK_EABI) return throw_gk(env, "eval_tab_rows");
    return mk_int(env, 0);
}

/* ------------------------------------------------------------- presolver */
/* npp*: the LP / MIP preprocessor (gk_npp_*, glpnpp01.js .. glpnpp05.js);
 * host code, no context.  The JS side (js/gk_core.js npp*, js/gk_shim.js)
 * rebinds the reference's npp_* entry points to these.  A workspace is a
 * small integer (an index into npp_tab), freed by nppFree when the JS side is
 * done with it and at environment teardown otherwise: no external with a
 * finalizer (libnode 12 runs those during its own teardown and can fault
 * there) */
static gk_npp **npp_tab = NULL;
static int npp_cap = 0;

static void npp_free_all(void)
{
    for (int k = 0; k < npp_cap; k++)
        if (npp_tab[k]) {
            gk_npp_destroy(npp_tab[k]);
            npp_tab[k] = NULL;
        }
}

static gk_npp *npp_get(napi_env env, napi_value v)
{
    int k = -1;
    if (napi_get_value_int32(env, v, &k) != napi_ok || k < 0 || k >= npp_cap || !npp_tab[k]) {
        napi_throw_error(env, NULL, "gk_addon: invalid preprocessor workspace");
        return NULL;
    }
    return npp_tab[k];
}

static napi_value js_npp_create(napi_env env, napi_callback_info info)
{
    (void)info;
    int k = 0;
    while (k < npp_cap && npp_tab[k]) k++;
    if (k == npp_cap) {
        int cap = npp_cap ? 2 * npp_cap : 16;
        gk_npp **t = (gk_npp **)realloc(npp_tab, (size_t)cap * sizeof *t);
        if (!t) {
            napi_throw_error(env, NULL, "gk_addon: out of memory");
            return NULL;
        }
        for (int q = npp_cap; q < cap; q++) t[q] = NULL;
        npp_tab = t;
        npp_cap = cap;
    }
    gk_npp *w = gk_npp_create();
    if (!w) return throw_gk(env, "npp_create_wksp");
    npp_tab[k] = w;
    return mk_int(env, k);
}

static napi_value js_npp_free(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    int k = -1;
    CHECK(napi_get_value_int32(env, argv[0], &k));
    if (k >= 0 && k < npp_cap && npp_tab[k]) {
        gk_npp_destroy(npp_tab[k]);
        npp_tab[k] = NULL;
    }
    return mk_int(env, 0);
}

static int npp_ret(napi_env env, int ret, const char *what, napi_value *out)
{
    if (ret == GK_EABI) {
        throw_gk(env, what);
        return 0;
    }
    *out = mk_int(env, ret);
    return 1;
}

/* nppLoad(npp, L, kind Int8Array | null, sol) */
static napi_value js_npp_load(napi_env env, napi_callback_info info)
{
    napi_value argv[4], r;
    if (!get_args(env, info, 4, argv)) return NULL;
    gk_lp lp;
    if (!fill_lp(env, argv[1], &lp)) return NULL;
    int sol = 0;
    CHECK(napi_get_value_int32(env, argv[3], &sol));
    const signed char *kind = (const signed char *)ta(env, argv[2]);
    return npp_ret(env, gk_npp_load(npp_get(env, argv[0]), &lp, kind, sol), "npp_load_prob", &r) ? r : NULL;
}

static napi_value js_npp_simplex(napi_env env, napi_callback_info info)
{
    napi_value argv[1], r;
    if (!get_args(env, info, 1, argv)) return NULL;
    return npp_ret(env, gk_npp_simplex(npp_get(env, argv[0])), "npp_simplex", &r) ? r : NULL;
}

/* nppInteger(npp, binarize, msg Int32Array(7)) */
static napi_value js_npp_integer(napi_env env, napi_callback_info info)
{
    napi_value argv[3], r;
    if (!get_args(env, info, 3, argv)) return NULL;
    int bin = 0;
    CHECK(napi_get_value_int32(env, argv[1], &bin));
    int *msg = (int *)ta(env, argv[2]);
    return npp_ret(env, gk_npp_integer(npp_get(env, argv[0]), bin, msg), "npp_integer", &r) ? r : NULL;
}

/* nppBuildSize(npp, out Int32Array(3)) -> m, n, nnz in out */
static napi_value js_npp_build_size(napi_env env, napi_callback_info info)
{
    napi_value argv[2], r;
    if (!get_args(env, info, 2, argv)) return NULL;
    int *o = (int *)ta(env, argv[1]);
    if (!o) {
        napi_throw_type_error(env, NULL, "nppBuildSize: Int32Array(3) expected");
        return NULL;
    }
    return npp_ret(env, gk_npp_build_size(npp_get(env, argv[0]), &o[0], &o[1], &o[2]), "npp_build_prob",
                   &r) ? r : NULL;
}

/* nppBuild(npp, row_type, row_lb, row_ub, col_type, col_lb, col_ub, col_coef,
 *          col_kind, A_ptr, A_ind, A_val, row_ref, col_ref, c0 Float64Array(1)) */
static napi_value js_npp_build(napi_env env, napi_callback_info info)
{
    napi_value argv[15], r;
    if (!get_args(env, info, 15, argv)) return NULL;
    void *a[15];
    for (int k = 1; k < 15; k++) {
        a[k] = ta(env, argv[k]);
        if (!a[k]) {
            napi_throw_type_error(env, NULL, "nppBuild: typed arrays expected");
            return NULL;
        }
    }
    int ret = gk_npp_build(npp_get(env, argv[0]), (signed char *)a[1], (double *)a[2], (double *)a[3],
                           (signed char *)a[4], (double *)a[5], (double *)a[6], (double *)a[7], (signed char *)a[8],
                           (int *)a[9], (int *)a[10], (double *)a[11], (int *)a[12], (int *)a[13], (double *)a[14]);
    return npp_ret(env, ret, "npp_build_prob", &r) ? r : NULL;
}

/* nppPostprocess(npp, stat1, stat2, row_stat, row_dual, col_stat, col_prim)
 * (the first three arrays null for a MIP solution; col_prim = mipx) */
static napi_value js_npp_postprocess(napi_env env, napi_callback_info info)
{
    napi_value argv[7], r;
    if (!get_args(env, info, 7, argv)) return NULL;
    int s1 = 0, s2 = 0;
    CHECK(napi_get_value_int32(env, argv[1], &s1));
    CHECK(napi_get_value_int32(env, argv[2], &s2));
    int ret = gk_npp_postprocess(npp_get(env, argv[0]), s1, s2, (const signed char *)ta(env, argv[3]),
                                 (const double *)ta(env, argv[4]), (const signed char *)ta(env, argv[5]),
                                 (const double *)ta(env, argv[6]));
    return npp_ret(env, ret, "npp_postprocess", &r) ? r : NULL;
}

/* nppUnloadSol(npp, L): statuses and values into L's arrays; L.pbs_stat,
 * L.dbs_stat, L.obj_val */
static napi_value js_npp_unload_sol(napi_env env, napi_callback_info info)
{
    napi_value argv[2], r;
    if (!get_args(env, info, 2, argv)) return NULL;
    gk_lp lp;
    if (!fill_lp(env, argv[1], &lp)) return NULL;
    if (!npp_ret(env, gk_npp_unload_sol(npp_get(env, argv[0]), &lp), "npp_unload_sol", &r)) return NULL;
    set_num(env, argv[1], "pbs_stat", lp.pbs_stat);
    set_num(env, argv[1], "dbs_stat", lp.dbs_stat);
    set_num(env, argv[1], "obj_val", lp.obj_val);
    return r;
}

/* nppUnloadMip(npp, L, kind, row_mipx, col_mipx): L.mip_stat, L.mip_obj */
static napi_value js_npp_unload_mip(napi_env env, napi_callback_info info)
{
    napi_value argv[5], r;
    if (!get_args(env, info, 5, argv)) return NULL;
    gk_lp lp;
    if (!fill_lp(env, argv[1], &lp)) return NULL;
    int st = 0;
    double obj = 0.0;
    int ret = gk_npp_unload_mip(npp_get(env, argv[0]), &lp, (const signed char *)ta(env, argv[2]),
                                (double *)ta(env, argv[3]), (double *)ta(env, argv[4]), &st, &obj);
    if (!npp_ret(env, ret, "npp_unload_sol", &r)) return NULL;
    set_num(env, argv[1], "mip_stat", st);
    set_num(env, argv[1], "mip_obj", obj);
    return r;
}

/* exitNow(code): the process leaves with code from node's 'exit' event, before
 * the environment teardown.  libnode 12 (the node of this image) runs the
 * second-pass phantom callbacks of N-API references during its teardown and
 * can fault inside them (node::...PendingPhantomCallback::Invoke) once
 * externals with finalizers exist: js/gk_core.js calls this from its 'exit'
 * listener as soon as it has created one.  stdout / stderr are synchronous
 * for files, pipes and terminals on Linux, so nothing written is lost. */
static napi_value js_exit_now(napi_env env, napi_callback_info info)
{
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    int code = 0;
    CHECK(napi_get_value_int32(env, argv[0], &code));
    fflush(stdout);
    fflush(stderr);
    _exit(code);
    return NULL;
}

#define FN(name, f) { name, NULL, f, NULL, NULL, NULL, napi_enumerable, NULL }

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
static void segv_trace(int sig)
{
    void *fr[64];
    int nf = backtrace(fr, 64);
    backtrace_symbols_fd(fr, nf, 2);
    _exit(128 + sig);
}

static napi_value init(napi_env env, napi_value exports)
{
    if (getenv("GK_SEGV_TRACE")) signal(SIGSEGV, segv_trace);
    napi_add_env_cleanup_hook(env, teardown_hook, NULL);
    napi_property_descriptor d[] = {
        FN("commCreate", js_comm_create), FN("commBackend", js_comm_backend), FN("commOption", js_comm_option),
        FN("bfdSetComm", js_bfd_set_comm),
        FN("create", js_create), FN("deviceCount", js_device_count), FN("abiVersion", js_abi_version),
        FN("lastError", js_last_error), FN("bfdCreate", js_bfd_create), FN("bfdSetParm", js_bfd_set_parm), FN("bfdResetParm", js_bfd_reset_parm),
        FN("bfdFactorizeCsc", js_bfd_factorize_csc), FN("bfdFtran", js_bfd_ftran), FN("bfdBtran", js_bfd_btran),
        FN("bfdUpdate", js_bfd_update), FN("bfdGetCount", js_bfd_get_count), FN("bfdValid", js_bfd_valid),
        FN("spx", js_spx), FN("ios", js_ios), FN("stats", js_stats), FN("scale", js_scale),
        FN("advBasis", js_adv_basis), FN("evalTabRows", js_eval_tab_rows),
        FN("nppCreate", js_npp_create), FN("nppLoad", js_npp_load), FN("nppSimplex", js_npp_simplex),
        FN("nppInteger", js_npp_integer), FN("nppBuildSize", js_npp_build_size), FN("nppBuild", js_npp_build),
        FN("nppPostprocess", js_npp_postprocess), FN("nppUnloadSol", js_npp_unload_sol),
        FN("nppUnloadMip", js_npp_unload_mip), FN("nppFree", js_npp_free), FN("exitNow", js_exit_now),
    };
    napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
