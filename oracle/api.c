/* ORACLE (test infrastructure only) — the slice of the problem-object API the
 * hot path needs, plus a flat C interface for the tests (ctypes).
 * Restates glpapi06.js (glp_simplex :1, solve_lp :3, trivial_lp :149,
 * SMCP :359), glpapi12.js (glp_factorize :5 with b_col :7, glp_ftran :198,
 * glp_btran :222, glp_get_bfcp :108, copy_bfcp :127, glp_eval_tab_row :401,
 * glp_dual_rtest :687), glpapi01.js (glp_set_row_bnds :214,
 * glp_set_col_bnds :247) and glpapi05.js (glp_set_row_stat,
 * glp_set_col_stat). */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "orc.h"

jmp_buf *orc_err_jmp = NULL;
char orc_err_msg[512];
orc_trace_fn orc_trace = NULL;
void *orc_trace_ctx = NULL;
long orc_instab_events = 0;
int orc_instab_last_it = -1;

long orc_instab_count(int *last_it)
{
    if (last_it) *last_it = orc_instab_last_it;
    return orc_instab_events;
}

void orc_fail(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(orc_err_msg, sizeof orc_err_msg, fmt, ap);
    va_end(ap);
    if (orc_err_jmp) longjmp(*orc_err_jmp, 1);
    fprintf(stderr, "oracle: %s\n", orc_err_msg);
    abort();
}

void *orc_alloc(size_t n, size_t sz)
{
    void *p = calloc(n ? n : 1, sz);
    if (!p) orc_fail("out of memory (%zu x %zu)", n, sz);
    return p;
}

void orc_free(void *p) { free(p); }

double orc_time(void)          /* xtime() in seconds (glpapi.js:53) */
{
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

void orc_smcp_default(orc_smcp *parm)                    /* glpapi06.js:359 */
{
    parm->msg_lev = GLP_MSG_ALL;
    parm->meth = GLP_PRIMAL;
    parm->pricing = GLP_PT_PSE;
    parm->r_test = GLP_RT_HAR;
    parm->tol_bnd = 1e-7;
    parm->tol_dj = 1e-7;
    parm->tol_piv = 1e-10;
    parm->obj_ll = -DBL_MAX;
    parm->obj_ul = +DBL_MAX;
    parm->it_lim = ORC_INT_MAX;
    parm->tm_lim = ORC_INT_MAX;
    parm->out_frq = 500;
    parm->out_dly = 0;
    parm->presolve = GLP_OFF;
}

int orc_bf_exists(orc_prob *lp) { return lp->m == 0 || lp->valid; }

void orc_get_bfcp(orc_prob *lp, orc_bfcp *parm)           /* glpapi12.js:108 */
{
    if (lp->bfcp == NULL) {
        parm->type = GLP_BF_FT;
        parm->lu_size = 0;
        parm->piv_tol = 0.10;
        parm->piv_lim = 4;
        parm->suhl = GLP_ON;
        parm->eps_tol = 1e-15;
        parm->max_gro = 1e+10;
        parm->nfs_max = 100;
        parm->upd_tol = 1e-6;
        parm->nrs_max = 100;
        parm->rs_size = 0;
    } else
        *parm = *lp->bfcp;
}

static int b_col(void *info, int j, int *ind, double *val)      /* glpapi12.js:7 */
{
    orc_prob *lp = (orc_prob *)info;
    int m = lp->m, k, len, ptr, c;
    ORC_ASSERT(1 <= j && j <= m);
    k = lp->head[j];
    if (k <= m) {
        len = 1; ind[1] = k; val[1] = 1.0;
    } else {
        c = k - m;
        len = 0;
        for (ptr = lp->A_ptr[c]; ptr < lp->A_ptr[c + 1]; ptr++) {
            len++;
            ind[len] = lp->A_ind[ptr];
            val[len] = -lp->rii[lp->A_ind[ptr]] * lp->A_val[ptr] * lp->sjj[c];
        }
    }
    return len;
}

int orc_factorize(orc_prob *lp)                                  /* glpapi12.js:5 */
{
    int m = lp->m, n = lp->n, j, k, stat, ret;
    lp->valid = 0;
    j = 0;
    for (k = 1; k <= m + n; k++) {
        if (k <= m) { stat = lp->row_stat[k]; lp->row_bind[k] = 0; }
        else { stat = lp->col_stat[k - m]; lp->col_bind[k - m] = 0; }
        if (stat == GLP_BS) {
            j++;
            if (j > m) return GLP_EBADB;
            lp->head[j] = k;
            if (k <= m) lp->row_bind[k] = j; else lp->col_bind[k - m] = j;
        }
    }
    if (j < m) return GLP_EBADB;
    if (m > 0) {
        if (lp->bfd == NULL) {
            orc_bfcp parm;
            lp->bfd = bfd_create_it();
            orc_get_bfcp(lp, &parm);
            bfd_set_parm(lp->bfd, &parm);
        }
        ret = bfd_factorize(lp->bfd, m, lp->head, b_col, lp);
        if (ret == BFD_ESING) return GLP_ESING;
        if (ret == BFD_ECOND) return GLP_ECOND;
        ORC_ASSERT(ret == 0);
        lp->valid = 1;
    }
    return 0;
}

void orc_ftran(orc_prob *lp, double *x)                        /* glpapi12.js:198 */
{
    int m = lp->m, i, k;
    if (!(m == 0 || lp->valid)) orc_fail("glp_ftran: basis factorization does not exist");
    for (i = 1; i <= m; i++) x[i] *= lp->rii[i];
    if (m > 0) bfd_ftran(lp->bfd, x);
    for (i = 1; i <= m; i++) {
        k = lp->head[i];
        if (k <= m) x[i] /= lp->rii[k]; else x[i] *= lp->sjj[k - m];
    }
}

void orc_btran(orc_prob *lp, double *x)                        /* glpapi12.js:222 */
{
    int m = lp->m, i, k;
    if (!(m == 0 || lp->valid)) orc_fail("glp_btran: basis factorization does not exist");
    for (i = 1; i <= m; i++) {
        k = lp->head[i];
        if (k <= m) x[i] /= lp->rii[k]; else x[i] *= lp->sjj[k - m];
    }
    if (m > 0) bfd_btran(lp->bfd, x);
    for (i = 1; i <= m; i++) x[i] *= lp->rii[i];
}

/* ---- glpapi01.js / glpapi05.js mutators --------------------------------- */
void orc_set_row_bnds(orc_prob *lp, int i, int type, double lb, double ub)   /* glpapi01.js:214 */
{
    if (!(1 <= i && i <= lp->m)) orc_fail("glp_set_row_bnds: i = %d; row number out of range", i);
    lp->row_type[i] = (signed char)type;
    switch (type) {
    case GLP_FR:
        lp->row_lb[i] = lp->row_ub[i] = 0.0;
        if (lp->row_stat[i] != GLP_BS) lp->row_stat[i] = GLP_NF;
        break;
    case GLP_LO:
        lp->row_lb[i] = lb; lp->row_ub[i] = 0.0;
        if (lp->row_stat[i] != GLP_BS) lp->row_stat[i] = GLP_NL;
        break;
    case GLP_UP:
        lp->row_lb[i] = 0.0; lp->row_ub[i] = ub;
        if (lp->row_stat[i] != GLP_BS) lp->row_stat[i] = GLP_NU;
        break;
    case GLP_DB:
        lp->row_lb[i] = lb; lp->row_ub[i] = ub;
        if (!(lp->row_stat[i] == GLP_BS || lp->row_stat[i] == GLP_NL || lp->row_stat[i] == GLP_NU))
            lp->row_stat[i] = (fabs(lb) <= fabs(ub) ? GLP_NL : GLP_NU);
        break;
    case GLP_FX:
        lp->row_lb[i] = lp->row_ub[i] = lb;
        if (lp->row_stat[i] != GLP_BS) lp->row_stat[i] = GLP_NS;
        break;
    default:
        orc_fail("glp_set_row_bnds: i = %d; type = %d; invalid row type", i, type);
    }
}

void orc_set_col_bnds(orc_prob *lp, int j, int type, double lb, double ub)   /* glpapi01.js:247 */
{
    if (!(1 <= j && j <= lp->n)) orc_fail("glp_set_col_bnds: j = %d; column number out of range", j);
    lp->col_type[j] = (signed char)type;
    switch (type) {
    case GLP_FR:
        lp->col_lb[j] = lp->col_ub[j] = 0.0;
        if (lp->col_stat[j] != GLP_BS) lp->col_stat[j] = GLP_NF;
        break;
    case GLP_LO:
        lp->col_lb[j] = lb; lp->col_ub[j] = 0.0;
        if (lp->col_stat[j] != GLP_BS) lp->col_stat[j] = GLP_NL;
        break;
    case GLP_UP:
        lp->col_lb[j] = 0.0; lp->col_ub[j] = ub;
        if (lp->col_stat[j] != GLP_BS) lp->col_stat[j] = GLP_NU;
        break;
    case GLP_DB:
        lp->col_lb[j] = lb; lp->col_ub[j] = ub;
        if (!(lp->col_stat[j] == GLP_BS || lp->col_stat[j] == GLP_NL || lp->col_stat[j] == GLP_NU))
            lp->col_stat[j] = (fabs(lb) <= fabs(ub) ? GLP_NL : GLP_NU);
        break;
    case GLP_FX:
        lp->col_lb[j] = lp->col_ub[j] = lb;
        if (lp->col_stat[j] != GLP_BS) lp->col_stat[j] = GLP_NS;
        break;
    default:
        orc_fail("glp_set_col_bnds: j = %d; type = %d; invalid column type", j, type);
    }
}

void orc_set_row_stat(orc_prob *lp, int i, int stat)              /* glpapi05.js */
{
    if (!(1 <= i && i <= lp->m)) orc_fail("glp_set_row_stat: i = %d; row number out of range", i);
    if (!(stat == GLP_BS || stat == GLP_NL || stat == GLP_NU || stat == GLP_NF || stat == GLP_NS))
        orc_fail("glp_set_row_stat: i = %d; stat = %d; invalid status", i, stat);
    if (stat != GLP_BS) {
        switch (lp->row_type[i]) {
        case GLP_FR: stat = GLP_NF; break;
        case GLP_LO: stat = GLP_NL; break;
        case GLP_UP: stat = GLP_NU; break;
        case GLP_DB: if (stat != GLP_NU) stat = GLP_NL; break;
        case GLP_FX: stat = GLP_NS; break;
        default: ORC_ASSERT(0);
        }
    }
    if ((lp->row_stat[i] == GLP_BS && stat != GLP_BS) || (lp->row_stat[i] != GLP_BS && stat == GLP_BS))
        lp->valid = 0;
    lp->row_stat[i] = (signed char)stat;
}

void orc_set_col_stat(orc_prob *lp, int j, int stat)              /* glpapi05.js */
{
    if (!(1 <= j && j <= lp->n)) orc_fail("glp_set_col_stat: j = %d; column number out of range", j);
    if (!(stat == GLP_BS || stat == GLP_NL || stat == GLP_NU || stat == GLP_NF || stat == GLP_NS))
        orc_fail("glp_set_col_stat: j = %d; stat = %d; invalid status", j, stat);
    if (stat != GLP_BS) {
        switch (lp->col_type[j]) {
        case GLP_FR: stat = GLP_NF; break;
        case GLP_LO: stat = GLP_NL; break;
        case GLP_UP: stat = GLP_NU; break;
        case GLP_DB: if (stat != GLP_NU) stat = GLP_NL; break;
        case GLP_FX: stat = GLP_NS; break;
        default: ORC_ASSERT(0);
        }
    }
    if ((lp->col_stat[j] == GLP_BS && stat != GLP_BS) || (lp->col_stat[j] != GLP_BS && stat == GLP_BS))
        lp->valid = 0;
    lp->col_stat[j] = (signed char)stat;
}

/* ---- glpapi06.js --------------------------------------------------------- */
static int solve_lp(orc_prob *P, const orc_smcp *parm)             /* :3 */
{
    int ret;
    if (!orc_bf_exists(P)) {
        ret = orc_factorize(P);
        if (ret != 0) return ret;
    }
    if (parm->meth == GLP_PRIMAL)
        ret = spx_primal(P, parm);
    else if (parm->meth == GLP_DUALP) {
        ret = spx_dual(P, parm);
        if (ret == GLP_EFAIL && P->valid) ret = spx_primal(P, parm);
    } else if (parm->meth == GLP_DUAL)
        ret = spx_dual(P, parm);
    else
        ORC_ASSERT(0);
    return ret;
}

static void trivial_lp(orc_prob *P, const orc_smcp *parm)           /* :149 */
{
    int i, j;
    double zeta;
    P->valid = 0;
    P->pbs_stat = P->dbs_stat = GLP_FEAS;
    P->obj_val = P->c0;
    P->some = 0;
    for (i = 1; i <= P->m; i++) {
        int t = P->row_type[i];
        P->row_stat[i] = GLP_BS;
        P->row_prim[i] = P->row_dual[i] = 0.0;
        if (t == GLP_LO || t == GLP_DB || t == GLP_FX) {
            if (P->row_lb[i] > +parm->tol_bnd) {
                P->pbs_stat = GLP_NOFEAS;
                if (P->some == 0 && parm->meth != GLP_PRIMAL) P->some = i;
            }
        }
        if (t == GLP_UP || t == GLP_DB || t == GLP_FX) {
            if (P->row_ub[i] < -parm->tol_bnd) {
                P->pbs_stat = GLP_NOFEAS;
                if (P->some == 0 && parm->meth != GLP_PRIMAL) P->some = i;
            }
        }
    }
    zeta = 1.0;
    for (j = 1; j <= P->n; j++)
        if (zeta < fabs(P->col_coef[j])) zeta = fabs(P->col_coef[j]);
    zeta = (P->dir == GLP_MIN ? +1.0 : -1.0) / zeta;
    for (j = 1; j <= P->n; j++) {
        int t = P->col_type[j];
        double coef = P->col_coef[j], dual;
        if (t == GLP_FR) { P->col_stat[j] = GLP_NF; P->col_prim[j] = 0.0; }
        else if (t == GLP_LO) { P->col_stat[j] = GLP_NL; P->col_prim[j] = P->col_lb[j]; }
        else if (t == GLP_UP) { P->col_stat[j] = GLP_NU; P->col_prim[j] = P->col_ub[j]; }
        else if (t == GLP_DB) {
            if (zeta * coef > 0.0) { P->col_stat[j] = GLP_NL; P->col_prim[j] = P->col_lb[j]; }
            else if (zeta * coef < 0.0) { P->col_stat[j] = GLP_NU; P->col_prim[j] = P->col_ub[j]; }
            else if (fabs(P->col_lb[j]) <= fabs(P->col_ub[j])) { P->col_stat[j] = GLP_NL; P->col_prim[j] = P->col_lb[j]; }
            else { P->col_stat[j] = GLP_NU; P->col_prim[j] = P->col_ub[j]; }
        } else if (t == GLP_FX) { P->col_stat[j] = GLP_NS; P->col_prim[j] = P->col_lb[j]; }
        dual = P->col_dual[j] = coef;
        P->obj_val += coef * P->col_prim[j];
        if (t == GLP_FR || t == GLP_LO) {
            if (zeta * dual < -parm->tol_dj) {
                P->dbs_stat = GLP_NOFEAS;
                if (P->some == 0 && parm->meth == GLP_PRIMAL) P->some = P->m + j;
            }
        }
        if (t == GLP_FR || t == GLP_UP) {
            if (zeta * dual > +parm->tol_dj) {
                P->dbs_stat = GLP_NOFEAS;
                if (P->some == 0 && parm->meth == GLP_PRIMAL) P->some = P->m + j;
            }
        }
    }
}

int orc_simplex(orc_prob *P, const orc_smcp *parm)                    /* :1 */
{
    int i, j, ret = 0;
    if (P->tree != NULL) { /* glp_simplex is allowed only outside callbacks (:265) */ }
    if (!(parm->msg_lev == GLP_MSG_OFF || parm->msg_lev == GLP_MSG_ERR || parm->msg_lev == GLP_MSG_ON ||
          parm->msg_lev == GLP_MSG_ALL || parm->msg_lev == GLP_MSG_DBG))
        orc_fail("glp_simplex: msg_lev = %d; invalid parameter", parm->msg_lev);
    if (!(parm->meth == GLP_PRIMAL || parm->meth == GLP_DUALP || parm->meth == GLP_DUAL))
        orc_fail("glp_simplex: meth = %d; invalid parameter", parm->meth);
    if (!(parm->pricing == GLP_PT_STD || parm->pricing == GLP_PT_PSE))
        orc_fail("glp_simplex: pricing = %d; invalid parameter", parm->pricing);
    if (!(parm->r_test == GLP_RT_STD || parm->r_test == GLP_RT_HAR))
        orc_fail("glp_simplex: r_test = %d; invalid parameter", parm->r_test);
    if (!(0.0 < parm->tol_bnd && parm->tol_bnd < 1.0)) orc_fail("glp_simplex: tol_bnd = %g; invalid parameter", parm->tol_bnd);
    if (!(0.0 < parm->tol_dj && parm->tol_dj < 1.0)) orc_fail("glp_simplex: tol_dj = %g; invalid parameter", parm->tol_dj);
    if (!(0.0 < parm->tol_piv && parm->tol_piv < 1.0)) orc_fail("glp_simplex: tol_piv = %g; invalid parameter", parm->tol_piv);
    if (parm->it_lim < 0) orc_fail("glp_simplex: it_lim = %d; invalid parameter", parm->it_lim);
    if (parm->tm_lim < 0) orc_fail("glp_simplex: tm_lim = %d; invalid parameter", parm->tm_lim);
    if (parm->out_frq < 1) orc_fail("glp_simplex: out_frq = %d; invalid parameter", parm->out_frq);
    if (parm->out_dly < 0) orc_fail("glp_simplex: out_dly = %d; invalid parameter", parm->out_dly);
    if (!(parm->presolve == GLP_ON || parm->presolve == GLP_OFF))
        orc_fail("glp_simplex: presolve = %d; invalid parameter", parm->presolve);
    P->pbs_stat = P->dbs_stat = GLP_UNDEF;
    P->obj_val = 0.0;
    P->some = 0;
    for (i = 1; i <= P->m; i++)
        if (P->row_type[i] == GLP_DB && P->row_lb[i] >= P->row_ub[i]) return GLP_EBOUND;
    for (j = 1; j <= P->n; j++)
        if (P->col_type[j] == GLP_DB && P->col_lb[j] >= P->col_ub[j]) return GLP_EBOUND;
    if (P->nnz == 0) {
        trivial_lp(P, parm);
        ret = 0;
    } else if (!parm->presolve)
        ret = solve_lp(P, parm);
    else
        orc_fail("glp_simplex: presolve is outside the oracle's scope");
    return ret;
}

/* ========================================================================
 * Flat interface for the tests (ctypes).  Arrays are 0-based on input;
 * the A matrix is CSC with 0-based column pointers and 1-based row indices
 * in the column-list order of the reference problem object.
 * ====================================================================== */
typedef struct { jmp_buf jb; } orc_guard;

#define GUARD_BEGIN(errval) \
    jmp_buf jb__; jmp_buf *prev__ = orc_err_jmp; \
    if (setjmp(jb__)) { orc_err_jmp = prev__; return errval; } \
    orc_err_jmp = &jb__;
#define GUARD_END() orc_err_jmp = prev__;

const char *orc_last_error(void) { return orc_err_msg; }

orc_prob *orc_prob_create(int m, int n, int dir, double c0,
                          const signed char *row_type, const double *row_lb, const double *row_ub,
                          const double *rii, const signed char *row_stat,
                          const signed char *col_type, const double *col_lb, const double *col_ub,
                          const double *col_coef, const double *sjj, const signed char *col_stat,
                          const signed char *col_kind,
                          const int *A_ptr, const int *A_ind, const double *A_val)
{
    orc_prob *P;
    int i, j, k, nnz;
    GUARD_BEGIN(NULL)
    P = (orc_prob *)orc_alloc(1, sizeof(orc_prob));
    P->m = m; P->n = n; P->dir = dir; P->c0 = c0;
    P->row_type = (signed char *)orc_alloc((size_t)(1 + m), 1);
    P->row_stat = (signed char *)orc_alloc((size_t)(1 + m), 1);
    P->row_lb = (double *)orc_alloc((size_t)(1 + m), sizeof(double));
    P->row_ub = (double *)orc_alloc((size_t)(1 + m), sizeof(double));
    P->rii = (double *)orc_alloc((size_t)(1 + m), sizeof(double));
    P->row_bind = (int *)orc_alloc((size_t)(1 + m), sizeof(int));
    P->row_prim = (double *)orc_alloc((size_t)(1 + m), sizeof(double));
    P->row_dual = (double *)orc_alloc((size_t)(1 + m), sizeof(double));
    P->row_mipx = (double *)orc_alloc((size_t)(1 + m), sizeof(double));
    P->col_type = (signed char *)orc_alloc((size_t)(1 + n), 1);
    P->col_kind = (signed char *)orc_alloc((size_t)(1 + n), 1);
    P->col_stat = (signed char *)orc_alloc((size_t)(1 + n), 1);
    P->col_lb = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    P->col_ub = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    P->col_coef = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    P->sjj = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    P->col_bind = (int *)orc_alloc((size_t)(1 + n), sizeof(int));
    P->col_prim = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    P->col_dual = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    P->col_mipx = (double *)orc_alloc((size_t)(1 + n), sizeof(double));
    for (i = 1; i <= m; i++) {
        P->row_type[i] = row_type[i - 1]; P->row_lb[i] = row_lb[i - 1]; P->row_ub[i] = row_ub[i - 1];
        P->rii[i] = rii ? rii[i - 1] : 1.0; P->row_stat[i] = row_stat ? row_stat[i - 1] : GLP_BS;
    }
    for (j = 1; j <= n; j++) {
        P->col_type[j] = col_type[j - 1]; P->col_lb[j] = col_lb[j - 1]; P->col_ub[j] = col_ub[j - 1];
        P->col_coef[j] = col_coef[j - 1]; P->sjj[j] = sjj ? sjj[j - 1] : 1.0;
        P->col_stat[j] = col_stat[j - 1]; P->col_kind[j] = col_kind ? col_kind[j - 1] : GLP_CV;
    }
    nnz = A_ptr[n];
    P->nnz = nnz;
    P->A_ptr = (int *)orc_alloc((size_t)(n + 2), sizeof(int));
    P->A_ind = (int *)orc_alloc((size_t)(nnz + 1), sizeof(int));
    P->A_val = (double *)orc_alloc((size_t)(nnz + 1), sizeof(double));
    for (j = 1; j <= n + 1; j++) P->A_ptr[j] = A_ptr[j - 1] + 1;
    for (k = 1; k <= nnz; k++) { P->A_ind[k] = A_ind[k - 1]; P->A_val[k] = A_val[k - 1]; }
    /* rows (any order within a row; see spx_dual.c eval_trow2) */
    P->AT_ptr = (int *)orc_alloc((size_t)(m + 2), sizeof(int));
    P->AT_ind = (int *)orc_alloc((size_t)(nnz + 1), sizeof(int));
    P->AT_val = (double *)orc_alloc((size_t)(nnz + 1), sizeof(double));
    {
        int *cnt = (int *)orc_alloc((size_t)(m + 2), sizeof(int));
        for (k = 1; k <= nnz; k++) cnt[P->A_ind[k]]++;
        P->AT_ptr[1] = 1;
        for (i = 1; i <= m; i++) P->AT_ptr[i + 1] = P->AT_ptr[i] + cnt[i];
        for (i = 1; i <= m; i++) cnt[i] = P->AT_ptr[i];
        for (j = 1; j <= n; j++)
            for (k = P->A_ptr[j]; k < P->A_ptr[j + 1]; k++) {
                int pos = cnt[P->A_ind[k]]++;
                P->AT_ind[pos] = j; P->AT_val[pos] = P->A_val[k];
            }
        orc_free(cnt);
    }
    P->head = (int *)orc_alloc((size_t)(1 + m + n), sizeof(int));
    P->valid = 0; P->bfd = NULL; P->bfcp = NULL;
    P->pbs_stat = P->dbs_stat = GLP_UNDEF;
    P->mip_stat = GLP_UNDEF;
    GUARD_END()
    return P;
}

void orc_prob_delete(orc_prob *P)
{
    if (!P) return;
    bfd_delete_it(P->bfd);
    orc_free(P->bfcp);
    orc_free(P->row_type); orc_free(P->row_stat); orc_free(P->row_lb); orc_free(P->row_ub); orc_free(P->rii);
    orc_free(P->row_bind); orc_free(P->row_prim); orc_free(P->row_dual); orc_free(P->row_mipx);
    orc_free(P->col_type); orc_free(P->col_kind); orc_free(P->col_stat); orc_free(P->col_lb); orc_free(P->col_ub);
    orc_free(P->col_coef); orc_free(P->sjj); orc_free(P->col_bind); orc_free(P->col_prim); orc_free(P->col_dual);
    orc_free(P->col_mipx);
    orc_free(P->A_ptr); orc_free(P->A_ind); orc_free(P->A_val);
    orc_free(P->AT_ptr); orc_free(P->AT_ind); orc_free(P->AT_val);
    orc_free(P->head);
    orc_free(P);
}

void orc_prob_set_bfcp(orc_prob *P, int type, int nfs_max, int nrs_max)
{
    /* glp_set_bfcp (glpapi12.js:133) with defaults except the given fields */
    if (P->bfcp == NULL) {
        P->bfcp = (orc_bfcp *)orc_alloc(1, sizeof(orc_bfcp));
        orc_get_bfcp(P, P->bfcp);      /* bfcp still NULL inside? no: fill defaults */
    }
    {
        orc_bfcp d; orc_bfcp *save = P->bfcp; P->bfcp = NULL; orc_get_bfcp(P, &d); P->bfcp = save;
        *P->bfcp = d;
    }
    P->bfcp->type = type;
    if (nfs_max > 0) P->bfcp->nfs_max = nfs_max;
    if (nrs_max > 0) P->bfcp->nrs_max = nrs_max;
    if (P->bfcp->rs_size == 0) P->bfcp->rs_size = 20 * P->bfcp->nrs_max;
    if (P->bfd != NULL) bfd_set_parm(P->bfd, P->bfcp);
}

void orc_prob_set_upd_tol(orc_prob *P, double upd_tol)
{
    /* glp_set_bfcp's upd_tol field (glpfhv.js:436-442 uses it), after
     * orc_prob_set_bfcp */
    ORC_ASSERT(P->bfcp != NULL);
    P->bfcp->upd_tol = upd_tol;
    if (P->bfd != NULL) bfd_set_parm(P->bfd, P->bfcp);
}

typedef struct {
    int meth, pricing, r_test, it_lim, tm_lim;
    double tol_bnd, tol_dj, tol_piv, obj_ll, obj_ul;
} orc_smcp_flat;                     /* 0 / 0.0 fields mean "default", as SMCP's || */

static void smcp_from_flat(orc_smcp *parm, const orc_smcp_flat *f)
{
    orc_smcp_default(parm);
    if (!f) return;
    if (f->meth) parm->meth = f->meth;
    if (f->pricing) parm->pricing = f->pricing;
    if (f->r_test) parm->r_test = f->r_test;
    if (f->it_lim) parm->it_lim = f->it_lim;
    if (f->tm_lim) parm->tm_lim = f->tm_lim;
    if (f->tol_bnd != 0.0) parm->tol_bnd = f->tol_bnd;
    if (f->tol_dj != 0.0) parm->tol_dj = f->tol_dj;
    if (f->tol_piv != 0.0) parm->tol_piv = f->tol_piv;
    if (f->obj_ll != 0.0) parm->obj_ll = f->obj_ll;
    if (f->obj_ul != 0.0) parm->obj_ul = f->obj_ul;
}

int orc_prob_simplex(orc_prob *P, const orc_smcp_flat *f, orc_trace_fn tr, void *ctx)
{
    orc_smcp parm;
    int ret;
    GUARD_BEGIN(-1)
    smcp_from_flat(&parm, f);
    orc_trace = tr; orc_trace_ctx = ctx;
    ret = orc_simplex(P, &parm);
    orc_trace = NULL; orc_trace_ctx = NULL;
    GUARD_END()
    return ret;
}

typedef struct {
    int pbs_stat, dbs_stat, some, it_cnt, valid, mip_stat;
    double obj_val, mip_obj;
} orc_result_flat;

void orc_prob_result(orc_prob *P, orc_result_flat *r,
                     signed char *row_stat, double *row_prim, double *row_dual,
                     signed char *col_stat, double *col_prim, double *col_dual,
                     double *row_mipx, double *col_mipx, int *head)
{
    int i, j;
    r->pbs_stat = P->pbs_stat; r->dbs_stat = P->dbs_stat; r->some = P->some; r->it_cnt = P->it_cnt;
    r->valid = P->valid; r->obj_val = P->obj_val; r->mip_stat = P->mip_stat; r->mip_obj = P->mip_obj;
    for (i = 1; i <= P->m; i++) {
        if (row_stat) row_stat[i - 1] = P->row_stat[i];
        if (row_prim) row_prim[i - 1] = P->row_prim[i];
        if (row_dual) row_dual[i - 1] = P->row_dual[i];
        if (row_mipx) row_mipx[i - 1] = P->row_mipx[i];
        if (head) head[i - 1] = P->head[i];
    }
    for (j = 1; j <= P->n; j++) {
        if (col_stat) col_stat[j - 1] = P->col_stat[j];
        if (col_prim) col_prim[j - 1] = P->col_prim[j];
        if (col_dual) col_dual[j - 1] = P->col_dual[j];
        if (col_mipx) col_mipx[j - 1] = P->col_mipx[j];
    }
}

/* factorization API used by tests: glp_factorize + glp_ftran/glp_btran on
 * 0-based vectors */
int orc_prob_factorize(orc_prob *P)
{
    int ret;
    GUARD_BEGIN(-1)
    ret = orc_factorize(P);
    GUARD_END()
    return ret;
}

int orc_prob_ftran(orc_prob *P, double *x0, int tr)
{
    int i, m = P->m;
    double *x = (double *)orc_alloc((size_t)(m + 1), sizeof(double));
    GUARD_BEGIN(-1)
    for (i = 1; i <= m; i++) x[i] = x0[i - 1];
    if (tr) orc_btran(P, x); else orc_ftran(P, x);
    for (i = 1; i <= m; i++) x0[i - 1] = x[i];
    GUARD_END()
    orc_free(x);
    return 0;
}
