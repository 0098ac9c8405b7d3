// gk_shim.js — concatenated into the reference bundle after lib/*.js (see
// js/load_glpk.js).  The bundle is one closure, so assigning to its function
// names rebinds every internal caller:
//   solve_lp (glpapi06.js:27-37)          -> spx_primal / spx_dual
//   glp_factorize / glp_ftran / glp_btran -> bfd_* (glpapi12.js:75-105, 211, 240)
//   npp_* (glpnpp01.js .. glpnpp05.js)    -> gk_npp_* (presolve = GLP_ON)
// Matrix and scale mutators bump lp.__gk_version so the device copy of A is
// re-uploaded only when A or the scaling changed (SURVEY.md §8(b).1).
var __gk = require(__gk_core_path);

spx_primal = function (lp, parm) { return __gk.spx(lp, parm, false, xprintf); };
spx_dual = function (lp, parm) { return __gk.spx(lp, parm, true, xprintf); };
bfd_create_it = function () { return __gk.bfdCreate(); };
bfd_set_parm = function (bfd, parm) { __gk.bfdSetParm(bfd, parm); };
// copy_bfcp (glpapi12.js:127-131, from glp_factorize and glp_set_bfcp): a
// problem with its own bfcp (glp_set_bfcp called with a parm) hands over
// exact values — nfs_max = 100 included; one without hands over the
// defaults, the re-inversion interval then left to the engine
copy_bfcp = function (lp) {
    if (lp.bfcp == null) { __gk.bfdResetParm(lp.bfd); return; }
    var parm = {};
    glp_get_bfcp(lp, parm);
    __gk.bfdSetParm(lp.bfd, parm);
};
bfd_factorize = function (bfd, m, bh, col, info) { return __gk.bfdFactorize(bfd, m, bh, col, info); };
bfd_ftran = function (bfd, x) { __gk.bfdFtran(bfd, x); };
bfd_btran = function (bfd, x) { __gk.bfdBtran(bfd, x); };
bfd_update_it = function (bfd, j, bh, len, ind, idx, val) { return __gk.bfdUpdate(bfd, j, bh, len, ind, idx, val); };
bfd_get_count = function (bfd) { return __gk.bfdGetCount(bfd); };
// ios_driver (glpios03.js:1, called by solve_mip glpapi09.js:79): the native
// batched B&B when the request is one it serves, else the reference's driver
var __gk_js_ios_driver = ios_driver;
ios_driver = function (T) { return __gk.nativeIos(T) ? __gk.iosDriver(T, xprintf) : __gk_js_ios_driver(T); };

// glp_scale_prob (glpscl.js:215-225): the factors from the device, the
// reference's report lines through its own xprintf, the factors stored
// through its own glp_unscale_prob / glp_set_rii / glp_set_sjj (which keep
// the basis-invalidation rules of glpapi04.js:1-28)
glp_scale_prob = exports["glp_scale_prob"] = function (lp, flags) {
    if (flags & ~(GLP_SF_GM | GLP_SF_EQ | GLP_SF_2N | GLP_SF_SKIP | GLP_SF_AUTO))
        xerror("glp_scale_prob: flags = " + flags + "; invalid scaling options");
    var r = __gk.scaleProb(lp, flags), rep = r.report, bits = rep[12], i, j;
    function line(tag, k) {
        xprintf(tag + ": min|aij| = " + rep[3 * k] + "  max|aij| = " + rep[3 * k + 1] + "  ratio = " + rep[3 * k + 2] + "");
    }
    xprintf("Scaling...");
    glp_unscale_prob(lp);
    line(" A", 0);
    if (bits & 1) xprintf("Problem data seem to be well scaled");
    if (!(bits & 16)) {
        if (bits & 2) line("GM", 1);
        if (bits & 4) line("EQ", 2);
        if (bits & 8) line("2N", 3);
    }
    for (i = 1; i <= lp.m; i++) glp_set_rii(lp, i, r.rii[i - 1]);
    for (j = 1; j <= lp.n; j++) glp_set_sjj(lp, j, r.sjj[j - 1]);
};

// glp_adv_basis (glpini01.js:356-362): the triangular basis from the native
// library (gk_adv_basis); the reference's lines through its own xprintf, the
// statuses (GLP_*) through its own glp_set_row_stat / glp_set_col_stat, which
// lpx_set_row_stat / lpx_set_col_stat forward to (glplpx01.js:233-240)
glp_adv_basis = exports["glp_adv_basis"] = function (lp, flags) {
    if (flags != 0)
        xerror("glp_adv_basis: flags = " + flags + "; invalid flags");
    if (lp.m == 0 || lp.n == 0) {
        glp_std_basis(lp);
        return;
    }
    xprintf("Constructing initial basis...");
    var r = __gk.advBasis(lp), i, j;
    if (lpx_get_int_parm(lp, LPX_K_MSGLEV) >= 3)
        xprintf("Size of triangular part = " + r.size + "");
    for (i = 1; i <= lp.m; i++) glp_set_row_stat(lp, i, r.row_stat[i]);
    for (j = 1; j <= lp.n; j++) glp_set_col_stat(lp, j, r.col_stat[j]);
};

// the LP / MIP preprocessor (glpnpp01.js .. glpnpp05.js, called by
// glp_simplex's preprocess_and_solve_lp glpapi06.js:41 and glp_intopt's
// preprocess_and_solve_mip glpapi09.js:116): the native workspace (gk_npp_*)
// for loads with names and scaling off, the reference's own otherwise; the
// reduced problem is built through the reference's glp_* API, as its
// npp_build_prob builds it (glpnpp01.js:396)
(function () {
    var js = {create: npp_create_wksp, load: npp_load_prob, simplex: npp_simplex, integer: npp_integer,
              build: npp_build_prob, post: npp_postprocess, unload: npp_unload_sol};
    npp_create_wksp = function () { return {__gk: null, __js: null}; };
    npp_load_prob = function (npp, orig, names, sol, scaling) {
        if (names || scaling || !(sol == GLP_SOL || sol == GLP_MIP)) {
            npp.__js = js.create();
            js.load(npp.__js, orig, names, sol, scaling);
            return;
        }
        npp.__gk = __gk.nppLoad(orig, sol);
    };
    npp_simplex = function (npp, parm) { return npp.__js ? js.simplex(npp.__js, parm) : __gk.nppSimplex(npp.__gk); };
    npp_integer = function (npp, parm) {
        return npp.__js ? js.integer(npp.__js, parm) : __gk.nppInteger(npp.__gk, parm, xprintf);
    };
    npp_build_prob = function (npp, prob) {
        if (npp.__js) { js.build(npp.__js, prob); return; }
        var r = __gk.nppBuild(npp.__gk), i, j, k, len, ind, val;
        glp_erase_prob(prob);
        glp_set_obj_dir(prob, r.dir);
        glp_set_obj_coef(prob, 0, r.c0[0]);
        for (i = 1; i <= r.m; i++) {
            glp_add_rows(prob, 1);
            glp_set_row_bnds(prob, i, r.row_type[i], r.row_lb[i], r.row_ub[i]);
        }
        ind = new Int32Array(1 + r.m);
        val = new Float64Array(1 + r.m);
        for (j = 1; j <= r.n; j++) {
            glp_add_cols(prob, 1);
            glp_set_col_kind(prob, j, r.col_kind[j]);
            glp_set_col_bnds(prob, j, r.col_type[j], r.col_lb[j], r.col_ub[j]);
            glp_set_obj_coef(prob, j, r.col_coef[j]);
            // the workspace's list order, which glp_set_mat_col reverses
            len = 0;
            for (k = r.A_ptr[j + 1] - 1; k >= r.A_ptr[j]; k--) {
                len++;
                ind[len] = r.A_ind[k];
                val[len] = r.A_val[k];
            }
            glp_set_mat_col(prob, j, len, ind, val);
        }
    };
    npp_postprocess = function (npp, prob) {
        if (npp.__js) return js.post(npp.__js, prob);
        __gk.nppPostprocess(npp.__gk, prob);
    };
    npp_unload_sol = function (npp, orig) {
        if (npp.__js) return js.unload(npp.__js, orig);
        __gk.nppUnload(npp.__gk, orig);
    };
})();

(function () {
    function versioned(f) {
        return function (lp) {
            var r = f.apply(this, arguments);
            lp.__gk_version = __gk.nextVersion();
            return r;
        };
    }
    // bounds, types, costs, dir and scale factors: lp.__gk_bversion (the
    // engine skips init_csa's rebuild while it is unchanged).  Outside the
    // wrapped mutators the reference writes them directly in two places:
    // glp_analyze_bound / _coef (glpapi12.js:1098-1120) on the lp they are
    // given — its version is unknown (0) during those calls — and
    // ios_feas_pump (glpios10.js:186-247) on its working copy of the MIP
    // (objective, dir, c0, column bounds and types between its glp_simplex
    // calls) — every solve runs without a version while it is active
    function bversioned(f) {
        return function (lp) {
            var r = f.apply(this, arguments);
            lp.__gk_bversion = __gk.nextVersion();
            return r;
        };
    }
    function bunknown(f) {
        return function (lp) {
            lp.__gk_bversion = 0;
            try { return f.apply(this, arguments); } finally { lp.__gk_bversion = __gk.nextVersion(); }
        };
    }
    ["glp_set_row_bnds", "glp_set_col_bnds", "glp_set_obj_coef", "glp_set_obj_dir", "glp_set_rii", "glp_set_sjj",
     "glp_unscale_prob", "glp_add_rows", "glp_add_cols", "glp_del_rows", "glp_del_cols", "glp_copy_prob",
     "glp_erase_prob"].forEach(function (name) {
        var f = eval(name);
        eval(name + " = exports[name] = bversioned(f)");
    });
    ["glp_analyze_bound", "glp_analyze_coef"].forEach(function (name) {
        var f = eval(name);
        eval(name + " = exports[name] = bunknown(f)");
    });
    var feas_pump = ios_feas_pump;
    ios_feas_pump = function (T) {
        __gk.bversionHold(+1);
        try { return feas_pump(T); } finally { __gk.bversionHold(-1); }
    };
    exports["__gk_ios_feas_pump"] = ios_feas_pump;
    glp_set_mat_row = exports["glp_set_mat_row"] = versioned(glp_set_mat_row);
    glp_set_mat_col = exports["glp_set_mat_col"] = versioned(glp_set_mat_col);
    glp_load_matrix = exports["glp_load_matrix"] = versioned(glp_load_matrix);
    glp_add_rows = exports["glp_add_rows"] = versioned(glp_add_rows);
    glp_add_cols = exports["glp_add_cols"] = versioned(glp_add_cols);
    glp_del_rows = exports["glp_del_rows"] = versioned(glp_del_rows);
    glp_del_cols = exports["glp_del_cols"] = versioned(glp_del_cols);
    glp_set_rii = exports["glp_set_rii"] = versioned(glp_set_rii);
    glp_set_sjj = exports["glp_set_sjj"] = versioned(glp_set_sjj);
    glp_scale_prob = exports["glp_scale_prob"] = versioned(glp_scale_prob);
    glp_unscale_prob = exports["glp_unscale_prob"] = versioned(glp_unscale_prob);
    glp_sort_matrix = exports["glp_sort_matrix"] = versioned(glp_sort_matrix);
    glp_erase_prob = exports["glp_erase_prob"] = versioned(glp_erase_prob);
    glp_copy_prob = exports["glp_copy_prob"] = versioned(glp_copy_prob);
})();
exports["__gk_core"] = __gk;
exports["__gk_ios_driver"] = ios_driver;
