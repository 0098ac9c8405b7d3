// gk_shim.js — concatenated into the reference bundle after lib/*.js (see
// js/load_glpk.js).  The bundle is one closure, so assigning to its function
// names rebinds every internal caller:
//   solve_lp (glpapi06.js:27-37)          -> spx_primal / spx_dual
//   glp_factorize / glp_ftran / glp_btran -> bfd_* (glpapi12.js:75-105, 211, 240)
// Matrix and scale mutators bump lp.__gk_version so the device copy of A is
// re-uploaded only when A or the scaling changed (SURVEY.md §8(b).1).
var __gk = require(__gk_core_path);

spx_primal = function (lp, parm) { return __gk.spx(lp, parm, false, xprintf); };
spx_dual = function (lp, parm) { return __gk.spx(lp, parm, true, xprintf); };
bfd_create_it = function () { return __gk.bfdCreate(); };
bfd_set_parm = function (bfd, parm) { __gk.bfdSetParm(bfd, parm); };
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

(function () {
    function versioned(f) {
        return function (lp) {
            var r = f.apply(this, arguments);
            lp.__gk_version = __gk.nextVersion();
            return r;
        };
    }
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
