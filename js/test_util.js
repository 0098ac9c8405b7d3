// Helpers of the JS GPU tests (node + the addon on the MI355X box; no
// reference code there): the reference's problem-object layout, glp_factorize
// with b_col, solve_lp's flow, IOCP defaults and the C5s generator.
'use strict';
var path = require('path');
var core = require(path.join(__dirname, 'gk_core.js'));

var GLP_BS = 1, GLP_PRIMAL = 1, GLP_DUALP = 2, GLP_DUAL = 3, GLP_EFAIL = 5;
var DBL_MAX = Number.MAX_VALUE, INT_MAX = 0x7FFFFFFF;

function smcp(o) {  // SMCP with the reference's `||` defaults (glpapi06.js:359-375)
    o = o || {};
    return {msg_lev: o.msg_lev || 3, meth: o.meth || GLP_PRIMAL, pricing: o.pricing || 0x22,
            r_test: o.r_test || 0x22, tol_bnd: o.tol_bnd || 1e-7, tol_dj: o.tol_dj || 1e-7,
            tol_piv: o.tol_piv || 1e-10, obj_ll: o.obj_ll || -DBL_MAX, obj_ul: o.obj_ul || +DBL_MAX,
            it_lim: o.it_lim || INT_MAX, tm_lim: o.tm_lim || INT_MAX, out_frq: o.out_frq || 500,
            out_dly: o.out_dly || 0, presolve: 0};
}

function buildLp(fx) {
    var lp = {m: fx.m, n: fx.n, nnz: fx.nnz, dir: fx.dir, c0: fx.c0, row: [null], col: [null],
              head: new Int32Array(fx.m + 1), valid: 0, bfd: null, it_cnt: 0};
    for (var i = 1; i <= fx.m; i++)
        lp.row.push({i: i, type: fx.row_type[i - 1], lb: fx.row_lb[i - 1], ub: fx.row_ub[i - 1],
                     rii: fx.row_rii[i - 1], stat: fx.row_stat[i - 1], bind: 0, prim: 0, dual: 0});
    for (var j = 1; j <= fx.n; j++) {
        var col = {j: j, type: fx.col_type[j - 1], lb: fx.col_lb[j - 1], ub: fx.col_ub[j - 1],
                   coef: fx.col_coef[j - 1], sjj: fx.col_sjj[j - 1], stat: fx.col_stat[j - 1],
                   bind: 0, prim: 0, dual: 0, ptr: null};
        var last = null;
        for (var t = fx.A_ptr[j - 1]; t < fx.A_ptr[j]; t++) {
            var aij = {row: lp.row[fx.A_ind[t]], col: col, val: fx.A_val[t], c_next: null};
            if (last === null) col.ptr = aij; else last.c_next = aij;
            last = aij;
        }
        lp.col.push(col);
    }
    return lp;
}

// glp_factorize (glpapi12.js:5-94) with b_col (:7-31)
function factorize(lp) {
    var m = lp.m, n = lp.n, j = 0;
    lp.valid = 0;
    for (var k = 1; k <= m + n; k++) {
        var rec = k <= m ? lp.row[k] : lp.col[k - m];
        rec.bind = 0;
        if (rec.stat === GLP_BS) {
            j++;
            if (j > m) return 0x02;               // GLP_EBADB
            lp.head[j] = k;
            rec.bind = j;
        }
    }
    if (j < m) return 0x02;
    if (lp.bfd === null) lp.bfd = core.bfdCreate();
    function bCol(lp, jj, ind, val) {
        var kk = lp.head[jj];
        if (kk <= m) { ind[1] = kk; val[1] = 1.0; return 1; }
        var len = 0;
        for (var aij = lp.col[kk - m].ptr; aij !== null; aij = aij.c_next) {
            len++;
            ind[len] = aij.row.i;
            val[len] = -aij.row.rii * aij.val * aij.col.sjj;
        }
        return len;
    }
    var ret = core.bfdFactorize(lp.bfd, m, lp.head, bCol, lp);
    if (ret === 1) return 0x03;                   // GLP_ESING
    if (ret === 2) return 0x04;                   // GLP_ECOND
    lp.valid = 1;
    return 0;
}

function simplex(lp, parm, print) {   // solve_lp (glpapi06.js:3-37)
    if (!lp.valid) {
        var r = factorize(lp);
        if (r) return r;
    }
    if (parm.meth === GLP_PRIMAL) return core.spx(lp, parm, false, print);
    if (parm.meth === GLP_DUALP) {
        var ret = core.spx(lp, parm, true, print);
        if (ret === GLP_EFAIL && lp.valid) ret = core.spx(lp, parm, false, print);
        return ret;
    }
    return core.spx(lp, parm, true, print);
}


// IOCP with the reference's defaults (glpapi09.js:392-414)
function iocp(o) {
    o = o || {};
    return {msg_lev: o.msg_lev || 3, br_tech: o.br_tech || 4, bt_tech: o.bt_tech || 4, tol_int: o.tol_int || 1e-5,
            tol_obj: o.tol_obj || 1e-7, tm_lim: o.tm_lim || INT_MAX, out_frq: o.out_frq || 5000,
            out_dly: o.out_dly || 10000, cb_func: null, cb_info: null, cb_size: 0, pp_tech: o.pp_tech || 2,
            mip_gap: o.mip_gap || 0.0, mir_cuts: 0, gmi_cuts: 0, cov_cuts: 0, clq_cuts: 0, presolve: 0,
            binarize: 0, fp_heur: 0};
}

// SURVEY.md §8(d) generators (splitmix64), for fixtures stored without A
function SplitMix(seed) { this.s = BigInt.asUintN(64, BigInt(seed)); }
SplitMix.prototype.u = function () {
    var M = 0xFFFFFFFFFFFFFFFFn;
    this.s = (this.s + 0x9E3779B97F4A7C15n) & M;
    var z = this.s;
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M;
    z = z ^ (z >> 31n);
    return Number(z >> 11n) * Math.pow(2, -53);
};

// C5s (12 x n correlated multi-knapsack): the explicit fixture layout
// (column lists in glp_load_matrix's row-descending order: glpapi01.js:512-528)
function genC5sFixture(fx) {
    var m = fx.gen.m, n = fx.gen.n, r = new SplitMix(fx.gen.seed), i, j, w = [];
    var out = Object.assign({}, fx);
    out.row_type = []; out.row_lb = []; out.row_ub = []; out.row_rii = []; out.row_stat = [];
    for (i = 0; i < m; i++) {
        w.push([]);
        var s = 0;
        for (j = 0; j < n; j++) { w[i].push(1 + Math.floor(1000 * r.u())); s += w[i][j]; }
        out.row_type.push(3); out.row_lb.push(0); out.row_ub.push(Math.floor(s / 2)); out.row_rii.push(1);
        out.row_stat.push(GLP_BS);
    }
    out.A_ptr = [0]; out.A_ind = []; out.A_val = [];
    for (j = 0; j < n; j++) {
        for (i = m - 1; i >= 0; i--) { out.A_ind.push(i + 1); out.A_val.push(w[i][j]); }
        out.A_ptr.push(out.A_ind.length);
    }
    return out;
}

// a MIP fixture with its root LP solved (glp_simplex's solve_lp flow)
function mipProblem(fx) {
    if (fx.gen && fx.gen.kind === 'c5s') fx = genC5sFixture(fx);
    var lp = buildLp(fx);
    for (var j = 1; j <= fx.n; j++) lp.col[j].kind = fx.col_kind[j - 1];
    var ret = simplex(lp, smcp(fx.root.opts));
    lp.mip_stat = 1; lp.mip_obj = 0.0;
    for (var i = 1; i <= fx.m; i++) lp.row[i].mipx = 0.0;
    for (j = 1; j <= fx.n; j++) lp.col[j].mipx = 0.0;
    return {lp: lp, ret: ret, fx: fx};
}

module.exports = {core: core, smcp: smcp, buildLp: buildLp, factorize: factorize, simplex: simplex, iocp: iocp,
                  genC5sFixture: genC5sFixture, mipProblem: mipProblem, GLP_BS: GLP_BS, INT_MAX: INT_MAX,
                  DBL_MAX: DBL_MAX};
