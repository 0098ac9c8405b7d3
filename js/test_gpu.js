// GPU parity of the JS boundary (runs on the MI355X box: node + the addon,
// no reference code there).  For every explicit LP fixture in tests/golden it
// builds a problem object with the reference's field layout (glpapi01.js:
// lp.row[i] / lp.col[j] records, column lists of aij elements), runs the
// solve_lp flow of glp_simplex (glpapi06.js:3-37) — glp_factorize through
// bfd_factorize with the reference's b_col column callback, then spx_* —
// through js/gk_core.js, and compares with the reference's recorded result.
'use strict';
var assert = require('assert');
var fs = require('fs');
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

// the display lines and messages the engine reported against the
// reference's (tests/golden lp_* runs[].lines, minus glp_simplex's own header
// lines): same text, numbers within 1e-7 relative
var NUM = /-?(?:\d+\.?\d*(?:e[+-]?\d+)?|Infinity)/g;
function linesClose(ours, ref) {
    if (ours.length !== ref.length) return false;
    for (var i = 0; i < ours.length; i++) {
        if (ours[i].replace(NUM, '#') !== ref[i].replace(NUM, '#')) return false;
        var a = ours[i].match(NUM) || [], b = ref[i].match(NUM) || [];
        for (var k = 0; k < a.length; k++) {
            var x = Number(a[k]), y = Number(b[k]);
            if (!(Math.abs(x - y) <= 1e-7 * Math.max(1, Math.abs(y)))) return false;
        }
    }
    return true;
}

var dir = path.join(__dirname, '..', 'tests', 'golden');
var files = fs.readdirSync(dir).filter(function (f) { return /^lp_.*\.json$/.test(f); }).sort();
var ncase = 0, nlines = 0;
files.forEach(function (f) {
    var fx = JSON.parse(fs.readFileSync(path.join(dir, f), 'utf8'));
    if (fx.gen || fx.row_type === undefined) return;          // generated instances: Python tests
    fx.runs.forEach(function (run, r) {
        var lp = buildLp(fx), lines = [];
        var ret = simplex(lp, smcp(run.opts), function (s) { lines.push(s); });
        var tag = f + '#' + r;
        if (run.lines && !run.lines.some(function (s) { return s[0] === '~'; })) {
            var ref = run.lines.slice(2);
            if (lp.it_cnt === run.it_cnt) assert.ok(linesClose(lines, ref), tag + ' lines ' + JSON.stringify([lines, ref]));
            else assert.strictEqual(lines[lines.length - 1], ref[ref.length - 1], tag + ' last line');
            nlines++;
        }
        assert.strictEqual(ret, run.ret, tag + ' ret');
        assert.strictEqual(lp.pbs_stat, run.pbs_stat, tag + ' pbs_stat');
        assert.strictEqual(lp.dbs_stat, run.dbs_stat, tag + ' dbs_stat');
        var scale = Math.max(1.0, Math.abs(run.obj_val));
        assert.ok(Math.abs(lp.obj_val - run.obj_val) <= 1e-9 * scale, tag + ' obj ' + lp.obj_val + ' vs ' + run.obj_val);
        if (run.opts && run.opts.it_lim) assert.strictEqual(lp.it_cnt, run.it_cnt, tag + ' it_cnt');
        ncase++;
    });
});
assert.ok(ncase > 50, 'too few cases: ' + ncase);
assert.ok(nlines > 50, 'too few line checks: ' + nlines);
if (global.gc) global.gc();   // finalize the LP section's factor handles now (node --expose-gc)



// MIP fixtures: root LP through solve_lp as above, then the native driver
// through gk_core.iosDriver with the tree object ios_driver receives
// (T.mip = the problem, T.parm = IOCP with the reference's defaults,
// glpapi09.js:392-414); solve_mip's FEAS -> OPT / NOFEAS (glpapi09.js:82-92)
function iocp() {
    return {msg_lev: 3, br_tech: 4, bt_tech: 4, tol_int: 1e-5, tol_obj: 1e-7, tm_lim: INT_MAX, out_frq: 5000,
            out_dly: 10000, cb_func: null, cb_info: null, cb_size: 0, pp_tech: 2, mip_gap: 0.0, mir_cuts: 0,
            gmi_cuts: 0, cov_cuts: 0, clq_cuts: 0, presolve: 0, binarize: 0, fp_heur: 0};
}
var nmip = 0;
fs.readdirSync(dir).filter(function (f) { return /^mip_.*\.json$/.test(f) && !/12x30/.test(f); }).sort()
    .forEach(function (f) {
        var fx = JSON.parse(fs.readFileSync(path.join(dir, f), 'utf8'));
        if (fx.gen || fx.A_ptr === undefined) return;              // generated instances: Python tests
        var lp = buildLp(fx);
        for (var j = 1; j <= fx.n; j++) lp.col[j].kind = fx.col_kind[j - 1];
        var ret = simplex(lp, smcp(fx.root.opts));
        assert.strictEqual(ret, fx.root.ret, f + ' root ret');
        if (lp.pbs_stat !== 2 || lp.dbs_stat !== 2) return;       // glp_intopt would return GLP_EROOT
        lp.mip_stat = 1; lp.mip_obj = 0.0;
        for (var i = 1; i <= fx.m; i++) lp.row[i].mipx = 0.0;
        for (j = 1; j <= fx.n; j++) lp.col[j].mipx = 0.0;
        var T = {mip: lp, parm: iocp()};
        assert.ok(core.nativeIos(T), f + ' not served natively');
        ret = core.iosDriver(T);
        if (ret === 0) lp.mip_stat = (lp.mip_stat === 2) ? 5 : 4;
        assert.strictEqual(ret, fx.mip.ret, f + ' ret');
        assert.strictEqual(lp.mip_stat, fx.mip.mip_stat, f + ' mip_stat');
        if (lp.mip_stat === 5) {
            var sc = Math.max(1.0, Math.abs(fx.mip.mip_obj));
            assert.ok(Math.abs(lp.mip_obj - fx.mip.mip_obj) <= 1e-9 * sc, f + ' mip_obj ' + lp.mip_obj);
            var obj = fx.c0;
            for (j = 1; j <= fx.n; j++) {
                var x = lp.col[j].mipx;
                if (fx.col_kind[j - 1] === 2) assert.strictEqual(x, Math.floor(x), f + ' integrality');
                obj += fx.col_coef[j - 1] * x;
            }
            assert.ok(Math.abs(obj - lp.mip_obj) <= 1e-7 * sc, f + ' objective of mipx');
        }
        nmip++;
    });
assert.ok(nmip >= 10, 'too few MIP cases: ' + nmip);

// glp_scale_prob through the addon: the factors the reference computed
// (tests/golden/scale_*.json), bit for bit, and its report numbers as JS
// prints them (the shim's report lines are built from these)
var nscale = 0;
fs.readdirSync(dir).filter(function (f) { return /^scale_.*\.json$/.test(f); }).sort().forEach(function (f) {
    var fx = JSON.parse(fs.readFileSync(path.join(dir, f)));
    var lp = buildLp(fx);
    fx.runs.forEach(function (r) {
        if (r.error) return;
        var out = core.scaleProb(lp, r.flags);
        assert.strictEqual(out.ret, 0, f + ' ret');
        for (var i = 0; i < fx.m; i++) assert.strictEqual(out.rii[i], r.rii[i], f + ' rii ' + i + ' flags ' + r.flags);
        for (var j = 0; j < fx.n; j++) assert.strictEqual(out.sjj[j], r.sjj[j], f + ' sjj ' + j + ' flags ' + r.flags);
        var a = out.report;
        assert.strictEqual(r.lines[1], ' A: min|aij| = ' + a[0] + '  max|aij| = ' + a[1] + '  ratio = ' + a[2], f + ' A line');
        nscale++;
    });
});
assert.ok(nscale >= 60, 'too few scaling runs: ' + nscale);
// tableau rows (tests/golden/tab_*.json: the reference's glp_eval_tab_row on
// the basis glp_simplex left) through gk_core.evalTabRows, both device paths
var ntab = 0;
fs.readdirSync(dir).filter(function (f) { return /^tab_.*\.json$/.test(f); }).sort().forEach(function (f) {
    var fx = JSON.parse(fs.readFileSync(path.join(dir, f), 'utf8'));
    var lp = buildLp(fx);
    assert.strictEqual(factorize(lp), 0, f + ' factorize');
    var ks = fx.tab_rows.map(function (r) { return r.k; }), w = fx.m + fx.n;
    [false, true].forEach(function (perRow) {
        var rows = core.evalTabRows(lp, ks, perRow);
        fx.tab_rows.forEach(function (r, t) {
            var ref = new Float64Array(w), big = 1.0;
            r.ind.forEach(function (j, q) { ref[j - 1] = r.val[q]; big = Math.max(big, Math.abs(r.val[q])); });
            for (var j = 0; j < w; j++)
                assert.ok(Math.abs(rows[t][j] - ref[j]) <= 1e-9 * big, f + ' k=' + r.k + ' j=' + (j + 1) + ': ' + rows[t][j] + ' vs ' + ref[j]);
        });
    });
    ntab++;
});
assert.ok(ntab >= 5, 'too few tab fixtures: ' + ntab);

console.log('ok js gpu parity: ' + ncase + ' runs, ' + nmip + ' MIPs, ' + nscale + ' scalings, ' + ntab + ' tableau-row fixtures');
// node 12's environment teardown can run pending N-API second-pass
// finalizers after the addon's environment is gone (a segfault inside
// libnode's PendingPhantomCallback::Invoke, seen when handles were
// collected just before exit); a checked script leaves without it
process.exit(0);
