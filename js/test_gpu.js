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


var U = require(path.join(__dirname, 'test_util.js'));
var smcp = U.smcp, buildLp = U.buildLp, factorize = U.factorize, simplex = U.simplex;

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
var iocp = U.iocp;
var nmip = 0;
// (C5s instances are stored with their generator: test_util.genC5sFixture
// rebuilds A, so the deep 12 x 30 tree runs here too)
fs.readdirSync(dir).filter(function (f) { return /^mip_.*\.json$/.test(f); }).sort()
    .forEach(function (f) {
        var fx = JSON.parse(fs.readFileSync(path.join(dir, f), 'utf8'));
        if (fx.A_ptr === undefined && !(fx.gen && fx.gen.kind === 'c5s')) return;
        var mp = U.mipProblem(fx), lp = mp.lp, j;
        fx = mp.fx;
        var ret = mp.ret;
        assert.strictEqual(ret, fx.root.ret, f + ' root ret');
        if (lp.pbs_stat !== 2 || lp.dbs_stat !== 2) return;       // glp_intopt would return GLP_EROOT
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
// no process.exit here: the library leaves from node's 'exit' event itself
// (js/gk_core.js armExit), so the script's exit code stands
