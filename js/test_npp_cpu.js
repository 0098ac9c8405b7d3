// The native preprocessor through the JS marshalling (js/gk_core.js npp*, the
// functions js/gk_shim.js binds to the reference's npp_* names), on the CPU:
// for every presolve_* / mippre_* fixture with its matrix stored (the
// reference's glp_simplex / glp_intopt with presolve = GLP_ON), the reduced
// problem equals the reference's bit for bit, and postprocessing the
// reference's solution of it gives the reference's final statuses and
// values.  Host code only (no device).
'use strict';
var assert = require('assert');
var fs = require('fs');
var path = require('path');
var U = require(path.join(__dirname, 'test_util.js'));
var core = U.core;

var gold = path.join(__dirname, '..', 'tests', 'golden');
var files = fs.readdirSync(gold).filter(function (f) { return /^(presolve|mippre)_.*\.json$/.test(f); }).sort();
var runs = 0;

function same(a, b, what) {
    assert.strictEqual(a.length, b.length, what + ' length');
    for (var k = 0; k < a.length; k++) assert.ok(a[k] === b[k], what + '[' + k + ']: ' + a[k] + ' != ' + b[k]);
}
function close(a, b, what) {
    var big = 1.0;
    b.forEach(function (v) { big = Math.max(big, Math.abs(v)); });
    for (var k = 0; k < b.length; k++) assert.ok(Math.abs(a[k] - b[k]) <= 1e-12 * big, what + '[' + k + ']');
}

files.forEach(function (f) {
    var fx = JSON.parse(fs.readFileSync(path.join(gold, f)));
    if (fx.gen) return;                          // generated instances carry no matrix
    var mip = /^mippre_/.test(f);
    fx.runs.forEach(function (run) {
        var lp = U.buildLp(fx), j, i;
        if (mip)
            for (j = 1; j <= fx.n; j++) { lp.col[j].kind = fx.col_kind[j - 1]; lp.col[j].mipx = 0; }
        for (i = 1; i <= fx.m; i++) lp.row[i].mipx = 0;
        var w = core.nppLoad(lp, mip ? 3 : 1);
        var ret = mip ? core.nppInteger(w, run.opts, function () {}) : core.nppSimplex(w);
        var red = run.reduced;
        if (red === null) {
            assert.strictEqual(ret, run.ret, f);
            runs++;
            return;
        }
        assert.strictEqual(ret, 0, f);
        var r = core.nppBuild(w);
        assert.deepStrictEqual([r.m, r.n, r.nnz], [red.m, red.n, red.nnz], f);
        same(Array.from(r.row_ref).slice(1), red.row_ref, f + ' row_ref');
        same(Array.from(r.col_ref).slice(1), red.col_ref, f + ' col_ref');
        assert.ok(r.c0[0] === red.c0, f + ' c0');
        ['row_type', 'row_lb', 'row_ub', 'col_type', 'col_lb', 'col_ub', 'col_coef'].forEach(function (k) {
            same(Array.from(r[k]).slice(1), red[k], f + ' ' + k);
        });
        same(Array.from(r.A_ind).slice(1), red.A_ind, f + ' A_ind');
        same(Array.from(r.A_val).slice(1), red.A_val, f + ' A_val');
        var s = run.reduced_sol;
        if (s === null) { runs++; return; }
        // the reduced problem's solution as the reference's problem object holds it
        var prob = {m: r.m, n: r.n, row: [null], col: [null], pbs_stat: s.pbs_stat, dbs_stat: s.dbs_stat,
                    mip_stat: s.mip_stat};
        for (i = 1; i <= r.m; i++) prob.row.push(mip ? {} : {stat: s.row_stat[i - 1], dual: s.row_dual[i - 1]});
        for (j = 1; j <= r.n; j++)
            prob.col.push(mip ? {mipx: s.col_mipx[j - 1]} : {stat: s.col_stat[j - 1], prim: s.col_prim[j - 1]});
        core.nppPostprocess(w, prob);
        core.nppUnload(w, lp);
        if (mip) {
            assert.strictEqual(lp.mip_stat, run.mip_stat, f);
            same(lp.col.slice(1).map(function (c) { return c.mipx; }), run.col_mipx, f + ' col_mipx');
            close(lp.row.slice(1).map(function (c) { return c.mipx; }), run.row_mipx, f + ' row_mipx');
        } else {
            assert.deepStrictEqual([lp.pbs_stat, lp.dbs_stat], [run.pbs_stat, run.dbs_stat], f);
            same(lp.row.slice(1).map(function (c) { return c.stat; }), run.row_stat, f + ' row_stat');
            same(lp.col.slice(1).map(function (c) { return c.stat; }), run.col_stat, f + ' col_stat');
            same(lp.col.slice(1).map(function (c) { return c.prim; }), run.col_prim, f + ' col_prim');
            same(lp.row.slice(1).map(function (c) { return c.dual; }), run.row_dual, f + ' row_dual');
            close(lp.row.slice(1).map(function (c) { return c.prim; }), run.row_prim, f + ' row_prim');
            close(lp.col.slice(1).map(function (c) { return c.dual; }), run.col_dual, f + ' col_dual');
            assert.ok(Math.abs(lp.obj_val - run.obj_val) <= 1e-12 * Math.max(1, Math.abs(run.obj_val)), f + ' obj');
        }
        runs++;
    });
});
assert.ok(runs >= 100, 'runs ' + runs);
console.log('ok js npp ' + runs + ' runs');
