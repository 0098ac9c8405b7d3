// CPU-side checks of the JS boundary (no GPU here): the addon loads and
// exports the binding, the reference bundle loads with the shim, the hot-path
// names are rebound, and a solve fails loudly (no fallback to the JS simplex).
'use strict';
var assert = require('assert');
var path = require('path');
var core = require(path.join(__dirname, 'gk_core.js'));

var names = ['create', 'deviceCount', 'abiVersion', 'lastError', 'bfdCreate', 'bfdSetParm', 'bfdFactorizeCsc',
             'bfdFtran', 'bfdBtran', 'bfdUpdate', 'bfdGetCount', 'bfdValid', 'spx', 'ios', 'stats', 'advBasis',
             'evalTabRows', 'nppCreate', 'nppLoad', 'nppSimplex', 'nppInteger', 'nppBuildSize', 'nppBuild',
             'nppPostprocess', 'nppUnloadSol', 'nppUnloadMip'];
names.forEach(function (k) { assert.strictEqual(typeof core.addon[k], 'function', k); });
assert.strictEqual(core.addon.abiVersion(), 11);

var ref = process.env.GLPK_REF || '/root/reference';
var fs = require('fs');
if (!fs.existsSync(path.join(ref, 'lib'))) {
    console.log('ok addon (reference tree absent: shim test skipped)');
    process.exit(0);
}
var glpk = require(path.join(__dirname, 'load_glpk.js'))(ref);
assert.ok(glpk.__gk_core, 'shim not concatenated');
assert.ok(/nativeIos/.test(String(glpk.__gk_ios_driver)), 'ios_driver not rebound');
// requests the native driver does not serve go to the reference's driver
assert.strictEqual(core.nativeIos({mip: {m: 2, n: 3}, parm: {cb_func: function () {}}}), false);
assert.strictEqual(core.nativeIos({mip: {m: 2, n: 3}, parm: {cb_func: null, mip_gap: 0.01}}), true);   // mip_gap is native
// show_progress lines (glpios03.js:45) from the native driver's records
assert.strictEqual(core.mipProgressLine(1, [3, 0, 57, 1, 0, -1.7976931348623157e308, 0]), '+57: mip = not found yet >= -inf  (1; 0)');
assert.strictEqual(core.mipProgressLine(1, [3, 3, 529, 133, 284, 259, 10]), '+529: >>>>> 284 >= 259   8.8% (133; 10)');
assert.strictEqual(core.mipProgressLine(1, [3, 6, 652, 0, 261, 0, 331]), '+652: mip = 261 >= tree is empty   0.0% (0; 331)');
assert.strictEqual(core.nativeIos({mip: {m: 2, n: 3}, parm: {cb_func: null, mip_gap: 0, gmi_cuts: 1}}), false);
assert.strictEqual(core.nativeIos({mip: {m: 2, n: 3}, parm: {cb_func: null, mip_gap: 0}}), true);
// node LPs beyond 64 KiB of LDS run natively too (HBM work area), and
// beyond 2 MiB on the engine: no size goes back to the reference's driver
assert.strictEqual(core.nativeIos({mip: {m: 80, n: 200}, parm: {cb_func: null, mip_gap: 0}}), true);
assert.strictEqual(core.nativeIos({mip: {m: 30000, n: 40000}, parm: {cb_func: null, mip_gap: 0}}), true);
glpk.glp_set_print_func(function () {});
// the feasibility pump writes its working lp's objective and bounds
// directly (glpios10.js:186-247): while it runs, every solve hands the
// engine b_version 0 (the hold is released on every exit, a throw included)
(function () {
    var seen = -1, fake = {};
    Object.defineProperty(fake, 'mip', {get: function () { seen = core.bversionHold(0); throw new Error('probe'); }});
    assert.throws(function () { glpk.__gk_ios_feas_pump(fake); }, /probe/);
    assert.strictEqual(seen, 1, 'b_version held inside ios_feas_pump');
    assert.strictEqual(core.bversionHold(0), 0, 'hold released');
})();
// glp_adv_basis through the shim (host code in the library, no device): the
// reference's statuses and printed lines on its fixtures (tests/golden/adv_*)
(function () {
    var gdir = path.join(__dirname, '..', 'tests', 'golden');
    var files = fs.readdirSync(gdir).filter(function (f) { return /^adv_.*\.json$/.test(f); }).sort();
    assert.ok(files.length > 0, 'no adv_* fixtures');
    files.forEach(function (f) {
        var d = JSON.parse(fs.readFileSync(path.join(gdir, f), 'utf8'));
        var P = glpk.glp_create_prob(), i, j, k;
        if (d.m) glpk.glp_add_rows(P, d.m);
        if (d.n) glpk.glp_add_cols(P, d.n);
        for (i = 1; i <= d.m; i++) glpk.glp_set_row_bnds(P, i, d.row_type[i - 1], d.row_lb[i - 1], d.row_ub[i - 1]);
        for (j = 1; j <= d.n; j++) glpk.glp_set_col_bnds(P, j, d.col_type[j - 1], d.col_lb[j - 1], d.col_ub[j - 1]);
        // glp_load_matrix leaves the column lists in descending row order
        // (glpapi01.js:512-528), glp_sort_matrix in ascending order (the
        // order glp_read_lp leaves): the recorded problems have one or the other
        var ia = [0], ja = [0], ar = [0];
        for (j = 1; j <= d.n; j++)
            for (k = d.A_ptr[j - 1]; k < d.A_ptr[j]; k++) { ia.push(d.A_ind[k]); ja.push(j); ar.push(d.A_val[k]); }
        if (ia.length > 1) glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
        var same = function () {
            for (j = 1; j <= d.n; j++) {
                var l = [];
                for (var a = P.col[j].ptr; a != null; a = a.c_next) l.push(a.row.i);
                if (JSON.stringify(l) !== JSON.stringify(d.A_ind.slice(d.A_ptr[j - 1], d.A_ptr[j]))) return false;
            }
            return true;
        };
        if (!same()) glpk.glp_sort_matrix(P);
        assert.ok(same(), f + ': column list order not reproduced');
        var lines = [];
        glpk.glp_set_print_func(function (s) { lines.push(s); });
        glpk.glp_adv_basis(P, 0);
        glpk.glp_set_print_func(function () {});
        assert.deepStrictEqual(lines, d.adv.lines, f + ': printed lines');
        for (i = 1; i <= d.m; i++) assert.strictEqual(P.row[i].stat, d.adv.row_stat[i - 1], f + ': row ' + i);
        for (j = 1; j <= d.n; j++) assert.strictEqual(P.col[j].stat, d.adv.col_stat[j - 1], f + ': col ' + j);
        if (d.adv.flags_error) {
            var err = null;
            try { glpk.glp_adv_basis(P, 1); } catch (e) { err = String(e.message); }
            assert.strictEqual(err, d.adv.flags_error, f + ': flags error');
        }
    });
    console.log('ok adv basis (' + files.length + ' reference fixtures)');
})();
// glp_simplex / glp_intopt with presolve = GLP_ON go through the native
// preprocessor (the shim's npp_* rebinding): the runs the reference's own
// preprocessor stops (no primal / no dual feasible solution) end there
// without a device, with the reference's return code and lines
(function () {
    var gdir = path.join(__dirname, '..', 'tests', 'golden');
    var calls = 0, keep = core.nppLoad;
    core.nppLoad = function () { calls++; return keep.apply(this, arguments); };
    var files = fs.readdirSync(gdir).filter(function (f) { return /^presolve_(wild|mix|sparse).*\.json$/.test(f); }).sort();
    var stopped = 0;
    files.forEach(function (f) {
        var d = JSON.parse(fs.readFileSync(path.join(gdir, f), 'utf8'));
        d.runs.forEach(function (run) {
            if (run.reduced !== null) return;
            var P = glpk.glp_create_prob(), i, j, k;
            glpk.glp_set_obj_dir(P, d.dir);
            glpk.glp_set_obj_coef(P, 0, d.c0);
            if (d.m) glpk.glp_add_rows(P, d.m);
            if (d.n) glpk.glp_add_cols(P, d.n);
            for (i = 1; i <= d.m; i++) glpk.glp_set_row_bnds(P, i, d.row_type[i - 1], d.row_lb[i - 1], d.row_ub[i - 1]);
            for (j = 1; j <= d.n; j++) {
                glpk.glp_set_col_bnds(P, j, d.col_type[j - 1], d.col_lb[j - 1], d.col_ub[j - 1]);
                glpk.glp_set_obj_coef(P, j, d.col_coef[j - 1]);
            }
            var ia = [0], ja = [0], ar = [0];
            for (j = 1; j <= d.n; j++)
                for (k = d.A_ptr[j - 1]; k < d.A_ptr[j]; k++) { ia.push(d.A_ind[k]); ja.push(j); ar.push(d.A_val[k]); }
            if (ia.length > 1) glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
            var lines = [];
            glpk.glp_set_print_func(function (s) { lines.push(s); });
            var ret = glpk.glp_simplex(P, new glpk.SMCP({meth: run.opts.meth, presolve: glpk.GLP_ON}));
            glpk.glp_set_print_func(function () {});
            assert.strictEqual(ret, run.ret, f);
            assert.deepStrictEqual(lines, run.lines, f + ': printed lines');
            stopped++;
        });
    });
    core.nppLoad = keep;
    assert.ok(stopped >= 10 && calls === stopped, 'presolve runs ' + stopped + ', native loads ' + calls);
    console.log('ok presolve stops (' + stopped + ' reference runs, native preprocessor)');
})();
var lp = glpk.glp_create_prob();
glpk.glp_set_obj_dir(lp, glpk.GLP_MAX);
glpk.glp_add_rows(lp, 1);
glpk.glp_set_row_bnds(lp, 1, glpk.GLP_UP, 0, 4);
glpk.glp_add_cols(lp, 2);
glpk.glp_set_col_bnds(lp, 1, glpk.GLP_LO, 0, 0);
glpk.glp_set_col_bnds(lp, 2, glpk.GLP_LO, 0, 0);
glpk.glp_set_obj_coef(lp, 1, 1);
glpk.glp_set_obj_coef(lp, 2, 2);
glpk.glp_load_matrix(lp, 2, [0, 1, 1], [0, 1, 2], [0, 1, 1]);
assert.ok(lp.__gk_version > 0, 'glp_load_matrix not versioned');
var threw = null;
try {
    glpk.glp_simplex(lp, new glpk.SMCP({presolve: glpk.GLP_OFF}));
} catch (e) { threw = e; }
if (core.addon.deviceCount() === 0) {
    assert.ok(threw && /gk_ctx_create|device/.test(threw.message), 'expected a loud device error, got ' + threw);
    console.log('ok shim (no device: ' + threw.message + ')');
} else {
    assert.ok(!threw, String(threw));
    assert.strictEqual(glpk.glp_get_obj_val(lp), 8);
    console.log('ok shim (device solve: obj ' + glpk.glp_get_obj_val(lp) + ')');
}
