// Golden-vector generator (run in the build container only; needs node and
// /root/reference). It builds a throw-away, runtime-instrumented copy of the
// reference bundle in /tmp (header + glpdebug.js + lib/*.js + hooks + footer,
// the same concatenation as build.sh:3), runs the reference's own
// glp_simplex / glp_intopt flows on each instance and writes the inputs and
// outputs as JSON fixtures next to this script. Nothing from the reference is
// copied into the repository: only generated numbers are.
//
// Hooks added to the throw-away copy:
//   * a per-pivot trace call in front of change_basis(csa) in the primal and
//     dual main loops (glpspx01.js:2051, glpspx02.js:1962);
//   * counters around ios_solve_node (glpios01.js:866) and bfd_factorize
//     (glpbfd.js:47), rebinding the closure names (SURVEY.md §0).
//
// usage: node tests/golden/gen_golden.js [--big] [--only PREFIX]
//        node tests/golden/gen_golden.js --lpf-fix --only bfcpfix_
//        node tests/golden/gen_golden.js --deep 12x34   (one deep C5s MIP)
//        node --max-old-space-size=12000 tests/golden/gen_golden.js --c3
//          (C3 4096x16384 at full size only: the reference's state after its
//           first 300 dual pivots, one it_lim=300 call and three it_lim=100
//           calls; about 10 minutes and a 7 GB heap)
'use strict';
var fs = require('fs');
var path = require('path');

var REF = process.env.GLPK_REF || '/root/reference';
var OUT = __dirname;
var BIG = process.argv.indexOf('--big') >= 0;
var C3 = process.argv.indexOf('--c3') >= 0;
var ONLY = process.argv.indexOf('--only') >= 0 ? process.argv[process.argv.indexOf('--only') + 1] : null;
// --lpf-fix: the throw-away copy with the two offsets of lpf_update_it
// corrected (glplpf.js:420, :422 pass 0 where the new column and row of C
// live at g = fg + m0 and w = vw + m0, as scf_update_exp reads them at :427);
// only the bfcp cases run, written as bfcpfix_*.json
var LPF_FIX = process.argv.indexOf('--lpf-fix') >= 0;

function buildBundle() {
    var lib = path.join(REF, 'lib');
    var files = fs.readdirSync(lib).filter(function (f) { return /\.js$/.test(f); }).sort();
    var parts = [fs.readFileSync(path.join(REF, 'header'), 'utf8'),
                 fs.readFileSync(path.join(REF, 'glpdebug.js'), 'utf8')];
    files.forEach(function (f) {
        var src = fs.readFileSync(path.join(lib, f), 'utf8');
        if (f === 'glpspx01.js')
            src = src.replace('\n        change_basis(csa);',
                '\n        if (__trace) __trace(1, csa.it_cnt, csa.phase, csa.p, csa.q, csa.head[csa.m+csa.q], csa.p > 0 ? csa.head[csa.p] : 0, csa.teta);' +
                '\n        change_basis(csa);');
        if (f === 'glpspx02.js')
            src = src.replace('\n        change_basis(csa);',
                '\n        if (__trace) __trace(2, csa.it_cnt, csa.phase, csa.p, csa.q, csa.head[csa.m+csa.q], csa.head[csa.p], csa.delta);' +
                '\n        change_basis(csa);');
        if (f === 'glplpf.js' && LPF_FIX) {
            var fixed = src.replace('s_prod(lpf, x, 0, -1.0, f);', 's_prod(lpf, x, m0, -1.0, f);')
                           .replace('rt_prod(lpf, y, 0, -1.0, v);', 'rt_prod(lpf, y, m0, -1.0, v);');
            if (fixed === src) throw new Error('lpf-fix: pattern not found');
            src = fixed;
        }
        parts.push(src);
    });
    parts.push([
        'var __trace = null;',
        'exports["__set_trace"] = function(f){ __trace = f; };',
        'var __cnt = {solve_node: 0, factorize: 0};',
        'exports["__cnt"] = __cnt;',
        'ios_solve_node = (function(f){ return function(t){ __cnt.solve_node++; return f(t); }; })(ios_solve_node);',
        'bfd_factorize = (function(f){ return function(a,b,c,d,e){ __cnt.factorize++; return f(a,b,c,d,e); }; })(bfd_factorize);',
        'exports["__glp_adv_basis"] = glp_adv_basis;',
        // presolve: the reduced problem npp_build_prob made and the solution
        // npp_postprocess receives (glpapi06.js:87, :51)
        'var __npp_hook = null;',
        'exports["__set_npp_hook"] = function(f){ __npp_hook = f; };',
        'npp_build_prob = (function(f){ return function(npp, prob){ f(npp, prob); if (__npp_hook) __npp_hook("build", npp, prob); }; })(npp_build_prob);',
        'npp_postprocess = (function(f){ return function(npp, prob){ if (__npp_hook) __npp_hook("post", npp, prob); f(npp, prob); }; })(npp_postprocess);',
        ''].join('\n'));
    parts.push(fs.readFileSync(path.join(REF, 'footer'), 'utf8'));
    var dst = LPF_FIX ? '/tmp/glpk_golden_bundle_lpffix.js' : '/tmp/glpk_golden_bundle.js';
    fs.writeFileSync(dst, parts.join('\n'));
    return require(dst);
}

var glpk = buildBundle();
glpk.glp_set_print_func(function () {});

// ---- deterministic generators (SURVEY.md §8(d)) --------------------------
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

function newProb() { return glpk.glp_create_prob(); }

function genDense(m, n, seed) {
    var r = new SplitMix(seed), P = newProb(), i, j;
    glpk.glp_set_obj_dir(P, glpk.GLP_MAX);
    glpk.glp_add_rows(P, m); glpk.glp_add_cols(P, n);
    for (j = 1; j <= n; j++) { glpk.glp_set_obj_coef(P, j, r.u()); glpk.glp_set_col_bnds(P, j, glpk.GLP_LO, 0, 0); }
    var ne = m * n, ia = new Int32Array(1 + ne), ja = new Int32Array(1 + ne), ar = new Float64Array(1 + ne), k = 0;
    for (i = 1; i <= m; i++) {
        glpk.glp_set_row_bnds(P, i, glpk.GLP_UP, 0, 0.25 * n);
        for (j = 1; j <= n; j++) { k++; ia[k] = i; ja[k] = j; ar[k] = 0.5 + r.u(); }
    }
    glpk.glp_load_matrix(P, ne, ia, ja, ar);
    return P;
}

function genC2s(m, n, nzc, seed) {
    var r = new SplitMix(seed), P = newProb(), i, j, t;
    glpk.glp_set_obj_dir(P, glpk.GLP_MAX);
    glpk.glp_add_rows(P, m); glpk.glp_add_cols(P, n);
    for (j = 1; j <= n; j++) { glpk.glp_set_obj_coef(P, j, r.u()); glpk.glp_set_col_bnds(P, j, glpk.GLP_LO, 0, 0); }
    var ia = [0], ja = [0], ar = [0];
    for (j = 1; j <= n; j++) {
        var used = {};
        for (t = 0; t < nzc; ) {
            i = 1 + Math.floor(r.u() * m);
            if (used[i]) continue;
            used[i] = 1; t++;
            ia.push(i); ja.push(j); ar.push(0.5 + r.u());
        }
    }
    for (i = 1; i <= m; i++) glpk.glp_set_row_bnds(P, i, glpk.GLP_UP, 0, 1 + 9 * r.u());
    glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
    return P;
}

function genC5s(m, n, seed) {
    var r = new SplitMix(seed), P = newProb(), i, j;
    glpk.glp_set_obj_dir(P, glpk.GLP_MAX);
    glpk.glp_add_rows(P, m); glpk.glp_add_cols(P, n);
    var w = [], ia = [0], ja = [0], ar = [0];
    for (i = 1; i <= m; i++) {
        w[i] = [];
        var s = 0;
        for (j = 1; j <= n; j++) { w[i][j] = 1 + Math.floor(1000 * r.u()); s += w[i][j]; ia.push(i); ja.push(j); ar.push(w[i][j]); }
        glpk.glp_set_row_bnds(P, i, glpk.GLP_UP, 0, Math.floor(s / 2));
    }
    for (j = 1; j <= n; j++) {
        var cs = 0;
        for (i = 1; i <= m; i++) cs += w[i][j];
        glpk.glp_set_obj_coef(P, j, Math.floor(cs / m) + 500);
        glpk.glp_set_col_kind(P, j, glpk.GLP_BV);
    }
    glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
    return P;
}

// random sparse LP with every bound type on rows and columns; exercises the
// phase-I/phase-II logic, free and fixed variables, infeasible/unbounded ends.
// feasible=true builds the bounds around a random point x0 (so the LP has a
// feasible solution; integer columns get integer x0 and integer bounds).
function genMix(seed, m, n, dens, withInt, feasible, colsBounded) {
    var r = new SplitMix(seed), P = newProb(), i, j;
    glpk.glp_set_obj_dir(P, r.u() < 0.5 ? glpk.GLP_MIN : glpk.GLP_MAX);
    glpk.glp_add_rows(P, m); glpk.glp_add_cols(P, n);
    var isint = [], x0 = [];
    for (j = 1; j <= n; j++) {
        isint[j] = withInt && r.u() < (typeof withInt === 'number' ? withInt : 0.7);
        x0[j] = isint[j] ? Math.floor(r.u() * 7) - 3 : Math.round((r.u() * 10 - 5) * 4) / 4;
    }
    function bnds(setter, idx, c, integral, boxed) {
        var t = r.u(), a = Math.round((r.u() * 20 - 10) * 4) / 4, w = 1 + Math.round(r.u() * 40) / 4,
            w2 = 1 + Math.round(r.u() * 40) / 4;
        if (integral) { w = Math.ceil(w); w2 = Math.ceil(w2); }
        if (boxed) { setter(P, idx, glpk.GLP_DB, c - w, c + w2); return; }
        if (feasible) {
            if (t < 0.08) setter(P, idx, glpk.GLP_FR, 0, 0);
            else if (t < 0.38) setter(P, idx, glpk.GLP_LO, c - w, 0);
            else if (t < 0.58) setter(P, idx, glpk.GLP_UP, 0, c + w);
            else if (t < 0.95) setter(P, idx, glpk.GLP_DB, c - w, c + w2);
            else setter(P, idx, glpk.GLP_FX, c, c);
            return;
        }
        if (t < 0.10) setter(P, idx, glpk.GLP_FR, 0, 0);
        else if (t < 0.45) setter(P, idx, glpk.GLP_LO, a, 0);
        else if (t < 0.65) setter(P, idx, glpk.GLP_UP, 0, a);
        else if (t < 0.92) setter(P, idx, glpk.GLP_DB, a, a + w);
        else setter(P, idx, glpk.GLP_FX, a, a);
    }
    for (j = 1; j <= n; j++) {
        glpk.glp_set_obj_coef(P, j, Math.round((r.u() * 20 - 10) * 8) / 8);
    }
    glpk.glp_set_obj_coef(P, 0, Math.round(r.u() * 100) / 4);
    var ia = [0], ja = [0], ar = [0], rowv = [];
    for (i = 1; i <= m; i++) {
        rowv[i] = 0;
        for (j = 1; j <= n; j++)
            if (r.u() < dens) {
                var v = Math.round((r.u() * 18 - 9) * 16) / 16 || 1;
                ia.push(i); ja.push(j); ar.push(v); rowv[i] += v * x0[j];
            }
    }
    for (i = 1; i <= m; i++) bnds(glpk.glp_set_row_bnds, i, rowv[i], false);
    for (j = 1; j <= n; j++) bnds(glpk.glp_set_col_bnds, j, x0[j], isint[j], !!colsBounded);
    glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
    if (withInt) {
        for (j = 1; j <= n; j++) if (isint[j]) glpk.glp_set_col_kind(P, j, glpk.GLP_IV);
    }
    return P;
}

function readLp(file) {
    var P = newProb();
    glpk.glp_read_lp_from_string(P, null, fs.readFileSync(path.join(REF, 'test', file)).toString());
    return P;
}

// ---- dump helpers ---------------------------------------------------------
function dumpProb(P, gen) {
    var m = P.m, n = P.n, i, j, d = {m: m, n: n, nnz: P.nnz, dir: P.dir, c0: P.col[0] ? 0 : P.c0};
    d.c0 = P.c0;
    if (gen) d.gen = gen;
    var rt = [], rl = [], ru = [], rr = [], rs = [];
    for (i = 1; i <= m; i++) { var R = P.row[i]; rt.push(R.type); rl.push(R.lb); ru.push(R.ub); rr.push(R.rii); rs.push(R.stat); }
    var ct = [], cl = [], cu = [], cc = [], cs = [], ck = [], cst = [];
    for (j = 1; j <= n; j++) { var C = P.col[j]; ct.push(C.type); cl.push(C.lb); cu.push(C.ub); cc.push(C.coef); cs.push(C.sjj); ck.push(C.kind); cst.push(C.stat); }
    Object.assign(d, {row_type: rt, row_lb: rl, row_ub: ru, row_rii: rr, row_stat: rs,
                      col_type: ct, col_lb: cl, col_ub: cu, col_coef: cc, col_sjj: cs, col_kind: ck, col_stat: cst});
    if (!gen) {
        // A by columns in list order (init_csa, glpspx01.js:96-105)
        var ptr = [0], ind = [], val = [];
        for (j = 1; j <= n; j++) {
            for (var a = P.col[j].ptr; a != null; a = a.c_next) { ind.push(a.row.i); val.push(a.val); }
            ptr.push(ind.length);
        }
        d.A_ptr = ptr; d.A_ind = ind; d.A_val = val;
    }
    return d;
}

function snapshotBasis(P) {
    var i, j, rs = [], cs = [];
    for (i = 1; i <= P.m; i++) rs.push(P.row[i].stat);
    for (j = 1; j <= P.n; j++) cs.push(P.col[j].stat);
    return {row_stat: rs, col_stat: cs};
}

function runLp(P, opts, traceCap) {
    var tr = [];
    glpk.__set_trace(function (kind, it, phase, p, q, kq, kp, t) {
        if (tr.length < traceCap) tr.push([it, phase, p, q, kq, kp, t]);
    });
    var parm = new glpk.SMCP(opts);
    var f0 = glpk.__cnt.factorize;
    var lines = [];
    glpk.glp_set_print_func(function (s) { lines.push(s); });
    var t0 = process.hrtime.bigint();
    var ret = glpk.glp_simplex(P, parm);
    var dt = Number(process.hrtime.bigint() - t0) / 1e9;
    glpk.glp_set_print_func(function () {});
    glpk.__set_trace(null);
    var i, j, out = {opts: opts, ret: ret, pbs_stat: P.pbs_stat, dbs_stat: P.dbs_stat, obj_val: P.obj_val,
                     it_cnt: P.it_cnt, some: P.some, factorizations: glpk.__cnt.factorize - f0, seconds: dt};
    var a = snapshotBasis(P);
    out.row_stat = a.row_stat; out.col_stat = a.col_stat;
    out.row_prim = []; out.row_dual = []; out.col_prim = []; out.col_dual = [];
    for (i = 1; i <= P.m; i++) { out.row_prim.push(P.row[i].prim); out.row_dual.push(P.row[i].dual); }
    for (j = 1; j <= P.n; j++) { out.col_prim.push(P.col[j].prim); out.col_dual.push(P.col[j].dual); }
    out.trace = tr;
    out.lines = lines;
    return out;
}

function writeJson(name, obj) {
    fs.writeFileSync(path.join(OUT, name + '.json'), JSON.stringify(obj));
    console.log('wrote', name, obj.runs ? obj.runs.map(function (r) { return 'meth' + (r.opts.meth || 1) + ':ret' + r.ret + ':it' + r.it_cnt + ':obj' + r.obj_val + (r.mip_obj !== undefined ? ':mip' + r.mip_obj : ''); }).join(' ') : '');
}

// LP instance: run primal and dual each on a fresh copy, from the initial basis.
function lpCase(name, mk, gen, methods, traceCap, extraRuns) {
    if (ONLY && name.indexOf(ONLY) !== 0) return;
    var P0 = mk();
    var d = dumpProb(P0, gen);
    d.name = name; d.kind = 'lp'; d.runs = [];
    (methods || [1, 3]).forEach(function (meth) {
        var P = mk();
        d.runs.push(runLp(P, {meth: meth}, traceCap === undefined ? 100000 : traceCap));
    });
    (extraRuns || []).forEach(function (opts) {
        var P = mk();
        d.runs.push(runLp(P, opts, traceCap === undefined ? 100000 : traceCap));
    });
    writeJson('lp_' + name, d);
}

// LP instance under glp_set_bfcp (glpapi12.js:133): the factorization type
// (FT / BG / GR: glpfhv, glplpf + glpscf) and the refactorization limit
// nfs_max / nrs_max; primal and dual from the initial basis, each on a fresh
// copy, it_lim 2000 (glp_set_bfcp's BG / GR do not converge on the dense
// LP: see --lpf-fix).  The records keep the factorization count of each run.
var BFCP_RUNS = [{type: 2}, {type: 3}, {nfs_max: 20}, {type: 2, nrs_max: 15}, {upd_tol: 0.5}];
function bfcpCase(name, mk, gen) {
    var pre = LPF_FIX ? 'bfcpfix_' : 'bfcp_';
    if (ONLY && (pre + name).indexOf(ONLY) !== 0) return;
    var d = dumpProb(mk(), gen);
    d.name = name; d.kind = 'lp'; d.runs = [];
    BFCP_RUNS.forEach(function (b) {
        [1, 3].forEach(function (meth) {
            var P = mk(), parm = {};
            glpk.glp_get_bfcp(P, parm);
            Object.keys(b).forEach(function (k) { parm[k] = b[k]; });
            glpk.glp_set_bfcp(P, parm);
            var r = runLp(P, {meth: meth, it_lim: 2000}, 100000);
            r.bfcp = b;
            d.runs.push(r);
        });
    });
    d.lpf_fix = LPF_FIX;
    writeJson(pre + name, d);
}

// LP instance through glp_simplex with presolve = GLP_ON (glpapi06.js:41,
// preprocess_and_solve_lp): per method the reduced problem (rows / columns in
// list order, A by columns in list order, row_ref / col_ref), the solution of
// the reduced problem handed to npp_postprocess, and the final solution.
function presolveCase(name, mk, gen) {
    if (ONLY && ('presolve_' + name).indexOf(ONLY) !== 0) return;
    var d = dumpProb(mk(), gen);
    d.name = name; d.kind = 'lp'; d.runs = [];
    [1, 3].forEach(function (meth) {
        var P = mk(), red = null, redsol = null;
        glpk.__set_npp_hook(function (what, npp, prob) {
            if (what === 'build') {
                red = dumpProb(prob, null);
                red.row_ref = Array.from(npp.row_ref).slice(1);
                red.col_ref = Array.from(npp.col_ref).slice(1);
            } else {
                var i, j, s = {pbs_stat: prob.pbs_stat, dbs_stat: prob.dbs_stat, obj_val: prob.obj_val,
                               row_stat: [], row_dual: [], col_stat: [], col_prim: []};
                for (i = 1; i <= prob.m; i++) { s.row_stat.push(prob.row[i].stat); s.row_dual.push(prob.row[i].dual); }
                for (j = 1; j <= prob.n; j++) { s.col_stat.push(prob.col[j].stat); s.col_prim.push(prob.col[j].prim); }
                redsol = s;
            }
        });
        var r = runLp(P, {meth: meth, presolve: glpk.GLP_ON}, 0);
        glpk.__set_npp_hook(null);
        r.reduced = red;
        r.reduced_sol = redsol;
        d.runs.push(r);
    });
    writeJson('presolve_' + name, d);
}

// MIP instance: root primal glp_simplex then glp_intopt (default IOCP), the
// flow of SURVEY.md §8(d) C4/C5.
function mipCase(name, mk, gen) {
    if (ONLY && ('mip_' + name).indexOf(ONLY) !== 0) return;
    var P = mk();
    var d = dumpProb(P, gen);
    d.name = name; d.kind = 'mip';
    var root = runLp(P, {}, 0);
    delete root.trace;
    var s0 = glpk.__cnt.solve_node, f0 = glpk.__cnt.factorize, it0 = P.it_cnt;
    var lines = [];
    glpk.glp_set_print_func(function (s) { lines.push(s); });
    var t0 = process.hrtime.bigint();
    var ret = glpk.glp_intopt(P, new glpk.IOCP({}));
    var dt = Number(process.hrtime.bigint() - t0) / 1e9;
    glpk.glp_set_print_func(function () {});
    var j, x = [];
    for (j = 1; j <= P.n; j++) x.push(P.col[j].mipx);
    var rx = [];
    for (j = 1; j <= P.m; j++) rx.push(P.row[j].mipx);
    d.root = root;
    d.mip = {ret: ret, mip_stat: P.mip_stat, mip_obj: P.mip_obj, col_mipx: x, row_mipx: rx,
             lp_solves: glpk.__cnt.solve_node - s0, factorizations: glpk.__cnt.factorize - f0,
             pivots: P.it_cnt - it0, seconds: dt, lines: lines};
    fs.writeFileSync(path.join(OUT, 'mip_' + name + '.json'), JSON.stringify(d));
    console.log('wrote mip', name, 'ret', ret, 'obj', P.mip_obj, 'lp', d.mip.lp_solves, 'piv', d.mip.pivots, 'sec', dt.toFixed(2));
}

// MIP instance through glp_intopt with presolve = GLP_ON (glpapi09.js:116,
// preprocess_and_solve_mip), no root LP beforehand: per option set
// ({presolve}, {presolve, binarize}) the reduced problem npp_build_prob made,
// the MIP solution npp_postprocess received, the printed lines and the final
// solution.
function mipPresolveCase(name, mk, gen) {
    if (ONLY && ('mippre_' + name).indexOf(ONLY) !== 0) return;
    var d = dumpProb(mk(), gen);
    d.name = name; d.kind = 'mip'; d.runs = [];
    [{presolve: glpk.GLP_ON}, {presolve: glpk.GLP_ON, binarize: glpk.GLP_ON}].forEach(function (opts) {
        var P = mk(), red = null, redsol = null, lines = [];
        glpk.__set_npp_hook(function (what, npp, prob) {
            if (what === 'build') {
                red = dumpProb(prob, null);
                red.row_ref = Array.from(npp.row_ref).slice(1);
                red.col_ref = Array.from(npp.col_ref).slice(1);
            } else {
                var j, x = [];
                for (j = 1; j <= prob.n; j++) x.push(prob.col[j].mipx);
                redsol = {mip_stat: prob.mip_stat, mip_obj: prob.mip_obj, col_mipx: x};
            }
        });
        glpk.glp_set_print_func(function (s) { lines.push(s); });
        var s0 = glpk.__cnt.solve_node;
        var ret = glpk.glp_intopt(P, new glpk.IOCP(opts));
        glpk.glp_set_print_func(function () {});
        glpk.__set_npp_hook(null);
        var j, x = [], rx = [];
        for (j = 1; j <= P.n; j++) x.push(P.col[j].mipx);
        for (j = 1; j <= P.m; j++) rx.push(P.row[j].mipx);
        d.runs.push({opts: opts, ret: ret, mip_stat: P.mip_stat, mip_obj: P.mip_obj, col_mipx: x, row_mipx: rx,
                     lp_solves: glpk.__cnt.solve_node - s0, lines: lines, reduced: red, reduced_sol: redsol});
    });
    fs.writeFileSync(path.join(OUT, 'mippre_' + name + '.json'), JSON.stringify(d));
    console.log('wrote mippre', name, d.runs.map(function (r) { return 'ret' + r.ret + ':stat' + r.mip_stat + ':obj' + r.mip_obj + ':lp' + r.lp_solves; }).join(' '));
}

// MIP instance under several IOCP option sets (branching rule br_tech,
// node selection bt_tech, preprocessing pp_tech; glpios09.js:1,
// glpios12.js:2, glpios03.js:643-656): one root solve per run, the
// reference's objective, incumbent and node-LP count for each.
function mipOptsCase(name, mk, optsList) {
    if (ONLY && ('mipopt_' + name).indexOf(ONLY) !== 0) return;
    var d = dumpProb(mk(), null);
    d.name = name; d.kind = 'mipopt'; d.runs = [];
    optsList.forEach(function (opts) {
        var P = mk();
        var root = runLp(P, {}, 0);
        var s0 = glpk.__cnt.solve_node, it0 = P.it_cnt;
        var lines = [];
        glpk.glp_set_print_func(function (s) { lines.push(s); });
        var t0 = process.hrtime.bigint();
        var ret = glpk.glp_intopt(P, new glpk.IOCP(opts));
        var dt = Number(process.hrtime.bigint() - t0) / 1e9;
        glpk.glp_set_print_func(function () {});
        var j, x = [];
        for (j = 1; j <= P.n; j++) x.push(P.col[j].mipx);
        d.runs.push({opts: opts, root_ret: root.ret, ret: ret, mip_stat: P.mip_stat, mip_obj: P.mip_obj, col_mipx: x,
                     lp_solves: glpk.__cnt.solve_node - s0, pivots: P.it_cnt - it0, seconds: dt, lines: lines});
    });
    fs.writeFileSync(path.join(OUT, 'mipopt_' + name + '.json'), JSON.stringify(d));
    console.log('wrote mipopt', name, d.runs.map(function (r) {
        return JSON.stringify(r.opts) + ':ret' + r.ret + ':mip' + r.mip_obj + ':lp' + r.lp_solves; }).join(' '));
}
var MIP_OPTS = [{br_tech: 1}, {br_tech: 2}, {br_tech: 3}, {br_tech: 5}, {bt_tech: 1}, {bt_tech: 2}, {bt_tech: 4},
                {br_tech: 3, bt_tech: 1}, {br_tech: 5, bt_tech: 4}, {pp_tech: 1}, {br_tech: 1, bt_tech: 2, pp_tech: 1},
                {mip_gap: 0.05}, {mip_gap: 0.01}, {mip_gap: 0.002, bt_tech: 2}];

// ---- C3 at full size (BASELINE.json configs[2]): the headline instance -----
// The reference's own timing run (BASELINE.md: first 300 dual pivots) as
// glp_simplex(SMCP{meth: GLP_DUAL, it_lim}) from the slack basis, once with
// it_lim = 300 and once as three it_lim = 100 calls continuing from the basis
// the previous call left (the bench's step definition: the factor and its
// update count persist in lp.bfd across calls).  Recorded: the pivot trace,
// statuses, objective, primal and dual values after the last call.  Gzipped
// (20k-entry vectors); A is not stored (the generator is exact, §8(d)).
function c3Case() {
    var zlib = require('zlib');
    var m = 4096, n = 16384, seed = 42;
    var d = {name: 'c3_itlim', kind: 'lp', gen: {kind: 'dense', m: m, n: n, seed: seed}, runs: []};
    [[300, 1], [100, 3]].forEach(function (c) {
        var t0 = Date.now();
        var P = genDense(m, n, seed);
        console.log('C3 built in', (Date.now() - t0) / 1000, 's');
        var calls = [], trace = [], lines = [], last = null;
        for (var k = 0; k < c[1]; k++) {
            last = runLp(P, {meth: glpk.GLP_DUAL, it_lim: c[0]}, 1000000);
            calls.push({ret: last.ret, it_cnt: last.it_cnt, obj_val: last.obj_val, factorizations: last.factorizations,
                        seconds: last.seconds});
            trace = trace.concat(last.trace);
            lines = lines.concat(last.lines);
            console.log('C3 call', k, 'ret', last.ret, 'it', last.it_cnt, 'obj', last.obj_val, last.seconds.toFixed(1), 's');
        }
        last.trace = trace; last.lines = lines; last.calls = calls;
        last.opts = {meth: glpk.GLP_DUAL, it_lim: c[0]}; last.ncalls = c[1];
        d.runs.push(last);
        P = null;
        if (global.gc) global.gc();
    });
    fs.writeFileSync(path.join(OUT, 'c3_itlim.json.gz'), zlib.gzipSync(JSON.stringify(d)));
    console.log('wrote c3_itlim.json.gz');
}
if (C3) { c3Case(); process.exit(0); }
// --deep MxN: one deep C5s instance (the multi-GPU B&B workload, SURVEY.md
// §8(d) generator) — the reference's glp_intopt on it, as mipCase records
// every MIP; minutes to hours of node time
if (process.argv.indexOf('--deep') >= 0) {
    var dm = process.argv[process.argv.indexOf('--deep') + 1].split('x').map(Number);
    mipCase('c5s_' + dm[0] + 'x' + dm[1], function () { return genC5s(dm[0], dm[1], 42); },
            {kind: 'c5s', m: dm[0], n: dm[1], seed: 42});
    process.exit(0);
}

// ---- instances ------------------------------------------------------------
lpCase('test', function () { return readLp('test.lpt'); }, null);
lpCase('todd', function () { return readLp('todd.lpt'); }, null);
lpCase('gap', function () { return readLp('gap.lpt'); }, null);
[[64, 256], [128, 512], [256, 1024]].forEach(function (s) {
    lpCase('dense_' + s[0] + 'x' + s[1], function () { return genDense(s[0], s[1], 42); },
           {kind: 'dense', m: s[0], n: s[1], seed: 42}, [1, 3], 100000,
           s[0] === 256 ? [{meth: 3, it_lim: 100}, {meth: 1, it_lim: 50}] : []);
});
for (var sd = 1; sd <= 32; sd++) {
    var mm = 4 + (sd * 7) % 29, nn = 5 + (sd * 13) % 41;
    (function (sd, mm, nn) {
        if (sd <= 12)
            lpCase('wild' + sd, function () { return genMix(sd, mm, nn, 0.35, false, false); }, null, [1, 2, 3]);
        else
            lpCase('mix' + sd, function () { return genMix(sd, mm, nn, 0.35, false, true); }, null, [1, 2, 3]);
    })(sd, mm, nn);
}
presolveCase('test', function () { return readLp('test.lpt'); }, null);
presolveCase('todd', function () { return readLp('todd.lpt'); }, null);
presolveCase('gap', function () { return readLp('gap.lpt'); }, null);
presolveCase('dense_64x256', function () { return genDense(64, 256, 42); }, {kind: 'dense', m: 64, n: 256, seed: 42});
for (var ps = 1; ps <= 32; ps++) {
    (function (sd, mm, nn) {
        presolveCase((sd <= 12 ? 'wild' : 'mix') + sd, function () { return genMix(sd, mm, nn, 0.35, false, sd > 12); }, null);
    })(ps, 4 + (ps * 7) % 29, 5 + (ps * 13) % 41);
}
for (var pz = 1; pz <= 12; pz++) {
    (function (sd) {
        presolveCase('sparse' + sd, function () { return genMix(200 + sd, 20 + 3 * sd, 25 + 4 * sd, 0.08, false, true, sd % 3 !== 0); }, null);
    })(pz);
}
bfcpCase('gap', function () { return readLp('gap.lpt'); }, null);
bfcpCase('todd', function () { return readLp('todd.lpt'); }, null);
bfcpCase('dense_64x256', function () { return genDense(64, 256, 42); }, {kind: 'dense', m: 64, n: 256, seed: 42});
bfcpCase('mix20', function () { return genMix(20, 4 + (20 * 7) % 29, 5 + (20 * 13) % 41, 0.35, false, true); }, null);
if (LPF_FIX) process.exit(0);
mipCase('gap', function () { return readLp('gap.lpt'); }, null);
mipCase('todd', function () { return readLp('todd.lpt'); }, null);
mipCase('c5s_12x20', function () { return genC5s(12, 20, 42); }, {kind: 'c5s', m: 12, n: 20, seed: 42});
for (var ms = 1; ms <= 12; ms++) {
    (function (ms) {
        mipCase('mixint' + ms, function () { return genMix(100 + ms, 6 + ms, 8 + 2 * ms, 0.5, true, true); }, null);
    })(ms);
}
mipPresolveCase('gap', function () { return readLp('gap.lpt'); }, null);
mipPresolveCase('todd', function () { return readLp('todd.lpt'); }, null);
mipPresolveCase('c5s_12x20', function () { return genC5s(12, 20, 42); }, {kind: 'c5s', m: 12, n: 20, seed: 42});
for (var mp = 1; mp <= 12; mp++) {
    (function (ms) {
        mipPresolveCase('mixint' + ms, function () { return genMix(100 + ms, 6 + ms, 8 + 2 * ms, 0.5, true, true); }, null);
    })(mp);
}
for (var mq = 1; mq <= 8; mq++) {
    (function (ms) {
        mipPresolveCase('sparseint' + ms, function () { return genMix(400 + ms, 20 + 2 * ms, 24 + 3 * ms, 0.1, 0.6, true, ms % 2 === 0); }, null);
    })(mq);
}
mipOptsCase('gap', function () { return readLp('gap.lpt'); }, MIP_OPTS);
mipOptsCase('c5s_12x20', function () { return genC5s(12, 20, 42); }, MIP_OPTS);
mipOptsCase('mixint4', function () { return genMix(104, 10, 16, 0.5, true, true); }, MIP_OPTS);
mipOptsCase('mixint9', function () { return genMix(109, 15, 26, 0.5, true, true); }, MIP_OPTS);
// glp_read_lp on CPLEX LP texts exercising every section and bound form
// (the Python reader problems.read_lp is pinned on these problem dumps; the
// texts travel in the fixture, the error cases record the reference's message)
function readCase(name, text) {
    if (ONLY && ('lpread_' + name).indexOf(ONLY) !== 0) return;
    var P = newProb(), d;
    try {
        glpk.glp_read_lp_from_string(P, null, text);
        d = dumpProb(P, null);
    } catch (e) {
        d = {error: String(e.message)};
    }
    d.text = text;
    fs.writeFileSync(path.join(OUT, 'lpread_' + name + '.json'), JSON.stringify(d));
    console.log('wrote lpread', name, d.error || (d.m + 'x' + d.n));
}
readCase('sections', [
    '\\ every bound form', 'Minimize', ' cost: 3 x + 2.5e-1 y - z + 0 w + 1e1 v', 'Subject To',
    ' c1: x + y + z >= 2', ' c2: - x + 3 y <= -1.5', ' 2 z - w = 4', ' c4: v + x - 0 y >= -3', 'Bounds',
    ' x <= 10', ' -5 <= y <= 5', ' z free', ' w >= -infinity', ' 0 <= v <= 0', ' q = 2', ' -inf <= r <= 7',
    ' s >= 1', 'Generals', ' y', 'Binaries', ' b', 'End', ''].join('\n'));
readCase('keywords', [
    'maximize', ' obj: x1 + x2 + x3', 'such that', ' x1 + x2 <= 4', ' r2: x2 + x3 <= 3',
    ' x1 + x3 =< 5', ' x3 => 0.5', 'bound', ' x1 <= 3', 'int', ' x2', 'end', ''].join('\n'));
readCase('st_dot', ['MIN', ' a + b', 'S.T.', ' a - b >= -2', ' a + 2 b <= 6', 'END', ''].join('\n'));
// the reference accepts any name but `inf' after `>= -' (glpcpx.js:543)
readCase('ge_quirk', ['Minimize', ' x + y', 'Subject To', ' x + y >= 1', 'Bounds', ' x >= -foo', 'End', ''].join('\n'));
readCase('err_geinf', ['Minimize', ' x + y', 'Subject To', ' x + y >= 1', 'Bounds', ' x >= -inf', 'End', ''].join('\n'));
readCase('err_noobj', ['Subject To', ' x + y <= 1', 'End', ''].join('\n'));
readCase('err_nost', ['Minimize', ' x + y', 'Bounds', ' x <= 1', 'End', ''].join('\n'));
readCase('err_dupvar', ['Minimize', ' x + x', 'Subject To', ' x <= 1', 'End', ''].join('\n'));
readCase('err_norhs', ['Minimize', ' x', 'Subject To', ' x <= y', 'End', ''].join('\n'));

// node LPs beyond the node kernel's 64 KiB of LDS (gk_mip.hip, HBM work area)
[[50, 80, 0.15], [60, 90, 0.15], [70, 100, 0.1], [48, 90, 0.35]].forEach(function (s, k) {
    mipCase('mixbig' + (k + 1), function () { return genMix(300 + k, s[0], s[1], 0.15, s[2], true, true); }, null);
});
// node LPs past the node kernel's work-area regime (m (2m + n) doubles of
// at least 2 MiB): glp_intopt's node LPs go to the engine (gk_mip.hip engine
// mode); sparse, a third of the columns integer, boxed columns (--bigmip)
if (process.argv.indexOf('--bigmip') >= 0) {
    [[250, 400, 0.012, 0.1], [320, 480, 0.01, 0.08], [400, 600, 0.008, 0.06], [800, 1200, 0.004, 0.05]].forEach(function (s, k) {
        mipCase('sparsebig' + (k + 1), function () { return genMix(700 + k, s[0], s[1], s[2], s[3], true, true); }, null);
    });
}
if (BIG) {
    lpCase('c2s', function () { return genC2s(821, 1571, 7, 42); }, {kind: 'c2s', m: 821, n: 1571, nzc: 7, seed: 42}, [3, 1], 0);
    lpCase('dense_512x2048', function () { return genDense(512, 2048, 42); }, {kind: 'dense', m: 512, n: 2048, seed: 42}, [1, 3], 0);
    mipCase('c5s_12x30', function () { return genC5s(12, 30, 42); }, {kind: 'c5s', m: 12, n: 30, seed: 42});
}

// ---- glp_scale_prob (glpscl.js:1): scale factors and printed lines ---------
// badly scaled sparse matrix with an empty row and an empty column
function genBadScale(seed, m, n, dens) {
    var r = new SplitMix(seed), P = newProb(), i, j;
    glpk.glp_add_rows(P, m); glpk.glp_add_cols(P, n);
    var ia = [0], ja = [0], ar = [0];
    for (i = 1; i <= m; i++) {
        if (i === 3) continue;
        for (j = 1; j <= n; j++) {
            if (j === 5 || r.u() >= dens) continue;
            var k = Math.floor(r.u() * 11) - 5;
            ia.push(i); ja.push(j); ar.push((r.u() < 0.5 ? -1 : 1) * Math.pow(10, k) * (1 + r.u()));
        }
    }
    glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
    return P;
}
function genWellScaled(seed, m, n) {
    var r = new SplitMix(seed), P = newProb(), i, j;
    glpk.glp_add_rows(P, m); glpk.glp_add_cols(P, n);
    var ia = [0], ja = [0], ar = [0];
    for (i = 1; i <= m; i++)
        for (j = 1; j <= n; j++)
            if (r.u() < 0.3) { ia.push(i); ja.push(j); ar.push(0.5 + 1.5 * r.u()); }
    glpk.glp_load_matrix(P, ia.length - 1, ia, ja, ar);
    return P;
}
var SCALE_FLAGS = [0, 0x01, 0x10, 0x20, 0x11, 0x31, 0x71, 0x80, 0x40, 0x21, 0x200];
function scaleCase(name, mk) {
    if (ONLY && ('scale_' + name).indexOf(ONLY) !== 0) return;
    var d = dumpProb(mk(), null);
    d.name = name; d.kind = 'scale'; d.runs = [];
    SCALE_FLAGS.forEach(function (flags) {
        var P = mk(), lines = [], run = {flags: flags};
        glpk.glp_set_print_func(function (s) { lines.push(s); });
        try {
            glpk.glp_scale_prob(P, flags);
            var i, j;
            run.rii = []; run.sjj = [];
            for (i = 1; i <= P.m; i++) run.rii.push(P.row[i].rii);
            for (j = 1; j <= P.n; j++) run.sjj.push(P.col[j].sjj);
        } catch (e) {
            run.error = String(e.message);
        }
        glpk.glp_set_print_func(function () {});
        run.lines = lines;
        d.runs.push(run);
    });
    fs.writeFileSync(path.join(OUT, 'scale_' + name + '.json'), JSON.stringify(d));
    console.log('wrote scale', name, d.m + 'x' + d.n);
}
scaleCase('test', function () { return readLp('test.lpt'); });
scaleCase('todd', function () { return readLp('todd.lpt'); });
scaleCase('gap', function () { return readLp('gap.lpt'); });
scaleCase('bad', function () { return genBadScale(77, 40, 60, 0.2); });
scaleCase('well', function () { return genWellScaled(78, 20, 30); });
scaleCase('dense_64x256', function () { return genDense(64, 256, 42); });
scaleCase('c2s', function () { return genC2s(821, 1571, 7, 42); });

// ---- glp_adv_basis (glpini01.js:1): the triangular starting basis ----------
// statuses and printed lines, the bad-flags error, and both simplex methods
// run from that basis
function advCase(name, mk) {
    if (ONLY && ('adv_' + name).indexOf(ONLY) !== 0) return;
    var P = mk(), d = dumpProb(P, null), lines = [];
    d.name = name; d.kind = 'adv';
    glpk.glp_set_print_func(function (s) { lines.push(s); });
    glpk.__glp_adv_basis(P, 0);
    glpk.glp_set_print_func(function () {});
    var b = snapshotBasis(P);
    d.adv = {row_stat: b.row_stat, col_stat: b.col_stat, lines: lines};
    try { glpk.__glp_adv_basis(mk(), 1); } catch (e) { d.adv.flags_error = String(e.message); }
    d.runs = [];
    [1, 3].forEach(function (meth) {
        var Q = mk();
        glpk.__glp_adv_basis(Q, 0);
        d.runs.push(runLp(Q, {meth: meth}, 0));
    });
    fs.writeFileSync(path.join(OUT, 'adv_' + name + '.json'), JSON.stringify(d));
    console.log('wrote adv', name, d.m + 'x' + d.n, d.adv.lines.join(' | '),
                d.runs.map(function (r) { return 'meth' + r.opts.meth + ':ret' + r.ret + ':it' + r.it_cnt + ':obj' + r.obj_val; }).join(' '));
}
advCase('test', function () { return readLp('test.lpt'); });
advCase('todd', function () { return readLp('todd.lpt'); });
advCase('gap', function () { return readLp('gap.lpt'); });
advCase('dense_64x256', function () { return genDense(64, 256, 42); });
advCase('c2s', function () { return genC2s(821, 1571, 7, 42); });
[13, 14, 15, 16, 17, 18].forEach(function (sd) {
    advCase('mix' + sd, function () { return genMix(sd, 8 + sd, 10 + 2 * sd, 0.35, false, true); });
});
[1, 2, 3].forEach(function (sd) {
    advCase('wild' + sd, function () { return genMix(sd, 6 + 2 * sd, 9 + 3 * sd, 0.35, false, false); });
});
advCase('mixbig1', function () { return genMix(300, 50, 80, 0.15, false, true, false); });
advCase('nocols', function () { var P = newProb(); glpk.glp_add_rows(P, 3); return P; });

// ---- glp_eval_tab_row (glpapi12.js:401) on optimal bases -------------------
// the problem (after scaling, when asked: rii / sjj in the dump), the basis
// glp_simplex left, and the tableau row of every basic variable (up to 48)
function tabCase(name, mk, scale) {
    if (ONLY && ('tab_' + name).indexOf(ONLY) !== 0) return;
    var P = mk();
    if (scale) glpk.glp_scale_prob(P, scale);
    var ret = glpk.glp_simplex(P, new glpk.SMCP({meth: glpk.GLP_DUAL, presolve: glpk.GLP_OFF}));
    var d = dumpProb(P, null);
    d.name = name; d.kind = 'tab'; d.simplex_ret = ret;
    var b = snapshotBasis(P), rows = [], k;
    d.row_stat = b.row_stat; d.col_stat = b.col_stat;
    for (k = 1; k <= P.m + P.n && rows.length < 48; k++) {
        var st = k <= P.m ? P.row[k].stat : P.col[k - P.m].stat;
        if (st !== glpk.GLP_BS) continue;
        var ind = new Int32Array(1 + P.n), val = new Float64Array(1 + P.n);
        var len = glpk.glp_eval_tab_row(P, k, ind, val);
        rows.push({k: k, ind: Array.from(ind.slice(1, len + 1)), val: Array.from(val.slice(1, len + 1))});
    }
    d.tab_rows = rows;
    fs.writeFileSync(path.join(OUT, 'tab_' + name + '.json'), JSON.stringify(d));
    console.log('wrote tab', name, d.m + 'x' + d.n, 'ret', ret, rows.length, 'rows');
}
tabCase('test', function () { return readLp('test.lpt'); }, 0);
tabCase('gap', function () { return readLp('gap.lpt'); }, 0);
tabCase('dense_64x256', function () { return genDense(64, 256, 42); }, 0);
tabCase('dense_64x256_scaled', function () { return genDense(64, 256, 42); }, glpk.GLP_SF_GM | glpk.GLP_SF_EQ | glpk.GLP_SF_2N);
tabCase('mix14_scaled', function () { return genMix(14, 22, 38, 0.35, false, true); }, glpk.GLP_SF_GM | glpk.GLP_SF_EQ);
tabCase('c2s_scaled', function () { return genC2s(821, 1571, 7, 42); }, glpk.GLP_SF_GM | glpk.GLP_SF_EQ);
