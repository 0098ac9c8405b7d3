// gk_core.js — JS side of the drop-in boundary (Node.js, CommonJS).
//
// Marshals the reference's problem object (`lp`, glpapi01.js) into the flat,
// 1-based typed arrays of gk_lp (include/glpk_mi355x.h) — exactly the fields
// init_csa reads (glpspx01.js:42-145 / glpspx02.js:89-190) — calls the native
// core through the N-API addon (js/gk_addon.c), and writes back what
// store_sol writes (glpspx01.js:1591-1681 / glpspx02.js:1499-1590).
//
// There is no CPU fallback: without a gfx950 device the first call throws
// the native error text.
'use strict';
var path = require('path');

var addon = require(path.join(__dirname, 'build', 'gk_addon.node'));

var GLP_BS = 1, GLP_UNDEF = 1, GLP_EFAIL = 0x05;
var ctx = null;
var version = 0;

// once an external with a finalizer exists (context, factor, communicator),
// the process leaves from node's 'exit' event with its exit code, before
// libnode 12's environment teardown (see exitNow in gk_addon.c); the
// listener is registered last-in at that moment, so listeners the program
// registered earlier still run
var exitArmed = false;
function armExit() {
    if (exitArmed) return;
    exitArmed = true;
    process.on('exit', function (code) { addon.exitNow(code === undefined ? process.exitCode || 0 : code); });
}

function context() {
    if (ctx === null) {
        armExit();
        ctx = addon.create(parseInt(process.env.GK_DEVICE || '0', 10));
    }
    return ctx;
}

function nextVersion() { return ++version; }
// while > 0 every solve hands the engine b_version 0 (bounds / costs
// unknown: init_csa rebuilds and compares): the shim holds it around
// reference code that writes an lp's bounds or costs directly
var bvHold = 0;
function bversionHold(d) { bvHold += d; return bvHold; }

// ---- lp.bfd (glpbfd.js) ------------------------------------------------------
function bfdCreate() {
    // the JS object the reference keeps in lp.bfd; the native factor is owned
    // by the addon external (freed by its finalizer)
    return {gk: addon.bfdCreate(context()), valid: 0, m: 0};
}

function bfdSetParm(bfd, parm) { addon.bfdSetParm(bfd.gk, parm); }
function bfdResetParm(bfd) { addon.bfdResetParm(bfd.gk); }

// bfd_factorize(bfd, m, bh, col, info) (glpbfd.js:47): the columns come from
// the reference's own callback col(info, j, ind, val) (b_col, glpapi12.js:7)
function bfdFactorize(bfd, m, bh, col, info) {
    var ptr = new Int32Array(m + 2), tind = new Int32Array(m + 1), tval = new Float64Array(m + 1);
    var ind = [0], val = [0];
    ptr[1] = 1;
    for (var j = 1; j <= m; j++) {
        var len = col(info, j, tind, tval);
        for (var t = 1; t <= len; t++) { ind.push(tind[t]); val.push(tval[t]); }
        ptr[j + 1] = ptr[j] + len;
    }
    var ret = addon.bfdFactorizeCsc(bfd.gk, m, ptr, Int32Array.from(ind), Float64Array.from(val));
    bfd.valid = ret === 0 ? 1 : 0;
    bfd.m = m;
    return ret;
}

function solve(bfd, x, tr) {
    var y = (x instanceof Float64Array) ? x : Float64Array.from(x);
    if (tr) addon.bfdBtran(bfd.gk, y); else addon.bfdFtran(bfd.gk, y);
    if (y !== x) for (var i = 1; i <= bfd.m; i++) x[i] = y[i];
}
function bfdFtran(bfd, x) { solve(bfd, x, 0); }
function bfdBtran(bfd, x) { solve(bfd, x, 1); }

function bfdUpdate(bfd, j, bh, len, ind, idx, val) {
    var ret = addon.bfdUpdate(bfd.gk, j, len, Int32Array.from(ind), idx, Float64Array.from(val));
    if (ret !== 0) bfd.valid = 0;
    return ret;
}
function bfdGetCount(bfd) { return addon.bfdGetCount(bfd.gk); }

// ---- spx_primal / spx_dual ---------------------------------------------------
function arrays(lp) {
    var m = lp.m, n = lp.n, g = lp.__gk;
    if (!g || g.m !== m || g.n !== n) {
        g = lp.__gk = {
            m: m, n: n,
            row_type: new Int8Array(m + 1), row_lb: new Float64Array(m + 1), row_ub: new Float64Array(m + 1),
            rii: new Float64Array(m + 1), row_stat: new Int8Array(m + 1), row_bind: new Int32Array(m + 1),
            row_prim: new Float64Array(m + 1), row_dual: new Float64Array(m + 1),
            col_type: new Int8Array(n + 1), col_lb: new Float64Array(n + 1), col_ub: new Float64Array(n + 1),
            col_coef: new Float64Array(n + 1), sjj: new Float64Array(n + 1), col_stat: new Int8Array(n + 1),
            col_bind: new Int32Array(n + 1), col_prim: new Float64Array(n + 1), col_dual: new Float64Array(n + 1),
            head: new Int32Array(m + 1), a_version: 0
        };
    }
    return g;
}

// A by columns in list order (init_csa glpspx01.js:96-108), unscaled; the
// device scales rii * a * sjj in the same order.  Re-walked only when a
// matrix/scale mutator ran since the last call (lp.__gk_version).
function marshalMatrix(lp, g) {
    if (lp.__gk_version === undefined) lp.__gk_version = nextVersion();
    if (g.a_version === lp.__gk_version && g.nnz === lp.nnz) return;
    var n = lp.n, nnz = lp.nnz;
    var ptr = new Int32Array(n + 2), ind = new Int32Array(nnz + 1), val = new Float64Array(nnz + 1);
    var loc = 1;
    for (var j = 1; j <= n; j++) {
        ptr[j] = loc;
        for (var aij = lp.col[j].ptr; aij !== null; aij = aij.c_next) {
            ind[loc] = aij.row.i;
            val[loc] = aij.val;
            loc++;
        }
    }
    ptr[n + 1] = loc;
    if (loc !== nnz + 1) throw new Error('assert');
    g.A_ptr = ptr; g.A_ind = ind; g.A_val = val; g.nnz = nnz;
    g.a_version = lp.__gk_version;
}

// the init_csa inputs of lp into the marshalled object L
function marshal(lp, g) {
    var m = lp.m, n = lp.n, i, j, row, col;
    for (i = 1; i <= m; i++) {
        row = lp.row[i];
        g.row_type[i] = row.type; g.row_lb[i] = row.lb; g.row_ub[i] = row.ub;
        g.rii[i] = row.rii; g.row_stat[i] = row.stat;
    }
    for (j = 1; j <= n; j++) {
        col = lp.col[j];
        g.col_type[j] = col.type; g.col_lb[j] = col.lb; g.col_ub[j] = col.ub;
        g.col_coef[j] = col.coef; g.sjj[j] = col.sjj; g.col_stat[j] = col.stat;
    }
    for (i = 1; i <= m; i++) g.head[i] = lp.head[i];
    marshalMatrix(lp, g);
    return {
        m: m, n: n, nnz: lp.nnz, dir: lp.dir, c0: lp.c0, a_version: g.a_version, it_cnt: lp.it_cnt,
        b_version: bvHold > 0 ? 0 : (lp.__gk_bversion || 0),
        row_type: g.row_type, row_lb: g.row_lb, row_ub: g.row_ub, rii: g.rii,
        col_type: g.col_type, col_lb: g.col_lb, col_ub: g.col_ub, col_coef: g.col_coef, sjj: g.sjj,
        A_ptr: g.A_ptr, A_ind: g.A_ind, A_val: g.A_val, head: g.head,
        row_stat: g.row_stat, col_stat: g.col_stat, row_bind: g.row_bind, col_bind: g.col_bind,
        row_prim: g.row_prim, row_dual: g.row_dual, col_prim: g.col_prim, col_dual: g.col_dual
    };
}

// the simplex's terminal output (gk_bfd_set_report) as the reference prints
// it (display, glpspx01.js:1587 / glpspx02.js:1492-1495, and the main loops'
// xprintf lines): one report -> its lines
var MSG = {1: 'OPTIMAL SOLUTION FOUND', 2: 'PROBLEM HAS NO DUAL FEASIBLE SOLUTION',
           3: 'PROBLEM HAS NO FEASIBLE SOLUTION', 4: 'PROBLEM HAS UNBOUNDED SOLUTION',
           5: 'ITERATION LIMIT EXCEEDED; SEARCH TERMINATED', 6: 'TIME LIMIT EXCEEDED; SEARCH TERMINATED',
           7: 'OBJECTIVE LOWER LIMIT REACHED; SEARCH TERMINATED', 8: 'OBJECTIVE UPPER LIMIT REACHED; SEARCH TERMINATED',
           10: 'Error: unable to choose basic variable on phase I'};
function reportLines(r) {
    var kind = r[0], code = r[1], it = r[2], phase = r[3], obj = r[4], inf = r[5], aux = r[6];
    if (kind === 1) {
        if (code === 1) return [(phase == 1 ? ' ' : '*') + it + ": obj = " + obj + "  infeas = " + inf + " (" + aux + ")"];
        if (phase == 1) return [" " + it + ":  infeas = " + inf + " (" + aux + ")"];
        return ["|" + it + ": obj = " + obj + "  infeas = " + inf + " (" + aux + ")"];
    }
    if (code === 9)
        return ["Warning: numerical instability (" + (aux == 1 ? "primal" : "dual") + " simplex, phase " +
                (phase == 1 ? "I" : "II") + ")"];
    if (code === 11)
        return ["Error: unable to factorize the basis matrix (" + aux + ")",
                "Sorry, basis recovery procedure not implemented yet"];
    return MSG[code] ? [MSG[code]] : [];
}
module.exports.reportLines = reportLines;

// print: the reference's xprintf (the shim passes it), called in order for
// every line the solve produced
function spx(lp, parm, dual, print) {
    var m = lp.m, n = lp.n, i, j, row, col;
    var g = arrays(lp);
    var L = marshal(lp, g);
    // init_csa asserts lp.valid and takes lp.bfd (glpspx01.js:129-132)
    if (!lp.valid || lp.bfd === null) throw new Error('assert');
    var ret = addon.spx(context(), lp.bfd.gk, L, parm, dual);
    if (print && L.reports)
        L.reports.forEach(function (r) { reportLines(r).forEach(function (s) { print(s); }); });
    lp.valid = L.valid;
    lp.bfd.valid = L.valid;
    lp.pbs_stat = L.pbs_stat;
    lp.dbs_stat = L.dbs_stat;
    lp.obj_val = L.obj_val;
    lp.it_cnt = L.it_cnt;
    lp.some = L.some;
    if (L.valid) {
        // store_sol
        for (i = 1; i <= m; i++) lp.head[i] = g.head[i];
        for (i = 1; i <= m; i++) {
            row = lp.row[i];
            row.stat = g.row_stat[i]; row.bind = g.row_bind[i];
            row.prim = g.row_prim[i]; row.dual = g.row_dual[i];
        }
        for (j = 1; j <= n; j++) {
            col = lp.col[j];
            col.stat = g.col_stat[j]; col.bind = g.col_bind[j];
            col.prim = g.col_prim[j]; col.dual = g.col_dual[j];
        }
    } else if (ret === GLP_EFAIL) {
        lp.pbs_stat = lp.dbs_stat = GLP_UNDEF;
        lp.obj_val = 0.0;
        lp.some = 0;
    }
    return ret;
}

// ---- ios_driver (glpios03.js:1) ---------------------------------------------
var GLP_IV = 2, GLP_FEAS = 2, GLP_OPT = 5;

// the requests the native driver serves: no callbacks (glpios03.js:533-897),
// no cut generators / feasibility pump (they stay in JS).  Any size: node LPs
// whose tableau fits the node kernel's work area (gk_mip.hip: LDS up to
// 64 KiB, HBM slices up to 2 MiB) run batched in it, larger ones on the
// engine's revised simplex (gk_mip.hip engine mode)
function nativeIos(T) {
    var parm = T.parm;
    if (parm.cb_func != null) return false;
    if (parm.gmi_cuts || parm.mir_cuts || parm.cov_cuts || parm.clq_cuts || parm.fp_heur) return false;
    return true;
}

// T = the tree of ios_create_tree: T.mip is the problem (its LP relaxation
// solved to optimality by glp_intopt's caller), T.parm the IOCP.  Writes what
// the reference's driver writes into the problem on an integer solution
// (record_solution, glpios03.js:113-135): mip_stat = GLP_FEAS, mip_obj, mipx;
// solve_mip then turns FEAS into OPT (glpapi09.js:82-92).
// show_progress (glpios03.js:2-48) for one GK_RPT_MIP record of the native
// driver: [kind, code (1 bingo | 2 incumbent | 4 tree empty), it_cnt,
// a_cnt, obj, best bound, fathomed]
function mipProgressLine(dir, r) {
    var code = r[1], best_mip, best_bound, rho, rel_gap, temp;
    best_mip = (code & 2) ? String(r[4]) : "not found yet";
    if (code & 4) best_bound = "tree is empty";
    else if (r[5] == -DBL_MAX) best_bound = "-inf";
    else if (r[5] == +DBL_MAX) best_bound = "+inf";
    else best_bound = r[5];
    rho = dir == GLP_MIN ? ">=" : "<=";
    if (!(code & 2)) temp = DBL_MAX;                      // ios_relative_gap (glpios01.js:842)
    else if (code & 4) temp = 0.0;
    else temp = Math.abs(r[4] - r[5]) / (Math.abs(r[4]) + DBL_EPSILON);
    if (temp == 0.0) rel_gap = "  0.0%";
    else if (temp < 0.001) rel_gap = " < 0.1%";
    else if (temp <= 9.999) rel_gap = "  " + Number(100.0 * temp).toFixed(1) + "%";
    else rel_gap = "";
    return "+" + r[2] + ": " + ((code & 1) ? ">>>>>" : "mip =") + " " + best_mip + " " + rho + " " + best_bound +
           " " + rel_gap + " (" + r[3] + "; " + r[6] + ")";
}
var GLP_MIN = 1, DBL_MAX = 1.7976931348623157e308, DBL_EPSILON = 2.220446049250313e-16;

// one process per GPU (SURVEY.md §8(e)): with GK_WORLD_SIZE (or WORLD_SIZE)
// above 1 in the environment, glp_intopt's search is sharded over the ranks
// through the library's collective (gk_comm: RCCL between distinct devices,
// TCP through rank 0 otherwise), rank from GK_RANK / RANK, rank 0's address
// from GK_COMM_ADDR or MASTER_ADDR:MASTER_PORT; every rank returns the same
// incumbent.  GK_RAMP_NODES < 0 hands the whole tree to rank 0 first (the
// open-node exchange feeds the others).
var __comm = undefined;
function comm() {
    if (__comm !== undefined) return __comm;
    var env = process.env;
    var size = parseInt(env.GK_WORLD_SIZE || env.WORLD_SIZE || '1', 10);
    if (!(size > 1)) { __comm = null; return __comm; }
    var rank = parseInt(env.GK_RANK || env.RANK || '0', 10);
    var addr = env.GK_COMM_ADDR || ((env.MASTER_ADDR || '127.0.0.1') + ':' + (env.MASTER_PORT || '29533'));
    __comm = addon.commCreate(context(), rank, size, addr, parseInt(env.GK_COMM_BACKEND || '0', 10));
    if (env.GK_RAMP_NODES) addon.commOption(__comm, 1, parseInt(env.GK_RAMP_NODES, 10));
    return __comm;
}

function iosDriver(T, print) {
    var P = T.mip, m = P.m, n = P.n, i, j;
    var g = arrays(P);
    var L = marshal(P, g);
    if (!g.col_kind || g.col_kind.length !== n + 1) {
        g.col_kind = new Int8Array(n + 1);
        g.row_mipx = new Float64Array(m + 1);
        g.col_mipx = new Float64Array(n + 1);
    }
    for (j = 1; j <= n; j++) g.col_kind[j] = P.col[j].kind;
    L.col_kind = g.col_kind; L.row_mipx = g.row_mipx; L.col_mipx = g.col_mipx;
    L.pbs_stat = P.pbs_stat; L.dbs_stat = P.dbs_stat; L.obj_val = P.obj_val;
    var cm = comm();
    var ret = cm ? addon.ios(context(), L, T.parm, cm) : addon.ios(context(), L, T.parm);
    if (print && L.reports)
        L.reports.forEach(function (r) { print(mipProgressLine(P.dir, r)); });
    if (L.mip_stat === GLP_OPT || (ret !== 0 && L.mip_stat === GLP_FEAS)) {
        P.mip_stat = GLP_FEAS;
        P.mip_obj = L.mip_obj;
        for (i = 1; i <= m; i++) P.row[i].mipx = g.row_mipx[i];
        for (j = 1; j <= n; j++) P.col[j].mipx = g.col_mipx[j];
    }
    return ret;
}

module.exports = {
    addon: addon, context: context, nextVersion: nextVersion, bversionHold: bversionHold,
    bfdCreate: bfdCreate, bfdSetParm: bfdSetParm, bfdResetParm: bfdResetParm, bfdFactorize: bfdFactorize,
    bfdFtran: bfdFtran, bfdBtran: bfdBtran, bfdUpdate: bfdUpdate, bfdGetCount: bfdGetCount,
    spx: spx, iosDriver: iosDriver, nativeIos: nativeIos, GLP_BS: GLP_BS, mipProgressLine: mipProgressLine,
    comm: comm
};

// ---- glp_scale_prob (glpscl.js:1) -------------------------------------------
// A by columns in list order (the row numbers of the aij elements), the
// factors and the report numbers from the device (gk_scale_prob)
function scaleProb(lp, flags) {
    var m = lp.m, n = lp.n, ptr = new Int32Array(n + 1), ind = [], val = [];
    for (var j = 1; j <= n; j++) {
        for (var a = lp.col[j].ptr; a != null; a = a.c_next) { ind.push(a.row.i); val.push(a.val); }
        ptr[j] = ind.length;
    }
    var rii = new Float64Array(Math.max(m, 1)), sjj = new Float64Array(Math.max(n, 1)), rep = new Float64Array(13);
    var ret = addon.scale(context(), m, n, ptr, Int32Array.from(ind), Float64Array.from(val), flags | 0, rii, sjj, rep);
    return {ret: ret, rii: rii, sjj: sjj, report: rep};
}
module.exports.scaleProb = scaleProb;

// ---- glp_adv_basis (glpini01.js:1) -------------------------------------------
// the statuses of the triangular starting basis (gk_adv_basis, host code)
function advBasis(lp) {
    var m = lp.m, n = lp.n, i, j, g = arrays(lp);
    for (i = 1; i <= m; i++) { var R = lp.row[i]; g.row_type[i] = R.type; g.row_lb[i] = R.lb; g.row_ub[i] = R.ub; }
    for (j = 1; j <= n; j++) { var Cj = lp.col[j]; g.col_type[j] = Cj.type; g.col_lb[j] = Cj.lb; g.col_ub[j] = Cj.ub; }
    marshalMatrix(lp, g);
    var rs = new Int8Array(m + 1), cs = new Int8Array(n + 1);
    var size = addon.advBasis(m, n, g.row_type, g.row_lb, g.row_ub, g.col_type, g.col_lb, g.col_ub,
                              g.A_ptr, g.A_ind, rs, cs);
    return {size: size, row_stat: rs, col_stat: cs};
}
module.exports.advBasis = advBasis;

// glp_eval_tab_row (glpapi12.js:401) for a batch of basic variables ks on
// the current factor: one Float64Array row of m + n entries per k (index
// j - 1 = alfa of variable j, 0 for basic variables), one device GEMM for
// the batch (gk_bfd_eval_tab_rows; perRow: the per-row device path)
function evalTabRows(lp, ks, perRow) {
    if (!(lp.m == 0 || lp.valid) || lp.bfd === null) throw new Error('glp_eval_tab_row: basis factorization does not exist');
    var g = arrays(lp), L = marshal(lp, g), w = lp.m + lp.n;
    var out = new Float64Array(ks.length * w);
    addon.evalTabRows(lp.bfd.gk, L, Int32Array.from(ks), out, perRow ? 1 : 0);
    var rows = [];
    for (var t = 0; t < ks.length; t++) rows.push(out.subarray(t * w, (t + 1) * w));
    return rows;
}
module.exports.evalTabRows = evalTabRows;

// ---- LP / MIP preprocessor (glpnpp01.js .. glpnpp05.js) ----------------------
// the native workspace (gk_npp_*) behind the reference's npp_* calls made by
// glp_simplex / glp_intopt (glpapi06.js:41, glpapi09.js:116)
var GLP_SOL = 1, GLP_MIP = 3;
function nppLoad(orig, sol) {
    var g = arrays(orig);
    var L = marshal(orig, g);
    var kind = null, j;
    if (sol === GLP_MIP) {
        kind = new Int8Array(orig.n + 1);
        for (j = 1; j <= orig.n; j++) kind[j] = orig.col[j].kind;
    }
    var h = addon.nppCreate();
    addon.nppLoad(h, L, kind, sol);
    return {h: h, sol: sol, dir: orig.dir};
}
// a stop of the preprocessor ends the caller's use of the workspace
// (glpapi06.js:84, glpapi09.js:162)
function nppDone(w) {
    if (w.h !== null) addon.nppFree(w.h);
    w.h = null;
}
function nppSimplex(w) {
    var ret = addon.nppSimplex(w.h);
    if (ret !== 0) nppDone(w);
    return ret;
}
// npp_integer's lines (glpnpp04.js:92-97, glpnpp05.js:475-514) through the
// reference's xprintf (term_out as the caller set it)
function nppInteger(w, parm, print) {
    var msg = new Int32Array(7);
    var ret = addon.nppInteger(w.h, parm && parm.binarize ? 1 : 0, msg);
    if (ret === 0) {
        if (msg[0] > 0) print(msg[0] + " integer variable(s) were replaced by " + msg[1] + " binary ones");
        if (msg[2] > 0) print(msg[2] + " row(s) were added due to binarization");
        if (msg[3] > 0) print("Binarization failed for " + msg[3] + " integer variable(s)");
        if (msg[4] > 0) print(msg[4] + " hidden packing inequaliti(es) were detected");
        if (msg[5] > 0) print(msg[5] + " hidden covering inequaliti(es) were detected");
        if (msg[6] > 0) print(msg[6] + " constraint coefficient(s) were reduced");
    } else
        nppDone(w);
    return ret;
}
// the reduced problem as arrays (1-based; A by columns in the order the
// reference's glp_set_mat_col leaves them)
function nppBuild(w) {
    var sz = new Int32Array(3);
    addon.nppBuildSize(w.h, sz);
    var m = sz[0], n = sz[1], nnz = sz[2];
    var r = {m: m, n: n, nnz: nnz, dir: w.dir,
             row_type: new Int8Array(m + 1), row_lb: new Float64Array(m + 1), row_ub: new Float64Array(m + 1),
             col_type: new Int8Array(n + 1), col_lb: new Float64Array(n + 1), col_ub: new Float64Array(n + 1),
             col_coef: new Float64Array(n + 1), col_kind: new Int8Array(n + 1), A_ptr: new Int32Array(n + 2),
             A_ind: new Int32Array(nnz + 1), A_val: new Float64Array(nnz + 1), row_ref: new Int32Array(m + 1),
             col_ref: new Int32Array(n + 1), c0: new Float64Array(1)};
    addon.nppBuild(w.h, r.row_type, r.row_lb, r.row_ub, r.col_type, r.col_lb, r.col_ub, r.col_coef, r.col_kind,
                   r.A_ptr, r.A_ind, r.A_val, r.row_ref, r.col_ref, r.c0);
    w.m = m; w.n = n;
    return r;
}
function nppPostprocess(w, prob) {
    var i, j, m = prob.m, n = prob.n;
    if (w.sol === GLP_MIP) {
        var mx = new Float64Array(n + 1);
        for (j = 1; j <= n; j++) mx[j] = prob.col[j].mipx;
        addon.nppPostprocess(w.h, prob.mip_stat, 0, null, null, null, mx);
        return;
    }
    var rs = new Int8Array(m + 1), rd = new Float64Array(m + 1), cs = new Int8Array(n + 1), cp = new Float64Array(n + 1);
    for (i = 1; i <= m; i++) { rs[i] = prob.row[i].stat; rd[i] = prob.row[i].dual; }
    for (j = 1; j <= n; j++) { cs[j] = prob.col[j].stat; cp[j] = prob.col[j].prim; }
    addon.nppPostprocess(w.h, prob.pbs_stat, prob.dbs_stat, rs, rd, cs, cp);
}
function nppUnload(w, orig) {
    var g = arrays(orig), L = marshal(orig, g), i, j, row, col;
    if (w.sol === GLP_MIP) {
        var kind = new Int8Array(orig.n + 1), rx = new Float64Array(orig.m + 1), cx = new Float64Array(orig.n + 1);
        for (j = 1; j <= orig.n; j++) kind[j] = orig.col[j].kind;
        addon.nppUnloadMip(w.h, L, kind, rx, cx);
        nppDone(w);
        orig.mip_stat = L.mip_stat;
        orig.mip_obj = L.mip_obj;
        for (j = 1; j <= orig.n; j++) orig.col[j].mipx = cx[j];
        for (i = 1; i <= orig.m; i++) orig.row[i].mipx = rx[i];
        return;
    }
    addon.nppUnloadSol(w.h, L);
    nppDone(w);
    orig.valid = 0;
    orig.pbs_stat = L.pbs_stat;
    orig.dbs_stat = L.dbs_stat;
    orig.obj_val = L.obj_val;
    orig.some = 0;
    for (i = 1; i <= orig.m; i++) {
        row = orig.row[i];
        row.stat = g.row_stat[i]; row.prim = g.row_prim[i]; row.dual = g.row_dual[i];
    }
    for (j = 1; j <= orig.n; j++) {
        col = orig.col[j];
        col.stat = g.col_stat[j]; col.prim = g.col_prim[j]; col.dual = g.col_dual[j];
    }
}
module.exports.nppLoad = nppLoad;
module.exports.nppSimplex = nppSimplex;
module.exports.nppInteger = nppInteger;
module.exports.nppBuild = nppBuild;
module.exports.nppPostprocess = nppPostprocess;
module.exports.nppUnload = nppUnload;
