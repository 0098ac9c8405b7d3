// Primal simplex pivot pipeline (glpspx01.js main loop :1705-2056) on the
// structure of the explicit inverse, the primal counterpart of gk_dual.hip.
//
// inv(B) e_c = e_{bind[c]} exactly for every basic slack c, so only the nr
// columns in rlist (the non-basic slacks) carry data; the commit kernel
// maintains the list.  A pivot is four kernels, each gated on st->stop, the
// choices that need a whole vector carried as per-wave / per-group
// candidates by the kernel that produces the vector:
//   k_primal_ftran   grid  chuzc (:646) from the commit's candidates, the
//                          PSE reset (:586), phase-I check (:1483); tcol =
//                          inv(B) h, h = -N[q] (eval_tcol :690) over the dense
//                          columns; per 64-row group: max |tcol|, the d_q
//                          check sum (:1901-1919), gamma_q partial and the
//                          PSE vector (update_gamma :1208-1218), and the
//                          Harris pass-1 candidate (chuzr :808-870)
//   k_primal_ratio   grid  the d_q check, pass-1 choice (with the bound flip
//                          of a double-bounded xN[q]), pass-2 candidates
//                          (:871-1028); extra blocks: u = inv(B)' v (update_gamma's
//                          bfd_btran :1220) over the dense columns
//   k_primal_row     grid  the pass-2 choice p, rho = row p of inv(B)
//   k_primal_col           (eval_rho :1030), the pivot row trow_j = -rho' N_j
//                          (eval_trow :1058) over the rows of AT in the
//                          support of rho (dense A) or the CSC entries (sparse
//                          A), and s_j = N_j' u (update_gamma :1230-1241)
//   k_primal_commit  grid  pivot check (:1950-1965), update_bbar (:1100),
//                          update_cbar (:1154), update_gamma (:1178),
//                          change_basis (:2035-2055) and the list maintenance,
//                          rank-1 update of inv(B); the chuzc candidates and
//                          the phase-I check of the next pivot
// The rigorous mode (after a failed accuracy check) keeps the earlier
// single-workgroup kernels (gk_kernels.hip: primal_iteration).
#include "gk_device.h"
#include <algorithm>

namespace gk {

// primal-only candidate / partial regions beyond the dual's (engine_alloc):
// per-row-group pass-1 candidates, then max |tcol|, d_q check sums and
// gamma_q sums of the groups (16 gv each)
__device__ __forceinline__ Cand *pcand1(const SpxDev &d) { return (Cand *)d.cand + 12 * gv_of(d.m, d.n); }
__device__ __forceinline__ double *ptmax(const SpxDev &d) { return d.gpart + 8 * gv_of(d.m, d.n); }
__device__ __forceinline__ double *pdsum(const SpxDev &d) { return d.gpart + 24 * gv_of(d.m, d.n); }
__device__ __forceinline__ double *pvsum(const SpxDev &d) { return d.gpart + 40 * gv_of(d.m, d.n); }

// the candidates carry the basic variable and its new status: aux = 8 k + stat
__device__ __forceinline__ int aux_k(int aux) { return aux >> 3; }
__device__ __forceinline__ int aux_stat(int aux) { return aux & 7; }

// ---------------------------------------------------------------------------
// the Harris ratio test of the primal (chuzr, glpspx01.js:808-1028): basic
// row i holding variable k with value bb; pass 1 against the bounds relaxed
// by rtol (1 + 0.1 |bound|), pass 2 against the exact bounds with t <= tmax;
// phase I only lets infeasible basics (coef != 0) reach the violated bound
// ---------------------------------------------------------------------------
struct PRatio {
    double eps, s, rtol;
    int phase;
};

template <int PASS>
__device__ __forceinline__ bool prow_cand(const PRatio &x, double tv, double bb, int tk, double lbk, double ubk,
                                          double ck, int i, int k, double tmax, Cand &e)
{
    if (tv == 0.0 || fabs(tv) < x.eps) return false;
    const double alfa = x.s * tv;
    double t;
    int ist;
    if (alfa > 0.0) {
        if (x.phase == 1 && ck < 0.0) {
            if (PASS == 1) t = ((lbk + x.rtol * (1.0 + 0.10 * fabs(lbk))) - bb) / alfa;
            else t = (lbk - bb) / alfa;
            ist = NL;
        } else if (x.phase == 1 && ck > 0.0) return false;
        else if (tk == UP || tk == DB || tk == FX) {
            if (PASS == 1) t = ((ubk + x.rtol * (1.0 + 0.10 * fabs(ubk))) - bb) / alfa;
            else t = (ubk - bb) / alfa;
            ist = NU;
        } else return false;
    } else {
        if (x.phase == 1 && ck > 0.0) {
            if (PASS == 1) t = ((ubk - x.rtol * (1.0 + 0.10 * fabs(ubk))) - bb) / alfa;
            else t = (ubk - bb) / alfa;
            ist = NU;
        } else if (x.phase == 1 && ck < 0.0) return false;
        else if (tk == LO || tk == DB || tk == FX) {
            if (PASS == 1) t = ((lbk - x.rtol * (1.0 + 0.10 * fabs(lbk))) - bb) / alfa;
            else t = (lbk - bb) / alfa;
            ist = NL;
        } else return false;
    }
    if (t < 0.0) t = 0.0;
    if (PASS == 2 && !(t <= tmax)) return false;
    e.k1 = t; e.k2 = fabs(alfa); e.idx = i + 1; e.aux = k * 8 + ist;
    return true;
}

__device__ __forceinline__ Cand prow_cand_at(const SpxDev &d, const PRatio &x, int i, int pass, double tmax)
{
    Cand e = no_cand(pass == 1 ? DBL_MAX : 0.0);
    if (i >= d.m) return e;
    const int k = d.head[i];
    Cand f;
    const bool ok = (pass == 1)
        ? prow_cand<1>(x, d.tcol[i], d.bbar[i], d.type[k - 1], d.lb[k - 1], d.ub[k - 1], d.coef[k - 1], i, k, tmax, f)
        : prow_cand<2>(x, d.tcol[i], d.bbar[i], d.type[k - 1], d.lb[k - 1], d.ub[k - 1], d.coef[k - 1], i, k, tmax, f);
    return ok ? f : e;
}

// chuzc candidate of non-basic j (glpspx01.js:646-688): d_j^2 / gamma_j
__device__ __forceinline__ Cand chuzc_cand(int j, int k, int sj, double dj, double g, double tol_dj)
{
    Cand e = no_cand(0.0);
    if (sj == NL) { if (dj >= -tol_dj) return e; }
    else if (sj == NU) { if (dj <= +tol_dj) return e; }
    else if (sj == NF) { if (-tol_dj <= dj && dj <= +tol_dj) return e; }
    else return e;
    const double temp = (dj * dj) / g;
    if (temp > 0.0) { e.k1 = temp; e.k2 = 0.0; e.idx = j + 1; e.aux = k; }
    return e;
}

// check_feas of phase I (glpspx01.js:1483): basic x_k still infeasible
__device__ __forceinline__ int primal_bad(double cf, double bb, double lbk, double ubk, double tol)
{
    if (cf < 0.0) return bb < lbk - tol * (1.0 + 0.10 * fabs(lbk));
    if (cf > 0.0) return bb > ubk + tol * (1.0 + 0.10 * fabs(ubk));
    return 0;
}

// batch start: chuzc candidates (gamma := 1 when the reference space is
// reset first) and the phase-I flag of the current state
__global__ void __launch_bounds__(256) k_primal_prep(SpxDev d)
{
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool reset = (st->pricing == PT_PSE && st->refct == 0);
    Cand c = no_cand(0.0);
    if (i < n) {
        const int k = d.head[m + i];
        c = chuzc_cand(i, k, d.stat[i], d.cbar[i], reset ? 1.0 : d.gamma[i], st->tol_dj);
    }
    const Cand b = wave_best<0>(c);
    if ((threadIdx.x & 63) == 0) cand_chuzr(d)[blockIdx.x * 4 + (threadIdx.x >> 6)] = b;
    if (st->phase == 1) {
        int bad = 0;
        if (i < m) {
            const int k = d.head[i];
            bad = primal_bad(d.coef[k - 1], d.bbar[i], d.lb[k - 1], d.ub[k - 1], st->tol_bnd);
        }
        if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
    }
}

// ---------------------------------------------------------------------------
// k_primal_ftran: RPB rows per block, the waves (and 64 / RPB slices of each
// wave) split the dense-column list; wave 0 finishes its rows.  The list
// entries and the q-independent inv(B) values are loaded before the chuzc
// choice resolves.
// ---------------------------------------------------------------------------
template <int RPB, int SP>
__global__ void __launch_bounds__(1024) k_primal_ftran(SpxDev d, int pse, int nr_cap, int ncc)
{
    __shared__ double sp[16][64];
    DState *st = d.st;
    const int m = d.m;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    constexpr int SL = 64 / RPB;
    const int sl = lane / RPB;
    const int r = blockIdx.x * RPB + (lane % RPB);
    const int gs = w * SL + sl, NSL = nw * SL;
    const bool act = r < m;
    const bool tail = (w == 0 && sl == 0);
    const bool lead = (blockIdx.x == 0);
    const size_t ldb = (size_t)d.ldb;
    const int *__restrict__ rl = d.rlist;
    const double *__restrict__ Bv = d.Binv;
    // ---- trip 1: state, chuzc candidates, list entries, this row's basic variable
    const int stop = st->stop;
    const int iter_left = st->iter_left, refact = st->refact_pending, refct = st->refct, phase = st->phase;
    const int pinf = st->dinf, nr = st->nr;
    const double tol_piv = st->tol_piv, tol_bnd = st->tol_bnd;
    const int rtest = st->rtest;
    Cand cc = no_cand(0.0);
    for (int b = lane; b < ncc; b += 64) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, cc)) cc = e;
    }
    constexpr int G = 8;
    int c0[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
        const int t = gs + u * NSL;
        c0[u] = (t < nr_cap) ? rl[t] : 0;
    }
    const int kh = (tail && act) ? d.head[r] : 1;
    const double bb = (tail && act) ? d.bbar[r] : 0.0;
    // ---- trip 2: q-independent inv(B) values, the row's bounds and cost
    double bv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) bv[u] = (act && gs + u * NSL < nr) ? Bv[(size_t)c0[u] * ldb + r] : 0.0;
    int tk = 0;
    double lbk = 0.0, ubk = 0.0, ck = 0.0;
    bool refk = false;
    if (tail && act) {
        tk = d.type[kh - 1];
        lbk = d.lb[kh - 1];
        ubk = d.ub[kh - 1];
        ck = d.coef[kh - 1];
        refk = pse && d.refsp[kh - 1] != 0;
    }
    if (stop) return;
    // ---- decisions (identical in every wave)
    int why = ST_RUN;
    if (iter_left <= 0 || refact) why = refact ? ST_REFACT : ST_BATCH;
    const bool reset = (why == ST_RUN && pse && refct == 0);
    if (why == ST_RUN && phase == 1 && !pinf) why = ST_PHASE;
    const Cand best = wave_best<0>(cc);
    if (why == ST_RUN && best.idx == 0) why = ST_Q0;
    if (lead) {
        if (why != ST_RUN) {
            if (threadIdx.x == 0) {
                if (why == ST_Q0) st->q = 0;
                st->stop = why;
            }
            return;
        }
        if (reset) {
            // the basic slacks in the reference space: none after the reset
            const int nsl = st->nwl;
            for (int l = threadIdx.x; l < nsl; l += blockDim.x) d.wpos[d.wlist[l]] = -1;
            reset_refsp_dev(d, 0);            // refsp := non-basic variables, gamma := 1 (syncs)
            if (threadIdx.x == 0) st->nwl = 0;
        }
    }
    if (why != ST_RUN) return;
    if (reset) refk = false;                  // no basic variable is in the new reference space
    const int q = best.idx, kq = best.aux;
    // ---- tcol = inv(B) h, h = -N[q]
    const double *hcol = (!SP && kq > m) ? d.A.A + (size_t)(kq - m - 1) * d.A.lda : nullptr;
    auto hval = [&](int c) { return hcol ? hcol[c] : (c == kq - 1 ? -1.0 : 0.0); };
    double a = 0.0, ua = 0.0;
    if (!SP && tail && act && kh <= m) ua = hval(kh - 1);
    if (SP) {
        // sparse h: the entries of column q, columns of inv(B) read whole
        if (kq > m) {
            const int cq = kq - m - 1;
            const int beg = d.A.cptr[cq], end = d.A.cptr[cq + 1];
            for (int t = beg + gs; t < end; t += NSL)
                a += d.A.cval[t] * (act ? Bv[(size_t)d.A.cind[t] * ldb + r] : 0.0);
        } else if (gs == 0) {
            a = act ? -Bv[(size_t)(kq - 1) * ldb + r] : 0.0;
        }
    } else {
        double xa[G];
#pragma unroll
        for (int u = 0; u < G; ++u) xa[u] = (gs + u * NSL < nr) ? hval(c0[u]) : 0.0;
#pragma unroll
        for (int u = 0; u < G; ++u) a += bv[u] * xa[u];
        int t = gs + G * NSL;
        for (; t + 3 * NSL < nr; t += 4 * NSL) {
            int c[4];
            double x[4], y[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = rl[t + u * NSL];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                x[u] = act ? Bv[(size_t)c[u] * ldb + r] : 0.0;
                y[u] = hval(c[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) a += x[u] * y[u];
        }
        for (; t < nr; t += NSL) {
            const int c = rl[t];
            a += (act ? Bv[(size_t)c * ldb + r] : 0.0) * hval(c);
        }
    }
    sp[w][lane] = a;
    const double dq = d.cbar[q - 1];          // sign of the ratio test
    __syncthreads();
    if (w != 0) return;
    double tv = 0.0;
    if (sl == 0 && act) {
        for (int k = 0; k < nw; ++k)
#pragma unroll
            for (int z = 0; z < SL; ++z) tv += sp[k][lane + z * RPB];
        tv += ua;
        d.tcol[r] = tv;
    }
    // ---- per-group outputs (wave 0; lanes with sl != 0 contribute nothing)
    const double bmax = wmax(fabs(tv));
    const double ds = wsum((tv != 0.0) ? ck * tv : 0.0);
    double vs = 0.0;
    if (pse) {
        const double v = (tv != 0.0 && refk) ? tv : 0.0;
        if (sl == 0 && act) d.h[r] = v;
        vs = wsum(v * v);
    }
    PRatio x;
    x.eps = tol_piv * (1.0 + 0.01 * bmax);    // group-local tolerance <= the global one
    x.s = (dq > 0.0 ? -1.0 : +1.0);
    x.rtol = (rtest == RT_HAR) ? 0.30 * tol_bnd : 0.0;
    x.phase = phase;
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (sl == 0 && act && prow_cand<1>(x, tv, bb, tk, lbk, ubk, ck, r, kh, 0.0, e)) c = e;
    const Cand b1 = wave_best<1>(c);
    if (lane == 0) {
        ptmax(d)[blockIdx.x] = bmax;
        pdsum(d)[blockIdx.x] = ds;
        if (pse) pvsum(d)[blockIdx.x] = vs;
        pcand1(d)[blockIdx.x] = b1;
        if (lead) {
            st->q = q;
            st->kq = kq;
        }
    }
}

// ---------------------------------------------------------------------------
// k_primal_ratio: blocks [0, gm) — every wave: the d_q check, the pass-1
// choice from the ng group candidates (a group whose candidate is not
// significant under the global tolerance is rescanned), the bound flip, then
// the pass-2 candidates of rows [256 b, 256 b + 256), one per wave; blocks
// [gm, ...) — u = inv(B)' v: the unit columns (u_c = v[bind[c]]) per thread,
// then one wave per dense column.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_primal_ratio(SpxDev d, int gm, int ng, int rpb, int pse)
{
    DState *st = d.st;
    const int stop = st->stop;
    const int m = d.m;
    const int lane = threadIdx.x & 63;
    if ((int)blockIdx.x >= gm) {
        const int b = blockIdx.x - gm;
        const int gu = (m + 255) / 256;
        if (b < gu) {
            const int c = b * 256 + threadIdx.x;
            if (c >= m) return;
            const int rp = d.rpos[c];
            const int pos = d.bind[c];
            const double v = (rp < 0) ? d.h[pos - 1] : 0.0;
            if (stop) return;
            if (rp < 0) d.u[c] = v;
            return;
        }
        const int t = (b - gu) * 4 + (threadIdx.x >> 6);
        const int nr = st->nr;
        if (t >= nr) return;
        const int c = d.rlist[t];
        const double *col = d.Binv + (size_t)c * d.ldb;
        double acc = 0.0;
        int r = lane;
        for (; r + 192 < m; r += 256) {
            double v[4], x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v[u] = d.h[r + 64 * u];
                x[u] = col[r + 64 * u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += x[u] * v[u];
        }
        for (; r < m; r += 64) acc += col[r] * d.h[r];
        acc = wsum(acc);
        if (stop) return;
        if (lane == 0) d.u[c] = acc;
        return;
    }
    // ---- trip 1: state, group partials and candidates, this thread's row
    const int q = max(st->q, 1), kq = max(st->kq, 1);
    const int phase = st->phase, rtest = st->rtest, rigorous = st->rigorous, cbar_fresh = st->cbar_fresh;
    const double tol_piv = st->tol_piv, tol_bnd = st->tol_bnd;
    const double d1 = d.cbar[q - 1], ckq = d.coef[kq - 1];
    const int tkq = d.type[kq - 1];
    const double lbq = d.lb[kq - 1], ubq = d.ub[kq - 1];
    const bool refq = pse && d.refsp[kq - 1] != 0;
    constexpr int CPL = 8;
    Cand cl[CPL];
    double vmax = 0.0, dsl = 0.0, vsl = 0.0;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        const int b = lane + u * 64;
        cl[u] = (b < ng) ? pcand1(d)[b] : no_cand(DBL_MAX);
        if (b < ng) {
            vmax = fmax(vmax, ptmax(d)[b]);
            dsl += pdsum(d)[b];
            if (pse) vsl += pvsum(d)[b];
        }
    }
    for (int b = lane + CPL * 64; b < ng; b += 64) {
        vmax = fmax(vmax, ptmax(d)[b]);
        dsl += pdsum(d)[b];
        if (pse) vsl += pvsum(d)[b];
    }
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool in_m = i < m;
    const double tv = in_m ? d.tcol[i] : 0.0;
    const double bb = in_m ? d.bbar[i] : 0.0;
    const int k = in_m ? d.head[i] : 1;
    const int tk = in_m ? d.type[k - 1] : 0;
    const double lbk = in_m ? d.lb[k - 1] : 0.0, ubk = in_m ? d.ub[k - 1] : 0.0, ck = in_m ? d.coef[k - 1] : 0.0;
    if (stop) return;
    const double big = wmax(vmax);
    const double dsum = wsum(dsl);
    // ---- the accuracy check of d_q (glpspx01.js:1901-1919)
    const double d2 = ckq + dsum;
    if (fabs(d1 - d2) > 1e-5 * (1.0 + fabs(d2)) || !((d1 < 0.0 && d2 < 0.0) || (d1 > 0.0 && d2 > 0.0))) {
        if (!cbar_fresh || !rigorous) {
            if (blockIdx.x == 0 && threadIdx.x == 0) st->stop = ST_DCHK;
            return;
        }
    }
    const double cq = (d1 > 0.0) ? (d2 > 0.0 ? d2 : +DBL_EPS) : (d2 < 0.0 ? d2 : -DBL_EPS);
    PRatio x;
    x.eps = tol_piv * (1.0 + 0.01 * big);
    x.s = (cq > 0.0 ? -1.0 : +1.0);
    x.rtol = (rtest == RT_HAR) ? 0.30 * tol_bnd : 0.0;
    x.phase = phase;
    // ---- pass 1: the group candidates under the global tolerance
    Cand c = no_cand(DBL_MAX);
    int fail = 0;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        if (cl[u].idx != 0 && cl[u].k2 < x.eps) fail = 1;
        else if (better<1>(cl[u], c)) c = cl[u];
    }
    for (int b = lane + CPL * 64; b < ng; b += 64) {
        const Cand f = pcand1(d)[b];
        if (f.idx != 0 && f.k2 < x.eps) fail = 1;
        else if (better<1>(f, c)) c = f;
    }
    if (__any(fail)) {
        // rare: rescan the groups whose candidate is not significant
        for (int b = 0; b < ng; ++b) {
            const Cand f = pcand1(d)[b];
            if (!(f.idx != 0 && f.k2 < x.eps)) continue;
            for (int rr = lane; rr < rpb; rr += 64) {
                const Cand g = prow_cand_at(d, x, b * rpb + rr, 1, 0.0);
                if (better<1>(g, c)) c = g;
            }
        }
    }
    const Cand b1 = wave_best<1>(c);
    // the bound flip of a double-bounded xN[q] competes (:830-840)
    int p;
    double teta, big0;
    if (tkq == DB) { p = -1; teta = ubq - lbq; big0 = 1.0; }
    else { p = 0; teta = DBL_MAX; big0 = 0.0; }
    int paux = 0;
    double palfa = 0.0;
    if (b1.idx != 0 && (b1.k1 < teta || (b1.k1 == teta && b1.k2 > big0))) {
        p = b1.idx;
        teta = b1.k1;
        paux = b1.aux;
        palfa = b1.k2;
    }
    const int need2 = !(x.rtol == 0.0 || p <= 0 || teta == 0.0);
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        const double vsum = pse ? wsum(vsl) : 0.0;
        if (threadIdx.x == 0) {
            d.cbar[q - 1] = cq;
            st->dq_ratio = cq;
            st->q1 = p;
            st->teta1 = teta;
            st->kq1 = paux;
            st->alfa1 = palfa;
            st->need2 = need2;
            st->tcol_max = big;
            st->delta = x.s;                  // sign of the step (teta = s * t)
            if (pse) {
                const double eta = refq ? 1.0 : 0.0;
                st->eta_pq = eta;
                st->gamma_pq = eta + vsum;
            }
        }
    }
    if (!need2) return;
    // ---- pass 2 candidates (:871-1028): exact bounds, t <= teta of pass 1
    Cand c2 = no_cand(0.0);
    {
        Cand f;
        if (in_m && prow_cand<2>(x, tv, bb, tk, lbk, ubk, ck, i, k, teta, f)) c2 = f;
    }
    const Cand b2 = wave_best<2>(c2);
    if (lane == 0) cand_pass2(d)[blockIdx.x * 4 + (threadIdx.x >> 6)] = b2;
}

// the leaving choice (pass 2 if needed) and its checks, identical in every
// wave of the calling grid; returns p (-1: bound flip), 0 when the
// iteration stops
struct PPick {
    int need2, q1, aux1, rigorous;
    double teta1, alfa1, big, s;
    Cand c;
};

__device__ __forceinline__ PPick ppick_load(const SpxDev &d, int gm)
{
    const DState *st = d.st;
    const int lane = threadIdx.x & 63;
    PPick pk;
    pk.need2 = st->need2;
    pk.q1 = st->q1;
    pk.aux1 = st->kq1;
    pk.rigorous = st->rigorous;
    pk.teta1 = st->teta1;
    pk.alfa1 = st->alfa1;
    pk.big = st->tcol_max;
    pk.s = st->delta;
    pk.c = no_cand(0.0);
    for (int b = lane; b < 4 * gm; b += 64) {
        const Cand e = cand_pass2(d)[b];
        if (better<2>(e, pk.c)) pk.c = e;
    }
    return pk;
}

__device__ __forceinline__ int ppick_resolve(const SpxDev &d, const PPick &pk, bool lead, int *kp_out, int *pstat_out,
                                             double *teta_out)
{
    DState *st = d.st;
    int p, aux;
    double teta, alfa;
    if (pk.need2) {
        const Cand b2 = wave_best<2>(pk.c);
        p = b2.idx; aux = b2.aux; teta = b2.k1; alfa = b2.k2;
    } else {
        p = pk.q1; aux = pk.aux1; teta = pk.teta1; alfa = pk.alfa1;
    }
    if (p == 0) {
        if (lead && threadIdx.x == 0) { st->p = 0; st->stop = ST_P0; }
        return 0;
    }
    int kp = 0, ps = 0;
    if (p > 0) {
        kp = aux_k(aux);
        ps = aux_stat(aux);
        if (alfa < 1e-5 * (1.0 + 0.01 * pk.big) && !pk.rigorous) {
            if (lead && threadIdx.x == 0) { st->p = p; st->stop = ST_SMALLPIV; }
            return 0;
        }
    }
    *kp_out = kp;
    *pstat_out = ps;
    *teta_out = pk.s * teta;
    return p;
}

// the pivot row of slots (structural column idx, slack row idx) from the
// row / column pass: trow = -rho' N_j (0 for a fixed non-basic), s = N_j' u
__device__ __forceinline__ void prow_emit(const SpxDev &d, int pse, int idx, int j1, int j2, int s1, int s2,
                                          double tr1, double tr2, double sv1, double sv2)
{
    if (j1 >= 0) {
        d.trow[j1] = (s1 == NS) ? 0.0 : tr1;
        if (pse) d.s[j1] = (s1 == NS) ? 0.0 : sv1;
    }
    if (j2 >= 0) {
        d.trow[j2] = (s2 == NS) ? 0.0 : tr2;
        if (pse) d.s[j2] = (s2 == NS) ? 0.0 : sv2;
    }
    (void)idx;
}

// ---------------------------------------------------------------------------
// k_primal_row (dense A): block b owns the 64 slots [64 b, 64 b + 64); its
// waves split the support of rho (rows of AT, 512-byte segments) and, with
// PSE, all m rows for s = N' u; the partial sums meet in LDS in wave order.
// Block 0 publishes the compact rho for the commit.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_primal_row(SpxDev d, int pse, int nr_cap, int gm)
{
    __shared__ double sp[2][16][64];
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    const int idx = blockIdx.x * 64 + lane;
    const bool lead = (blockIdx.x == 0);
    const int stop = st->stop, nr = st->nr;
    const PPick pk = ppick_load(d, gm);
    int c0[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int t = w + u * nw;
        c0[u] = (t < nr_cap) ? d.rlist[t] : 0;
    }
    int pos1 = 0, pos2 = 0, s1 = 0, s2 = 0;
    if (w == 0) {
        pos1 = (idx < n) ? d.bind[m + idx] : 0;
        pos2 = (idx < m) ? d.bind[idx] : 0;
    }
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    if (j1 >= 0) s1 = d.stat[j1];
    if (j2 >= 0) s2 = d.stat[j2];
    if (stop) return;
    int kp = 0, ps = 0;
    double teta = 0.0;
    const int p = ppick_resolve(d, pk, lead, &kp, &ps, &teta);
    if (p == 0) return;
    if (lead && threadIdx.x == 0) {
        st->p = p;
        st->kp = kp;
        st->p_stat = (p > 0 && d.type[kp - 1] == FX) ? NS : ps;
        st->teta = teta;
        st->ns = (p > 0) ? nr + (kp <= m ? 1 : 0) : 0;
        st->dinf = 0;
    }
    if (p < 0) return;                        // bound flip: no pivot row
    const int ns = nr + (kp <= m ? 1 : 0);
    const double *__restrict__ brow = d.Binv + (p - 1);
    const size_t ldb = (size_t)d.ldb;
    const double *__restrict__ col = d.A.AT + min(idx, n - 1);
    const size_t ldt = (size_t)d.A.ldt;
    double v0[8], a0[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int t = w + u * nw;
        int c = c0[u];
        if (t == nr) c = kp - 1;
        v0[u] = (t < nr) ? brow[(size_t)c * ldb] : 1.0;
        a0[u] = (t < ns) ? col[(size_t)c * ldt] : 0.0;
        c0[u] = c;
    }
    const double rho2 = (j2 >= 0) ? brow[(size_t)idx * ldb] : 0.0;
    const double u2 = (pse && j2 >= 0) ? d.u[idx] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (w + u * nw < ns) acc += v0[u] * a0[u];
    if (lead && lane == 0) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = w + u * nw;
            if (t < ns) {
                d.rho_idx[t] = c0[u];
                d.rho_val[t] = v0[u];
            }
        }
    }
    for (int t = w + 8 * nw; t < ns; t += 4 * nw) {
        int c[4];
        double v[4], a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int tt = t + u * nw;
            c[u] = (tt < nr) ? d.rlist[tt] : kp - 1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int tt = t + u * nw;
            v[u] = (tt < nr) ? brow[(size_t)c[u] * ldb] : 1.0;
            a[u] = (tt < ns) ? col[(size_t)c[u] * ldt] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (t + u * nw < ns) acc += v[u] * a[u];
        if (lead && lane == 0) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int tt = t + u * nw;
                if (tt < ns) {
                    d.rho_idx[tt] = c[u];
                    d.rho_val[tt] = v[u];
                }
            }
        }
    }
    // s = -A[:, idx]' u (the second pass of update_gamma): u = inv(B)' v with
    // v = tcol on the basic variables of the reference space is zero outside
    // the dense columns of inv(B) and the basic slacks of the reference space
    // (a basic slack c has u_c = v[bind[c]]), so the pass runs over the rows
    // of AT in rlist and slist only
    double sa = 0.0;
    if (pse) {
        const int nsl = st->nwl;
        const int nu = nr + nsl;
        int t = w;
        for (; t + 3 * nw < nu; t += 4 * nw) {
            int c[4];
            double uu[4], aa[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int tt = t + u * nw;
                c[u] = (tt < nr) ? d.rlist[tt] : d.wlist[tt - nr];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uu[u] = d.u[c[u]];
                aa[u] = col[(size_t)c[u] * ldt];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) sa += uu[u] * aa[u];
        }
        for (; t < nu; t += nw) {
            const int c = (t < nr) ? d.rlist[t] : d.wlist[t - nr];
            sa += d.u[c] * col[(size_t)c * ldt];
        }
    }
    sp[0][w][lane] = (idx < n) ? acc : 0.0;
    sp[1][w][lane] = (idx < n) ? sa : 0.0;
    __syncthreads();
    if (w != 0) return;
    double tsum = 0.0, ssum = 0.0;
    for (int k = 0; k < nw; ++k) {
        tsum += sp[0][k][lane];
        ssum += sp[1][k][lane];
    }
    prow_emit(d, pse, idx, j1, j2, s1, s2, tsum, -rho2, -ssum, u2);
}

// ---------------------------------------------------------------------------
// k_primal_col (sparse A): every wave owns 64 slots; the CSC entries of the
// slot's column are loaded before the pivot choice; rho_i is read straight
// from row p of inv(B).  The compact rho is published by the whole grid.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_primal_col(SpxDev d, int pse, int nr_cap, int gm)
{
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int grp = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int idx = grp * 64 + lane;
    const bool lead = (blockIdx.x == 0);
    const int stop = st->stop, nr = st->nr;
    const PPick pk = ppick_load(d, gm);
    const int pos1 = (idx < n) ? d.bind[m + idx] : 0;
    const int pos2 = (idx < m) ? d.bind[idx] : 0;
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    constexpr int CU = 8;
    int beg = 0, end = 0;
    if (j1 >= 0) {
        beg = d.A.cptr[idx];
        end = d.A.cptr[idx + 1];
    }
    int ci[CU];
    double cv[CU];
#pragma unroll
    for (int u = 0; u < CU; ++u) {
        const bool ok = beg + u < end;
        ci[u] = ok ? d.A.cind[beg + u] : 0;
        cv[u] = ok ? d.A.cval[beg + u] : 0.0;
    }
    const int s1 = (j1 >= 0) ? d.stat[j1] : 0;
    const int s2 = (j2 >= 0) ? d.stat[j2] : 0;
    constexpr int PU = 4;
    const int tpub = blockIdx.x * blockDim.x + threadIdx.x, npub = gridDim.x * blockDim.x;
    int cpub[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
        const int t = tpub + u * npub;
        cpub[u] = (t < nr_cap) ? d.rlist[t] : 0;
    }
    // s = N' u does not depend on the pivot choice
    double sv1 = 0.0;
    if (pse) {
        double uv[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) uv[u] = (beg + u < end) ? d.u[ci[u]] : 0.0;
#pragma unroll
        for (int u = 0; u < CU; ++u) sv1 += cv[u] * uv[u];
        for (int t = beg + CU; t < end; ++t) sv1 += d.A.cval[t] * d.u[d.A.cind[t]];
    }
    const double u2 = (pse && j2 >= 0) ? d.u[idx] : 0.0;
    if (stop) return;
    int kp = 0, ps = 0;
    double teta = 0.0;
    const int p = ppick_resolve(d, pk, lead, &kp, &ps, &teta);
    if (p == 0) return;
    if (lead && threadIdx.x == 0) {
        st->p = p;
        st->kp = kp;
        st->p_stat = (p > 0 && d.type[kp - 1] == FX) ? NS : ps;
        st->teta = teta;
        st->ns = (p > 0) ? nr + (kp <= m ? 1 : 0) : 0;
        st->dinf = 0;
    }
    if (p < 0) return;
    const int ns = nr + (kp <= m ? 1 : 0);
    const double *__restrict__ brow = d.Binv + (p - 1);
    const size_t ldb = (size_t)d.ldb;
    double rv[CU];
#pragma unroll
    for (int u = 0; u < CU; ++u) rv[u] = (beg + u < end) ? brow[(size_t)ci[u] * ldb] : 0.0;
    const double rho2 = (j2 >= 0) ? brow[(size_t)idx * ldb] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < CU; ++u) acc += cv[u] * rv[u];
    for (int t = beg + CU; t < end; ++t) acc += d.A.cval[t] * brow[(size_t)d.A.cind[t] * ldb];
    {
        double vpub[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int t = tpub + u * npub;
            if (t == nr) cpub[u] = kp - 1;
            vpub[u] = (t < nr) ? brow[(size_t)cpub[u] * ldb] : 1.0;
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int t = tpub + u * npub;
            if (t < ns) {
                d.rho_idx[t] = cpub[u];
                d.rho_val[t] = vpub[u];
            }
        }
        for (int t = tpub + PU * npub; t < ns; t += npub) {
            const int c = (t < nr) ? d.rlist[t] : kp - 1;
            d.rho_idx[t] = c;
            d.rho_val[t] = (t < nr) ? brow[(size_t)c * ldb] : 1.0;
        }
    }
    prow_emit(d, pse, idx, j1, j2, s1, s2, acc, -rho2, -sv1, u2);
}

// ---------------------------------------------------------------------------
// k_primal_commit: the first nvb blocks — pivot check, the vector updates,
// the next pivot's chuzc candidates and phase-I flag, and (block 0) the
// change of basis and the list maintenance; the others — the rank-1 update
// of the dense columns of inv(B) over the compact rho (as k_dual_commit).
// Reads of the header patch the change block 0 writes (idempotent).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_primal_commit(SpxDev d, int pse, int nvb, int tiles, int lpsu,
                                                       double bytes_fixed, int rowmode)
{
    DState *st = d.st;
    const int stop = st->stop;
    const int m = d.m, n = d.n;
    const int p = st->p, q = max(st->q, 1), kq = max(st->kq, 1);
    const int pp = max(p, 1), kp = max(st->kp, 1);
    if ((int)blockIdx.x < nvb) {
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        const bool in_m = i < m, in_n = i < n;
        const int kold = in_m ? d.head[i] : 1;
        double bb = in_m ? d.bbar[i] : 0.0;
        const double ti = in_m ? d.tcol[i] : 0.0;
        double cb = in_n ? d.cbar[i] : 0.0;
        const double tri = in_n ? d.trow[i] : 0.0;
        double g = in_n ? d.gamma[i] : 0.0;
        const double si = (pse && in_n) ? d.s[i] : 0.0;
        const int kn_old = in_n ? d.head[m + i] : 1;
        const int sn_old = in_n ? d.stat[i] : 0;
        const bool refn = (pse && in_n) ? d.refsp[kn_old - 1] != 0 : false;
        const double piv1 = d.tcol[pp - 1], piv2 = d.trow[q - 1];
        const double cbq = st->dq_ratio;          // = cbar[q] (its owner rewrites the entry below)
        const int sq = d.stat[q - 1];
        const double xq = get_xN(d.stat, d.lb, d.ub, kq, q);
        const int tkp = d.type[kp - 1];
        const double ckp = d.coef[kp - 1];
        const int p_stat = st->p_stat;
        const double teta = st->teta, gamma_p = st->gamma_pq, eta_p = st->eta_pq;
        const int phase = st->phase, refct = st->refct, binv_fresh = st->binv_fresh, rig = st->rigorous;
        const int upd_cnt = st->upd_cnt, upd_lim = st->upd_lim, it_cnt = st->it_cnt, npiv = st->npiv;
        const int iter_left = st->iter_left;
        const double tol_bnd = st->tol_bnd, tol_dj = st->tol_dj;
        const int knew = (p > 0 && i == p - 1) ? kq : kold;
        const double lbn = in_m ? d.lb[knew - 1] : 0.0, ubn = in_m ? d.ub[knew - 1] : 0.0;
        const double cfn = in_m ? d.coef[knew - 1] : 0.0;
        const bool maint = (blockIdx.x == 0 && threadIdx.x == 64);
        int rq = -1, rlast = 0, nr0 = 0, sp = -1, slast = 0, nsl0 = 0;
        bool refkq = false;
        if (maint) {
            nr0 = st->nr;
            nsl0 = st->nwl;
            if (kq <= m) rq = d.rpos[kq - 1];
            rlast = d.rlist[max(nr0 - 1, 0)];
            if (pse) {
                if (kp <= m) sp = d.wpos[kp - 1];
                slast = d.wlist[max(nsl0 - 1, 0)];
                refkq = kq <= m && d.refsp[kq - 1] != 0;
            }
        }
        if (stop) return;
        // every block's entry loads (the header and the counters block 0
        // rewrites below) are done before block 0 stores them (gk_device.h)
        gate_arrive(st);
        double pivot = 0.0, new_dq = 0.0, cq_new = 0.0;
        if (p > 0) {
            const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                             !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
            if (bad && (!binv_fresh || !rig)) {
                if (blockIdx.x == 0 && threadIdx.x == 0) {
                    gate_wait(st);
                    st->stop = ST_PIVCHK;
                }
                return;
            }
            pivot = bad ? piv1 : piv2;
            new_dq = cbq / pivot;
            cq_new = new_dq;
            if (phase == 1) cq_new -= ckp;
        }
        // update_bbar (:1100)
        if (in_m) {
            if (p > 0 && i == p - 1) bb = xq + teta;
            else if (teta != 0.0) bb += ti * teta;
            d.bbar[i] = bb;
        }
        // update_cbar (:1154), update_gamma (:1178)
        const int new_refct = (p > 0 && pse && refct > 0) ? refct - 1 : refct;
        if (in_n && p > 0) {
            if (i == q - 1) cb = cq_new;
            else if (tri != 0.0) cb -= tri * new_dq;
            d.cbar[i] = cb;
            if (pse && refct > 0) {
                if (i == q - 1) {
                    if (tkp == FX) g = 1.0;
                    else {
                        g = gamma_p / (pivot * pivot);
                        if (g < DBL_EPS) g = DBL_EPS;
                    }
                    d.gamma[i] = g;
                } else if (tri != 0.0) {
                    const double t = tri / pivot;
                    const double t1 = g + t * t * gamma_p + 2.0 * t * si;
                    const double t2 = (refn ? 1.0 : 0.0) + eta_p * t * t;
                    g = (t1 >= t2 ? t1 : t2);
                    if (g < DBL_EPS) g = DBL_EPS;
                    d.gamma[i] = g;
                }
            }
        }
        // the next pivot: chuzc candidates and the phase-I check
        {
            Cand c = no_cand(0.0);
            if (in_n) {
                int sn = sn_old, kn = kn_old;
                if (i == q - 1) {
                    if (p > 0) { sn = (tkp == FX) ? NS : p_stat; kn = kp; }
                    else sn = (sq == NL) ? NU : NL;
                }
                const bool reset = pse && new_refct == 0;
                c = chuzc_cand(i, kn, sn, cb, reset ? 1.0 : g, tol_dj);
            }
            const Cand b = wave_best<0>(c);
            if ((threadIdx.x & 63) == 0) cand_chuzr(d)[blockIdx.x * 4 + (threadIdx.x >> 6)] = b;
        }
        if (phase == 1) {
            const int bad = in_m && primal_bad((p > 0 && knew == kp) ? 0.0 : cfn, bb, lbn, ubn, tol_bnd);
            if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            gate_wait(st);
            // change_basis (:2035-2055) and the counters of finish_pivot
            if (p > 0) {
                d.head[p - 1] = kq;
                d.head[m + q - 1] = kp;
                d.bind[kq - 1] = p;
                d.bind[kp - 1] = m + q;
                d.stat[q - 1] = (signed char)((tkp == FX) ? NS : p_stat);
                if (phase == 1) d.coef[kp - 1] = 0.0;
                st->refct = new_refct;
                st->upd_cnt = upd_cnt + 1;
                st->binv_fresh = 0;
                st->cbar_fresh = 0;
                if (upd_cnt + 1 >= upd_lim) st->refact_pending = 1;
                st->pivot = pivot;
                st->new_dq = new_dq;
            } else {
                d.stat[q - 1] = (signed char)((sq == NL) ? NU : NL);
            }
            st->it_cnt = it_cnt + 1;
            st->npiv = npiv + 1;
            st->iter_left = iter_left - 1;
            if (rig > 0) st->rigorous = rig - 1;
        }
        if (maint && p > 0) {
            int nr = nr0;
            if (kq <= m) {
                d.rlist[rq] = rlast;
                d.rpos[rlast] = rq;
                d.rpos[kq - 1] = -1;
                nr--;
            }
            if (kp <= m) {
                d.rlist[nr] = kp - 1;
                d.rpos[kp - 1] = nr;
                nr++;
            }
            st->nr = nr;
            if (pse) {
                // basic slacks in the reference space: a slack leaving drops
                // out, a slack of the reference space entering joins
                int nsl = nsl0;
                if (sp >= 0) {
                    d.wlist[sp] = slast;
                    d.wpos[slast] = sp;
                    d.wpos[kp - 1] = -1;
                    nsl--;
                }
                if (refkq) {
                    d.wlist[nsl] = kq - 1;
                    d.wpos[kq - 1] = nsl;
                    nsl++;
                }
                st->nwl = nsl;
            }
            // algorithmic bytes: the pivot row (rows of AT in the support of
            // rho, or the CSC), s = N' u (rows of AT in the support of u, or
            // the CSC), inv(B) for the FTRAN and the PSE BTRAN, the rank-1
            // update and the vectors
            const int ns = st->ns;
            const double rowb = rowmode == 1 ? 8.0 * (double)ns * n : 12.0 * (double)d.A.nnz;
            const double sb = pse ? (rowmode == 1 ? 8.0 * (double)(nr0 + nsl0) * n : 12.0 * (double)d.A.nnz) : 0.0;
            st->bytes += rowb + sb + 8.0 * (double)m * (nr0 + 1) * (pse ? 2.0 : 1.0) +
                         16.0 * (double)m * (nr0 + (kp <= m ? 1 : 0)) + bytes_fixed;
        }
        return;
    }
    // rank-1 update over the dense columns (the compact rho: ns entries);
    // every thread loads, then passes the entry gate, then works (or not)
    const int b = blockIdx.x - nvb;
    const int tile = b % tiles, chunk = b / tiles;
    const int t0 = chunk * lpsu;
    const int r = (tile * 256 + threadIdx.x) * 2;
    const bool act = p > 0 && r < m;
    const bool two = act && (r + 1 < m);
    const double tr0 = act ? d.tcol[r] : 0.0, tr1 = two ? d.tcol[r + 1] : 0.0;
    constexpr int U = 4;
    int cc[U];
    double rl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = t0 + u;
        cc[u] = (t <= m && u < lpsu) ? d.rho_idx[t] : 0;
        rl[u] = (t <= m && u < lpsu) ? d.rho_val[t] : 0.0;
    }
    const int ns = st->ns;
    const int binv_fresh = st->binv_fresh, rig = st->rigorous;
    const int t1 = act ? min(ns, t0 + lpsu) : t0;
    const double piv1 = d.tcol[pp - 1], piv2 = d.trow[q - 1];
    const int ce = (kq <= m) ? kq - 1 : -1;
    double2 v0[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (t0 + u < t1) v0[u] = *(const double2 *)(d.Binv + (size_t)cc[u] * d.ldb + r);
    if (stop) return;
    gate_arrive(st);
    if (!act) return;
    const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                     !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
    if (bad && (!binv_fresh || !rig)) return;
    const double tp = piv1;
    const bool z0 = (r == p - 1), z1 = (r + 1 == p - 1);
    const double f0 = z0 ? 1.0 / tp : tr0 / tp;
    const double f1 = two ? (z1 ? 1.0 / tp : tr1 / tp) : 0.0;
    auto upd = [&](int c, double rv, double2 v) {
        double *ptr = d.Binv + (size_t)c * d.ldb + r;
        if (c == ce) {
            v.x = z0 ? 1.0 : 0.0;
            v.y = z1 ? 1.0 : 0.0;
        } else {
            v.x = (z0 ? 0.0 : v.x) - f0 * rv;
            v.y = (z1 ? 0.0 : v.y) - f1 * rv;
        }
        if (two) *(double2 *)ptr = v;
        else ptr[0] = v.x;
    };
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (t0 + u < t1) upd(cc[u], rl[u], v0[u]);
    for (int t = t0 + U; t < t1; t += U) {
        int c[U];
        double rv[U];
        double2 v[U];
        const int cnt = min(U, t1 - t);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < cnt) {
                c[u] = d.rho_idx[t + u];
                rv[u] = d.rho_val[t + u];
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < cnt) v[u] = *(const double2 *)(d.Binv + (size_t)c[u] * d.ldb + r);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < cnt) upd(c[u], rv[u], v[u]);
    }
}

// ---------------------------------------------------------------------------
// the primal pivot on the sparse factor (gk_sparse.hip): the
// same stages with the inverse's reads replaced by solves —
//   k_sp_primal_top     1 WG  stop tests, PSE reset, chuzc (:646), h = -N[q]
//   FTRAN               tcol = inv(B) h (eval_tcol :690)
//   k_sp_primal_groups  grid  per 64-row group: max |tcol|, the d_q check
//                       sum, the PSE vector v and its sum of squares, the
//                       Harris pass-1 candidate (the tail of k_primal_ftran)
//   k_primal_ratio      grid  (its pass blocks only) d_q check, pass 1, bound
//                       flip, pass-2 candidates
//   k_sp_primal_pick    1 WG  the pass-2 choice p (ppick)
//   BTRAN x 2           rho = inv(B)' e_p, u = inv(B)' v (eval_rho :1030,
//                       update_gamma :1220)
//   column pass         trow_j = -rho' N_j, s_j = N_j' u (:1058, :1230-1241)
//   k_primal_commit     (vector blocks only) the updates, change_basis
//   factor update       the Schur-complement column of the pivot
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_sp_primal_top(SpxDev d, int pse, int ncc)
{
    DState *st = d.st;
    const int lane = threadIdx.x & 63;
    const int stop = st->stop;
    const int iter_left = st->iter_left, refact = st->refact_pending, refct = st->refct, phase = st->phase;
    const int pinf = st->dinf;
    Cand cc = no_cand(0.0);
    for (int b = lane; b < ncc; b += 64) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, cc)) cc = e;
    }
    if (stop) return;
    int why = ST_RUN;
    if (iter_left <= 0 || refact) why = refact ? ST_REFACT : ST_BATCH;
    const bool reset = (why == ST_RUN && pse && refct == 0);
    if (why == ST_RUN && phase == 1 && !pinf) why = ST_PHASE;
    const Cand best = wave_best<0>(cc);
    if (why == ST_RUN && best.idx == 0) why = ST_Q0;
    if (why != ST_RUN) {
        if (threadIdx.x == 0) {
            if (why == ST_Q0) st->q = 0;
            st->stop = why;
        }
        return;
    }
    if (reset) {
        const int nsl = st->nwl;
        for (int l = threadIdx.x; l < nsl; l += blockDim.x) d.wpos[d.wlist[l]] = -1;
        reset_refsp_dev(d, 0);                // refsp := non-basic variables, gamma := 1 (syncs)
        if (threadIdx.x == 0) st->nwl = 0;
    }
    const int q = best.idx, kq = best.aux;
    build_hq(d, q);                           // h = -N[q] (syncs)
    if (threadIdx.x == 0) {
        st->q = q;
        st->kq = kq;
    }
}

__global__ void __launch_bounds__(256) k_sp_primal_groups(SpxDev d, int pse)
{
    DState *st = d.st;
    const int m = d.m;
    const int lane = threadIdx.x & 63;
    const int grp = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int r = blockIdx.x * 256 + threadIdx.x;
    const bool act = r < m;
    const int stop = st->stop;
    const int q = max(st->q, 1), phase = st->phase, rtest = st->rtest;
    const double tol_piv = st->tol_piv, tol_bnd = st->tol_bnd;
    const double tv = act ? d.tcol[r] : 0.0, bb = act ? d.bbar[r] : 0.0;
    const int kh = act ? d.head[r] : 1;
    const int tk = act ? d.type[kh - 1] : 0;
    const double lbk = act ? d.lb[kh - 1] : 0.0, ubk = act ? d.ub[kh - 1] : 0.0, ck = act ? d.coef[kh - 1] : 0.0;
    const bool refk = act && pse && d.refsp[kh - 1] != 0;
    const double dq = d.cbar[q - 1];
    if (stop) return;
    const double bmax = wmax(fabs(tv));
    const double ds = wsum((tv != 0.0) ? ck * tv : 0.0);
    double vs = 0.0;
    if (pse) {
        const double v = (tv != 0.0 && refk) ? tv : 0.0;
        if (act) d.h[r] = v;                  // v for update_gamma's BTRAN (h is free after the FTRAN)
        vs = wsum(v * v);
    }
    PRatio x;
    x.eps = tol_piv * (1.0 + 0.01 * bmax);    // group-local tolerance <= the global one
    x.s = (dq > 0.0 ? -1.0 : +1.0);
    x.rtol = (rtest == RT_HAR) ? 0.30 * tol_bnd : 0.0;
    x.phase = phase;
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (act && prow_cand<1>(x, tv, bb, tk, lbk, ubk, ck, r, kh, 0.0, e)) c = e;
    const Cand b1 = wave_best<1>(c);
    if (lane == 0) {
        ptmax(d)[grp] = bmax;
        pdsum(d)[grp] = ds;
        if (pse) pvsum(d)[grp] = vs;
        pcand1(d)[grp] = b1;
    }
}

__global__ void __launch_bounds__(1024) k_sp_primal_pick(SpxDev d, int gm)
{
    DState *st = d.st;
    const int m = d.m;
    const int stop = st->stop, nr = st->nr;
    const PPick pk = ppick_load(d, gm);
    if (stop) return;
    int kp = 0, ps = 0;
    double teta = 0.0;
    const int p = ppick_resolve(d, pk, true, &kp, &ps, &teta);
    if (p == 0) return;
    if (threadIdx.x == 0) {
        st->p = p;
        st->kp = kp;
        st->p_stat = (p > 0 && d.type[kp - 1] == FX) ? NS : ps;
        st->teta = teta;
        st->ns = (p > 0) ? nr + (kp <= m ? 1 : 0) : 0;
        st->dinf = 0;
    }
}

void colpass_gated(hipStream_t s, const MatDev &A, int mode, int off, int cnt, const int *head,
                   const signed char *stat, const double *coef, const double *h, const double *x,
                   const double *y, double *out1, double *out2, unsigned long long *maxbits,
                   const DState *st, int need_p);

void primal_iteration_sparse(hipStream_t s, const SpxDev &d, int pse)
{
    const int m = d.m, n = d.n;
    const int gv = cdiv(std::max(m, n), 256), gm = cdiv(m, 256), tiles_m = cdiv(m, 512);
    const int ng = cdiv(m, 64);
    hipLaunchKernelGGL(k_sp_primal_top, dim3(1), dim3(1024), 0, s, d, pse, 4 * gv);
    sp_pivot_ftran(*d.sp, s, d.st, d.h, nullptr, d.tcol, nullptr, 0);
    hipLaunchKernelGGL(k_sp_primal_groups, dim3(gm), dim3(256), 0, s, d, pse);
    hipLaunchKernelGGL(k_primal_ratio, dim3(gm), dim3(256), 0, s, d, gm, ng, 64, pse);
    hipLaunchKernelGGL(k_sp_primal_pick, dim3(1), dim3(1024), 0, s, d, gm);
    if (pse) sp_pivot_btran2(*d.sp, s, d.st, d.h, d.rho, d.u);
    else sp_pivot_btran(*d.sp, s, d.st, d.rho);
    colpass_gated(s, d.A, pse ? CP_TROW_S : CP_TROW, m, n, d.head, d.stat, d.coef, nullptr, d.rho, pse ? d.u : nullptr,
                  d.trow, pse ? d.s : nullptr, nullptr, d.st, 1);
    hipLaunchKernelGGL(k_primal_commit, dim3(gv), dim3(256), 0, s, d, pse, gv, tiles_m, 1, 96.0 * ((double)m + n), 0);
    sp_pivot_update(*d.sp, s, d.st);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
DualPlan primal_plan(const SpxDev &d, int nr_max, int pse)
{
    const int m = d.m;
    DualPlan pl{};
    pl.pse = pse;
    nr_max = std::min(std::max(nr_max, 0), m);
    const int ns_max = std::min(m, nr_max + 1);
    pl.nr_cap = nr_max;
    pl.ns_cap = ns_max;
    pl.rowpath = (d.A.dense && d.A.AT) ? 1 : 0;
    pl.colpath = d.A.dense ? 0 : 1;
    pl.fwaves = nr_max <= 32 ? 4 : (nr_max <= 128 ? 8 : 16);
    pl.twaves = (ns_max <= 32 && !pse) ? 4 : (ns_max <= 128 && !pse ? 8 : 16);
    const int tiles_f = cdiv(m, 512);
    pl.uchunks = std::max(1, std::min(2048 / tiles_f, cdiv(ns_max, 4)));
    pl.lpsu = cdiv(ns_max, pl.uchunks);
    pl.uchunks = cdiv(ns_max, pl.lpsu);
    pl.fused = (m <= 2048) ? 16 : 64;         // rows per block of k_primal_ftran
    return pl;
}

bool primal_fast_ok(const SpxDev &d)
{
    // the row path needs the row-major copy of dense A
    return !d.A.dense || d.A.AT != nullptr;
}

void primal_batch_begin(hipStream_t s, const SpxDev &d)
{
    hipLaunchKernelGGL(k_primal_prep, dim3(cdiv(std::max(d.m, d.n), 256)), dim3(256), 0, s, d);
}

void primal_iteration2(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    const int m = d.m, n = d.n;
    const int gv = cdiv(std::max(m, n), 256), gm = cdiv(m, 256), tiles_m = cdiv(m, 512);
    const int ncc = 4 * gv;
    const int rpb = pl.fused;
    const int ng = cdiv(m, rpb);
    const dim3 bf(64 * pl.fwaves);
    if (d.A.dense) {
        if (rpb == 16) hipLaunchKernelGGL((k_primal_ftran<16, 0>), dim3(ng), bf, 0, s, d, pl.pse, pl.nr_cap, ncc);
        else hipLaunchKernelGGL((k_primal_ftran<64, 0>), dim3(ng), bf, 0, s, d, pl.pse, pl.nr_cap, ncc);
    } else {
        if (rpb == 16) hipLaunchKernelGGL((k_primal_ftran<16, 1>), dim3(ng), bf, 0, s, d, pl.pse, pl.nr_cap, ncc);
        else hipLaunchKernelGGL((k_primal_ftran<64, 1>), dim3(ng), bf, 0, s, d, pl.pse, pl.nr_cap, ncc);
    }
    const int ub = pl.pse ? cdiv(m, 256) + cdiv(std::max(pl.nr_cap, 1), 4) : 0;
    hipLaunchKernelGGL(k_primal_ratio, dim3(gm + ub), dim3(256), 0, s, d, gm, ng, rpb, pl.pse);
    if (pl.rowpath)
        hipLaunchKernelGGL(k_primal_row, dim3(cdiv(std::max(m, n), 64)), dim3(64 * pl.twaves), 0, s, d, pl.pse,
                           pl.nr_cap, gm);
    else
        hipLaunchKernelGGL(k_primal_col, dim3(gv), dim3(256), 0, s, d, pl.pse, pl.nr_cap, gm);
    hipLaunchKernelGGL(k_primal_commit, dim3(gv + tiles_m * pl.uchunks), dim3(256), 0, s, d, pl.pse, gv, tiles_m,
                       pl.lpsu, 96.0 * ((double)m + n), pl.rowpath);
}

}  // namespace gk
