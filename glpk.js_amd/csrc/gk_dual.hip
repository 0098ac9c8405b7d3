// Dual simplex pivot pipeline (glpspx02.js main loop :1614-1966) on the
// structure of the explicit inverse.
//
// inv(B) e_c = e_{bind[c]} for every basic slack c, exactly (the unit columns
// are written exactly at re-inversion and whenever a slack enters the basis),
// so only the nr columns of inv(B) listed in rlist[] — the non-basic slacks —
// carry data.  Every pass over inv(B) runs over that list:
//   rho  = row p of inv(B)            nr strided loads + the unit entry
//   tcol = inv(B) h, u = inv(B) w     2-RHS GEMV over the nr dense columns
//   rank-1 update                     the nr dense columns (+1 when a slack leaves)
// and rho has at most nr + 1 non-zeros, so for dense A the pivot row
// trow = -rho' N is formed from the rows of A in the support of rho (row-major
// copy AT), reading 8 * ns * n bytes instead of 8 * m * n.  With the basis
// growing from the slack basis, nr is the number of basic structurals.
//
// A pivot is seven kernels, each gated on st->stop; the decisions that need
// the whole of a vector are prepared as per-block candidates by the kernel
// that produces the vector, so that no kernel rescans m or n entries in one
// workgroup:
//   k_dual_top     1 WG  change_basis of the previous pivot (:1954-1964),
//                        reference-space reset (:497), phase-I / limit checks,
//                        chuzr (:572) from the candidates of k_dual_commit,
//                        rho = row p of inv(B) (eval_rho :627)
//   k_lgemv_part   grid  trow partials over the rows of AT      (eval_trow :655-791)
//   k_trow_finish  grid  trow, max|trow|, PSE vectors, gamma_p partials,
//                        Harris pass-1 candidates per block     (:820-869)
//   k_dual_ratio   grid  pass-1 choice, pass-2 candidates (:870-950); A w over
//                        the reference-space columns            (update_gamma :1103-1134)
//   k_dual_ftran   grid  pass-2 choice, h = -N[q], tcol = inv(B) h and
//                        u = inv(B)(ys - A w) over the dense columns (eval_tcol :937)
//   k_dual_ftran_reduce
//   k_dual_commit  grid  pivot check (:1913-1933), update_bbar/cbar/gamma
//                        (:1020-1134), rank-1 update of inv(B); chuzr candidates
//                        and the phase-I check of the next iteration
#include "gk_device.h"
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace gk {

// ---------------------------------------------------------------------------
// list GEMV of one 512-row tile over list entries [t0, t1):
//   o[k*rows + r] = sum_t M[list[t]*ld + r] * x_k(t, list[t])
// r + 1 < ld always (ld is a multiple of 8 and r even), so the 16-byte load
// stays inside the allocation even for the last odd row.
// ---------------------------------------------------------------------------
template <int NRHS, typename XF>
__device__ __forceinline__ void lgemv_tile(const double *__restrict__ M, size_t ld, int rows,
                                           const int *__restrict__ list, int t0, int t1, int r, XF xf,
                                           double *__restrict__ o)
{
    if (r >= rows) return;
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
    int t = t0;
    for (; t + 4 <= t1; t += 4) {
        int c[4];
        double xa[4], xb[4];
        bool any = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            c[u] = list[t + u];
            xf(t + u, c[u], xa[u], xb[u]);
            any = any || xa[u] != 0.0 || xb[u] != 0.0;
        }
        if (!any) continue;
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const double2 *)(M + (size_t)c[u] * ld + r);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a0 += v[u].x * xa[u];
            a1 += v[u].y * xa[u];
            if (NRHS == 2) {
                b0 += v[u].x * xb[u];
                b1 += v[u].y * xb[u];
            }
        }
    }
    for (; t < t1; ++t) {
        const int c = list[t];
        double xa, xb;
        xf(t, c, xa, xb);
        if (xa == 0.0 && xb == 0.0) continue;
        const double2 v = *(const double2 *)(M + (size_t)c * ld + r);
        a0 += v.x * xa;
        a1 += v.y * xa;
        if (NRHS == 2) {
            b0 += v.x * xb;
            b1 += v.y * xb;
        }
    }
    o[r] = a0;
    if (r + 1 < rows) o[r + 1] = a1;
    if (NRHS == 2) {
        o[rows + r] = b0;
        if (r + 1 < rows) o[rows + r + 1] = b1;
    }
}

// the same with the multipliers staged in LDS, 256 list entries at a time:
// thread k evaluates xf for entry k of the chunk once per block (xf may be a
// chain of loads), instead of every thread evaluating it for every entry.
// Called by the whole block (it synchronises); rows beyond `rows` idle.
template <int NRHS, typename XF>
__device__ __forceinline__ void lgemv_tile_staged(const double *__restrict__ M, size_t ld, int rows,
                                                  const int *__restrict__ list, int t0, int t1, int r, XF xf,
                                                  double *__restrict__ o)
{
    __shared__ double sxa[256], sxb[256];
    __shared__ int sc[256];
    const bool act = r < rows;
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
    for (int c0 = t0; c0 < t1; c0 += 256) {
        const int cn = min(256, t1 - c0);
        __syncthreads();
        if ((int)threadIdx.x < cn) {
            const int c = list[c0 + threadIdx.x];
            double xa, xb;
            xf(c0 + threadIdx.x, c, xa, xb);
            sc[threadIdx.x] = c;
            sxa[threadIdx.x] = xa;
            sxb[threadIdx.x] = xb;
        }
        __syncthreads();
        if (!act) continue;
        int k = 0;
        for (; k + 4 <= cn; k += 4) {
            double xa[4], xb[4];
            bool any = false;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                xa[u] = sxa[k + u];
                xb[u] = (NRHS == 2) ? sxb[k + u] : 0.0;
                any = any || xa[u] != 0.0 || xb[u] != 0.0;
            }
            if (!any) continue;
            double2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *(const double2 *)(M + (size_t)sc[k + u] * ld + r);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a0 += v[u].x * xa[u];
                a1 += v[u].y * xa[u];
                if (NRHS == 2) {
                    b0 += v[u].x * xb[u];
                    b1 += v[u].y * xb[u];
                }
            }
        }
        for (; k < cn; ++k) {
            const double xa = sxa[k], xb = (NRHS == 2) ? sxb[k] : 0.0;
            if (xa == 0.0 && xb == 0.0) continue;
            const double2 v = *(const double2 *)(M + (size_t)sc[k] * ld + r);
            a0 += v.x * xa;
            a1 += v.y * xa;
            if (NRHS == 2) {
                b0 += v.x * xb;
                b1 += v.y * xb;
            }
        }
    }
    if (!act) return;
    o[r] = a0;
    if (r + 1 < rows) o[r + 1] = a1;
    if (NRHS == 2) {
        o[rows + r] = b0;
        if (r + 1 < rows) o[rows + r + 1] = b1;
    }
}

// trow partials: part[s*n + c] = sum over the support of rho in chunk s of rho_i A[i, c].
// With st, block (0,0) stamps the device wall clock at entry and every block
// at exit (tslots), so the kernel's span is measured inside captured graphs.
__global__ void __launch_bounds__(256) k_lgemv_part(const double *__restrict__ M, size_t ld, int rows,
                                                      const int *__restrict__ list, const int *cntp,
                                                      const double *__restrict__ xv, double *__restrict__ part,
                                                      DState *st, unsigned long long *tslots)
{
    if (st && st->stop) return;
    if (st && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) st->tk_start = wall_clock64();
    const int cnt = *cntp;
    const int splits = gridDim.y;
    const int lps = (cnt + splits - 1) / splits;
    const int t0 = blockIdx.y * lps, t1 = min(cnt, t0 + lps);
    const int r = (blockIdx.x * 256 + threadIdx.x) * 2;
    lgemv_tile<1>(M, ld, rows, list, t0, t1, r,
                  [&](int t, int, double &xa, double &xb) { xa = xv[t]; xb = 0.0; },
                  part + (size_t)blockIdx.y * rows);
    if (tslots) {
        __syncthreads();
        if (threadIdx.x == 0) tslots[blockIdx.y * gridDim.x + blockIdx.x] = wall_clock64();
    }
}

// ---------------------------------------------------------------------------
// the Harris ratio test pieces (glpspx02.js:820-950)
// ---------------------------------------------------------------------------
struct RatioCtx {
    double eps, s, rtol;
};

// the scalars of the ratio test, loaded early (with the kernel's first loads)
struct RatioIn {
    double tol_bnd, delta, tol_dj;
    int rtest;
};

__device__ __forceinline__ RatioIn ratio_in(const DState *st)
{
    RatioIn r;
    r.tol_bnd = st->tol_bnd;
    r.delta = st->delta;
    r.tol_dj = st->tol_dj;
    r.rtest = st->rtest;
    return r;
}

__device__ __forceinline__ RatioCtx ratio_ctx(const RatioIn &r, double big)
{
    RatioCtx x;
    x.eps = r.tol_bnd * (1.0 + 0.01 * big);       // sort_trow with tol_bnd (:1851)
    x.s = (r.delta > 0.0 ? +1.0 : -1.0);
    x.rtol = (r.rtest == RT_HAR) ? 0.30 * r.tol_dj : 0.0;
    return x;
}

__device__ __forceinline__ RatioCtx ratio_ctx(const DState *st, double big) { return ratio_ctx(ratio_in(st), big); }

__device__ __forceinline__ double trow_big(const DState *st)
{
    return __longlong_as_double((long long)st->trow_max_bits);
}

// candidates carry k2 = |trow_j| and aux = the variable number of xN[j]
__device__ __forceinline__ bool pass1_cand(const RatioCtx &x, double tr, double cb, int sj, int j, int k, Cand &e)
{
    if (tr == 0.0 || fabs(tr) < x.eps) return false;
    const double alfa = x.s * tr;
    double t;
    if (alfa > 0.0) {
        if (sj == NL || sj == NF) t = (cb + x.rtol) / alfa; else return false;
    } else {
        if (sj == NU || sj == NF) t = (cb - x.rtol) / alfa; else return false;
    }
    if (t < 0.0) t = 0.0;
    e.k1 = t; e.k2 = fabs(alfa); e.idx = j + 1; e.aux = k;
    return true;
}

__device__ __forceinline__ bool pass2_cand(const RatioCtx &x, double tr, double cb, int sj, int j, int k, double tmax,
                                           Cand &e)
{
    if (tr == 0.0 || fabs(tr) < x.eps) return false;
    const double alfa = x.s * tr;
    double t;
    if (alfa > 0.0) {
        if (sj == NL || sj == NF) t = cb / alfa; else return false;
    } else {
        if (sj == NU || sj == NF) t = cb / alfa; else return false;
    }
    if (t < 0.0) t = 0.0;
    if (!(t <= tmax)) return false;
    e.k1 = t; e.k2 = fabs(alfa); e.idx = j + 1; e.aux = k;
    return true;
}

// pass-1 candidate of the non-basic variable(s) of slot idx (structural
// column idx and slack row idx)
__device__ __forceinline__ Cand pass1_slot(const SpxDev &d, const RatioCtx &x, int idx)
{
    const int m = d.m, n = d.n;
    Cand best = no_cand(DBL_MAX);
    if (idx < n) {
        const int pos = d.bind[m + idx];
        if (pos > m) {
            const int j = pos - m - 1;
            Cand e;
            if (pass1_cand(x, d.trow[j], d.cbar[j], d.stat[j], j, m + idx + 1, e) && better<1>(e, best)) best = e;
        }
    }
    if (idx < m) {
        const int pos = d.bind[idx];
        if (pos > m) {
            const int j = pos - m - 1;
            Cand e;
            if (pass1_cand(x, d.trow[j], d.cbar[j], d.stat[j], j, idx + 1, e) && better<1>(e, best)) best = e;
        }
    }
    return best;
}

// ---------------------------------------------------------------------------
// change_basis (glpspx02.js:1954-1964) of the committed pivot: the header
// writes and the scalar state.  k_dual_commit already maintained the lists
// (rlist / wlist) and precomputed kp, kq and the flags, so this part does no
// dependent loads.  Every thread computes the updated scalars (returned);
// threads 0-2 write.
// ---------------------------------------------------------------------------
struct TopState {
    int iter_left, refact, refct;
    double obj;
};

struct FinishIn {
    int pend, p, q, kp, kq, fxp, rclr, upd_cnt, it_cnt, npiv, rig;
    double delta;
    TopState t;
};

// every field is loaded unconditionally before any of them is tested (a
// short-circuit test between two loads makes the compiler issue the second
// only after the first returned: one memory round trip per test)
__device__ __forceinline__ FinishIn finish_load(const SpxDev &d)
{
    const DState *st = d.st;
    FinishIn f;
    const int pend = st->pend, iter_left = st->iter_left, rpend = st->refact_pending, upd_cnt = st->upd_cnt,
              upd_lim = st->upd_lim, pricing = st->pricing, refct = st->refct, phase = st->phase;
    const double obj = st->obj, cqo = st->cbar_q_old, zeta = st->zeta, delta = st->delta, pivot = st->pivot;
    f.p = st->p; f.q = st->q; f.kp = st->kp; f.kq = st->kq;
    f.fxp = st->fxp; f.rclr = st->rclr; f.it_cnt = st->it_cnt; f.npiv = st->npiv;
    f.rig = st->rigorous;
    f.pend = pend;
    f.upd_cnt = upd_cnt;
    f.delta = delta;
    f.t.iter_left = iter_left - pend;
    f.t.refact = (rpend != 0) | ((pend != 0) & (upd_cnt + 1 >= upd_lim));
    f.t.refct = ((pend != 0) & (pricing == PT_PSE) & (refct > 0)) ? refct - 1 : refct;
    const double dobj = (cqo / zeta) * (delta / pivot);
    f.t.obj = ((pend != 0) & (phase == 2)) ? obj + dobj : obj;
    return f;
}

__device__ TopState finish_apply(const SpxDev &d, const FinishIn &f, bool tail_sync)
{
    DState *st = d.st;
    const int m = d.m;
    __syncthreads();                          // every wave has read st before it is written
    if (f.pend) {
        if (threadIdx.x == 0) {
            d.head[f.p - 1] = f.kq;
            d.head[m + f.q - 1] = f.kp;
            d.bind[f.kq - 1] = f.p;
            d.bind[f.kp - 1] = m + f.q;
            d.stat[f.q - 1] = f.fxp ? NS : (f.delta > 0.0 ? NL : NU);
        } else if (threadIdx.x == 1) {
            if (f.rclr) d.refsp[f.kp - 1] = 0;
        } else if (threadIdx.x == 2) {
            st->obj = f.t.obj;
            st->upd_cnt = f.upd_cnt + 1;
            st->binv_fresh = 0;
            st->cbar_fresh = 0;
            st->refact_pending = f.t.refact;
            st->it_cnt = f.it_cnt + 1;
            st->npiv = f.npiv + 1;
            st->iter_left = f.t.iter_left;
            if (f.rig > 0) st->rigorous = f.rig - 1;
            st->refct = f.t.refct;
            st->pend = 0;
        }
    }
    if (tail_sync) __syncthreads();
    return f.t;
}

// finish_apply split for the gated multi-block kernels (k_dual_row,
// k_dual_top_grid, k_dual_col): the header arrays early (every other block
// patches what they change, idempotently), the scalars by one thread of the
// writer after gate_wait — refct = 1000 when the reference space was reset
// in between (reset_refsp_dev with set_refct false)
__device__ __forceinline__ void finish_arrays(const SpxDev &d, const FinishIn &f)
{
    const int m = d.m;
    __syncthreads();                          // every wave of this block has read the header
    if (f.pend) {
        if (threadIdx.x == 0) {
            d.head[f.p - 1] = f.kq;
            d.head[m + f.q - 1] = f.kp;
            d.bind[f.kq - 1] = f.p;
            d.bind[f.kp - 1] = m + f.q;
            d.stat[f.q - 1] = f.fxp ? NS : (f.delta > 0.0 ? NL : NU);
        } else if (threadIdx.x == 64) {
            if (f.rclr) d.refsp[f.kp - 1] = 0;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void finish_scalars(const SpxDev &d, const FinishIn &f, bool refsp_reset)
{
    DState *st = d.st;
    if (f.pend) {
        st->obj = f.t.obj;
        st->upd_cnt = f.upd_cnt + 1;
        st->binv_fresh = 0;
        st->cbar_fresh = 0;
        st->refact_pending = f.t.refact;
        st->it_cnt = f.it_cnt + 1;
        st->npiv = f.npiv + 1;
        st->iter_left = f.t.iter_left;
        if (f.rig > 0) st->rigorous = f.rig - 1;
        st->refct = f.t.refct;
        st->pend = 0;
    }
    if (refsp_reset) st->refct = 1000;
}

__device__ TopState dual_finish_block(const SpxDev &d, bool tail_sync)
{
    return finish_apply(d, finish_load(d), tail_sync);
}

__global__ void k_dual_finish(SpxDev d)
{
    (void)dual_finish_block(d, true);
}

// chuzr candidate of basic position i holding variable k (glpspx02.js:572-626)
__device__ __forceinline__ Cand chuzr_cand_v(int i, int k, int t, double lb, double ub, double bb, double g,
                                             double tol_bnd)
{
    double ri = 0.0;
    if (t == LO || t == DB || t == FX) {
        const double eps = tol_bnd * (1.0 + 0.10 * fabs(lb));
        if (bb < lb - eps) ri = lb - bb;
    }
    if (t == UP || t == DB || t == FX) {
        const double eps = tol_bnd * (1.0 + 0.10 * fabs(ub));
        if (bb > ub + eps) ri = ub - bb;
    }
    Cand e = no_cand(0.0);
    if (ri == 0.0) return e;
    if (g < DBL_EPS) g = DBL_EPS;
    const double temp = (ri * ri) / g;
    if (temp > 0.0) { e.k1 = temp; e.k2 = ri; e.idx = i + 1; e.aux = k; }
    return e;
}

// check_feas (glpspx02.js:1296): dual infeasibility of non-basic j
__device__ __forceinline__ int dual_bad(const SpxDev &d, int k, double cb, double tol)
{
    const int ot = d.orig_type[k - 1];
    if (cb < -tol && (ot == LO || ot == FR)) return 1;
    if (cb > +tol && (ot == UP || ot == FR)) return 1;
    return 0;
}

// batch start: chuzr candidates (one per 64 rows) and the phase-I check of
// the current state; the candidate slots [4 ceil(m / 256), gm) of a finer
// layout (k_dual_update: one per 16 rows) are cleared
__global__ void __launch_bounds__(256) k_dual_prep(SpxDev d, int gm, int panel)
{
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int s = 4 * ((m + 255) / 256) + i; s < gm; s += gridDim.x * blockDim.x) cand_chuzr(d)[s] = no_cand(0.0);
    // a batch without the MFMA panel (gk_panel.hip) changes the basis without
    // updating it: the panel is kept only across batches that maintain it
    if (i == 0 && !panel) st->pvalid = 0;
    const bool reset = (st->pricing == PT_PSE && st->refct == 0);
    if ((int)blockIdx.x * 256 < m) {
        Cand c = no_cand(0.0);
        if (i < m) {
            const int k = d.head[i];
            c = chuzr_cand_v(i, k, d.type[k - 1], d.lb[k - 1], d.ub[k - 1], d.bbar[i], reset ? 1.0 : d.gamma[i],
                             st->tol_bnd);
        }
        const Cand b = wave_best<0>(c);
        if ((threadIdx.x & 63) == 0) cand_chuzr(d)[blockIdx.x * 4 + (threadIdx.x >> 6)] = b;
    }
    if (st->phase == 1) {
        const int bad = (i < n) ? dual_bad(d, d.head[m + i], d.cbar[i], st->tol_dj) : 0;
        if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
    }
}

// ---------------------------------------------------------------------------
// k_dual_top (1 WG of 256): change_basis of the previous pivot, stop checks,
// chuzr, rho = row p of inv(B) in compact form.  The chuzr candidates (with
// the leaving variable in aux) and the dense-column list are loaded at entry
// (the list speculatively up to nr_cap); every wave makes the chuzr choice on
// its own, so the only block barrier is the one inside change_basis and the
// only dependent load is inv(B)[p, :].
// ---------------------------------------------------------------------------
constexpr int TOP_WG = 256;

__global__ void __launch_bounds__(TOP_WG) k_dual_top(SpxDev d, int rowpath, int nr_cap)
{
    const TraceScope trace_(d, 0);
    DState *st = d.st;
    const int stop = st->stop;               // tested before the first store
    const int m = d.m, n = d.n;
    const int gm = 4 * ((m + 255) / 256);
    // more candidates than 4 per lane (m > 16,384: the sparse factor's
    // problems): the block's waves split them and meet in LDS (better<0> is
    // a total order: the choice of one wave's walk over all of them)
    const bool split = gm > 256;
    const int lane = threadIdx.x & 63;
    Cand c = no_cand(0.0);
    for (int b = split ? (int)threadIdx.x : lane; b < gm; b += split ? TOP_WG : 64) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, c)) c = e;
    }
    if (split) {
        __shared__ Cand scw[TOP_WG / 64];
        const Cand cw = wave_best<0>(c);
        if (lane == 0) scw[threadIdx.x >> 6] = cw;
        __syncthreads();
        c = scw[0];
        for (int k = 1; k < TOP_WG / 64; ++k)
            if (better<0>(scw[k], c)) c = scw[k];
    }
    constexpr int RPT = 16;                   // list entries prefetched per thread
    int cl[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int t = threadIdx.x + u * TOP_WG;
        cl[u] = (t < nr_cap) ? d.rlist[t] : 0;
    }
    const FinishIn fin = finish_load(d);
    const int pricing = st->pricing, phase = st->phase, dinf = st->dinf, nr = st->nr;
    const double zeta = st->zeta, obj_ll = st->obj_ll, obj_ul = st->obj_ul;
    if (stop) return;
    const TopState ts = finish_apply(d, fin, false);
    if (ts.iter_left <= 0 || ts.refact) {
        if (threadIdx.x == 0) st->stop = ts.refact ? ST_REFACT : ST_BATCH;
        return;
    }
    if (pricing == PT_PSE && ts.refct == 0) {
        __syncthreads();                   // the header writes of change_basis are visible
        reset_refsp_dev(d, 1);             // refsp := basic variables, gamma := 1
        for (int l = threadIdx.x; l < n; l += blockDim.x) d.wpos[l] = -1;
        if (threadIdx.x == 0) st->nwl = 0;
        __syncthreads();
    }
    if (phase == 1) {
        if (!dinf) {
            if (threadIdx.x == 0) st->stop = ST_PHASE;
            return;
        }
    } else {
        // objective limits (:1729-1760)
        const double z = zeta, obj = ts.obj;
        const bool hit = (z < 0.0 && obj_ll > -DBL_MAX && obj <= obj_ll) ||
                         (z > 0.0 && obj_ul < +DBL_MAX && obj >= obj_ul);
        if (hit) {
            if (threadIdx.x == 0) st->stop = ST_OBJLIM;
            return;
        }
    }
    // chuzr from the per-wave candidates (the same choice in every wave)
    const Cand best = wave_best<0>(c);
    if (best.idx == 0) {
        if (threadIdx.x == 0) { st->p = 0; st->stop = ST_P0; }
        return;
    }
    const int p = best.idx, kp = best.aux;
    if (rowpath == 3) {
        // sparse factor: rho = inv(B)' e_p is the BTRAN that follows
        // (gk_sparse.hip sp_pivot_btran), nothing of inv(B) is stored here
        if (threadIdx.x == 0) {
            st->p = p;
            st->kp = kp;
            st->delta = best.k2;
            st->trow_max_bits = 0ull;
            st->ns = 0;
            st->dinf = 0;
        }
        return;
    }
    if (!rowpath) {
        for (int l = threadIdx.x; l < m; l += blockDim.x) d.rho[l] = 0.0;
        __syncthreads();
    }
    const double *brow = d.Binv + (p - 1);
    const size_t ldb = (size_t)d.ldb;
    double v[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int t = threadIdx.x + u * TOP_WG;
        v[u] = (t < nr) ? brow[(size_t)cl[u] * ldb] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int t = threadIdx.x + u * TOP_WG;
        if (t < nr) {
            if (!rowpath) d.rho[cl[u]] = v[u];
            d.rho_idx[t] = cl[u];
            d.rho_val[t] = v[u];
        }
    }
    for (int t = threadIdx.x + RPT * TOP_WG; t < nr; t += blockDim.x) {   // nr > 4096 only
        const int cc = d.rlist[t];
        const double vv = brow[(size_t)cc * ldb];
        if (!rowpath) d.rho[cc] = vv;
        d.rho_idx[t] = cc;
        d.rho_val[t] = vv;
    }
    if (threadIdx.x == 0) {
        int ns = nr;
        if (kp <= m) {   // the basic slack at position p: unit column of inv(B)
            if (!rowpath) d.rho[kp - 1] = 1.0;
            d.rho_idx[nr] = kp - 1;
            d.rho_val[nr] = 1.0;
            ns++;
        }
        st->p = p;
        st->kp = kp;
        st->delta = best.k2;
        st->trow_max_bits = 0ull;
        st->ns = ns;
        st->dinf = 0;
    }
}

// ---------------------------------------------------------------------------
// k_dual_top_grid (column-pass path, dense A, nr large): k_dual_top spread
// over the grid.  Every block makes the chuzr choice itself; block 0 applies
// the pending change of basis, the stop tests and the reference-space reset.
// The dense rho is written by rows (rho_i = inv(B)[p, i] for a dense column
// i, else 1 at the leaving slack, else 0: the unit columns are exact), the
// compact rho by list position; 256 rows / list entries per thread block.
// ---------------------------------------------------------------------------
// (PANEL = 0: no panel pick compiled in, so the plans without the panel do
// not reserve its 24 KB candidate array in LDS — ADVICE r5)
template <int PANEL>
__global__ void __launch_bounds__(256) k_dual_top_grid(SpxDev d, int pcap, int page_max)
{
    const TraceScope trace_(d, 0);
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const bool lead = (blockIdx.x == 0);
    const int stop = st->stop;
    const FinishIn fin = finish_load(d);
    const int pricing = st->pricing, phase = st->phase, dinf = st->dinf, nr = st->nr;
    const double zeta = st->zeta, obj_ll = st->obj_ll, obj_ul = st->obj_ul;
    const int gm = 4 * ((m + 255) / 256);
    Cand cc = no_cand(0.0);
    for (int b = lane; b < gm; b += 64) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, cc)) cc = e;
    }
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int rp = (i < m) ? d.rpos[i] : -1;
    const int cl = (i < nr) ? d.rlist[i] : 0;
    if (stop) return;
    const TopState ts = fin.t;
    int why = ST_RUN;
    if (ts.iter_left <= 0 || ts.refact) why = ts.refact ? ST_REFACT : ST_BATCH;
    else if (phase == 1 && !dinf) why = ST_PHASE;
    else if (phase != 1 && ((zeta < 0.0 && obj_ll > -DBL_MAX && ts.obj <= obj_ll) ||
                            (zeta > 0.0 && obj_ul < +DBL_MAX && ts.obj >= obj_ul)))
        why = ST_OBJLIM;
    const Cand best = wave_best<0>(cc);
    if (why == ST_RUN && best.idx == 0) why = ST_P0;
    // every block passes the entry gate before block 0 stores the state
    // (gk_device.h); the header arrays it changes are not read here
    gate_arrive(st);
    if (why != ST_RUN) {
        if (lead) {
            if (threadIdx.x == 0) gate_wait(st);
            finish_arrays(d, fin);
            if (threadIdx.x == 0) {
                finish_scalars(d, fin, false);
                if (why == ST_P0) st->p = 0;
                st->stop = why;
            }
        }
        return;
    }
    const bool reset = pricing == PT_PSE && ts.refct == 0;
    if (lead) {
        if (threadIdx.x == 0) gate_wait(st);
        finish_arrays(d, fin);
        if (reset) {
            reset_refsp_dev(d, 1, false);     // refsp := basic variables, gamma := 1
            for (int l = threadIdx.x; l < n; l += blockDim.x) d.wpos[l] = -1;
            if (threadIdx.x == 0) st->nwl = 0;
        }
        if (threadIdx.x == 0) finish_scalars(d, fin, reset);
    }
    const int p = best.idx, kp = best.aux;
    const double *brow = d.Binv + (p - 1);
    const size_t ldb = (size_t)d.ldb;
    const double vr = (i < m && rp >= 0) ? brow[(size_t)i * ldb] : 0.0;
    const double vl = (i < nr) ? brow[(size_t)cl * ldb] : 0.0;
    if (i < m) d.rho[i] = (rp >= 0) ? vr : (i == kp - 1 ? 1.0 : 0.0);
    if (i < nr) {
        d.rho_idx[i] = cl;
        d.rho_val[i] = vl;
    }
    if (lead && threadIdx.x == 0) {
        int ns = nr;
        if (kp <= m) {
            d.rho_idx[nr] = kp - 1;
            d.rho_val[nr] = 1.0;
            ns++;
        }
        st->p = p;
        st->kp = kp;
        st->delta = best.k2;
        st->trow_max_bits = 0ull;
        st->ns = ns;
        st->dinf = 0;
    }
    // the pricing panel's pick for this p (pcap > 0: the plan has the panel;
    // k_panel_pick's work, one launch fewer)
    if (PANEL && lead && pcap > 0) panel_pick_dev(d, gm, pcap, page_max, p);
}

// ---------------------------------------------------------------------------
// k_trow_finish (column-pass path: sparse A, or rho too dense for the row
// path): structural column c / slack row c of the pivot row computed by the
// column pass; the PSE vectors of update_gamma (:1103-1134), per-block sums
// of those trow^2 (gamma_p), and the block's Harris pass-1 candidate under the
// block-local significance tolerance (k_dual_ratio re-checks it).
// ---------------------------------------------------------------------------
// (panel: the pivot row read from the pricing panel here — k_panel_trow's
// work: the panel row of p at a structural, -rho at an auxiliary, 0 at a
// fixed variable, stored to trow with its maximum — one launch fewer)
// flags: 1 — the row comes from the MFMA panel; 2 — column-sharded pricing:
// work holds the exchanged A w, made work = ys - A w here
__global__ void __launch_bounds__(256) k_trow_finish(SpxDev d, int pse, int flags)
{
    const int panel = flags & 1;
    const TraceScope trace_(d, 5);
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    // sparse factor: h is free from the previous pivot's FTRAN to this
    // pivot's pick, so its zero fill runs here on the grid instead of in the
    // pick's single workgroup (build_hq then writes the column only)
    if (d.sp && idx < m) d.h[idx] = 0.0;
    const int pos1 = (idx < n) ? d.bind[m + idx] : 0;
    const int pos2 = (idx < m) ? d.bind[idx] : 0;
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    int s1 = 0, s2 = 0;
    double cb1 = 0.0, cb2 = 0.0, tv1 = 0.0, tv2 = 0.0;
    bool ref1 = false, ref2 = false;
    if (j1 >= 0) {
        s1 = d.stat[j1];
        cb1 = d.cbar[j1];
        if (panel) {
            tv1 = (s1 != NS) ? d.pnl[(size_t)st->pcur * d.ldp + idx] : 0.0;
            d.trow[j1] = tv1;
        } else
            tv1 = d.trow[j1];
        if (pse) ref1 = d.refsp[m + idx] != 0;
    }
    if (j2 >= 0) {
        s2 = d.stat[j2];
        cb2 = d.cbar[j2];
        if (panel) {
            tv2 = (s2 != NS) ? -d.rho[idx] : 0.0;
            d.trow[j2] = tv2;
        } else
            tv2 = d.trow[j2];
        if (pse) ref2 = d.refsp[idx] != 0;
    }
    double gsum = 0.0;
    if (pse) {
        const double w1 = ref1 ? tv1 : 0.0, w2 = ref2 ? tv2 : 0.0;
        if (idx < n) d.wcol[idx] = w1;
        if (idx < m) d.ys[idx] = w2;
        if ((flags & 2) && idx < m) d.work[idx] = w2 - d.work[idx];
        gsum = w1 * w1 + w2 * w2;
    }
    // per 64-slot group (one wave): max |trow|, gamma_p partial, pass-1
    // candidate with eps_g = tol_bnd (1 + 0.01 max_g) <= eps
    const int grp = blockIdx.x * 4 + (threadIdx.x >> 6);
    const double bmax = wmax(fmax(fabs(tv1), fabs(tv2)));
    const double g = pse ? wsum(gsum) : 0.0;
    const RatioCtx x = ratio_ctx(st, bmax);
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (j1 >= 0 && pass1_cand(x, tv1, cb1, s1, j1, m + idx + 1, e) && better<1>(e, c)) c = e;
    if (j2 >= 0 && pass1_cand(x, tv2, cb2, s2, j2, idx + 1, e) && better<1>(e, c)) c = e;
    const Cand b = wave_best<1>(c);
    if ((threadIdx.x & 63) == 0) {
        if (pse) d.gpart[grp] = g;
        tmax_part(d)[grp] = bmax;
        cand_pass1(d)[grp] = b;
        if (panel && bmax > 0.0) atomicMax(&st->trow_max_bits, dbits(bmax));
    }
}

// ---------------------------------------------------------------------------
// k_trow_rows (row path, dense A): the pivot row and the work of
// k_trow_finish in one kernel.  Block b owns the 64 slots [64 b, 64 b + 64)
// (structural column c and slack row c of each slot).  Its waves split the
// support of rho (rows t = w, w + nw, ... of AT, 512-byte coalesced segments
// of the 64 columns; the first group of rho entries is loaded before ns is
// known), the partial sums meet in LDS in wave order, and wave 0 finishes the
// slots with wave-level reductions: trow, the PSE vectors, the gamma_p
// partial, max |trow| and the Harris pass-1 candidate of the block.
// Block 0 stamps the device clock at entry and every block at exit (tslots).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_trow_rows(SpxDev d, int pse)
{
    const TraceScope trace_(d, 1);
    __shared__ double sp[16][64];
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    const int idx = blockIdx.x * 64 + lane;
    // trip 1: the state, the slot positions (wave 0) and the first group of
    // rho entries (inside the allocation: m + 1 entries); stop is tested
    // before the first store, not before the first load
    const int stop = st->stop, ns = st->ns;
    const RatioIn rin = ratio_in(st);
    int pos1 = 0, pos2 = 0, rp2 = -1;
    if (w == 0) {
        pos1 = (idx < n) ? d.bind[m + idx] : 0;
        pos2 = (idx < m) ? d.bind[idx] : 0;
        rp2 = (idx < m) ? d.rpos[idx] : -1;
    }
    const int *__restrict__ ri = d.rho_idx;
    const double *__restrict__ rv = d.rho_val;
    int r0[8];
    double v0[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int t = w + u * nw;
        r0[u] = (t <= m) ? ri[t] : 0;
        v0[u] = (t <= m) ? rv[t] : 0.0;
    }
    // trip 2: the slot operands (wave 0) and the first rows of AT
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    int s1 = 0, s2 = 0;
    double cb1 = 0.0, cb2 = 0.0, rho2 = 0.0;
    bool ref1 = false, ref2 = false;
    if (j1 >= 0) {
        s1 = d.stat[j1];
        cb1 = d.cbar[j1];
        if (pse) ref1 = d.refsp[m + idx] != 0;
    }
    if (j2 >= 0) {
        s2 = d.stat[j2];
        cb2 = d.cbar[j2];
        rho2 = d.rho_val[rp2];
        if (pse) ref2 = d.refsp[idx] != 0;
    }
    double acc = 0.0;
    const double *__restrict__ col = d.A.AT + min(idx, n - 1);
    const size_t ldt = (size_t)d.A.ldt;
    {
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = (w + u * nw < ns) ? col[(size_t)r0[u] * ldt] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (w + u * nw < ns) acc += v0[u] * a[u];
    }
    if (stop) return;
    if (d.tslots && blockIdx.x == 0 && threadIdx.x == 0) st->tk_start = wall_clock64();
    TPH(1, 0);
    {
        int t = w + 8 * nw;
        for (; t + 7 * nw < ns; t += 8 * nw) {
            int r[8];
            double v[8], a[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                r[u] = ri[t + u * nw];
                v[u] = rv[t + u * nw];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] = col[(size_t)r[u] * ldt];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u] * a[u];
        }
        for (; t < ns; t += nw) acc += rv[t] * col[(size_t)ri[t] * ldt];
    }
    TPH(1, 1);
    sp[w][lane] = (idx < n) ? acc : 0.0;
    __syncthreads();
    TPH(1, 2);
    if (w != 0) return;                      // wave 0 only from here: no block barriers
    // the waves' partial sums in wave order; the LDS loads issued together
    // (a loop over the runtime wave count waited for each load in turn)
    double tp16[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) tp16[k] = (k < nw) ? sp[k][lane] : 0.0;
    double tsum = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < nw) tsum += tp16[k];
    double tv1 = (j1 >= 0) ? tsum : 0.0;
    double tv2 = (j2 >= 0) ? -rho2 : 0.0;    // a non-basic slack is a dense column of inv(B)
    if (s1 == NS) tv1 = 0.0;
    if (s2 == NS) tv2 = 0.0;
    TPH(1, 3);
    if (j1 >= 0) d.trow[j1] = tv1;
    if (j2 >= 0) d.trow[j2] = tv2;
    double gsum = 0.0;
    if (pse) {
        const double w1 = ref1 ? tv1 : 0.0, w2 = ref2 ? tv2 : 0.0;
        if (idx < n) d.wcol[idx] = w1;
        if (idx < m) d.ys[idx] = w2;
        gsum = w1 * w1 + w2 * w2;
    }
    const double bmax = wmax(fmax(fabs(tv1), fabs(tv2)));
    const double g = pse ? wsum(gsum) : 0.0;
    // pass-1 candidate with eps_b = tol_bnd (1 + 0.01 max_b) <= eps
    const RatioCtx x = ratio_ctx(rin, bmax);
    TPH(1, 4);
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (j1 >= 0 && pass1_cand(x, tv1, cb1, s1, j1, m + idx + 1, e) && better<1>(e, c)) c = e;
    if (j2 >= 0 && pass1_cand(x, tv2, cb2, s2, j2, idx + 1, e) && better<1>(e, c)) c = e;
    const Cand b = wave_best<1>(c);
    TPH(1, 5);
    if (lane == 0) {
        tmax_part(d)[blockIdx.x] = bmax;
        if (pse) d.gpart[blockIdx.x] = g;
        cand_pass1(d)[blockIdx.x] = b;
        if (d.tslots) d.tslots[blockIdx.x] = wall_clock64();
    }
}

// ---------------------------------------------------------------------------
// k_dual_row (row path, dense A): k_dual_top and k_trow_rows in ONE kernel.
// Every block makes the chuzr choice itself (wave reduction over the
// commit's per-wave candidates, the leaving variable in aux), reads its rho
// entries straight from inv(B) (rho_t = inv(B)[p, rlist[t]], plus the unit
// entry 1 at row kp - 1 when the leaving variable is a slack) and forms its
// 64 slots of the pivot row.  The pending change of basis of the previous
// pivot is applied by block 0; the other blocks patch the few entries it
// changes (bind of kp / kq, stat of q, refsp of kp) where they read them, so
// the race with block 0's writes is benign (the patch is idempotent).  Block
// 0 also publishes the compact rho (rho_idx / rho_val, read by the commit),
// the scalar state and, every 1000 pivots, the reference-space reset.
// ---------------------------------------------------------------------------
// NP: list entries per wave loaded in trips 1-2 (8, or 16 when ns may exceed
// 8 per wave: the entries past them are read by a loop whose every
// iteration is two dependent trips)
template <int NP>
__global__ void __launch_bounds__(1024) k_dual_row(SpxDev d, int pse, int nr_cap, int gm)
{
    const TraceScope trace_(d, 1);
    __shared__ double sp[16][64];
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    const int idx = blockIdx.x * 64 + lane;
    // the block that applies the pending change of basis, publishes rho and the
    // scalar state: the last one (no slack slots when n > m, so the lightest)
    const bool lead = (blockIdx.x == gridDim.x - 1);
    // ---- trip 1: state, chuzr candidates, the wave's list entries, slots
    const int stop = st->stop;
    const FinishIn fin = finish_load(d);
    const int pricing = st->pricing, phase = st->phase, dinf = st->dinf, nr = st->nr;
    const double zeta = st->zeta, obj_ll = st->obj_ll, obj_ul = st->obj_ul;
    const RatioIn rin = ratio_in(st);
    // unconditional loads at clamped indices, selected afterwards: no load
    // waits for another (see finish_load)
    Cand ce[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) ce[u] = cand_chuzr(d)[min(lane + 64 * u, gm - 1)];
    int c0[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) c0[u] = d.rlist[min(w + u * nw, m - 1)];
    int pos1 = d.bind[m + min(idx, n - 1)];
    int pos2 = d.bind[min(idx, m - 1)];
    // the wave's rows of AT depend on the list alone: issued now, in flight
    // while the chuzr choice below resolves (the rho entries wait for it)
    const double *__restrict__ col = d.A.AT + min(idx, n - 1);
    const size_t ldt = (size_t)d.A.ldt;
    double a0[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) a0[u] = col[(size_t)min(max(c0[u], 0), m - 1) * ldt];
    Cand cc = no_cand(0.0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (lane + 64 * u < gm && better<0>(ce[u], cc)) cc = ce[u];
    for (int b = lane + 256; b < gm; b += 64) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, cc)) cc = e;
    }
#pragma unroll
    for (int u = 0; u < NP; ++u) c0[u] = (w + u * nw < nr_cap) ? c0[u] : 0;
    if (w != 0 || idx >= n) pos1 = 0;
    if (w != 0 || idx >= m) pos2 = 0;
    if (stop) return;
    if (d.tslots && lead && threadIdx.x == 0) st->tk_start = wall_clock64();
    // ---- decisions (identical in every block)
    const TopState ts = fin.t;
    int why = ST_RUN;
    if (ts.iter_left <= 0 || ts.refact) why = ts.refact ? ST_REFACT : ST_BATCH;
    else if (phase == 1 && !dinf) why = ST_PHASE;
    else if (phase != 1 && ((zeta < 0.0 && obj_ll > -DBL_MAX && ts.obj <= obj_ll) ||
                            (zeta > 0.0 && obj_ul < +DBL_MAX && ts.obj >= obj_ul)))
        why = ST_OBJLIM;
    const Cand best = wave_best<0>(cc);
    if (why == ST_RUN && best.idx == 0) why = ST_P0;
    const bool reset = (why == ST_RUN && pricing == PT_PSE && ts.refct == 0);
    if (why != ST_RUN) {
        // (every block agrees: the state it decided on is not stored until
        // all blocks have read it)
        gate_arrive(st);
        if (lead) {
            if (threadIdx.x == 0) gate_wait(st);
            finish_arrays(d, fin);
            if (threadIdx.x == 0) {
                finish_scalars(d, fin, false);
                if (why == ST_P0) st->p = 0;
                st->stop = why;
            }
        }
        return;
    }
    if (lead) {
        finish_arrays(d, fin);
        if (reset) {
            reset_refsp_dev(d, 1, false);     // refsp := basic variables, gamma := 1
            for (int l = threadIdx.x; l < n; l += blockDim.x) d.wpos[l] = -1;
            if (threadIdx.x == 0) st->nwl = 0;
        }
    }
    const int p = best.idx, kp = best.aux;
    const int ns = nr + (kp <= m ? 1 : 0);
    // the pending change of basis, as seen by this block
    auto bind_new = [&](int k1, int v) {
        if (!fin.pend) return v;
        if (k1 == fin.kq) return fin.p;
        if (k1 == fin.kp) return m + fin.q;
        return v;
    };
    // only slots that exist (structural idx < n, slack idx < m) and only in
    // wave 0, which holds the positions
    if (w == 0 && idx < n) pos1 = bind_new(m + idx + 1, pos1);
    if (w == 0 && idx < m) pos2 = bind_new(idx + 1, pos2);
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    // ---- trip 2: rho entries of the wave and their rows of AT; slot operands
    const double *__restrict__ brow = d.Binv + (p - 1);
    const size_t ldb = (size_t)d.ldb;
    double v0[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const int t = w + u * nw;
        int c = c0[u];
        double av = a0[u];
        if (t == nr) {                       // the unit entry (only when kp <= m: t < ns)
            c = kp - 1;
            av = col[(size_t)min(max(c, 0), m - 1) * ldt];
        }
        // list entries past nr are stale (or never written): clamp the
        // address, the value is not used
        const int ca = min(max(c, 0), m - 1);
        const double bv = brow[(size_t)ca * ldb];
        v0[u] = (t < nr) ? bv : 1.0;
        a0[u] = (t < ns) ? av : 0.0;
        c0[u] = c;
    }
    const signed char stq = fin.fxp ? NS : (fin.delta > 0.0 ? NL : NU);
    int s1 = 0, s2 = 0;
    double cb1 = 0.0, cb2 = 0.0, rho2 = 0.0;
    bool ref1 = false, ref2 = false;
    if (w == 0) {
        // the slot operands, loaded at clamped indices with the trip-2 loads
        const int j1c = max(j1, 0), j2c = max(j2, 0);
        const int l1 = d.stat[j1c], l2 = d.stat[j2c];
        const double c1 = d.cbar[j1c], c2 = d.cbar[j2c];
        const double r2 = brow[(size_t)min(idx, m - 1) * ldb];   // a non-basic slack: column idx of inv(B) is dense
        const int f1 = d.refsp[m + min(idx, n - 1)], f2 = d.refsp[min(idx, m - 1)];
        if (j1 >= 0) {
            s1 = (fin.pend && j1 == fin.q - 1) ? stq : l1;
            cb1 = c1;
            if (pse && !reset) ref1 = f1 != 0 && !(fin.pend && fin.rclr && m + idx + 1 == fin.kp);
        }
        if (j2 >= 0) {
            s2 = (fin.pend && j2 == fin.q - 1) ? stq : l2;
            cb2 = c2;
            rho2 = r2;
            if (pse && !reset) ref2 = f2 != 0 && !(fin.pend && fin.rclr && idx + 1 == fin.kp);
        }
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < NP; ++u)
        if (w + u * nw < ns) acc += v0[u] * a0[u];
    if (lead && lane == 0) {
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int t = w + u * nw;
            if (t < ns) {
                d.rho_idx[t] = c0[u];
                d.rho_val[t] = v0[u];
            }
        }
    }
    TPH(1, 0);
    {
        int t = w + NP * nw;
        for (; t < ns; t += 4 * nw) {
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
    }
    TPH(1, 1);
    sp[w][lane] = (idx < n) ? acc : 0.0;
    __syncthreads();
    TPH(1, 2);
    if (w != 0) return;                      // wave 0 only from here: no block barriers
    // the waves' partial sums in wave order; the LDS loads issued together
    // (a loop over the runtime wave count waited for each load in turn)
    double tp16[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) tp16[k] = (k < nw) ? sp[k][lane] : 0.0;
    double tsum = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < nw) tsum += tp16[k];
    double tv1 = (j1 >= 0) ? tsum : 0.0;
    double tv2 = (j2 >= 0) ? -rho2 : 0.0;
    if (s1 == NS) tv1 = 0.0;
    if (s2 == NS) tv2 = 0.0;
    if (j1 >= 0) d.trow[j1] = tv1;
    if (j2 >= 0) d.trow[j2] = tv2;
    double gsum = 0.0;
    if (pse) {
        const double w1 = ref1 ? tv1 : 0.0, w2 = ref2 ? tv2 : 0.0;
        if (idx < n) d.wcol[idx] = w1;
        if (idx < m) d.ys[idx] = w2;
        gsum = w1 * w1 + w2 * w2;
    }
    const double bmax = wmax(fmax(fabs(tv1), fabs(tv2)));
    const double g = pse ? wsum(gsum) : 0.0;
    // pass-1 candidate with eps_b = tol_bnd (1 + 0.01 max_b) <= eps; the
    // sign of delta is that of the chosen row
    RatioIn rin2 = rin;
    rin2.delta = best.k2;
    const RatioCtx x = ratio_ctx(rin2, bmax);
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (j1 >= 0 && pass1_cand(x, tv1, cb1, s1, j1, m + idx + 1, e) && better<1>(e, c)) c = e;
    if (j2 >= 0 && pass1_cand(x, tv2, cb2, s2, j2, idx + 1, e) && better<1>(e, c)) c = e;
    const Cand b = wave_best<1>(c);
    TPH(1, 5);
    if (lane == 0) {
        tmax_part(d)[blockIdx.x] = bmax;
        if (pse) d.gpart[blockIdx.x] = g;
        cand_pass1(d)[blockIdx.x] = b;
        if (d.tslots) d.tslots[blockIdx.x] = wall_clock64();
        // the choice goes to the outbox, which no block of this launch reads;
        // the scalar state every block read at entry (the pending pivot, the
        // counters, dinf) is rewritten by k_dual_ratio's block 0 from it
        if (lead) {
            st->ob_p = p;
            st->ob_kp = kp;
            st->ob_delta = best.k2;
            st->ob_ns = ns;
            st->ob_reset = reset ? 1 : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// k_dual_col (column path, sparse A): k_dual_top, the CSC column pass and
// k_trow_finish in ONE kernel — the sparse counterpart of k_dual_row.  Every
// wave owns 64 slots (structural column c and slack row c of each slot) and
// is one 64-slot group of the candidates.  The CSC entries of the slot's
// column are loaded before the pivot decision (they do not depend on it);
// after the chuzr choice (made in every wave from the commit's candidates)
// rho_i is read straight from row p of inv(B) — the unit columns of the
// basic slacks are stored exactly — so trow_c = sum_t cval[t] rho_cind[t]
// (eval_trow glpspx02.js:655-791, -rho' N_j) takes two dependent trips
// whatever the column length up to CU entries.  Block 0 applies the pending
// change of basis and publishes the compact rho (rho_idx / rho_val, read by
// the commit) and the scalar state; the other blocks patch what it changes,
// as in k_dual_row.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dual_col(SpxDev d, int pse, int nr_cap, int gm)
{
    const TraceScope trace_(d, 1);
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int grp = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int idx = grp * 64 + lane;
    const bool lead = (blockIdx.x == 0);
    // ---- trip 1: state, chuzr candidates, slot positions, CSC entries
    const int stop = st->stop;
    const FinishIn fin = finish_load(d);
    const int pricing = st->pricing, phase = st->phase, dinf = st->dinf, nr = st->nr;
    const double zeta = st->zeta, obj_ll = st->obj_ll, obj_ul = st->obj_ul;
    const RatioIn rin = ratio_in(st);
    Cand cc = no_cand(0.0);
    for (int b = lane; b < gm; b += 64) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, cc)) cc = e;
    }
    int pos1 = (idx < n) ? d.bind[m + idx] : 0;
    int pos2 = (idx < m) ? d.bind[idx] : 0;
    constexpr int CU = 8;                    // CSC entries per column loaded ahead
    int beg = 0, end = 0;
    if (idx < n) {
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
    // the dense-column list entries this thread publishes rho for
    constexpr int PU = 4;
    const int tpub = blockIdx.x * blockDim.x + threadIdx.x, npub = gridDim.x * blockDim.x;
    int cpub[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
        const int t = tpub + u * npub;
        cpub[u] = (t < nr_cap) ? d.rlist[t] : 0;
    }
    if (stop) return;
    if (d.tslots && lead && threadIdx.x == 0) st->tk_start = wall_clock64();
    // ---- decisions (identical in every wave)
    const TopState ts = fin.t;
    int why = ST_RUN;
    if (ts.iter_left <= 0 || ts.refact) why = ts.refact ? ST_REFACT : ST_BATCH;
    else if (phase == 1 && !dinf) why = ST_PHASE;
    else if (phase != 1 && ((zeta < 0.0 && obj_ll > -DBL_MAX && ts.obj <= obj_ll) ||
                            (zeta > 0.0 && obj_ul < +DBL_MAX && ts.obj >= obj_ul)))
        why = ST_OBJLIM;
    const Cand best = wave_best<0>(cc);
    if (why == ST_RUN && best.idx == 0) why = ST_P0;
    const bool reset = (why == ST_RUN && pricing == PT_PSE && ts.refct == 0);
    // every block passes the entry gate before block 0 stores the state
    // (gk_device.h); the header arrays it changes early are patched below
    gate_arrive(st);
    if (why != ST_RUN) {
        if (lead) {
            if (threadIdx.x == 0) gate_wait(st);
            finish_arrays(d, fin);
            if (threadIdx.x == 0) {
                finish_scalars(d, fin, false);
                if (why == ST_P0) st->p = 0;
                st->stop = why;
            }
        }
        return;
    }
    if (lead) {
        finish_arrays(d, fin);
        if (reset) {
            reset_refsp_dev(d, 1, false);     // refsp := basic variables, gamma := 1
            for (int l = threadIdx.x; l < n; l += blockDim.x) d.wpos[l] = -1;
            if (threadIdx.x == 0) st->nwl = 0;
        }
    }
    const int p = best.idx, kp = best.aux;
    const int ns = nr + (kp <= m ? 1 : 0);
    auto bind_new = [&](int k1, int v) {
        if (!fin.pend) return v;
        if (k1 == fin.kq) return fin.p;
        if (k1 == fin.kp) return m + fin.q;
        return v;
    };
    if (idx < n) pos1 = bind_new(m + idx + 1, pos1);
    if (idx < m) pos2 = bind_new(idx + 1, pos2);
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    // ---- trip 2: rho at the column's rows, the slot operands
    const double *__restrict__ brow = d.Binv + (p - 1);
    const size_t ldb = (size_t)d.ldb;
    double rv[CU];
#pragma unroll
    for (int u = 0; u < CU; ++u) rv[u] = (j1 >= 0 && beg + u < end) ? brow[(size_t)ci[u] * ldb] : 0.0;
    const signed char stq = fin.fxp ? NS : (fin.delta > 0.0 ? NL : NU);
    int s1 = 0, s2 = 0;
    double cb1 = 0.0, cb2 = 0.0, rho2 = 0.0;
    bool ref1 = false, ref2 = false;
    if (j1 >= 0) {
        s1 = (fin.pend && j1 == fin.q - 1) ? stq : d.stat[j1];
        cb1 = d.cbar[j1];
        if (pse && !reset) ref1 = d.refsp[m + idx] != 0 && !(fin.pend && fin.rclr && m + idx + 1 == fin.kp);
    }
    if (j2 >= 0) {
        s2 = (fin.pend && j2 == fin.q - 1) ? stq : d.stat[j2];
        cb2 = d.cbar[j2];
        rho2 = brow[(size_t)idx * ldb];      // a non-basic slack: column idx of inv(B) is dense
        if (pse && !reset) ref2 = d.refsp[idx] != 0 && !(fin.pend && fin.rclr && idx + 1 == fin.kp);
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < CU; ++u) acc += cv[u] * rv[u];
    if (j1 >= 0)
        for (int t = beg + CU; t < end; ++t) acc += d.A.cval[t] * brow[(size_t)d.A.cind[t] * ldb];
    {
        // the compact rho for the rank-1 update of the commit, spread over
        // the grid (list entries loaded at entry)
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
    if (lead && threadIdx.x == 0) {
        gate_wait(st);
        finish_scalars(d, fin, reset);
        st->p = p;
        st->kp = kp;
        st->delta = best.k2;
        st->trow_max_bits = 0ull;
        st->ns = ns;
        st->dinf = 0;
    }
    double tv1 = (j1 >= 0) ? acc : 0.0;
    double tv2 = (j2 >= 0) ? -rho2 : 0.0;
    if (s1 == NS) tv1 = 0.0;
    if (s2 == NS) tv2 = 0.0;
    if (j1 >= 0) d.trow[j1] = tv1;
    if (j2 >= 0) d.trow[j2] = tv2;
    double gsum = 0.0;
    if (pse) {
        const double w1 = ref1 ? tv1 : 0.0, w2 = ref2 ? tv2 : 0.0;
        if (idx < n) d.wcol[idx] = w1;
        if (idx < m) d.ys[idx] = w2;
        gsum = w1 * w1 + w2 * w2;
    }
    const double bmax = wmax(fmax(fabs(tv1), fabs(tv2)));
    const double g = pse ? wsum(gsum) : 0.0;
    RatioIn rin2 = rin;
    rin2.delta = best.k2;
    const RatioCtx x = ratio_ctx(rin2, bmax);
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (j1 >= 0 && pass1_cand(x, tv1, cb1, s1, j1, m + idx + 1, e) && better<1>(e, c)) c = e;
    if (j2 >= 0 && pass1_cand(x, tv2, cb2, s2, j2, idx + 1, e) && better<1>(e, c)) c = e;
    const Cand b = wave_best<1>(c);
    if (lane == 0) {
        tmax_part(d)[grp] = bmax;
        if (pse) d.gpart[grp] = g;
        cand_pass1(d)[grp] = b;
        if (d.tslots) d.tslots[grp] = wall_clock64();
    }
}

// ---------------------------------------------------------------------------
// k_dual_ratio: blocks [0, gn) — pass-1 choice from the ncb group candidates
// (a group whose candidate fails the global significance tolerance is
// rescanned), then the pass-2 candidates of positions [256 b, 256 b + 256),
// one per wave; blocks [gn, ...) — partials of A w over the reference-space
// columns.  Every wave makes the pass-1 choice on its own (no block barrier).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dual_ratio(SpxDev d, int gn, int tiles_m, int rowpath, int ncb, int nwl_cap,
                                                    int nprev)
{
    const TraceScope trace_(d, 2);
    DState *st = d.st;
    const int stop = st->stop;               // tested before the first store
    const int m = d.m, n = d.n;
    if ((int)blockIdx.x >= gn && d.A.dense && nwl_cap > 0) {
        // work = ys - A w in one pass (nwl <= nwl_cap): 64 rows per block,
        // lane = row, the 4 waves split wlist (entries loaded ahead up to the
        // cap, before nwl is known), partials combined in wave order
        __shared__ double sw[4][64];
        const int lane = threadIdx.x & 63, w4 = threadIdx.x >> 6;
        const int r = (blockIdx.x - gn) * 64 + lane;
        const int rc = min(r, m - 1);
        constexpr int WU = 16;
        // unconditional loads at clamped indices (no load waits for another)
        int cl[WU];
#pragma unroll
        for (int u = 0; u < WU; ++u) cl[u] = d.wlist[min(w4 + 4 * u, n - 1)];
        const int cnt = st->nwl;
        const double ysr = d.ys[rc];
        if (stop) return;
        const double *__restrict__ A = d.A.A;
        const size_t lda = (size_t)d.A.lda;
        double wv[WU], av[WU];
#pragma unroll
        for (int u = 0; u < WU; ++u) {
            // entries past nwl are stale (or never written): clamped address
            const int c = (w4 + 4 * u < nwl_cap) ? min(max(cl[u], 0), n - 1) : 0;
            wv[u] = d.wcol[c];
            av[u] = A[(size_t)c * lda + rc];
        }
#pragma unroll
        for (int u = 0; u < WU; ++u) {
            const bool ok = w4 + 4 * u < cnt && r < m;
            wv[u] = ok ? wv[u] : 0.0;
            av[u] = ok ? av[u] : 0.0;
        }
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < WU; ++u) acc += av[u] * wv[u];
        for (int t = w4 + 4 * WU; t < cnt; t += 4) {
            const int c = d.wlist[t];
            acc += (r < m ? A[(size_t)c * lda + r] : 0.0) * d.wcol[c];
        }
        sw[w4][lane] = acc;
        __syncthreads();
        if (w4 == 0 && r < m) d.work[r] = ysr - (((sw[0][lane] + sw[1][lane]) + sw[2][lane]) + sw[3][lane]);
        return;
    }
    if (!d.A.dense && (int)blockIdx.x >= gn + (m + 255) / 256) {
        // sparse A, one long row per block: the 4 waves stride its entries,
        // partials summed in wave order
        __shared__ double lw[4];
        const int r = d.A.lrow[blockIdx.x - gn - (m + 255) / 256];
        const int beg = d.A.rptr[r], end = d.A.rptr[r + 1];
        const double ysr = d.ys[r];
        if (stop) return;
        double acc = 0.0;
        for (int t = beg + (int)threadIdx.x; t < end; t += 256) acc += d.A.rval[t] * d.wcol[d.A.rcol[t]];
        acc = wsum(acc);
        if ((threadIdx.x & 63) == 0) lw[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) d.work[r] = ysr - (((lw[0] + lw[1]) + lw[2]) + lw[3]);
        return;
    }
    if ((int)blockIdx.x >= gn && !d.A.dense) {
        // sparse A: work = ys - A w, one row per thread over its CSR entries
        // (update_gamma :1103-1134; entries loaded ahead, fixed order)
        // (rows longer than CSR_LONG: the whole wave, below)
        const int r = (blockIdx.x - gn) * 256 + threadIdx.x;
        const int rc = min(r, m - 1);
        const int beg = d.A.rptr[rc], end = (r < m) ? d.A.rptr[rc + 1] : beg;
        const bool lng = end - beg > CSR_LONG;
        constexpr int RU = 16;
        int cc[RU];
        double av[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            const bool ok = !lng && beg + u < end;
            cc[u] = ok ? d.A.rcol[beg + u] : 0;
            av[u] = ok ? d.A.rval[beg + u] : 0.0;
        }
        const double ysr = d.ys[rc];
        if (stop) return;
        if (!lng && r < m) {
            double wv[RU];
#pragma unroll
            for (int u = 0; u < RU; ++u) wv[u] = (beg + u < end) ? d.wcol[cc[u]] : 0.0;
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < RU; ++u) acc += av[u] * wv[u];
            for (int t = beg + RU; t < end; ++t) acc += d.A.rval[t] * d.wcol[d.A.rcol[t]];
            d.work[r] = ysr - acc;
        }
        return;                                  // long rows: the blocks above
    }
    if ((int)blockIdx.x >= gn) {
        const int b = blockIdx.x - gn;
        const int tile = b % tiles_m, split = b / tiles_m, splits = (gridDim.x - gn) / tiles_m;
        const int cnt = st->nwl;
        if (stop) return;
        const int lps = (cnt + splits - 1) / splits;
        const int t0 = split * lps, t1 = min(cnt, t0 + lps);
        const int r = (tile * 256 + threadIdx.x) * 2;
        const double *wc = d.wcol;
        lgemv_tile<1>(d.A.A, (size_t)d.A.lda, m, d.wlist, t0, t1, r,
                      [&](int, int c, double &xa, double &xb) { xa = wc[c]; xb = 0.0; },
                      d.awpart + (size_t)split * m);
        // the last split to arrive at this tile forms work = ys - A w for its
        // rows, summing the partials in split order (deterministic)
        __shared__ int last;
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) last = (atomicAdd(&d.awcnt[tile], 1) == splits - 1);
        __syncthreads();
        if (!last) return;
        __threadfence();
        for (int rr = r; rr < min(r + 2, m); ++rr) {
            double acc = 0.0;
            for (int sp = 0; sp < splits; ++sp) acc += d.awpart[(size_t)sp * m + rr];
            d.work[rr] = d.ys[rr] - acc;
        }
        if (threadIdx.x == 0) d.awcnt[tile] = 0;
        return;
    }
    const int lane = threadIdx.x & 63;
    // roofline stamps (benches only: d.tslots set): the span of the pivot-row
    // kernel and of the previous pivot's k_dual_update, reduced from the
    // per-block exit stamps by block 0's first wave
    const bool stamps = d.tslots != nullptr;
    const unsigned long long t_entry = (stamps && rowpath && blockIdx.x == 0 && threadIdx.x == 0) ? wall_clock64() : 0ull;
    // the row path's k_dual_row left the new pivot's delta in the outbox
    // (st->delta still holds the pending pivot's until block 0 below)
    RatioIn rin = ratio_in(st);
    if (rowpath == 1) rin.delta = st->ob_delta;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int jc = min(j, n - 1);
    // unconditional loads at clamped indices, selected afterwards (no load
    // waits for another)
    double trj = d.trow[jc], cbj = d.cbar[jc];
    int sj = d.stat[jc], kj = d.head[m + jc];
    const bool lead = (blockIdx.x == 0 && threadIdx.x < 64);
    constexpr int CPL = 8;                    // group candidates per lane held in registers
    // more groups than a wave holds (large n: the sparse factor's problems):
    // the block's 4 waves split them and meet in LDS, instead of every wave
    // walking all of them one load per iteration
    const bool bsplit = ncb > CPL * 64;
    const int tb = bsplit ? (int)threadIdx.x : lane, tst = bsplit ? (int)blockDim.x : 64;
    Cand cl[CPL];
    double tv[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        const int b = min(tb + u * tst, ncb - 1);
        cl[u] = cand_pass1(d)[b];
        tv[u] = tmax_part(d)[b];
    }
    unsigned long long e = 0, xp = 0, u0 = 0;
    double uticks = 0.0, un = 0.0;
    if (stamps && rowpath && lead) {
        u0 = st->tk_upd0;
        uticks = st->upd_ticks;
        un = st->upd_n;
        unsigned long long te[CPL], tx[4];
#pragma unroll
        for (int u = 0; u < CPL; ++u) te[u] = d.tslots[min(lane + u * 64, ncb - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) tx[u] = d.xslots[min(lane + u * 64, max(nprev - 1, 0))];
#pragma unroll
        for (int u = 0; u < CPL; ++u) e = max(e, te[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) xp = max(xp, tx[u]);
        for (int b = lane + CPL * 64; b < ncb; b += 64) e = max(e, d.tslots[b]);
        for (int b = lane + 4 * 64; b < nprev; b += 64) xp = max(xp, d.xslots[b]);
    }
    if (j >= n) { trj = 0.0; cbj = 0.0; sj = 0; kj = 0; }
    double v = 0.0;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        if (tb + u * tst >= ncb) cl[u] = no_cand(DBL_MAX);
        else v = fmax(v, tv[u]);
    }
    for (int b = tb + CPL * tst; b < ncb; b += tst) v = fmax(v, tmax_part(d)[b]);
    double big = wmax(v);
    if (stop) return;
    __shared__ double rbig[4];
    __shared__ Cand rc1[4];
    __shared__ int rfl[4];
    if (bsplit) {
        if (lane == 0) rbig[threadIdx.x >> 6] = big;
        __syncthreads();
        big = fmax(fmax(rbig[0], rbig[1]), fmax(rbig[2], rbig[3]));
    }
    if (rowpath == 1 && blockIdx.x == 0 && threadIdx.x == 0) {
        // k_dual_row's outbox: the pending pivot's counters (finish_apply's
        // scalar half, from the state every block of k_dual_row read), then
        // the new pivot — no other block of this launch reads these fields
        const FinishIn f = finish_load(d);
        const int ob_p = st->ob_p, ob_kp = st->ob_kp, ob_ns = st->ob_ns, ob_reset = st->ob_reset;
        const double ob_delta = st->ob_delta;
        finish_scalars(d, f, ob_reset != 0);
        st->p = ob_p;
        st->kp = ob_kp;
        st->delta = ob_delta;
        st->ns = ob_ns;
        st->dinf = 0;
    }
    TPH(2, 0);
    if (lead) {
        // publish max |trow| and the end of the pivot-row kernel (latest
        // block exit stamp), and the last exit of the kernel before it
        const unsigned long long ee = stamps ? wmax_u64(e) : 0ull, xx = stamps ? wmax_u64(xp) : 0ull;
        if (lane == 0) {
            st->trow_max_bits = dbits(big);
            if (stamps && rowpath) {
                st->tk_next = t_entry;
                st->tk_end = ee;
                st->tk_prev = xx;
                // the previous pivot's k_dual_update: entry of its block 0 to
                // its last block exit (not across a batch boundary)
                if (u0 != 0ull && xx > u0 && xx - u0 < 20000ull) {
                    st->upd_ticks = uticks + (double)(xx - u0);
                    st->upd_n = un + 1.0;
                }
                st->tk_upd0 = 0ull;
            }
        }
    }
    const RatioCtx x = ratio_ctx(rin, big);
    Cand c = no_cand(DBL_MAX);
    int fail = 0;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        if (cl[u].idx != 0 && cl[u].k2 < x.eps) fail = 1;
        else if (better<1>(cl[u], c)) c = cl[u];
    }
    for (int b = tb + CPL * tst; b < ncb; b += tst) {
        const Cand f = cand_pass1(d)[b];
        if (f.idx != 0 && f.k2 < x.eps) fail = 1;
        else if (better<1>(f, c)) c = f;
    }
    if (bsplit) {
        // the waves' choices combined (better<1> is a total order: the same
        // choice as one wave's walk over every group); with a failing group
        // anywhere, every wave walks them all as below
        const Cand cw = wave_best<1>(c);
        const int fw = __any(fail) ? 1 : 0;
        if (lane == 0) {
            rc1[threadIdx.x >> 6] = cw;
            rfl[threadIdx.x >> 6] = fw;
        }
        __syncthreads();
        fail = rfl[0] | rfl[1] | rfl[2] | rfl[3];
        if (!fail) {
            c = rc1[0];
            for (int k = 1; k < 4; ++k)
                if (better<1>(rc1[k], c)) c = rc1[k];
        } else {
            c = no_cand(DBL_MAX);
            for (int b = lane; b < ncb; b += 64) {
                const Cand f = cand_pass1(d)[b];
                if (!(f.idx != 0 && f.k2 < x.eps) && better<1>(f, c)) c = f;
            }
        }
    }
    if (__any(fail)) {
        // rare: rescan the groups whose candidate is not significant (lane =
        // slot of the 64-slot group)
        for (int b = 0; b < ncb; ++b) {
            const Cand f = cand_pass1(d)[b];
            if (!(f.idx != 0 && f.k2 < x.eps)) continue;
            const Cand g = pass1_slot(d, x, b * 64 + lane);
            if (better<1>(g, c)) c = g;
        }
    }
    const Cand b1 = wave_best<1>(c);
    TPH(2, 1);
    const int q1 = b1.idx;
    const double teta1 = q1 ? b1.k1 : DBL_MAX;
    const int need2 = !(x.rtol == 0.0 || q1 == 0 || teta1 == 0.0);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->q1 = q1;
        st->teta1 = teta1;
        st->need2 = need2;
        st->kq1 = b1.aux;
        st->alfa1 = b1.k2;
    }
    if (!need2) return;
    Cand c2 = no_cand(0.0);
    if (j < n) {
        Cand f;
        if (pass2_cand(x, trj, cbj, sj, j, kj, teta1, f)) c2 = f;
    }
    const Cand b2 = wave_best<2>(c2);
    TPH(2, 2);
    if (lane == 0) cand_pass2(d)[blockIdx.x * 4 + (threadIdx.x >> 6)] = b2;
}

// the entering choice q (pass 2 if needed), its checks and the st fields;
// every wave of the calling grid evaluates it identically (no block
// barrier).  pick_load issues every load the choice needs (so a caller can
// put them in its first trip); pick_resolve returns q (kq through *kq_out),
// or 0 when the iteration stops.  The candidates carry |trow_q| (k2) and the
// entering variable (aux).
struct PickIn {
    int need2, q1, kq1, rigorous;
    double teta1, alfa1, big, delta;
    Cand c;                                   // this lane's best pass-2 candidate
    double g;                                 // lead wave: this lane's share of gamma_p
};

__device__ __forceinline__ PickIn pick_load(const SpxDev &d, int pse, int gn, int ncb)
{
    const DState *st = d.st;
    const int lane = threadIdx.x & 63;
    const bool lead = (blockIdx.x == 0 && blockIdx.y == 0);
    PickIn pi;
    pi.need2 = st->need2;
    pi.q1 = st->q1;
    pi.kq1 = st->kq1;
    pi.rigorous = st->rigorous;
    pi.teta1 = st->teta1;
    pi.alfa1 = st->alfa1;
    pi.big = trow_big(st);
    pi.delta = st->delta;
    pi.c = no_cand(0.0);
    for (int b = lane; b < 4 * gn; b += 64) {
        const Cand e = cand_pass2(d)[b];
        if (better<2>(e, pi.c)) pi.c = e;
    }
    // gamma_p (update_gamma :1103-1132) from the group sums, fixed order
    pi.g = 0.0;
    if (lead && pse && threadIdx.x < 64)
        for (int b = lane; b < ncb; b += 64) pi.g += d.gpart[b];
    return pi;
}

__device__ int pick_resolve(const SpxDev &d, const PickIn &pi, int pse, int *kq_out)
{
    DState *st = d.st;
    const bool lead = (blockIdx.x == 0 && blockIdx.y == 0);
    int q, kq;
    double teta, alfa;
    if (pi.need2) {
        const Cand b2 = wave_best<2>(pi.c);
        q = b2.idx;
        teta = b2.k1;
        kq = b2.aux;
        alfa = b2.k2;
    } else {
        q = pi.q1;
        teta = pi.teta1;
        kq = pi.kq1;
        alfa = pi.alfa1;
    }
    if (q == 0) {
        if (lead && threadIdx.x == 0) { st->q = 0; st->stop = ST_Q0; }
        return 0;
    }
    if (alfa < 1e-5 * (1.0 + 0.01 * pi.big) && !pi.rigorous) {
        if (lead && threadIdx.x == 0) { st->q = q; st->stop = ST_SMALLPIV; }
        return 0;
    }
    if (lead && threadIdx.x < 64) {
        const double g = pse ? wsum(pi.g) : 0.0;
        if (threadIdx.x == 0) {
            if (pse) {
                const double eta = d.refsp[st->kp - 1] ? 1.0 : 0.0;
                st->eta_pq = eta;
                st->gamma_pq = eta + g;
            }
            st->q = q;
            st->kq = kq;
            st->new_dq = (pi.delta > 0.0 ? +1.0 : -1.0) * teta;
            st->cbar_q_old = d.cbar[q - 1];
        }
    }
    *kq_out = kq;
    return q;
}

__device__ __forceinline__ int dual_pick(const SpxDev &d, int pse, int gn, int ncb, int *kq_out)
{
    const PickIn pi = pick_load(d, pse, gn, ncb);
    return pick_resolve(d, pi, pse, kq_out);
}

// sparse A / rigorous mode: the pick and h = -N[q] in one workgroup.  The
// pass-2 candidates and gamma_p's group sums are split over the block's
// waves (thousands of them on the sparse factor's problems, where one wave's
// walk cost one load round trip per 64) and combined in LDS in wave order
__global__ void __launch_bounds__(1024) k_dual_pick(SpxDev d, int pse, int gn, int ncb)
{
    const DState *st = d.st;
    if (st->stop) return;
    __shared__ Cand pc[16];
    __shared__ double pg[16];
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, w = tid >> 6, nw = nt >> 6;
    PickIn pi;
    pi.need2 = st->need2;
    pi.q1 = st->q1;
    pi.kq1 = st->kq1;
    pi.rigorous = st->rigorous;
    pi.teta1 = st->teta1;
    pi.alfa1 = st->alfa1;
    pi.big = trow_big(st);
    pi.delta = st->delta;
    Cand c = no_cand(0.0);
    for (int b = tid; b < 4 * gn; b += nt) {
        const Cand e = cand_pass2(d)[b];
        if (better<2>(e, c)) c = e;
    }
    c = wave_best<2>(c);
    double g = 0.0;
    if (pse)
        for (int b = tid; b < ncb; b += nt) g += d.gpart[b];
    g = wsum(g);
    if (lane == 0) {
        pc[w] = c;
        pg[w] = g;
    }
    __syncthreads();
    pi.c = pc[0];
    double gt = pg[0];
    for (int k = 1; k < nw; ++k) {
        if (better<2>(pc[k], pi.c)) pi.c = pc[k];
        gt += pg[k];
    }
    pi.g = (lane == 0) ? gt : 0.0;         // (pick_resolve's wave sum of it is gt exactly)
    int kq = 0;
    const int q = pick_resolve(d, pi, pse, &kq);
    if (q) build_hq(d, q, d.sp != nullptr);
}

// work_c = ys_c - (A w)_c from the partials, fixed order
__device__ __forceinline__ double aw_value(const SpxDev &d, int c, int awsplits)
{
    double acc = 0.0;
#pragma unroll 8
    for (int s = 0; s < awsplits; ++s) acc += d.awpart[(size_t)s * d.m + c];
    return d.ys[c] - acc;
}

// ---------------------------------------------------------------------------
// k_dual_ftran (split path, many dense columns): tcol = inv(B) h,
// u = inv(B) work over the dense columns, partials over fsplits list chunks.
// FUSED (dense A): the pick runs here and h_c = A[c, q] is read from A.
// AW: work from the A w partials (dense A), else from d.work.
// ---------------------------------------------------------------------------
template <int NRHS, int FUSED, int AW>
__global__ void __launch_bounds__(256) k_dual_ftran(SpxDev d, int tiles, int gn, int awsplits, int ncb)
{
    const TraceScope trace_(d, 6);
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m;
    int q, kq = 0;
    if (FUSED) {
        q = dual_pick(d, NRHS == 2, gn, ncb, &kq);
        if (!q) return;
    } else {
        q = st->q;
        kq = d.head[m + q - 1];
    }
    const double *hcol = (kq > m) ? d.A.A + (size_t)(kq - m - 1) * d.A.lda : nullptr;
    const int b = blockIdx.x;
    const int tile = b % tiles, split = b / tiles, splits = gridDim.x / tiles;
    const int cnt = st->nr;
    const int lps = (cnt + splits - 1) / splits;
    const int t0 = split * lps, t1 = min(cnt, t0 + lps);
    const int r = (tile * 256 + threadIdx.x) * 2;
    const double *h = d.h, *work = d.work;
    lgemv_tile_staged<NRHS>(d.Binv, (size_t)d.ldb, m, d.rlist, t0, t1, r,
                            [&](int, int c, double &xa, double &xb) {
                                if (FUSED) xa = hcol ? hcol[c] : (c == kq - 1 ? -1.0 : 0.0);
                                else xa = h[c];
                                if (NRHS == 2) xb = work[c];   // AW: formed by k_dual_ratio
                                else xb = 0.0;
                            },
                            d.partial + (size_t)split * NRHS * m);
}

// tcol[i] / u[i] = sum of the partials + the unit column of a basic slack
// at position i; 64 rows per block, 8 waves over the splits in fixed order
template <int NRHS, int FUSED, int AW>
__global__ void __launch_bounds__(512) k_dual_ftran_reduce(SpxDev d, int splits, int awsplits)
{
    const TraceScope trace_(d, 7);
    __shared__ double sh[NRHS][8][64];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 64 + lane;
    const double *part = d.partial;
    double a = 0.0, b = 0.0;
    if (r < m) {
#pragma unroll 4
        for (int s = w; s < splits; s += 8) {
            a += part[(size_t)s * NRHS * m + r];
            if (NRHS == 2) b += part[(size_t)s * NRHS * m + m + r];
        }
    }
    sh[0][w][lane] = a;
    if (NRHS == 2) sh[NRHS - 1][w][lane] = b;
    __syncthreads();
    if (w != 0 || r >= m) return;
    double va = sh[0][0][lane], vb = (NRHS == 2) ? sh[NRHS - 1][0][lane] : 0.0;
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        va += sh[0][k][lane];
        if (NRHS == 2) vb += sh[NRHS - 1][k][lane];
    }
    const int kh = d.head[r];
    if (kh <= m) {
        const int c = kh - 1;
        if (FUSED) {
            const int kq = st->kq;
            va += (kq > m) ? d.A.A[(size_t)(kq - m - 1) * d.A.lda + c] : (c == kq - 1 ? -1.0 : 0.0);
        } else
            va += d.h[c];
        if (NRHS == 2) vb += d.work[c];
    }
    d.tcol[r] = va;
    if (NRHS == 2) d.u[r] = vb;
}

// ---------------------------------------------------------------------------
// k_dual_ftran1 (dense A, nr <= FONE_MAX): the pick, tcol = inv(B) h and
// u = inv(B)(ys - A w) in ONE kernel.  Block b owns rows [64 b, 64 b + 64);
// its waves split the dense-column list (entries t = w, w + nw, ...; each
// wave reads 512-byte segments of the columns).  A wave's entries, and with
// them the multipliers h_c = A[c, q] and work_c, are wave-uniform.  The list
// entries, work_c and the first group of inv(B) values are loaded before the
// pick resolves (they do not depend on q); the wave partials meet in LDS in
// wave order (the only block barrier).
// ---------------------------------------------------------------------------
constexpr int FONE_MAX = 2048;

template <int NRHS, int SP, int RPB>
__global__ void __launch_bounds__(1024) k_dual_ftran1(SpxDev d, int gn, int awsplits, int ncb, int nr_cap)
{
    const TraceScope trace_(d, 3);
    __shared__ double sp[NRHS][16][64];
    DState *st = d.st;
    const int stop = st->stop;               // tested before the pick's stores
    const int m = d.m;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    constexpr int SL = 64 / RPB;             // list slices per wave (RPB rows per block)
    const int sl = lane / RPB;
    const int r = blockIdx.x * RPB + (lane % RPB);
    const int gs = w * SL + sl, NSL = nw * SL;
    const bool act = r < m;
    const size_t ldb = (size_t)d.ldb;
    const int *__restrict__ rl = d.rlist;
    const double *__restrict__ Bv = d.Binv;
    // trip 1: the pick's inputs, the wave's first list entries, this row's
    // basic variable
    const PickIn pin = pick_load(d, NRHS == 2, gn, ncb);
    constexpr int G = 8;
    int c0[G];
    double bv[G], wv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
        const int t = gs + u * NSL;
        c0[u] = (t < nr_cap) ? rl[t] : 0;
    }
    const int nr = st->nr;
    const int kh = (w == 0 && sl == 0 && act) ? d.head[r] : m + 1;
    // trip 2: q-independent inv(B) values and work_c
#pragma unroll
    for (int u = 0; u < G; ++u) {
        const bool ok = gs + u * NSL < nr;
        bv[u] = (act && ok) ? Bv[(size_t)c0[u] * ldb + r] : 0.0;
        wv[u] = (NRHS == 2 && ok) ? d.work[c0[u]] : 0.0;
    }
    double ub = 0.0;
    if (NRHS == 2 && kh <= m) ub = d.work[kh - 1];
    if (stop) return;
    TPH(3, 0);
    int kq = 0;
    const int q = pick_resolve(d, pin, NRHS == 2, &kq);
    if (!q) return;
    const double *hcol = (!SP && kq > m) ? d.A.A + (size_t)(kq - m - 1) * d.A.lda : nullptr;
    TPH(3, 1);
    auto hval = [&](int c) { return hcol ? hcol[c] : (c == kq - 1 ? -1.0 : 0.0); };
    double ua = 0.0;
    if (!SP && kh <= m) ua = hval(kh - 1);
    double a = 0.0, b = 0.0;
    if (SP) {
        // sparse h = -N[q]: tcol = inv(B) h over the entries of column q,
        // the waves splitting them; the columns of inv(B) are read whole
        // (unit columns included), so no unit part is added
        if (kq > m) {
            const int cq = kq - m - 1;
            const int beg = d.A.cptr[cq], end = d.A.cptr[cq + 1];
            for (int t = beg + gs; t < end; t += NSL)
                a += d.A.cval[t] * (act ? Bv[(size_t)d.A.cind[t] * ldb + r] : 0.0);
        } else if (gs == 0) {
            a = act ? -Bv[(size_t)(kq - 1) * ldb + r] : 0.0;
        }
    }
    {
        double xa[G];
#pragma unroll
        for (int u = 0; u < G; ++u) xa[u] = (!SP && gs + u * NSL < nr) ? hval(c0[u]) : 0.0;
#pragma unroll
        for (int u = 0; u < G; ++u) {
            if (!SP) a += bv[u] * xa[u];
            if (NRHS == 2) b += bv[u] * wv[u];
        }
    }
    if (!SP || NRHS == 2) {
        int t = gs + G * NSL;
        for (; t + 3 * NSL < nr; t += 4 * NSL) {
            int c[4];
            double x[4], xa[4], xb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = rl[t + u * NSL];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                x[u] = act ? Bv[(size_t)c[u] * ldb + r] : 0.0;
                xa[u] = SP ? 0.0 : hval(c[u]);
                xb[u] = (NRHS == 2) ? d.work[c[u]] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (!SP) a += x[u] * xa[u];
                if (NRHS == 2) b += x[u] * xb[u];
            }
        }
        for (; t < nr; t += NSL) {
            const int c = rl[t];
            const double x = act ? Bv[(size_t)c * ldb + r] : 0.0;
            if (!SP) a += x * hval(c);
            if (NRHS == 2) b += x * d.work[c];
        }
    }
    sp[0][w][lane] = a;
    if (NRHS == 2) sp[NRHS - 1][w][lane] = b;
    TPH(3, 2);
    __syncthreads();
    TPH(3, 3);
    if (w != 0 || sl != 0 || !act) return;
    double va = 0.0, vb = 0.0;
    for (int k = 0; k < nw; ++k)
#pragma unroll
        for (int z = 0; z < SL; ++z) {
            va += sp[0][k][lane + z * RPB];
            if (NRHS == 2) vb += sp[NRHS - 1][k][lane + z * RPB];
        }
    d.tcol[r] = va + ua;
    if (NRHS == 2) d.u[r] = vb + ub;
}

// ---------------------------------------------------------------------------
// k_dual_commit: pivot check (:1913-1933), update_bbar (:1042), update_cbar
// (:1020), update_gamma (:1075-1134) in the first `nvb` blocks, together with
// the chuzr candidates and the phase-I check of the next iteration; the
// rank-1 update of the dense columns of inv(B) in the others (row p :=
// rho / alpha_p, row i -= alpha_i / alpha_p rho) over the compact rho
// (entries [chunk lpsu, ...) loaded at entry).  A slack leaving the basis
// turns its unit column dense (the extra rho entry, value 1); a slack
// entering turns its column into exactly e_p.  Block 0 also maintains the
// dense-column and reference-space lists for the change of basis and
// accounts the pivot's algorithmic bytes.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dual_commit(SpxDev d, int pse, int nvb, int tiles, int lpsu, int rowpath,
                                                     double bytes_fixed, int pfrom)
{
    const TraceScope trace_(d, 4);
    const ExitStamp xs_(d.xslots, blockIdx.x);
    DState *st = d.st;
    // all loads first, stop tested before the first store; the pivot indices
    // are clamped so that the loads of a stopped iteration stay in bounds
    const int stop = st->stop;
    const int m = d.m, n = d.n;
    const int p = max(st->p, 1), q = max(st->q, 1), kp = max(st->kp, 1), kq = max(st->kq, 1);
    if ((int)blockIdx.x < nvb) {
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        // gathers first: the row / column operands and what the next
        // iteration's chuzr and check_feas read
        const bool in_m = i < m, in_n = i < n;
        const int kold = in_m ? d.head[i] : 1;
        double bb = in_m ? d.bbar[i] : 0.0;
        const double ti = in_m ? d.tcol[i] : 0.0;
        double g = in_m ? d.gamma[i] : 0.0;
        const double ui = (pse && in_m) ? d.u[i] : 0.0;
        double cb = in_n ? d.cbar[i] : 0.0;
        const double tri = in_n ? d.trow[i] : 0.0;
        const int kn = in_n ? ((i == q - 1) ? kp : d.head[m + i]) : 1;
        const double piv1 = d.tcol[p - 1], piv2 = d.trow[q - 1];
        const int tkq = d.type[kq - 1], tkp = d.type[kp - 1];
        const bool refkp = pse && d.refsp[kp - 1] != 0;
        const int knew = (i == p - 1) ? kq : kold;
        const int tkold = in_m ? d.type[kold - 1] : 0;
        const bool refk = (pse && in_m) ? d.refsp[kold - 1] != 0 : false;
        const int tknew = in_m ? d.type[knew - 1] : 0;
        const double lbn = in_m ? d.lb[knew - 1] : 0.0, ubn = in_m ? d.ub[knew - 1] : 0.0;
        const int ot = in_n ? d.orig_type[kn - 1] : 0;
        const double xq = (i == p - 1) ? get_xN(d.stat, d.lb, d.ub, kq, q) : 0.0;
        // list maintenance operands (block 0, wave 1)
        const bool maint = (blockIdx.x == 0 && threadIdx.x == 64);
        int rq = -1, wq = -1, rlast = 0, wlast = 0, nr0 = 0, nwl0 = 0;
        if (maint) {
            nr0 = st->nr;
            nwl0 = st->nwl;
            if (kq <= m) rq = d.rpos[kq - 1];
            if (kq > m) wq = d.wpos[kq - m - 1];
            rlast = d.rlist[max(nr0 - 1, 0)];
            if (pse) wlast = d.wlist[max(nwl0 - 1, 0)];
        }
        const int binv_fresh = st->binv_fresh, rig = st->rigorous, phase = st->phase, refct = st->refct;
        const double delta = st->delta, new_dq = st->new_dq, gamma_p = st->gamma_pq, eta_p = st->eta_pq;
        const double tol_bnd = st->tol_bnd, tol_dj = st->tol_dj, upd_tol = st->upd_tol;
        if (stop) return;
        const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                         !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
        if (bad && (!binv_fresh || !rig)) {
            if (blockIdx.x == 0 && threadIdx.x == 0) st->stop = ST_PIVCHK;
            return;
        }
        TPH(4, 0);
        const double tp = bad ? piv2 : piv1;
        const double teta = delta / tp;
        if (in_m) {
            if (i == p - 1) bb = xq + teta;
            else if (teta != 0.0) bb += ti * teta;
            d.bbar[i] = bb;
        }
        if (in_n) {
            if (i == q - 1) cb = new_dq;
            else if (new_dq != 0.0) cb -= tri * new_dq;
            d.cbar[i] = cb;
        }
        if (pse && in_m) {
            if (i == p - 1) {
                if (tkq == FR) g = 1.0;
                else {
                    g = gamma_p / (tp * tp);
                    if (g < DBL_EPS) g = DBL_EPS;
                }
            } else if (ti != 0.0 && tkold != FR) {
                const double t = ti / tp;
                const double t1 = g + t * t * gamma_p + 2.0 * t * ui;
                const double t2 = (refk ? 1.0 : 0.0) + eta_p * t * t;
                g = (t1 >= t2 ? t1 : t2);
                if (g < DBL_EPS) g = DBL_EPS;
            }
            if (tkp == FX && refkp && ti != 0.0) {
                double t = 0.0;
                bool apply = true;
                if (i == p - 1) {
                    if (tkq == FR) apply = false; else t = 1.0 / tp;
                } else {
                    if (tkold == FR) apply = false; else t = ti / tp;
                }
                if (apply) {
                    g -= t * t;
                    if (g < DBL_EPS) g = DBL_EPS;
                }
            }
            d.gamma[i] = g;
        }
        // next iteration: chuzr candidates (gamma := 1 if the reference space
        // is reset before it) and check_feas (:1296) on the updated state
        if ((int)blockIdx.x * 256 < m) {
            Cand c = no_cand(0.0);
            if (in_m) {
                const bool reset = (pse && refct == 1);
                c = chuzr_cand_v(i, knew, tknew, lbn, ubn, bb, reset ? 1.0 : g, tol_bnd);
            }
            const Cand b = wave_best<0>(c);
            if ((threadIdx.x & 63) == 0) cand_chuzr(d)[blockIdx.x * 4 + (threadIdx.x >> 6)] = b;
            TPH(4, 1);
            // growth check of the product-form update (see k_dual_update)
            const bool grow = in_m && i != p - 1 && fabs(ti) * upd_tol > fabs(tp);
            if (__any(grow) && (threadIdx.x & 63) == 0) {
                atomicOr(&st->refact_pending, 1);
                atomicAdd(&st->echk, 1);
            }
            const double gr = (in_m && i != p - 1) ? fabs(ti) / fabs(tp) : 0.0;
            if (__any(gr > 100.0)) {
                const double gw = wmax(gr);
                if ((threadIdx.x & 63) == 0) atomicMax(&st->grow_bits, dbits(gw));
            }
        }
        if (phase == 1) {
            const double tol = tol_dj;
            const int badj = in_n && ((cb < -tol && (ot == LO || ot == FR)) || (cb > +tol && (ot == UP || ot == FR)));
            if (__syncthreads_or(badj) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->teta = teta;
            st->pivot = tp;
            st->pend = 1;
            st->fxp = (tkp == FX);
            st->rclr = (tkp == FX && refkp);
        }
        if (maint) {
            // dense columns of inv(B): an entering slack's column is now e_p,
            // a leaving slack's column became dense
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
                // reference-space non-basic structurals (update_gamma's A w)
                int nwl = nwl0;
                if (wq >= 0) {
                    d.wlist[wq] = wlast;
                    d.wpos[wlast] = wq;
                    d.wpos[kq - m - 1] = -1;
                    nwl--;
                }
                if (kp > m && refkp && tkp != FX) {
                    d.wlist[nwl] = kp - m - 1;
                    d.wpos[kp - m - 1] = nwl;
                    nwl++;
                }
                st->nwl = nwl;
            }
            // algorithmic HBM bytes of this pivot: the pivot row (rows of A in
            // the support of rho, or all of A), A w over the reference-space
            // columns, inv(B) once for both right-hand sides, read + write of
            // the updated columns, and the O(m + n) vectors
            const int ns = st->ns;
            const double rowb = rowpath == 1 ? 8.0 * (double)ns * n
                                : rowpath == 2 ? 12.0 * (double)d.A.nnz : 8.0 * (double)m * n;
            const unsigned long long tk0 = st->tk_start, tk1 = st->tk_end, tk2 = st->tk_next, tkp = st->tk_prev;
            if (d.tslots && rowpath && tk1 > tk0) {
                st->bytes_trow += rowb;
                st->trow_ticks += (double)(tk1 - tk0);
                st->trow_ticks_b += (double)(tk2 - tk0);
                st->trow_n += 1.0;
                // from the last exit of the kernel before it (the previous
                // pivot's commit / update; not the first pivot of a batch)
                if (tkp < tk0 && tk0 - tkp < 20000ull) {
                    st->trow_ticks_r += (double)(tk1 - tkp);
                    st->trow_nr += 1.0;
                }
            }
            st->tk_end = 0;
            // (rowpath 3, the sparse factor: bytes_fixed carries the whole
            // pivot's chain-independent bytes, sp_pivot_bytes; the host adds
            // the Schur correction's, which grow with the chain)
            st->bytes += rowpath == 3 ? bytes_fixed
                                      : rowb + 8.0 * (double)m * nwl0 + 8.0 * (double)m * (nr0 + 1) +
                                            16.0 * (double)m * (nr0 + (kp <= m ? 1 : 0)) + bytes_fixed;
        }
        return;
    }
    if (pfrom > 0 && (int)blockIdx.x >= pfrom) {
        // the pricing panel's rows t != pcur follow the rank-1 update
        // (k_panel_update's work, gk_panel.hip: G[t] -= (tcol[pos_t] / alpha)
        // G[pcur], one read-modify-write per thread); row pcur, which these
        // read, is replaced by k_panel_update_cur after this launch
        const int nbx = (n + 255) / 256;
        const int pb = blockIdx.x - pfrom, t = pb / nbx;
        const int j = (pb % nbx) * 256 + threadIdx.x;
        const int pk = st->pk, cur = st->pcur;
        const int binv_fresh = st->binv_fresh, rig = st->rigorous;
        const double piv1 = d.tcol[p - 1], piv2 = d.trow[q - 1];
        if (stop || t >= pk || t == cur || j >= n) return;
        const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                         !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
        if (bad && (!binv_fresh || !rig)) return;
        const double tp = bad ? piv2 : piv1;
        const size_t ldp = (size_t)d.ldp;
        const double gp = d.pnl[(size_t)cur * ldp + j];
        double *g = d.pnl + (size_t)t * ldp + j;
        const double f = d.tcol[d.ppos[t] - 1] / tp;
        if (f != 0.0) *g -= f * gp;
        return;
    }
    // rank-1 update over the dense columns (the compact rho: ns entries)
    const int b = blockIdx.x - nvb;
    const int tile = b % tiles, chunk = b / tiles;
    const int t0 = chunk * lpsu;
    const int r = (tile * 256 + threadIdx.x) * 2;
    if (r >= m) return;
    const bool two = (r + 1 < m);
    const double tr0 = d.tcol[r], tr1 = two ? d.tcol[r + 1] : 0.0;
    constexpr int U = 16;
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
    const int t1 = min(ns, t0 + lpsu);
    const double piv1 = d.tcol[p - 1], piv2 = d.trow[q - 1];
    const int ce = (kq <= m) ? kq - 1 : -1;
    double2 v0[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (t0 + u < t1) v0[u] = *(const double2 *)(d.Binv + (size_t)cc[u] * d.ldb + r);
    if (stop) return;
    const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                     !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
    if (bad && (!binv_fresh || !rig)) return;
    const double tp = bad ? piv2 : piv1;
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
// k_dual_update (nr + 1 <= GM * 4 * waves): k_dual_ftran1 and k_dual_commit
// in ONE kernel.  Block b owns the UPD_RPB = 16 rows [16 b, 16 b + 16); its
// lanes are (list slice, row) pairs, its waves split the compact rho
// (rho_idx[t] = rlist[t] for t < nr, then the unit entry of a leaving slack).
// A thread loads its GM entries of inv(B)[r, rho_idx[t]] once, into
// registers, and uses them twice:
//   eval_tcol / update_gamma's FTRAN (glpspx02.js:937, :1103-1134):
//     tcol_r = sum_{t < nr} inv(B)[r, c_t] h_c (+ h at a basic slack's row),
//     u_r    = sum_{t < nr} inv(B)[r, c_t] work_c (+ the same unit part);
//   then, once tcol_r is combined in LDS, the product-form update of those
//     same entries: row r -= tcol_r / alpha_p rho (row p := rho / alpha_p).
// alpha_p = tcol[p] = rho' h is formed by every block the same way (one
// wave over the compact rho, fixed order), so no block waits for the block
// that owns row p.  Everything else is k_dual_commit's per-row and per-column
// work (update_bbar / update_cbar / update_gamma :1020-1134, the next chuzr
// candidates — one per block — and the phase-I check), each block for its
// 16 rows and an n / grid slice of the columns; the pick (pass 2) runs in
// every wave as in k_dual_ftran1.  One kernel boundary and one read of the
// active columns of inv(B) less per pivot than ftran1 + commit.
// ---------------------------------------------------------------------------
// rows per block of k_dual_update: 16 (GM = 4 entries per thread) or 32
// (GM = 8: spills to scratch at 1024 threads and 128 VGPRs — 68 bytes per
// thread, 2.3x the algorithmic write traffic in the PMC counts);
// GK_UPD_RPB=32 selects it (experiments)
static int upd_rpb()
{
    static const int v = [] {
        const char *e = std::getenv("GK_UPD_RPB");
        return (e && std::atoi(e) == 32) ? 32 : 16;
    }();
    return v;
}

struct PickOut {
    int q, kq;
    double teta, alfa;
};

// pick_resolve's choice without its state writes (every block of the caller
// needs the same values)
__device__ __forceinline__ PickOut pick_choose(const PickIn &pi)
{
    PickOut o;
    if (pi.need2) {
        const Cand b2 = wave_best<2>(pi.c);
        o.q = b2.idx; o.teta = b2.k1; o.kq = b2.aux; o.alfa = b2.k2;
    } else {
        o.q = pi.q1; o.teta = pi.teta1; o.kq = pi.kq1; o.alfa = pi.alfa1;
    }
    return o;
}

// the books of a committed pivot (k_dual_update's block 0, its last wave):
// the dense-column list of inv(B) — an entering slack's column is now e_p, a
// leaving slack's column became dense —, the reference-space list of
// update_gamma's A w, and the algorithmic bytes and device-clock spans of the
// pivot.  Its operands are loaded with the kernel's second
// trip and parked in LDS (holding them in registers to the end of the kernel
// spills), so the bookkeeping at the end is stores only.
struct Books {
    int nwl0, rlast, wlast, rq, wq;
    unsigned long long tk0, tk1, tk2, tkp;
    double ab, abt, att, attb, atn, attr, atnr, abu;
};

template <int NRHS>
__device__ __forceinline__ void books_load(const SpxDev &d, Books &b, int nr, int kqc)
{
    const DState *st = d.st;
    const int m = d.m, n = d.n;
    const int nwl0 = (NRHS == 2) ? st->nwl : 0;
    const int rlast = d.rlist[max(nr - 1, 0)];
    const int wlast = (NRHS == 2) ? d.wlist[max(nwl0 - 1, 0)] : 0;
    const int rq = d.rpos[min(kqc, m) - 1];
    const int wq = (NRHS == 2) ? d.wpos[min(max(kqc - m, 1), n) - 1] : -1;
    b.nwl0 = nwl0; b.rlast = rlast; b.wlast = wlast; b.rq = rq; b.wq = wq;
    if (d.tslots) {                           // byte / clock accounting: benches only
        b.tk0 = st->tk_start; b.tk1 = st->tk_end; b.tk2 = st->tk_next; b.tkp = st->tk_prev;
        b.ab = st->bytes; b.abt = st->bytes_trow; b.att = st->trow_ticks; b.attb = st->trow_ticks_b;
        b.atn = st->trow_n; b.attr = st->trow_ticks_r; b.atnr = st->trow_nr; b.abu = st->bytes_upd;
    }
}

template <int NRHS>
__device__ __forceinline__ void books_store(const SpxDev &d, const Books &b, int kp, int kq, int tkp, bool refkp,
                                            int nr, int ns, int rowpath, double bytes_fixed)
{
    // straight-line code (selects and stores to a spare slot past the end of
    // each list instead of branches): this runs in one wave per pivot, and
    // each branch of it costs an instruction fetch on the critical path
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int ds = m, dw = max(m, n);                     // spare slots of rlist / rpos and wlist / wpos
    const bool ent = kq <= m, lv = kp <= m;
    d.rlist[ent ? b.rq : ds] = b.rlast;
    d.rpos[ent ? b.rlast : ds] = b.rq;
    d.rpos[ent ? kq - 1 : ds] = -1;
    const int nr1 = nr - (ent ? 1 : 0);
    d.rlist[lv ? nr1 : ds] = kp - 1;
    d.rpos[lv ? kp - 1 : ds] = nr1;
    st->nr = nr1 + (lv ? 1 : 0);
    if (NRHS == 2) {
        const bool wout = kq > m && b.wq >= 0, win = kp > m && refkp && tkp != FX;
        d.wlist[wout ? b.wq : dw] = b.wlast;
        d.wpos[wout ? b.wlast : dw] = b.wq;
        d.wpos[wout ? kq - m - 1 : dw] = -1;
        const int nw1 = b.nwl0 - (wout ? 1 : 0);
        d.wlist[win ? nw1 : dw] = kp - m - 1;
        d.wpos[win ? kp - m - 1 : dw] = nw1;
        st->nwl = nw1 + (win ? 1 : 0);
    }
    if (!d.tslots) return;
    // (benches) the pivot row, A w, and inv(B) read once and written once
    // over the support of rho; the device-clock spans of the pivot-row
    // kernel, from its entry and from the last exit of the kernel before it
    // (the previous pivot's commit / update; not the first pivot of a batch);
    // k_dual_update's own algorithmic bytes: the touched entries of inv(B)
    // read and written (16 m ns), h = -N[q] and the PSE work vector, the
    // O(m) row vectors (head, bbar, gamma, tcol, type, bounds) and the O(n)
    // column vectors (cbar read + write, trow, head, orig_type)
    const double rowb = rowpath == 1 ? 8.0 * (double)ns * n
                        : rowpath == 2 ? 12.0 * (double)d.A.nnz : 8.0 * (double)m * n;
    const bool tm = rowpath && b.tk1 > b.tk0;
    const bool tr = tm && b.tkp < b.tk0 && b.tk0 - b.tkp < 20000ull;
    st->bytes_trow = tm ? b.abt + rowb : b.abt;
    st->trow_ticks = tm ? b.att + (double)(b.tk1 - b.tk0) : b.att;
    st->trow_ticks_b = tm ? b.attb + (double)(b.tk2 - b.tk0) : b.attb;
    st->trow_n = tm ? b.atn + 1.0 : b.atn;
    st->trow_ticks_r = tr ? b.attr + (double)(b.tk1 - b.tkp) : b.attr;
    st->trow_nr = tr ? b.atnr + 1.0 : b.atnr;
    st->tk_end = 0;
    st->bytes = b.ab + (rowb + 8.0 * (double)m * b.nwl0 + 16.0 * (double)m * ns + bytes_fixed);
    st->bytes_upd = b.abu + (16.0 * (double)m * ns + 16.0 * (double)m + 48.0 * (double)m + 29.0 * (double)n);
}

template <int NRHS, int SP, int GM, int RPB>
__global__ void __launch_bounds__(1024) k_dual_update(SpxDev d, int gn, int ncb, int nr_cap, int rowpath,
                                                      double bytes_fixed)
{
    const TraceScope trace_(d, 3);
    const ExitStamp xs_(d.xslots, blockIdx.x);
    if (d.tslots && blockIdx.x == 0 && threadIdx.x == 0) d.st->tk_upd0 = wall_clock64();
    constexpr int SL = 64 / RPB;
    __shared__ double sp[NRHS][16][64];
    __shared__ double srow[NRHS][RPB];
    __shared__ double sub[RPB];
    __shared__ double salp[16 * SL];
    __shared__ double salpha;
    __shared__ Books sbk;
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    const int wa = nw - 1;                          // the wave that forms alpha_p
    const int sl = lane / RPB, rl = lane % RPB;
    // block 0 keeps the books (list maintenance, the scalar state and the
    // byte / clock accounting of the pivot), in its last wave
    const bool bk = blockIdx.x == 0;
    const int r = blockIdx.x * RPB + rl;
    const int gs = w * SL + sl, NSL = nw * SL;
    const bool act = r < m;
    const bool rowlane = (w == 0 && sl == 0 && act);
    const size_t ldb = (size_t)d.ldb;
    const double *__restrict__ Bv = d.Binv;
    // ---- trip 1: everything independent of the entering choice.  Every
    // load is unconditional at a clamped index and selected afterwards, so
    // the trip is one batch of loads (a load guarded by a test of another
    // load's value waits for it: one memory round trip per guard)
    const int stop = st->stop;
    PickIn pin;
    pin.need2 = st->need2; pin.q1 = st->q1; pin.kq1 = st->kq1; pin.rigorous = st->rigorous;
    pin.teta1 = st->teta1; pin.alfa1 = st->alfa1; pin.big = trow_big(st); pin.delta = st->delta;
    const int np2 = 4 * gn;
    Cand c2l[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c2l[u] = cand_pass2(d)[min(lane + 64 * u, np2 - 1)];
    double gp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) gp[u] = (NRHS == 2) ? d.gpart[min(lane + 64 * u, ncb - 1)] : 0.0;
    const int nr = st->nr, ns = st->ns, p = max(st->p, 1), kp = max(st->kp, 1);
    const double delta = st->delta;
    const int binv_fresh = st->binv_fresh, rig = st->rigorous, phase = st->phase, refct = st->refct;
    const double tol_bnd = st->tol_bnd, tol_dj = st->tol_dj, upd_tol = st->upd_tol;
    int c0[GM];
    double rv[GM];
#pragma unroll
    for (int u = 0; u < GM; ++u) {
        const int t = min(gs + u * NSL, m);
        c0[u] = d.rho_idx[t];
        rv[u] = d.rho_val[t];
    }
    // the block's rows
    const int rc = min(r, m - 1);
    const int kold_l = d.head[rc];
    double bb = d.bbar[rc];
    double g = (NRHS == 2) ? d.gamma[rc] : 0.0;
    // the block's columns (update_cbar, check_feas)
    const int JPB = (n + gridDim.x - 1) / gridDim.x;
    const int j = blockIdx.x * JPB + (int)threadIdx.x;
    const bool colth = (int)threadIdx.x < JPB && j < n;
    const int jc = min(j, n - 1);
    double cb = d.cbar[jc];
    double tri = d.trow[jc];
    int hkj = d.head[m + jc];
    // ---- the selections of trip 1
    pin.c = no_cand(0.0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (lane + 64 * u < np2 && better<2>(c2l[u], pin.c)) pin.c = c2l[u];
    for (int b = lane + 256; b < np2; b += 64) {
        const Cand e = cand_pass2(d)[b];
        if (better<2>(e, pin.c)) pin.c = e;
    }
    pin.g = 0.0;                                    // gamma_p in every block, fixed order
    if (NRHS == 2 && w == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (lane + 64 * u < ncb) pin.g += gp[u];
        for (int b = lane + 256; b < ncb; b += 64) pin.g += d.gpart[b];
    }
#pragma unroll
    for (int u = 0; u < GM; ++u)
        if (gs + u * NSL > nr_cap) { c0[u] = 0; rv[u] = 0.0; }
    const int kold = rowlane ? kold_l : 1;
    if (!rowlane) { bb = 0.0; g = 0.0; }
    if (!colth) { cb = 0.0; tri = 0.0; hkj = 1; }
    TPH(3, 0);
    const double gsum = (NRHS == 2 && w == 0) ? wsum(pin.g) : 0.0;
    // ---- the entering choice (every wave)
    const PickOut pk = pick_choose(pin);
    const int q = pk.q, kq = pk.kq;
    const int qc = min(max(q, 1), n), kqc = min(max(kq, 1), m + n);
    // ---- trip 2: inv(B) entries, the multipliers, the choice's operands
    // (issued before the stop tests; addresses clamped)
    const bool hdense = !SP && kqc > m;
    const double *__restrict__ hcolv = d.A.A + (size_t)(hdense ? kqc - m - 1 : 0) * d.A.lda;
    double bv[GM], xa[GM], xb[GM];
#pragma unroll
    for (int u = 0; u < GM; ++u) {
        const int ca = min(max(c0[u], 0), m - 1);
        bv[u] = Bv[(size_t)ca * ldb + rc];
        xa[u] = SP ? 0.0 : hcolv[ca];
        xb[u] = (NRHS == 2) ? d.work[ca] : 0.0;
    }
    const int kou = min(max(kold - 1, 0), m - 1);          // a basic slack's row (kold <= m)
    const double ua_l = SP ? 0.0 : hcolv[kou];
    const double ub_l = (NRHS == 2) ? d.work[kou] : 0.0;
    const int tkp = d.type[kp - 1];
    const bool refkp = NRHS == 2 && d.refsp[kp - 1] != 0;
    const int knew = (r == p - 1) ? kqc : kold;
    const int tkold_l = d.type[kold - 1];
    const int refk_l = (NRHS == 2) ? d.refsp[kold - 1] : 0;
    const int tknew_l = d.type[knew - 1];
    const double lbn_l = d.lb[knew - 1], ubn_l = d.ub[knew - 1];
    const int stq_l = d.stat[qc - 1];
    const double lbq = d.lb[kqc - 1], ubq = d.ub[kqc - 1];
    const int tkq = d.type[kqc - 1];
    const double piv2 = d.trow[qc - 1];
    const int kn = colth ? ((j == q - 1) ? kp : hkj) : 1;
    const int ot_l = d.orig_type[kn - 1];
    if (bk && w == wa) {
        Books b;
        books_load<NRHS>(d, b, nr, kqc);
        if (lane == 0) sbk = b;
    }
    if (stop) return;
    const bool lead = bk && threadIdx.x == 0;
    if (q == 0) {
        if (lead) { st->q = 0; st->stop = ST_Q0; }
        return;
    }
    if (pk.alfa < 1e-5 * (1.0 + 0.01 * pin.big) && !pin.rigorous) {
        if (lead) { st->q = q; st->stop = ST_SMALLPIV; }
        return;
    }
    const double new_dq = (delta > 0.0 ? +1.0 : -1.0) * pk.teta;
    // h = -N[q]: a structural's column of A, or -e at a slack's row
    auto hsel = [&](int c, double v) { return hdense ? v : (c == kq - 1 ? -1.0 : 0.0); };
    double a = 0.0, b = 0.0, al = 0.0;
#pragma unroll
    for (int u = 0; u < GM; ++u) {
        // alpha_p = rho' h over the slice's entries (the unit entry t = nr
        // included); the FTRAN over t < nr only (unit columns per row)
        const int t = gs + u * NSL;
        const double h = (!SP && t < ns) ? hsel(c0[u], xa[u]) : 0.0;
        const double bvu = (act && t < ns) ? bv[u] : 0.0;
        bv[u] = bvu;
        if (!SP) {
            al += rv[u] * h;
            if (t < nr) a += bvu * h;
        }
        if (NRHS == 2 && t < nr) b += bvu * xb[u];
    }
    double ua = 0.0, ub = 0.0;                      // unit columns of a basic slack at this row
    if (rowlane && kold <= m) {
        if (!SP) ua = hsel(kold - 1, ua_l);
        if (NRHS == 2) ub = ub_l;
    }
    if (SP) {
        // sparse h = -N[q]: tcol = inv(B) h over the entries of column q, the
        // columns of inv(B) read whole (unit columns included: no unit part)
        if (kq > m) {
            const int cq = kq - m - 1;
            const int beg = d.A.cptr[cq], end = d.A.cptr[cq + 1];
            for (int t = beg + gs; t < end; t += NSL)
                a += d.A.cval[t] * (act ? Bv[(size_t)d.A.cind[t] * ldb + r] : 0.0);
        } else if (gs == 0) {
            a = act ? -Bv[(size_t)(kq - 1) * ldb + r] : 0.0;
        }
    }
    // alpha_p: dense — the slices' partial sums of rho' h (lanes of row 0
    // of each slice), combined in slice order below; sparse — row p of inv(B)
    // times the CSC column, one wave
    if (!SP && rl == 0) salp[gs] = al;
    if (SP && w == wa) {
        double s = 0.0;
        if (kq > m) {
            const int cq = kq - m - 1;
            const int beg = d.A.cptr[cq], end = d.A.cptr[cq + 1];
            for (int t = beg + lane; t < end; t += 64) s += d.A.cval[t] * Bv[(size_t)d.A.cind[t] * ldb + (p - 1)];
        } else if (lane == 0) {
            s = -Bv[(size_t)(kq - 1) * ldb + (p - 1)];
        }
        s = wsum(s);
        if (lane == 0) salpha = s;
    }
    // operands of the row updates that depend on the choice
    const int tkold = rowlane ? tkold_l : 0;
    const bool refk = (NRHS == 2 && rowlane) ? refk_l != 0 : false;
    const int tknew = rowlane ? tknew_l : 0;
    const double lbn = rowlane ? lbn_l : 0.0, ubn = rowlane ? ubn_l : 0.0;
    // get_xN (glpspx01.js:442) of the entering variable
    const double xq_v = (stq_l == NU) ? ubq : (stq_l == NF ? 0.0 : lbq);
    const double xq = (rowlane && r == p - 1) ? xq_v : 0.0;
    const int ot = colth ? ot_l : 0;
    sp[0][w][lane] = a;
    if (NRHS == 2) sp[NRHS - 1][w][lane] = b;
    if (NRHS == 2 && w == 0 && sl == 0) sub[rl] = ub;
    TPH(3, 2);
    // (the block barrier of the LDS combine) every block's entry loads —
    // st->nr among them — are done before block 0's books store the lists
    gate_arrive(st);
    // the three fixed-order sums (tcol and u of the block's rows, alpha_p)
    // are independent chains of nw * SL dependent adds: each in its own wave
    // (the lanes of the block's rows in the waves of tcol and u) so that they
    // run side by side; one wave does all when the block has fewer
    {
        const int wb = NRHS == 2 ? min(1, nw - 1) : 0, wl = min(2, nw - 1);
        // each sum in its fixed order (waves, then slices); the outer loop
        // unrolled so that the LDS loads of several waves are in flight
        if (w == 0 && sl == 0) {
            double sa = 0.0;
#pragma unroll 4
            for (int k = 0; k < nw; ++k)
#pragma unroll
                for (int z = 0; z < SL; ++z) sa += sp[0][k][rl + z * RPB];
            srow[0][rl] = sa + ua;
        }
        if (NRHS == 2 && w == wb && sl == 0) {
            double sb = 0.0;
#pragma unroll 4
            for (int k = 0; k < nw; ++k)
#pragma unroll
                for (int z = 0; z < SL; ++z) sb += sp[NRHS - 1][k][rl + z * RPB];
            srow[NRHS - 1][rl] = sb + sub[rl];
        }
        if (!SP && w == wl && lane == 0) {
            double s = 0.0;
#pragma unroll 8
            for (int k = 0; k < NSL; ++k) s += salp[k];
            salpha = s;
        }
    }
    __syncthreads();
    TPH(3, 3);
    const double piv1 = salpha;
    const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                     !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
    if (bad && (!binv_fresh || !rig)) {
        if (lead) {
            gate_wait(st);                          // (resets the gate: no books this launch)
            st->q = q; st->kq = kq; st->stop = ST_PIVCHK;
        }
        return;
    }
    const double tp = bad ? piv2 : piv1;
    const double teta = delta / tp;
    const double ti = srow[0][rl];
    const double ui = (NRHS == 2) ? srow[NRHS - 1][rl] : 0.0;
    // the books, as soon as the pivot is committed: their straight-line
    // code runs once per launch with a cold instruction cache (≈2.5 µs of
    // fetches), so the books wave starts it here, under wave 0's row and
    // column updates and the phase-I barrier below, instead of after them.
    // Nothing later in this kernel reads what it writes (the other blocks
    // read the compact rho, not the lists); st->nr / st->nwl, which every
    // block reads in trip 1, only once all blocks have passed the gate
    if (bk && w == wa && lane == 0) {
        gate_wait(st);
        books_store<NRHS>(d, sbk, kp, kq, tkp, refkp, nr, ns, rowpath, bytes_fixed);
    }
    // ---- product-form update of the entries held in registers
    {
        const bool z = (r == p - 1);
        const double f = z ? 1.0 / tp : ti / tp;
        const int ce = (kq <= m) ? kq - 1 : -1;
#pragma unroll
        for (int u = 0; u < GM; ++u) {
            const int t = gs + u * NSL;
            if (!act || t >= ns) continue;
            const int c = c0[u];
            double v = bv[u];
            if (c == ce) v = z ? 1.0 : 0.0;
            else v = (z ? 0.0 : v) - f * rv[u];
            d.Binv[(size_t)c * ldb + r] = v;
        }
    }
    TPH(3, 4);
    // ---- rows: update_bbar / update_gamma, the next chuzr candidates
    if (w == 0) {
        Cand cnd = no_cand(0.0);
        if (rowlane) {
            d.tcol[r] = ti;
            if (r == p - 1) bb = xq + teta;
            else if (teta != 0.0) bb += ti * teta;
            d.bbar[r] = bb;
            if (NRHS == 2) {
                const double eta_p = refkp ? 1.0 : 0.0;
                const double gamma_p = eta_p + gsum;
                if (r == p - 1) {
                    if (tkq == FR) g = 1.0;
                    else {
                        g = gamma_p / (tp * tp);
                        if (g < DBL_EPS) g = DBL_EPS;
                    }
                } else if (ti != 0.0 && tkold != FR) {
                    const double t = ti / tp;
                    const double t1 = g + t * t * gamma_p + 2.0 * t * ui;
                    const double t2 = (refk ? 1.0 : 0.0) + eta_p * t * t;
                    g = (t1 >= t2 ? t1 : t2);
                    if (g < DBL_EPS) g = DBL_EPS;
                }
                if (tkp == FX && refkp && ti != 0.0) {
                    double t = 0.0;
                    bool apply = true;
                    if (r == p - 1) {
                        if (tkq == FR) apply = false; else t = 1.0 / tp;
                    } else {
                        if (tkold == FR) apply = false; else t = ti / tp;
                    }
                    if (apply) {
                        g -= t * t;
                        if (g < DBL_EPS) g = DBL_EPS;
                    }
                }
                d.gamma[r] = g;
            }
            const bool reset = (NRHS == 2 && refct == 1);
            cnd = chuzr_cand_v(r, knew, tknew, lbn, ubn, bb, reset ? 1.0 : g, tol_bnd);
        }
        const Cand best = wave_best<0>(cnd);
        if (lane == 0) cand_chuzr(d)[blockIdx.x] = best;
        // growth of the product-form update: row i of the new inverse gains
        // tcol_i / alpha_p times row p, so a pivot with |alpha_p| < upd_tol
        // |tcol_i| amplifies the inverse's error by more than 1 / upd_tol —
        // the explicit inverse's counterpart of the Forrest-Tomlin check
        // |u_k2k2| < upd_tol max |u| (glpfhv.js:436-442): re-invert before
        // the next pivot (refact_pending ends the batch there)
        const bool grow = rowlane && r != p - 1 && fabs(ti) * upd_tol > fabs(tp);
        if (__any(grow) && lane == 0) {
            atomicOr(&st->refact_pending, 1);
            atomicAdd(&st->echk, 1);
        }
        const double gr = (rowlane && r != p - 1) ? fabs(ti) / fabs(tp) : 0.0;
        if (__any(gr > 100.0)) {
            const double gw = wmax(gr);
            if (lane == 0) atomicMax(&st->grow_bits, dbits(gw));
        }
    }
    TPH(3, 5);
    // ---- columns: update_cbar (:1020), check_feas of phase I (:1296)
    int badj = 0;
    if (colth) {
        const double cb_old = cb;
        if (j == q - 1) {
            cb = new_dq;
            st->cbar_q_old = cb_old;
        } else if (new_dq != 0.0)
            cb -= tri * new_dq;
        d.cbar[j] = cb;
        badj = phase == 1 && ((cb < -tol_dj && (ot == LO || ot == FR)) || (cb > +tol_dj && (ot == UP || ot == FR)));
    }
    TPH(3, 6);
    if (phase == 1 && __syncthreads_or(badj) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
    if (lead) {
        st->q = q;
        st->kq = kq;
        st->new_dq = new_dq;
        st->teta = teta;
        st->pivot = tp;
        st->pend = 1;
        st->fxp = (tkp == FX);
        st->rclr = (tkp == FX && refkp);
    }
    TPH(3, 7);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// ---- column-sharded pricing (gk_bfd_set_comm) ---------------------------
// The exchange block of a rank: its slice of the pivot row (L doubles), its
// max |trow| (as bits), and with PSE its partial A w over the members of W
// whose non-basic position is in its slice (m doubles): update_gamma's A w
// (glpspx02.js:1103-1134) sharded like the pivot row, the partials summed in
// rank order on every rank
__host__ __device__ static inline int shard_blk(int L, int m, int pse) { return L + 1 + (pse ? m : 0); }

// this rank's partial A w: k_dual_ratio's one-pass A w blocks (64 rows per
// block, the 4 waves split wlist, partials in wave order) over the members
// at positions [lo, hi) only — with one rank the sum is k_dual_ratio's, bit
// for bit
__global__ void __launch_bounds__(256) k_shard_aw(SpxDev d, int lo, int hi, double *out)
{
    __shared__ double sw[4][64];
    const DState *st = d.st;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63, w4 = threadIdx.x >> 6;
    const int r = blockIdx.x * 64 + lane;
    const int rc = min(r, m - 1);
    const int cnt = st->nwl;
    if (st->stop) return;
    const double *__restrict__ A = d.A.A;
    const size_t lda = (size_t)d.A.lda;
    double acc = 0.0;
    for (int t = w4; t < cnt; t += 4) {
        const int c = d.wlist[t];
        const int j = d.bind[m + c] - m - 1;              // its non-basic position
        const double wv = (j >= lo && j < hi) ? d.trow[j] : 0.0;
        acc += (r < m ? A[(size_t)c * lda + rc] : 0.0) * wv;
    }
    (void)n;
    sw[w4][lane] = acc;
    __syncthreads();
    if (w4 == 0 && r < m) out[r] = ((sw[0][lane] + sw[1][lane]) + sw[2][lane]) + sw[3][lane];
}

// this rank's slice of the pivot row and its max |trow| (as bits) into the
// send block; then every rank's slice into trow and the largest max, and the
// rank-ordered sum of the A w partials into work (k_trow_finish forms
// work = ys - A w from it)
__global__ void __launch_bounds__(256) k_shard_pack(const double *trow, int lo, int cnt, int L,
                                                    const unsigned long long *maxbits, double *send)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < L) send[i] = (i < cnt) ? trow[lo + i] : 0.0;
    if (i == 0) send[L] = __longlong_as_double((long long)*maxbits);
}

__global__ void __launch_bounds__(256) k_shard_unpack(const double *recv, int size, int L, int n, int m, int pse,
                                                      double *trow, unsigned long long *maxbits, double *aw)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int B = shard_blk(L, m, pse);
    if (j < n) {
        const int r = j / L, i = j - r * L;
        trow[j] = recv[(size_t)r * B + i];
    }
    if (pse && j < m) {
        double a = recv[(size_t)L + 1 + j];
        for (int r = 1; r < size; r++) a += recv[(size_t)r * B + L + 1 + j];
        aw[j] = a;
    }
    if (j == 0) {
        unsigned long long b = 0;
        for (int r = 0; r < size; r++) {
            const unsigned long long x = (unsigned long long)__double_as_longlong(recv[(size_t)r * B + L]);
            b = x > b ? x : b;
        }
        *maxbits = b;
    }
}

LpShard::~LpShard()
{
    if (dsend) (void)hipFree(dsend);
    if (drecv) (void)hipFree(drecv);
}

bool lp_force_colpass()
{
    static const bool on = [] {
        const char *e = std::getenv("GK_FORCE_COLPASS");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

// launched after this rank's column pass: the slices are all-gathered, so
// every rank holds the pivot row the single-GPU column pass forms — the same
// values, bit for bit (a column's dot product does not depend on the
// slicing), and with them the same pivot path
void lp_shard_trow(hipStream_t s, const SpxDev &d, int pse)
{
    LpShard &sh = *d.shard;
    const int n = d.n, m = d.m, L = sh.L;
    const int lo = std::min(n, sh.rank * L), cnt = std::min(n, lo + L) - lo;
    if (pse)
        hipLaunchKernelGGL(k_shard_aw, dim3(cdiv(m, 64)), dim3(256), 0, s, d, lo, lo + cnt, sh.dsend + L + 1);
    hipLaunchKernelGGL(k_shard_pack, dim3(cdiv(L, 256)), dim3(256), 0, s, (const double *)d.trow, lo, cnt, L,
                       (const unsigned long long *)&d.st->trow_max_bits, sh.dsend);
    const size_t bytes = (size_t)shard_blk(L, m, pse) * sizeof(double);
    if (gk_comm_allgather_dev(sh.comm, sh.dsend, bytes, sh.drecv, s, sh.hsend.data(), sh.hrecv.data()) != 0) {
        sh.failed = true;
        throw std::runtime_error("column-sharded pricing: the exchange failed");
    }
    hipLaunchKernelGGL(k_shard_unpack, dim3(cdiv(std::max(n, m), 256)), dim3(256), 0, s, (const double *)sh.drecv,
                       sh.size, L, n, m, pse, d.trow, &d.st->trow_max_bits, d.work);
}

DualPlan dual_plan(const SpxDev &d, int nr_max, int nwl_max, int pse, int rigorous)
{
    const int m = d.m, n = d.n;
    DualPlan pl{};
    pl.pse = pse;
    pl.rigorous = rigorous;
    nr_max = std::min(std::max(nr_max, 0), m);
    const int ns_max = std::min(m, nr_max + 1);
    pl.nr_cap = nr_max;
    pl.ns_cap = ns_max;
    // the row path reads 8 ns n bytes of AT, the column pass all of A plus a
    // dense rho; GK_ROWPATH_FRAC (experiments) moves the switch point ns / m
    static const double row_frac = [] {
        const char *e = std::getenv("GK_ROWPATH_FRAC");
        return e ? std::atof(e) : 0.5;
    }();
    // (column-sharded pricing: the column pass, whose slices the ranks own)
    const bool cp_only = d.shard || lp_force_colpass();
    pl.rowpath = (d.A.dense && d.A.AT && !rigorous && ns_max <= row_frac * m && !cp_only) ? 1 : 0;
    pl.fused = (d.A.dense && !rigorous) ? 1 : 0;
    const int tiles_t = cdiv(n, 512), tiles_f = cdiv(m, 512);
    pl.tsplits = std::max(1, std::min(2048 / tiles_t, cdiv(ns_max, 8)));
    pl.tsplits = std::max(1, std::min<int>(pl.tsplits, (int)(d.partial_cap / std::max(n, 1))));
    pl.twaves = ns_max <= 32 ? 4 : (ns_max <= 64 ? 8 : 16);    // 8 list entries per wave in trip 2
    const int nrhs = pse ? 2 : 1;
    pl.fsplits = std::max(1, std::min(2048 / tiles_f, cdiv(std::max(nr_max, 1), 8)));
    pl.fsplits = std::max(1, std::min<int>(pl.fsplits, (int)(d.partial_cap / ((size_t)nrhs * m))));
    pl.fone = (pl.fused && nr_max <= FONE_MAX) ? 1 : 0;
    pl.fwaves = nr_max <= 32 ? 4 : (nr_max <= 128 ? 8 : 16);
    pl.uchunks = std::max(1, std::min(2048 / tiles_f, cdiv(ns_max, 4)));
    pl.lpsu = cdiv(ns_max, pl.uchunks);
    pl.uchunks = cdiv(ns_max, pl.lpsu);
    pl.colpath = (!d.A.dense && !rigorous && nr_max <= FONE_MAX) ? 1 : 0;
    pl.awsplits = std::max(1, std::min(cdiv(std::max(nwl_max, 1), 32), 64));
    pl.awsplits = std::max(1, std::min<int>(pl.awsplits, (int)(d.awpart_cap / std::max(m, 1))));
    // FTRAN + commit in one kernel while the active columns of inv(B) fit the
    // registers of a 16-row block (4 entries per thread — 124 VGPRs at 1024
    // threads; 8 would spill —, 4 list slices per wave, up to 16 waves: at
    // most 256 entries); GK_DUAL_UPDATE=0 keeps the two-kernel path
    static const int upd_on = [] {
        const char *e = std::getenv("GK_DUAL_UPDATE");
        return e ? std::atoi(e) : 1;
    }();
    pl.gm = 4 * cdiv(m, 256);
    const int need = ns_max + 1;
    const int rpb = upd_rpb(), sl = 64 / rpb;
    const int rows_blocks = cdiv(m, rpb);
    if (upd_on && !rigorous && (pl.rowpath || pl.colpath) && (pl.fone || pl.colpath) && need <= 4 * 4 * 16 &&
        n <= rows_blocks * 1024) {
        pl.ugm = rpb == 32 ? 8 : 4;
        pl.uwaves = std::min(16, std::max(1, cdiv(need, pl.ugm * sl)));
        // every thread of the block also covers a column slot of update_cbar
        while (pl.uwaves < 16 && cdiv(n, rows_blocks) > 64 * pl.uwaves) pl.uwaves++;
        pl.fupd = 1;
        pl.gm = rows_blocks;
    }
    pl.awone = (pse && d.A.dense && nwl_max <= 512) ? std::max(nwl_max, 1) : 0;
    pl.panel = cp_only ? 0 : panel_wanted(d, pl);
    pl.panel_age = pl.panel ? panel_age_max() : 0;
    return pl;
}

void refine_rho_dev(hipStream_t s, const SpxDev &d);
void refine_tcol_dev(hipStream_t s, const SpxDev &d, int need_p);
void colpass_gated(hipStream_t s, const MatDev &A, int mode, int off, int cnt, const int *head,
                   const signed char *stat, const double *coef, const double *h, const double *x,
                   const double *y, double *out1, double *out2, unsigned long long *maxbits,
                   const DState *st, int need_p);

// GK_SHARD_SIM: every simulated rank's column pass, A w partial and pack in
// rank order, written into its receive block, then the unpack every rank of
// a real run executes (the same blocks, so the same row, maximum and A w)
void lp_shard_sim(hipStream_t s, const SpxDev &d, int pse)
{
    LpShard &sh = *d.shard;
    const int n = d.n, m = d.m, L = sh.L, G = sh.vsize;
    const size_t blk = (size_t)shard_blk(L, m, pse);
    for (int v = 0; v < G; ++v) {
        const int lo = std::min(n, v * L), cnt = std::min(n, lo + L) - lo;
        double *out = sh.drecv + (size_t)v * blk;
        colpass_gated(s, d.A, CP_TROW, m + lo, cnt, d.head, d.stat + lo, d.coef, nullptr, d.rho, nullptr, d.trow + lo,
                      nullptr, &d.st->trow_max_bits, d.st, 0);
        if (pse)
            hipLaunchKernelGGL(k_shard_aw, dim3(cdiv(m, 64)), dim3(256), 0, s, d, lo, lo + cnt, out + L + 1);
        hipLaunchKernelGGL(k_shard_pack, dim3(cdiv(L, 256)), dim3(256), 0, s, (const double *)d.trow, lo, cnt, L,
                           (const unsigned long long *)&d.st->trow_max_bits, out);
    }
    hipLaunchKernelGGL(k_shard_unpack, dim3(cdiv(std::max(n, m), 256)), dim3(256), 0, s, (const double *)sh.drecv, G,
                       L, n, m, pse, d.trow, &d.st->trow_max_bits, d.work);
}


double launch_trow_rows(hipStream_t s, const SpxDev &d, const DualPlan &pl, int ns)
{
    const int n = d.n;
    hipLaunchKernelGGL(k_lgemv_part, dim3(cdiv(n, 512), pl.tsplits), dim3(256), 0, s, d.A.AT, (size_t)d.A.ldt, n,
                       d.rho_idx, &d.st->ns, d.rho_val, d.partial, (DState *)nullptr, (unsigned long long *)nullptr);
    return 8.0 * (double)ns * n + 12.0 * ns;
}

static double bytes_fixed(const SpxDev &d) { return 96.0 * ((double)d.m + d.n); }

// algorithmic bytes of a dual pivot on the sparse factor, the
// part that does not depend on the Schur chain: 12 B per stored L / U entry
// per sweep — the BTRAN's two sweeps once, the 2-RHS FTRAN's two sweeps once
// (each entry read once, applied to both right-hand sides) —, the pivot
// row's CSC column pass and update_gamma's A w over the CSR rows (12 nnz(A)
// each), the new Y column written and the O(m + n) vectors.  The chain's
// Y / inv(M) reads (16 m k + 8 k^2 at chain length k) are added by the host
// per batch (sp_chain_bytes)
double sp_pivot_bytes(const SpxDev &d)
{
    long long nnz_lu = 0;
    int lv[4];
    double tl = 0.0;
    sp_info(d.sp, &nnz_lu, lv, &tl);
    return 24.0 * (double)nnz_lu + 24.0 * (double)d.A.nnz + 8.0 * d.m + bytes_fixed(d);
}

void dual_batch_begin(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    hipLaunchKernelGGL(k_dual_prep, dim3(cdiv(std::max(d.m, d.n), 256)), dim3(256), 0, s, d,
                       std::max(pl.gm, 4 * cdiv(d.m, 256)), pl.panel);
}

// blocks of the kernel that ends a pivot (their exit stamps: xslots)
static int prev_blocks(const SpxDev &d, const DualPlan &pl)
{
    if (pl.fupd) return cdiv(d.m, pl.ugm == 8 ? 32 : 16);
    return cdiv(std::max(d.m, d.n), 256) + cdiv(d.m, 512) * pl.uchunks;
}

template <int NRHS, int SP>
static void launch_update(hipStream_t s, const SpxDev &d, const DualPlan &pl, int gn, int ncb, int rowpath,
                          hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr)
{
    const dim3 grid(cdiv(d.m, pl.ugm == 8 ? 32 : 16)), block(64 * pl.uwaves);
    // (the extended launch only with events: graph capture takes the plain one)
    if (pl.ugm == 8) {
        if (e0)
            hipExtLaunchKernelGGL((k_dual_update<NRHS, SP, 8, 32>), grid, block, 0, s, e0, e1, 0, d, gn, ncb,
                                  pl.nr_cap, rowpath, bytes_fixed(d));
        else
            hipLaunchKernelGGL((k_dual_update<NRHS, SP, 8, 32>), grid, block, 0, s, d, gn, ncb, pl.nr_cap, rowpath,
                               bytes_fixed(d));
    } else {
        if (e0)
            hipExtLaunchKernelGGL((k_dual_update<NRHS, SP, 4, 16>), grid, block, 0, s, e0, e1, 0, d, gn, ncb,
                                  pl.nr_cap, rowpath, bytes_fixed(d));
        else
            hipLaunchKernelGGL((k_dual_update<NRHS, SP, 4, 16>), grid, block, 0, s, d, gn, ncb, pl.nr_cap, rowpath,
                               bytes_fixed(d));
    }
}

void dual_batch_end(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    (void)pl;
    hipLaunchKernelGGL(k_dual_finish, dim3(1), dim3(64), 0, s, d);
}

template <int NRHS, int FUSED, int AW>
static void launch_ftran(hipStream_t s, const SpxDev &d, const DualPlan &pl, int gn, int ncb)
{
    const int tiles_f = cdiv(d.m, 512);
    hipLaunchKernelGGL((k_dual_ftran<NRHS, FUSED, AW>), dim3(tiles_f * pl.fsplits), dim3(256), 0, s, d, tiles_f, gn,
                       pl.awsplits, ncb);
    hipLaunchKernelGGL((k_dual_ftran_reduce<NRHS, FUSED, AW>), dim3(cdiv(d.m, 64)), dim3(512), 0, s, d, pl.fsplits,
                       pl.awsplits);
}

void dual_iteration2(hipStream_t s, const SpxDev &d, const DualPlan &pl, hipEvent_t ev0, hipEvent_t ev1,
                     hipEvent_t ev2, hipEvent_t ev3)
{
    const int m = d.m, n = d.n;
    const int gv = cdiv(std::max(m, n), 256), gn = cdiv(n, 256), tiles_m = cdiv(m, 512);
    int ncb = 4 * gv;                                  // 64-slot groups of the pivot row
    if (pl.sparse) {
        // sparse factor (gk_sparse.hip): chuzr, BTRAN of e_p, the pivot row
        // as a CSC column pass, the ratio test (with update_gamma's A w over
        // the CSR rows), the pick and h = -N[q], the 2-RHS FTRAN (tcol, u),
        // the vector updates, then the Schur-complement update of the factor
        hipLaunchKernelGGL(k_dual_top, dim3(1), dim3(TOP_WG), 0, s, d, 3, 0);
        sp_pivot_btran(*d.sp, s, d.st, d.rho);
        if (ev0) (void)hipEventRecord(ev0, s);
        // (no max |trow| from the pass: k_trow_finish's group maxima give it,
        // and one atomic per block on a single word cost most of the pass)
        colpass_gated(s, d.A, CP_TROW, m, n, d.head, d.stat, d.coef, nullptr, d.rho, nullptr, d.trow, nullptr,
                      nullptr, d.st, 0);
        if (ev1) (void)hipEventRecord(ev1, s);
        hipLaunchKernelGGL(k_trow_finish, dim3(gv), dim3(256), 0, s, d, pl.pse, 0);
        hipLaunchKernelGGL(k_dual_ratio, dim3(gn + (pl.pse ? cdiv(m, 256) + d.A.nlr : 0)), dim3(256), 0, s, d, gn,
                           tiles_m, 0, ncb, 0, 0);
        hipLaunchKernelGGL(k_dual_pick, dim3(1), dim3(1024), 0, s, d, pl.pse, gn, ncb);
        sp_pivot_ftran(*d.sp, s, d.st, d.h, d.work, d.tcol, d.u, pl.pse);
        hipLaunchKernelGGL(k_dual_commit, dim3(gv), dim3(256), 0, s, d, pl.pse, gv, tiles_m, pl.lpsu, 3,
                           sp_pivot_bytes(d), 0);
        sp_pivot_update(*d.sp, s, d.st);
        return;
    }
    if (pl.colpath) {
        // sparse A: four kernels, as the dense row path
        if (ev0) (void)hipEventRecord(ev0, s);
        hipLaunchKernelGGL(k_dual_col, dim3(gv), dim3(256), 0, s, d, pl.pse, pl.nr_cap, pl.gm);
        if (ev1) (void)hipEventRecord(ev1, s);
        hipLaunchKernelGGL(k_dual_ratio, dim3(gn + (pl.pse ? cdiv(m, 256) + d.A.nlr : 0)), dim3(256), 0, s, d, gn,
                           tiles_m, 2, ncb, 0, prev_blocks(d, pl));
        if (pl.fupd) {
            if (pl.pse) launch_update<2, 1>(s, d, pl, gn, ncb, 2);
            else launch_update<1, 1>(s, d, pl, gn, ncb, 2);
            return;
        }
        // 16 rows per block (4 list slices per wave): 4x the blocks of the
        // dense layout for the small m of sparse problems
        if (pl.pse)
            hipLaunchKernelGGL((k_dual_ftran1<2, 1, 16>), dim3(cdiv(m, 16)), dim3(64 * pl.fwaves), 0, s, d, gn,
                               pl.awsplits, ncb, pl.nr_cap);
        else
            hipLaunchKernelGGL((k_dual_ftran1<1, 1, 16>), dim3(cdiv(m, 16)), dim3(64 * pl.fwaves), 0, s, d, gn,
                               pl.awsplits, ncb, pl.nr_cap);
        hipLaunchKernelGGL(k_dual_commit, dim3(gv + tiles_m * pl.uchunks), dim3(256), 0, s, d, pl.pse, gv, tiles_m,
                           pl.lpsu, 2, bytes_fixed(d), 0);
        return;
    }
    if (pl.rowpath) {
        // chuzr, rho and the pivot row in one kernel
        ncb = cdiv(std::max(m, n), 64);
        // (16 entries per wave in trips 1-2 measured slower on C3 — 11.6 against
        // 9.0 us of span, profiles/r04_trace_pivot_np16_reverted.txt — than 8
        // plus the dependent loop: k_dual_row<16> is kept for experiments)
        if (ev0)
            hipExtLaunchKernelGGL(k_dual_row<8>, dim3(ncb), dim3(64 * pl.twaves), 0, s, ev0, ev1, 0, d, pl.pse,
                                  pl.nr_cap, pl.gm);
        else
            hipLaunchKernelGGL(k_dual_row<8>, dim3(ncb), dim3(64 * pl.twaves), 0, s, d, pl.pse, pl.nr_cap, pl.gm);
    } else {
        const bool tgrid = !pl.rigorous && d.A.dense && m >= 1024;
        if (tgrid && pl.panel)
            hipLaunchKernelGGL(k_dual_top_grid<1>, dim3(cdiv(m, 256)), dim3(256), 0, s, d, pl.panel, pl.panel_age);
        else if (tgrid)
            hipLaunchKernelGGL(k_dual_top_grid<0>, dim3(cdiv(m, 256)), dim3(256), 0, s, d, 0, pl.panel_age);
        else
            hipLaunchKernelGGL(k_dual_top, dim3(1), dim3(TOP_WG), 0, s, d, pl.rowpath, pl.nr_cap);
        if (pl.rigorous) refine_rho_dev(s, d);
        if (ev0) (void)hipEventRecord(ev0, s);
        if (pl.panel)   // the row of p from the MFMA panel (gk_panel.hip)
            panel_trow(s, d, pl, tgrid);
        else if (d.shard && d.shard->vsize > 1)
            lp_shard_sim(s, d, pl.pse);
        else if (d.shard) {
            // this rank's slice of the non-basic positions, then the exchange
            const LpShard &sh = *d.shard;
            const int lo = std::min(n, sh.rank * sh.L), hi = std::min(n, lo + sh.L);
            colpass_gated(s, d.A, CP_TROW, m + lo, hi - lo, d.head, d.stat + lo, d.coef, nullptr, d.rho, nullptr,
                          d.trow + lo, nullptr, &d.st->trow_max_bits, d.st, 0);
            lp_shard_trow(s, d, pl.pse);
        } else
            colpass_gated(s, d.A, CP_TROW, m, n, d.head, d.stat, d.coef, nullptr, d.rho, nullptr, d.trow, nullptr,
                          nullptr, d.st, 0);
        if (ev1) (void)hipEventRecord(ev1, s);
        hipLaunchKernelGGL(k_trow_finish, dim3(gv), dim3(256), 0, s, d, pl.pse, (pl.panel ? 1 : 0) | (d.shard ? 2 : 0));
    }
    // (sharded: A w came with the exchange; k_trow_finish formed work)
    const int aw = (pl.pse && d.A.dense && !d.shard) ? 1 : 0;
    const int awone = (aw && pl.fused) ? pl.awone : 0;
    hipLaunchKernelGGL(k_dual_ratio, dim3(gn + (aw ? (awone ? cdiv(m, 64) : tiles_m * pl.awsplits) : 0)), dim3(256), 0,
                       s, d, gn, tiles_m, pl.rowpath, ncb, awone, prev_blocks(d, pl));
    if (pl.fupd) {
        if (pl.pse) launch_update<2, 0>(s, d, pl, gn, ncb, pl.rowpath, ev2, ev3);
        else launch_update<1, 0>(s, d, pl, gn, ncb, pl.rowpath, ev2, ev3);
        return;
    }
    if (pl.fused) {
        if (pl.fone) {
            if (pl.pse)
                hipLaunchKernelGGL((k_dual_ftran1<2, 0, 64>), dim3(cdiv(m, 64)), dim3(64 * pl.fwaves), 0, s, d, gn,
                                   pl.awsplits, ncb, pl.nr_cap);
            else
                hipLaunchKernelGGL((k_dual_ftran1<1, 0, 64>), dim3(cdiv(m, 64)), dim3(64 * pl.fwaves), 0, s, d, gn,
                                   pl.awsplits, ncb, pl.nr_cap);
        } else if (pl.pse)
            launch_ftran<2, 1, 1>(s, d, pl, gn, ncb);
        else
            launch_ftran<1, 1, 0>(s, d, pl, gn, ncb);
    } else {
        hipLaunchKernelGGL(k_dual_pick, dim3(1), dim3(1024), 0, s, d, pl.pse, gn, ncb);
        if (pl.pse) {
            if (aw) launch_ftran<2, 0, 1>(s, d, pl, gn, ncb);
            else {
                aprod_neg_gated(s, d.A, d.wcol, d.ys, d.work, d.partial, d.partial_cap, d.st, 0);   // work = ys - A w
                launch_ftran<2, 0, 0>(s, d, pl, gn, ncb);
            }
        } else
            launch_ftran<1, 0, 0>(s, d, pl, gn, ncb);
        if (pl.rigorous) refine_tcol_dev(s, d, 0);
    }
    const int nvb = gv;
    // (with the pricing panel: its rows t != pcur updated by extra blocks of
    // the commit, row pcur by panel_update after it)
    const int pfrom = pl.panel ? nvb + tiles_m * pl.uchunks : 0;
    const int pblocks = pl.panel ? cdiv(n, 256) * PANEL_MAX : 0;
    hipLaunchKernelGGL(k_dual_commit, dim3(nvb + tiles_m * pl.uchunks + pblocks), dim3(256), 0, s, d, pl.pse, nvb,
                       tiles_m, pl.lpsu, pl.rowpath, bytes_fixed(d), pfrom);
    if (pl.panel) panel_update(s, d, pl);
}

// ---------------------------------------------------------------------------
// inv(B) x and inv(B)' x on the structure of the inverse (dual path, where
// rlist is maintained): the nr dense columns plus the exact unit columns of
// the basic slacks.  Used by eval_beta / eval_pi between batches instead of
// passes over all m columns.
// ---------------------------------------------------------------------------
// y[i] = sum_t inv(B)[i, rlist[t]] x[rlist[t]] + (head[i] <= m ? x[head[i] - 1] : 0);
// 64 rows per block, its waves split the list, partials meet in wave order
static __host__ __device__ __forceinline__ int binv_list_waves(int nr) { return nr <= 32 ? 4 : (nr <= 128 ? 8 : 16); }

__global__ void __launch_bounds__(1024) k_binv_list(SpxDev d, int nr, const double *__restrict__ x,
                                                    double *__restrict__ y, const DState *eg, int accum)
{
    __shared__ double sp[16][64];
    const int m = d.m;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int nw = blockDim.x >> 6;
    if (eg) {
        // the epilogue's form: the list length of the finished batch, and the
        // waves the host would have launched for it (the same partial sums)
        if (eg->stop > ST_BATCH) return;
        nr = eg->nr;
        nw = binv_list_waves(nr);
    }
    const int r = blockIdx.x * 64 + lane;
    const bool act = r < m;
    const size_t ldb = (size_t)d.ldb;
    double acc = 0.0;
    int t = w < nw ? w : nr;
    for (; t + 3 * nw < nr; t += 4 * nw) {
        int c[4];
        double xv[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            c[u] = d.rlist[t + u * nw];
            xv[u] = x[c[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) bv[u] = (act && xv[u] != 0.0) ? d.Binv[(size_t)c[u] * ldb + r] : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += bv[u] * xv[u];
    }
    for (; t < nr; t += nw) {
        const int c = d.rlist[t];
        const double xv = x[c];
        if (act && xv != 0.0) acc += d.Binv[(size_t)c * ldb + r] * xv;
    }
    sp[w][lane] = acc;
    __syncthreads();
    if (w != 0 || !act) return;
    double v = 0.0;
    for (int k = 0; k < nw; ++k) v += sp[k][lane];
    const int kh = d.head[r];
    if (kh <= m) v += x[kh - 1];
    y[r] = accum ? y[r] + v : v;
}

// y[c] = inv(B)[:, c]' x: block t < nr — the dense column rlist[t]; the
// other blocks — the unit columns of the basic slacks (y[head[i] - 1] = x[i])
__global__ void __launch_bounds__(256) k_binvt_list(SpxDev d, int nr, const double *__restrict__ x,
                                                    double *__restrict__ y, const DState *eg)
{
    __shared__ double sh[4];
    const int m = d.m;
    int nrd = nr;                    // (eg: nr bounds the finished batch's list length)
    if (eg) {
        if (eg->stop > ST_BATCH) return;
        nrd = eg->nr;
    }
    if ((int)blockIdx.x < nr) {
        if ((int)blockIdx.x >= nrd) return;
        const int c = d.rlist[blockIdx.x];
        const double *col = d.Binv + (size_t)c * d.ldb;
        double acc = 0.0;
        int r = threadIdx.x * 2;
        for (; r + 1 < m; r += 512) {
            const double2 v = *(const double2 *)(col + r);
            acc += v.x * x[r];
            acc += v.y * x[r + 1];
        }
        if (r < m) acc += col[r] * x[r];
        acc = wsum(acc);
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) y[c] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
        return;
    }
    const int i = (blockIdx.x - nr) * 256 + threadIdx.x;
    if (i < m) {
        const int k = d.head[i];
        if (k <= m) y[k - 1] = x[i];
    }
}

void binv_ftran_list(hipStream_t s, const SpxDev &d, int nr, const double *x, double *y, const DState *eg, int acc)
{
    const int nw = eg ? 16 : binv_list_waves(nr);
    hipLaunchKernelGGL(k_binv_list, dim3(cdiv(d.m, 64)), dim3(64 * nw), 0, s, d, nr, x, y, eg, acc);
}

// ---------------------------------------------------------------------------
// eval_pi's residual and eval_cbar (glpspx02.js:426-495, glpspx01.js:514-584)
// by rows of AT, dense A: pi = inv(B)' cB vanishes outside the dense columns
// of inv(B) and the basic slacks c with a nonzero cost (pi_c = cB[bind[c]]:
// none in the dual, the primal's phase-I costs), so N_k' pi runs over those
// rows of AT (rlist, then `extra`) instead of all m rows of A.
// Block b owns the 64 variable slots [64 b, 64 b + 64) (structural column c
// and slack row c); waves split the list rows, partial sums meet in LDS.
//   CP_CBAR:  out[j] = coef[k] - N_k' pi for the non-basic position j of k
//   CP_RESID: out[i] = h[i]   - N_k' pi for the basic position i of k
// ---------------------------------------------------------------------------
static __host__ __device__ __forceinline__ int rowpass_waves(int cnt) { return cnt <= 64 ? 4 : (cnt <= 256 ? 8 : 16); }

__global__ void __launch_bounds__(1024) k_rowpass_pi(SpxDev d, int mode, int nr, const double *__restrict__ pi,
                                                     const double *__restrict__ h, double *__restrict__ out,
                                                     const int *__restrict__ extra, int nextra, const DState *eg,
                                                     const double *__restrict__ pi2)
{
    // (pi2: the multipliers are pi + pi2, eval_pi's refinement step taken
    // here instead of by an axpy)
    auto PI = [&](int c) { return pi2 ? pi[c] + pi2[c] : pi[c]; };
    __shared__ double sp[16][64];
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    int nw = blockDim.x >> 6;
    if (eg) {                        // (as k_binv_list)
        if (eg->stop > ST_BATCH) return;
        nr = eg->nr;
        nw = rowpass_waves(nr + nextra);
    }
    const int idx = blockIdx.x * 64 + lane;
    const double *__restrict__ col = d.A.AT + min(idx, n - 1);
    const size_t ldt = (size_t)d.A.ldt;
    double acc = 0.0;
    int t = w < nw ? w : nr;
    for (; t + 3 * nw < nr; t += 4 * nw) {
        int c[4];
        double v[4], a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = d.rlist[t + u * nw];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            v[u] = PI(c[u]);
            a[u] = col[(size_t)c[u] * ldt];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u] * a[u];
    }
    for (; t < nr; t += nw) {
        const int c = d.rlist[t];
        acc += PI(c) * col[(size_t)c * ldt];
    }
    for (t = w < nw ? w : nextra; t < nextra; t += nw) {        // basic slacks with a cost (primal phase I)
        const int c = extra[t];
        acc += PI(c) * col[(size_t)c * ldt];
    }
    sp[w][lane] = acc;
    __syncthreads();
    if (w != 0) return;
    double dot = 0.0;
    for (int k = 0; k < nw; ++k) dot += sp[k][lane];
    if (idx < n) {
        const int pos = d.bind[m + idx];
        if (mode == CP_CBAR && pos > m) out[pos - m - 1] = d.coef[m + idx] + dot;
        if (mode == CP_RESID && pos <= m) out[pos - 1] = h[pos - 1] + dot;
    }
    if (idx < m) {
        const int pos = d.bind[idx];
        if (mode == CP_CBAR && pos > m) out[pos - m - 1] = d.coef[idx] - PI(idx);
        if (mode == CP_RESID && pos <= m) out[pos - 1] = h[pos - 1] - PI(idx);
    }
}

void rowpass_pi(hipStream_t s, const SpxDev &d, int mode, int nr, const double *pi, const double *h, double *out,
                const int *extra, int nextra, const DState *eg, const double *pi2)
{
    const int nw = eg ? 16 : rowpass_waves(nr + nextra);
    hipLaunchKernelGGL(k_rowpass_pi, dim3(cdiv(std::max(d.m, d.n), 64)), dim3(64 * nw), 0, s, d, mode, nr, pi, h,
                       out, extra, nextra, eg, pi2);
}

void binv_btran_list(hipStream_t s, const SpxDev &d, int nr, const double *x, double *y, const DState *eg)
{
    hipLaunchKernelGGL(k_binvt_list, dim3(nr + cdiv(d.m, 256)), dim3(256), 0, s, d, nr, x, y, eg);
}

// AT[r*ldt + c] = A[c*lda + r], 64 x 64 tiles through LDS
__global__ void __launch_bounds__(256) k_transpose(const double *__restrict__ A, int m, int n, int lda,
                                                     double *__restrict__ AT, int ldt)
{
    __shared__ double tile[64][65];
    const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int cc = ty; cc < 64; cc += 4) {
        const int r = r0 + tx, c = c0 + cc;
        tile[cc][tx] = (r < m && c < n) ? A[(size_t)c * lda + r] : 0.0;
    }
    __syncthreads();
    for (int rr = ty; rr < 64; rr += 4) {
        const int r = r0 + rr, c = c0 + tx;
        if (r < m && c < ldt) AT[(size_t)r * ldt + c] = (c < n) ? tile[tx][rr] : 0.0;
    }
}

void transpose_dense(hipStream_t s, const double *A, int m, int n, int lda, double *AT, int ldt)
{
    dim3 g(cdiv(m, 64), cdiv(ldt, 64));
    hipLaunchKernelGGL(k_transpose, g, dim3(256), 0, s, A, m, n, lda, AT, ldt);
}

}  // namespace gk
