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
#include <algorithm>

namespace gk {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__device__ __forceinline__ int gv_of(int m, int n) { return (max(m, n) + 255) / 256; }
__device__ __forceinline__ Cand *cand_chuzr(const SpxDev &d) { return (Cand *)d.cand; }
// per-block outputs: chuzr candidates [gv); pass-1 candidates of the pivot-row
// blocks [4 gv) (64-slot blocks of k_trow_rows, or 256-slot blocks of
// k_trow_finish); pass-2 candidates [gv).  gpart: gamma_p sums [4 gv), then
// max |trow| [4 gv) of the same blocks.
__device__ __forceinline__ Cand *cand_pass1(const SpxDev &d) { return (Cand *)d.cand + gv_of(d.m, d.n); }
__device__ __forceinline__ Cand *cand_pass2(const SpxDev &d) { return (Cand *)d.cand + 5 * gv_of(d.m, d.n); }
__device__ __forceinline__ double *tmax_part(const SpxDev &d) { return d.gpart + 4 * gv_of(d.m, d.n); }
__device__ __forceinline__ Cand no_cand(double k1)
{
    Cand c; c.k1 = k1; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    return c;
}

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

__device__ __forceinline__ RatioCtx ratio_ctx(const DState *st, double big)
{
    RatioCtx x;
    x.eps = st->tol_bnd * (1.0 + 0.01 * big);     // sort_trow with tol_bnd (:1851)
    x.s = (st->delta > 0.0 ? +1.0 : -1.0);
    x.rtol = (st->rtest == RT_HAR) ? 0.30 * st->tol_dj : 0.0;
    return x;
}

__device__ __forceinline__ double trow_big(const DState *st)
{
    return __longlong_as_double((long long)st->trow_max_bits);
}

__device__ __forceinline__ bool pass1_cand(const RatioCtx &x, double tr, double cb, int sj, int j, Cand &e)
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
    e.k1 = t; e.k2 = fabs(alfa); e.idx = j + 1; e.aux = 0;
    return true;
}

__device__ __forceinline__ bool pass2_cand(const RatioCtx &x, double tr, double cb, int sj, int j, double tmax, Cand &e)
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
    e.k1 = t; e.k2 = fabs(alfa); e.idx = j + 1; e.aux = 0;
    return true;
}

// pass-1 candidate of the non-basic variable(s) handled by thread slot idx
// of k_trow_finish (structural column idx and slack row idx)
__device__ __forceinline__ Cand pass1_slot(const SpxDev &d, const RatioCtx &x, int idx)
{
    const int m = d.m, n = d.n;
    Cand best = no_cand(DBL_MAX);
    if (idx < n) {
        const int pos = d.bind[m + idx];
        if (pos > m) {
            const int j = pos - m - 1;
            Cand e;
            if (pass1_cand(x, d.trow[j], d.cbar[j], d.stat[j], j, e) && better<1>(e, best)) best = e;
        }
    }
    if (idx < m) {
        const int pos = d.bind[idx];
        if (pos > m) {
            const int j = pos - m - 1;
            Cand e;
            if (pass1_cand(x, d.trow[j], d.cbar[j], d.stat[j], j, e) && better<1>(e, best)) best = e;
        }
    }
    return best;
}

// ---------------------------------------------------------------------------
// change_basis (glpspx02.js:1954-1964) of the committed pivot, plus the lists
// of dense inv(B) columns and of reference-space non-basic structurals.
// Called by a whole block (>= 4 threads); four threads do independent parts.
// ---------------------------------------------------------------------------
__device__ void dual_finish_block(const SpxDev &d, int rowpath, double bytes_fixed)
{
    DState *st = d.st;
    const int pend = st->pend;
    const int role = threadIdx.x;
    const int m = d.m, n = d.n;
    int p = 0, q = 0, kp = 0, kq = 0, nr0 = 0, nwl0 = 0, ns = 0, tkp = 0, refkp = 0, wq = -1, rq = -1;
    if (pend && role < 4) {
        p = st->p; q = st->q;
        kp = d.head[p - 1];
        kq = d.head[m + q - 1];
        nr0 = st->nr; nwl0 = st->nwl; ns = st->ns;
        tkp = d.type[kp - 1];
        refkp = d.refsp[kp - 1];
        if (kq > m) wq = d.wpos[kq - m - 1];
        if (kq <= m) rq = d.rpos[kq - 1];
    }
    __syncthreads();
    if (pend && role == 0) {
        d.head[p - 1] = kq;
        d.head[m + q - 1] = kp;
        d.bind[kq - 1] = p;
        d.bind[kp - 1] = m + q;
        if (tkp == FX) d.stat[q - 1] = NS;
        else if (st->delta > 0.0) d.stat[q - 1] = NL;
        else d.stat[q - 1] = NU;
    } else if (pend && role == 1) {
        int nr = nr0;
        if (kq <= m) {           // entering slack: its column is now e_p
            const int last = d.rlist[nr - 1];
            d.rlist[rq] = last;
            d.rpos[last] = rq;
            d.rpos[kq - 1] = -1;
            nr--;
        }
        if (kp <= m) {           // leaving slack: its column became dense
            d.rlist[nr] = kp - 1;
            d.rpos[kp - 1] = nr;
            nr++;
        }
        st->nr = nr;
    } else if (pend && role == 2 && st->pricing == PT_PSE) {
        if (tkp == FX && refkp) {
            d.refsp[kp - 1] = 0;
            refkp = 0;
        }
        int nwl = nwl0;
        if (wq >= 0) {
            const int last = d.wlist[nwl - 1];
            d.wlist[wq] = last;
            d.wpos[last] = wq;
            d.wpos[kq - m - 1] = -1;
            nwl--;
        }
        if (kp > m && refkp) {
            d.wlist[nwl] = kp - m - 1;
            d.wpos[kp - m - 1] = nwl;
            nwl++;
        }
        st->nwl = nwl;
        if (st->refct > 0) st->refct--;
    } else if (pend && role == 3) {
        if (st->phase == 2) st->obj += (st->cbar_q_old / st->zeta) * (st->delta / st->pivot);
        st->upd_cnt++;
        st->binv_fresh = 0;
        st->cbar_fresh = 0;
        if (st->upd_cnt >= st->upd_lim) st->refact_pending = 1;
        st->it_cnt++;
        st->npiv++;
        st->iter_left--;
        if (st->rigorous > 0) st->rigorous--;
        st->pend = 0;
        // algorithmic HBM bytes of this pivot: the pivot row (rows of A in the
        // support of rho, or all of A), A w over the reference-space columns,
        // inv(B) once for both right-hand sides, read + write of the updated
        // columns, and the O(m + n) vectors
        const double rowb = rowpath ? 8.0 * (double)ns * n : 8.0 * (double)m * n;
        if (rowpath && st->tk_end > st->tk_start) {
            st->bytes_trow += rowb;
            st->trow_ticks += (double)(st->tk_end - st->tk_start);
            st->trow_ticks_b += (double)(st->tk_next - st->tk_start);
            st->trow_n += 1.0;
        }
        st->tk_end = 0;
        st->bytes += rowb + 8.0 * (double)m * nwl0 + 8.0 * (double)m * (nr0 + 1) +
                     16.0 * (double)m * (nr0 + (kp <= m ? 1 : 0)) + bytes_fixed;
    }
    __syncthreads();
}

__global__ void k_dual_finish(SpxDev d, int rowpath, double bytes_fixed)
{
    dual_finish_block(d, rowpath, bytes_fixed);
}

// chuzr candidate of basic position i (glpspx02.js:572-626)
__device__ __forceinline__ Cand chuzr_cand_v(int i, int t, double lb, double ub, double bb, double g, double tol_bnd)
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
    if (temp > 0.0) { e.k1 = temp; e.k2 = ri; e.idx = i + 1; }
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

// batch start: chuzr candidates and the phase-I check of the current state
__global__ void __launch_bounds__(256) k_dual_prep(SpxDev d)
{
    __shared__ Cand shc[16];
    DState *st = d.st;
    const int m = d.m, n = d.n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool reset = (st->pricing == PT_PSE && st->refct == 0);
    if ((int)blockIdx.x * 256 < m) {
        Cand c = no_cand(0.0);
        if (i < m) {
            const int k = d.head[i];
            c = chuzr_cand_v(i, d.type[k - 1], d.lb[k - 1], d.ub[k - 1], d.bbar[i], reset ? 1.0 : d.gamma[i],
                             st->tol_bnd);
        }
        const Cand b = block_best<0>(c, shc);
        if (threadIdx.x == 0) cand_chuzr(d)[blockIdx.x] = b;
    }
    if (st->phase == 1) {
        const int bad = (i < n) ? dual_bad(d, d.head[m + i], d.cbar[i], st->tol_dj) : 0;
        if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
    }
}

// ---------------------------------------------------------------------------
// k_dual_top
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(WG) k_dual_top(SpxDev d, int rowpath, double bytes_fixed)
{
    __shared__ Cand shc[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    // the next pivot's chuzr candidates are already final: load them while
    // the previous pivot's change_basis is applied
    const int gm = (m + 255) / 256;
    Cand c = no_cand(0.0);
    for (int b = threadIdx.x; b < gm; b += blockDim.x) {
        const Cand e = cand_chuzr(d)[b];
        if (better<0>(e, c)) c = e;
    }
    dual_finish_block(d, rowpath, bytes_fixed);
    if (st->iter_left <= 0 || st->refact_pending) {
        __syncthreads();
        if (threadIdx.x == 0) st->stop = st->refact_pending ? ST_REFACT : ST_BATCH;
        return;
    }
    if (st->pricing == PT_PSE && st->refct == 0) {
        reset_refsp_dev(d, 1);             // refsp := basic variables, gamma := 1
        for (int l = threadIdx.x; l < n; l += blockDim.x) d.wpos[l] = -1;
        if (threadIdx.x == 0) st->nwl = 0;
        __syncthreads();
    }
    if (st->phase == 1) {
        if (!st->dinf) {
            __syncthreads();
            if (threadIdx.x == 0) st->stop = ST_PHASE;
            return;
        }
    } else {
        // objective limits (:1729-1760)
        const double z = st->zeta, obj = st->obj;
        const bool hit = (z < 0.0 && st->obj_ll > -DBL_MAX && obj <= st->obj_ll) ||
                         (z > 0.0 && st->obj_ul < +DBL_MAX && obj >= st->obj_ul);
        if (hit) {
            __syncthreads();
            if (threadIdx.x == 0) st->stop = ST_OBJLIM;
            return;
        }
    }
    // chuzr from the per-block candidates
    const Cand best = block_best<0>(c, shc);
    if (best.idx == 0) {
        if (threadIdx.x == 0) { st->p = 0; st->stop = ST_P0; }
        return;
    }
    const int p = best.idx;
    // rho in compact form; the dense copy only for the column pass
    if (!rowpath) {
        for (int l = threadIdx.x; l < m; l += blockDim.x) d.rho[l] = 0.0;
        __syncthreads();
    }
    const int nr = st->nr;
    for (int t = threadIdx.x; t < nr; t += blockDim.x) {
        const int cc = d.rlist[t];
        const double v = d.Binv[(size_t)(p - 1) + (size_t)cc * d.ldb];
        if (!rowpath) d.rho[cc] = v;
        d.rho_idx[t] = cc;
        d.rho_val[t] = v;
    }
    if (threadIdx.x == 0) {
        const int kp = d.head[p - 1];
        int ns = nr;
        if (kp <= m) {   // the basic slack at position p: unit column of inv(B)
            if (!rowpath) d.rho[kp - 1] = 1.0;
            d.rho_idx[nr] = kp - 1;
            d.rho_val[nr] = 1.0;
            ns++;
        }
        st->p = p;
        st->delta = best.k2;
        st->trow_max_bits = 0ull;
        st->ns = ns;
        st->dinf = 0;
    }
}

// ---------------------------------------------------------------------------
// k_trow_finish: structural column c / slack row c of the pivot row.
// FROM_PART: trow from the row-path partials (structurals) and -rho (slacks);
// else trow was written by the column pass.  Also the PSE vectors of
// update_gamma (:1103-1134): wcol[c] / ys[c] = trow of a non-basic variable of
// the reference space, per-block sums of those trow^2 (gamma_p), and the
// block's Harris pass-1 candidate under the block-local significance
// tolerance (k_dual_ratio re-checks it against the global one).
// ---------------------------------------------------------------------------
template <int FROM_PART>
__global__ void __launch_bounds__(256) k_trow_finish(SpxDev d, const double *__restrict__ part, int splits, int pse,
                                                       int nslots)
{
    __shared__ double shd[16];
    __shared__ Cand shc[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (FROM_PART && blockIdx.x == 0) {
        // end of the pivot-row kernel: latest block stamp (one block, plain
        // store: same-address atomics from every block serialise)
        if (threadIdx.x == 0) st->tk_next = wall_clock64();
        unsigned long long e = 0;
        for (int t = threadIdx.x; t < nslots; t += blockDim.x) e = max(e, d.tslots[t]);
        __shared__ unsigned long long she;
        if (threadIdx.x == 0) she = 0;
        __syncthreads();
        if (e) atomicMax(&she, e);
        __syncthreads();
        if (threadIdx.x == 0 && she) st->tk_end = she;
    }
    // all gathers first (bind -> stat/cbar/refsp/partials), reductions after
    const int pos1 = (idx < n) ? d.bind[m + idx] : 0;
    const int pos2 = (idx < m) ? d.bind[idx] : 0;
    const int rp2 = (FROM_PART && idx < m) ? d.rpos[idx] : -1;   // a non-basic slack is a dense column of inv(B)
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    int s1 = 0, s2 = 0;
    double cb1 = 0.0, cb2 = 0.0, tv1 = 0.0, tv2 = 0.0;
    bool ref1 = false, ref2 = false;
    if (j1 >= 0) {
        s1 = d.stat[j1];
        cb1 = d.cbar[j1];
        if (FROM_PART) {
            double acc = 0.0;
#pragma unroll 8
            for (int s = 0; s < splits; ++s) acc += part[(size_t)s * n + idx];
            tv1 = acc;
        } else
            tv1 = d.trow[j1];
        if (pse) ref1 = d.refsp[m + idx] != 0;
    }
    if (j2 >= 0) {
        s2 = d.stat[j2];
        cb2 = d.cbar[j2];
        tv2 = FROM_PART ? -d.rho_val[rp2] : d.trow[j2];
        if (pse) ref2 = d.refsp[idx] != 0;
    }
    if (FROM_PART) {
        if (s1 == NS) tv1 = 0.0;
        if (s2 == NS) tv2 = 0.0;
        if (j1 >= 0) d.trow[j1] = tv1;
        if (j2 >= 0) d.trow[j2] = tv2;
    }
    double gsum = 0.0;
    if (pse) {
        const double w1 = ref1 ? tv1 : 0.0, w2 = ref2 ? tv2 : 0.0;
        if (idx < n) d.wcol[idx] = w1;
        if (idx < m) d.ys[idx] = w2;
        gsum = w1 * w1 + w2 * w2;
    }
    const double bmax = block_max(fmax(fabs(tv1), fabs(tv2)), shd);
    // per-block max |trow|; k_dual_ratio reduces them into st->trow_max_bits
    if (FROM_PART && threadIdx.x == 0) tmax_part(d)[blockIdx.x] = bmax;
    if (pse) {
        const double g = block_sum(gsum, shd);
        if (threadIdx.x == 0) d.gpart[blockIdx.x] = g;
    }
    // pass-1 candidate with eps_b = tol_bnd (1 + 0.01 max_b) <= eps
    const RatioCtx x = ratio_ctx(st, bmax);
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (j1 >= 0 && pass1_cand(x, tv1, cb1, s1, j1, e) && better<1>(e, c)) c = e;
    if (j2 >= 0 && pass1_cand(x, tv2, cb2, s2, j2, e) && better<1>(e, c)) c = e;
    const Cand b = block_best<1>(c, shc);
    if (threadIdx.x == 0) cand_pass1(d)[blockIdx.x] = b;
}

// ---------------------------------------------------------------------------
// k_trow_rows (row path, dense A): the pivot row and the work of
// k_trow_finish in one kernel.  Block b owns the 64 slots [64 b, 64 b + 64)
// (structural column c and slack row c of each slot).  Its waves split the
// support of rho (rows t = w, w + nw, ... of AT, 512-byte coalesced segments
// of the 64 columns), the partial sums meet in LDS in wave order, and wave 0
// finishes the slots with wave-level reductions: trow, the PSE vectors, the
// gamma_p partial, max |trow| and the Harris pass-1 candidate of the block.
// Block 0 stamps the device clock at entry and every block at exit (tslots).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_trow_rows(SpxDev d, int pse)
{
    __shared__ double sp[16][64];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nw = blockDim.x >> 6;
    const int idx = blockIdx.x * 64 + lane;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->tk_start = wall_clock64();
    // wave 0 gathers its slot operands first; their latency overlaps the rows
    int pos1 = 0, pos2 = 0, rp2 = -1;
    if (w == 0) {
        pos1 = (idx < n) ? d.bind[m + idx] : 0;
        pos2 = (idx < m) ? d.bind[idx] : 0;
        rp2 = (idx < m) ? d.rpos[idx] : -1;
    }
    const int ns = st->ns;
    double acc = 0.0;
    if (idx < n) {
        const double *__restrict__ col = d.A.AT + idx;
        const size_t ldt = (size_t)d.A.ldt;
        const int *__restrict__ ri = d.rho_idx;
        const double *__restrict__ rv = d.rho_val;
        int t = w;
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
    sp[w][lane] = acc;
    __syncthreads();
    if (w != 0) return;                      // wave 0 only from here: no block barriers
    double tsum = 0.0;
    for (int k = 0; k < nw; ++k) tsum += sp[k][lane];
    const int j1 = (pos1 > m) ? pos1 - m - 1 : -1;
    const int j2 = (pos2 > m) ? pos2 - m - 1 : -1;
    int s1 = 0, s2 = 0;
    double cb1 = 0.0, cb2 = 0.0, tv1 = 0.0, tv2 = 0.0;
    bool ref1 = false, ref2 = false;
    if (j1 >= 0) {
        s1 = d.stat[j1];
        cb1 = d.cbar[j1];
        tv1 = tsum;
        if (pse) ref1 = d.refsp[m + idx] != 0;
    }
    if (j2 >= 0) {
        s2 = d.stat[j2];
        cb2 = d.cbar[j2];
        tv2 = -d.rho_val[rp2];               // a non-basic slack is a dense column of inv(B)
        if (pse) ref2 = d.refsp[idx] != 0;
    }
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
    // pass-1 candidate with eps_b = tol_bnd (1 + 0.01 max_b) <= eps
    const RatioCtx x = ratio_ctx(st, bmax);
    Cand c = no_cand(DBL_MAX);
    Cand e;
    if (j1 >= 0 && pass1_cand(x, tv1, cb1, s1, j1, e) && better<1>(e, c)) c = e;
    if (j2 >= 0 && pass1_cand(x, tv2, cb2, s2, j2, e) && better<1>(e, c)) c = e;
    const Cand b = wave_best<1>(c);
    if (lane == 0) {
        tmax_part(d)[blockIdx.x] = bmax;
        if (pse) d.gpart[blockIdx.x] = g;
        cand_pass1(d)[blockIdx.x] = b;
        d.tslots[blockIdx.x] = wall_clock64();
    }
}

// ---------------------------------------------------------------------------
// k_dual_ratio: blocks [0, gn) — pass-1 choice from the block candidates
// (a block whose candidate fails the global significance tolerance is
// rescanned), then the pass-2 candidates of positions [256 b, 256 b + 256);
// blocks [gn, ...) — partials of A w over the reference-space columns.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dual_ratio(SpxDev d, int gn, int tiles_m, int rowpath, int ncb, int slotw)
{
    __shared__ Cand shc[16];
    __shared__ double shd[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    if ((int)blockIdx.x >= gn) {
        const int b = blockIdx.x - gn;
        const int tile = b % tiles_m, split = b / tiles_m, splits = (gridDim.x - gn) / tiles_m;
        const int cnt = st->nwl;
        const int lps = (cnt + splits - 1) / splits;
        const int t0 = split * lps, t1 = min(cnt, t0 + lps);
        const int r = (tile * 256 + threadIdx.x) * 2;
        const double *wc = d.wcol;
        lgemv_tile<1>(d.A.A, (size_t)d.A.lda, m, d.wlist, t0, t1, r,
                      [&](int, int c, double &xa, double &xb) { xa = wc[c]; xb = 0.0; },
                      d.awpart + (size_t)split * m);
        return;
    }
    double big;
    if (rowpath) {
        // max |trow| from the pivot-row blocks; block 0 publishes it and the
        // end of the pivot-row kernel (latest block exit stamp)
        double v = 0.0;
        unsigned long long e = 0;
        for (int b = threadIdx.x; b < ncb; b += blockDim.x) {
            v = fmax(v, tmax_part(d)[b]);
            if (blockIdx.x == 0) e = max(e, d.tslots[b]);
        }
        big = block_max(v, shd);
        if (blockIdx.x == 0) {
            __shared__ unsigned long long she;
            if (threadIdx.x == 0) {
                she = 0;
                st->tk_next = wall_clock64();
            }
            __syncthreads();
            if (e) atomicMax(&she, e);
            __syncthreads();
            if (threadIdx.x == 0) {
                st->trow_max_bits = dbits(big);
                st->tk_end = she;
            }
        }
    } else
        big = trow_big(st);
    const RatioCtx x = ratio_ctx(st, big);
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const double trj = (j < n) ? d.trow[j] : 0.0;
    const double cbj = (j < n) ? d.cbar[j] : 0.0;
    const int sj = (j < n) ? d.stat[j] : 0;
    Cand c = no_cand(DBL_MAX);
    int fail = 0;
    for (int b = threadIdx.x; b < ncb; b += blockDim.x) {
        const Cand e = cand_pass1(d)[b];
        if (e.idx != 0 && e.k2 < x.eps) fail = 1;
        else if (better<1>(e, c)) c = e;
    }
    if (__syncthreads_or(fail)) {
        // rare: rescan the blocks whose candidate is not significant
        for (int b = 0; b < ncb; ++b) {
            const Cand e = cand_pass1(d)[b];
            if (!(e.idx != 0 && e.k2 < x.eps)) continue;
            if ((int)threadIdx.x < slotw) {
                const Cand f = pass1_slot(d, x, b * slotw + threadIdx.x);
                if (better<1>(f, c)) c = f;
            }
        }
    }
    const Cand b1 = block_best<1>(c, shc);
    const int q1 = b1.idx;
    const double teta1 = q1 ? b1.k1 : DBL_MAX;
    const int need2 = !(x.rtol == 0.0 || q1 == 0 || teta1 == 0.0);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->q1 = q1;
        st->teta1 = teta1;
        st->need2 = need2;
    }
    if (!need2) return;
    Cand c2 = no_cand(0.0);
    if (j < n) {
        Cand e;
        if (pass2_cand(x, trj, cbj, sj, j, teta1, e)) c2 = e;
    }
    const Cand b2 = block_best<2>(c2, shc);
    if (threadIdx.x == 0) cand_pass2(d)[blockIdx.x] = b2;
}

// the entering choice q (pass 2 if needed), its checks and the st fields;
// every block of the calling grid evaluates it identically.  Returns q, or 0
// when the iteration stops.
__device__ int dual_pick(const SpxDev &d, Cand *shc, double *shd, int pse, int gn, int ncb)
{
    DState *st = d.st;
    int q;
    double teta;
    if (st->need2) {
        Cand c = no_cand(0.0);
        for (int b = threadIdx.x; b < gn; b += blockDim.x) {
            const Cand e = cand_pass2(d)[b];
            if (better<2>(e, c)) c = e;
        }
        const Cand b2 = block_best<2>(c, shc);
        q = b2.idx;
        teta = b2.k1;
    } else {
        q = st->q1;
        teta = st->teta1;
    }
    const bool lead = (blockIdx.x == 0 && blockIdx.y == 0);
    if (q == 0) {
        __syncthreads();
        if (lead && threadIdx.x == 0) { st->q = 0; st->stop = ST_Q0; }
        return 0;
    }
    const double big = trow_big(st);
    const double piv = d.trow[q - 1];
    if (fabs(piv) < 1e-5 * (1.0 + 0.01 * big) && !st->rigorous) {
        __syncthreads();
        if (lead && threadIdx.x == 0) { st->q = q; st->stop = ST_SMALLPIV; }
        return 0;
    }
    if (lead) {
        if (pse) {
            // gamma_p (update_gamma :1103-1132) from the per-block sums, fixed order
            double g = 0.0;
            for (int b = threadIdx.x; b < ncb; b += blockDim.x) g += d.gpart[b];
            g = block_sum(g, shd);
            if (threadIdx.x == 0) {
                const double eta = d.refsp[d.head[st->p - 1] - 1] ? 1.0 : 0.0;
                st->eta_pq = eta;
                st->gamma_pq = eta + g;
            }
        }
        if (threadIdx.x == 0) {
            st->q = q;
            st->new_dq = (st->delta > 0.0 ? +1.0 : -1.0) * teta;
            st->cbar_q_old = d.cbar[q - 1];
        }
    }
    return q;
}

// sparse A / rigorous mode: the pick and h = -N[q] in one workgroup
__global__ void __launch_bounds__(1024) k_dual_pick(SpxDev d, int pse, int gn, int ncb)
{
    __shared__ Cand shc[16];
    __shared__ double shd[16];
    if (d.st->stop) return;
    const int q = dual_pick(d, shc, shd, pse, gn, ncb);
    if (q) build_hq(d, q);
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
// k_dual_ftran: tcol = inv(B) h, u = inv(B) work over the dense columns.
// FUSED (dense A): the pick runs here and h_c = A[c, q] is read from A.
// AW: work from the A w partials (dense A), else from d.work.
// ---------------------------------------------------------------------------
template <int NRHS, int FUSED, int AW>
__global__ void __launch_bounds__(256) k_dual_ftran(SpxDev d, int tiles, int gn, int awsplits, int ncb)
{
    __shared__ Cand shc[16];
    __shared__ double shd[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m;
    int q;
    if (FUSED) {
        q = dual_pick(d, shc, shd, NRHS == 2, gn, ncb);
        if (!q) return;
    } else
        q = st->q;
    const int kq = d.head[m + q - 1];
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
                         if (NRHS == 2) xb = AW ? aw_value(d, c, awsplits) : work[c];
                         else xb = 0.0;
                     },
                     d.partial + (size_t)split * NRHS * m);
}

// tcol[i] / u[i] = sum of the partials + the unit column of a basic slack
// at position i; 64 rows per block, 8 waves over the splits in fixed order
template <int NRHS, int FUSED, int AW>
__global__ void __launch_bounds__(512) k_dual_ftran_reduce(SpxDev d, int splits, int awsplits)
{
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
            const int kq = d.head[m + st->q - 1];
            va += (kq > m) ? d.A.A[(size_t)(kq - m - 1) * d.A.lda + c] : (c == kq - 1 ? -1.0 : 0.0);
        } else
            va += d.h[c];
        if (NRHS == 2) vb += AW ? aw_value(d, c, awsplits) : d.work[c];
    }
    d.tcol[r] = va;
    if (NRHS == 2) d.u[r] = vb;
}

// ---------------------------------------------------------------------------
// k_dual_commit: pivot check (:1913-1933), update_bbar (:1042), update_cbar
// (:1020), update_gamma (:1075-1134) in the first `nvb` blocks, together with
// the chuzr candidates and the phase-I check of the next iteration; the
// rank-1 update of the dense columns of inv(B) in the others (row p :=
// rho / alpha_p, row i -= alpha_i / alpha_p rho).  A slack leaving the basis
// turns its unit column dense (virtual list entry nr, rho = 1); a slack
// entering turns its column into exactly e_p.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dual_commit(SpxDev d, int pse, int nvb, int tiles)
{
    __shared__ Cand shc[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n, p = st->p, q = st->q;
    const double piv1 = d.tcol[p - 1], piv2 = d.trow[q - 1];
    const bool bad = fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) ||
                     !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0));
    if (bad && (!st->binv_fresh || !st->rigorous)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) st->stop = ST_PIVCHK;
        return;
    }
    const double tp = bad ? piv2 : piv1;
    const double delta = st->delta;
    const int kq = d.head[m + q - 1];
    const int kp = d.head[p - 1];
    if ((int)blockIdx.x < nvb) {
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        // gathers first: the row / column operands and what the next
        // iteration's chuzr and check_feas read
        const bool in_m = i < m, in_n = i < n;
        const int kold = in_m ? d.head[i] : 1;
        const int knew = (i == p - 1) ? kq : kold;
        double bb = in_m ? d.bbar[i] : 0.0;
        const double ti = in_m ? d.tcol[i] : 0.0;
        double g = in_m ? d.gamma[i] : 0.0;
        const double ui = (pse && in_m) ? d.u[i] : 0.0;
        const int tkold = in_m ? d.type[kold - 1] : 0;
        const bool refk = (pse && in_m) ? d.refsp[kold - 1] != 0 : false;
        const int tknew = in_m ? d.type[knew - 1] : 0;
        const double lbn = in_m ? d.lb[knew - 1] : 0.0, ubn = in_m ? d.ub[knew - 1] : 0.0;
        double cb = in_n ? d.cbar[i] : 0.0;
        const double tri = in_n ? d.trow[i] : 0.0;
        const int kn = in_n ? ((i == q - 1) ? kp : d.head[m + i]) : 1;
        const int ot = (st->phase == 1 && in_n) ? d.orig_type[kn - 1] : 0;
        const double teta = delta / tp;
        const double new_dq = st->new_dq;
        if (in_m) {
            if (i == p - 1) bb = get_xN(d.stat, d.lb, d.ub, kq, q) + teta;
            else if (teta != 0.0) bb += ti * teta;
            d.bbar[i] = bb;
        }
        if (in_n) {
            if (i == q - 1) cb = new_dq;
            else if (new_dq != 0.0) cb -= tri * new_dq;
            d.cbar[i] = cb;
        }
        if (pse && in_m) {
            const double gamma_p = st->gamma_pq, eta_p = st->eta_pq;
            const int tkq = d.type[kq - 1];
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
            if (d.type[kp - 1] == FX && d.refsp[kp - 1] && ti != 0.0) {
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
                const bool reset = (pse && st->refct == 1);
                c = chuzr_cand_v(i, tknew, lbn, ubn, bb, reset ? 1.0 : g, st->tol_bnd);
            }
            const Cand b = block_best<0>(c, shc);
            if (threadIdx.x == 0) cand_chuzr(d)[blockIdx.x] = b;
        }
        if (st->phase == 1) {
            const double tol = st->tol_dj;
            const int badj = in_n && ((cb < -tol && (ot == LO || ot == FR)) || (cb > +tol && (ot == UP || ot == FR)));
            if (__syncthreads_or(badj) && threadIdx.x == 0) atomicOr(&st->dinf, 1);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->teta = teta;
            st->pivot = tp;
            st->pend = 1;
        }
        return;
    }
    // rank-1 update over the dense columns
    const int b = blockIdx.x - nvb;
    const int tile = b % tiles, chunk = b / tiles, chunks = (gridDim.x - nvb) / tiles;
    const int nr = st->nr;
    const int cnt = nr + (kp <= m ? 1 : 0);
    const int ce = (kq <= m) ? kq - 1 : -1;
    const int lps = (cnt + chunks - 1) / chunks;
    const int t0 = chunk * lps, t1 = min(cnt, t0 + lps);
    const int r = (tile * 256 + threadIdx.x) * 2;
    if (r >= m) return;
    const bool two = (r + 1 < m);
    const bool z0 = (r == p - 1), z1 = (r + 1 == p - 1);
    const double f0 = z0 ? 1.0 / tp : d.tcol[r] / tp;
    const double f1 = two ? (z1 ? 1.0 / tp : d.tcol[r + 1] / tp) : 0.0;
    for (int t = t0; t < t1; ++t) {
        const int c = (t < nr) ? d.rlist[t] : kp - 1;
        const double rl = (t < nr) ? d.rho_val[t] : 1.0;
        double *ptr = d.Binv + (size_t)c * d.ldb + r;
        double2 v;
        if (c == ce) {
            v.x = z0 ? 1.0 : 0.0;
            v.y = z1 ? 1.0 : 0.0;
        } else {
            v = *(double2 *)ptr;
            v.x = (z0 ? 0.0 : v.x) - f0 * rl;
            v.y = (z1 ? 0.0 : v.y) - f1 * rl;
        }
        if (two) *(double2 *)ptr = v;
        else ptr[0] = v.x;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
DualPlan dual_plan(const SpxDev &d, int nr_max, int nwl_max, int pse, int rigorous)
{
    const int m = d.m, n = d.n;
    DualPlan pl{};
    pl.pse = pse;
    pl.rigorous = rigorous;
    nr_max = std::min(std::max(nr_max, 0), m);
    const int ns_max = std::min(m, nr_max + 1);
    pl.rowpath = (d.A.dense && d.A.AT && !rigorous && 2 * ns_max <= m) ? 1 : 0;
    pl.fused = (d.A.dense && !rigorous) ? 1 : 0;
    const int tiles_t = cdiv(n, 512), tiles_f = cdiv(m, 512);
    pl.tsplits = std::max(1, std::min(2048 / tiles_t, cdiv(ns_max, 8)));
    pl.tsplits = std::max(1, std::min<int>(pl.tsplits, (int)(d.partial_cap / std::max(n, 1))));
    pl.twaves = ns_max <= 32 ? 4 : (ns_max <= 128 ? 8 : 16);
    const int nrhs = pse ? 2 : 1;
    pl.fsplits = std::max(1, std::min(2048 / tiles_f, cdiv(std::max(nr_max, 1), 8)));
    pl.fsplits = std::max(1, std::min<int>(pl.fsplits, (int)(d.partial_cap / ((size_t)nrhs * m))));
    pl.uchunks = std::max(1, std::min(2048 / tiles_f, cdiv(nr_max + 1, 4)));
    pl.awsplits = std::max(1, std::min(cdiv(std::max(nwl_max, 1), 32), 64));
    pl.awsplits = std::max(1, std::min<int>(pl.awsplits, (int)(d.awpart_cap / std::max(m, 1))));
    return pl;
}

void refine_rho_dev(hipStream_t s, const SpxDev &d);
void refine_tcol_dev(hipStream_t s, const SpxDev &d, int need_p);
void colpass_gated(hipStream_t s, const MatDev &A, int mode, int off, int cnt, const int *head,
                   const signed char *stat, const double *coef, const double *h, const double *x,
                   const double *y, double *out1, double *out2, unsigned long long *maxbits,
                   const DState *st, int need_p);
void aprod_neg_gated(hipStream_t s, const MatDev &A, const double *w, const double *base, double *y,
                     double *partial, size_t cap, const DState *st, int need_p);

double launch_trow_rows(hipStream_t s, const SpxDev &d, const DualPlan &pl, int ns)
{
    const int n = d.n;
    hipLaunchKernelGGL(k_lgemv_part, dim3(cdiv(n, 512), pl.tsplits), dim3(256), 0, s, d.A.AT, (size_t)d.A.ldt, n,
                       d.rho_idx, &d.st->ns, d.rho_val, d.partial, (DState *)nullptr, (unsigned long long *)nullptr);
    return 8.0 * (double)ns * n + 12.0 * ns;
}

static double bytes_fixed(const SpxDev &d) { return 96.0 * ((double)d.m + d.n); }

void dual_batch_begin(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    (void)pl;
    hipLaunchKernelGGL(k_dual_prep, dim3(cdiv(std::max(d.m, d.n), 256)), dim3(256), 0, s, d);
}

void dual_batch_end(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    hipLaunchKernelGGL(k_dual_finish, dim3(1), dim3(64), 0, s, d, pl.rowpath, bytes_fixed(d));
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

void dual_iteration2(hipStream_t s, const SpxDev &d, const DualPlan &pl, hipEvent_t ev0, hipEvent_t ev1)
{
    const int m = d.m, n = d.n;
    const int gv = cdiv(std::max(m, n), 256), gn = cdiv(n, 256), tiles_m = cdiv(m, 512);
    const double bf = bytes_fixed(d);
    hipLaunchKernelGGL(k_dual_top, dim3(1), dim3(WG), 0, s, d, pl.rowpath, bf);
    if (pl.rigorous) refine_rho_dev(s, d);
    int ncb = gv, slotw = 256;
    if (pl.rowpath) {
        ncb = cdiv(std::max(m, n), 64);
        slotw = 64;
        if (ev0) (void)hipEventRecord(ev0, s);
        hipLaunchKernelGGL(k_trow_rows, dim3(ncb), dim3(64 * pl.twaves), 0, s, d, pl.pse);
        if (ev1) (void)hipEventRecord(ev1, s);
    } else {
        if (ev0) (void)hipEventRecord(ev0, s);
        colpass_gated(s, d.A, CP_TROW, m, n, d.head, d.stat, d.coef, nullptr, d.rho, nullptr, d.trow, nullptr,
                      &d.st->trow_max_bits, d.st, 0);
        if (ev1) (void)hipEventRecord(ev1, s);
        hipLaunchKernelGGL(k_trow_finish<0>, dim3(gv), dim3(256), 0, s, d, (const double *)nullptr, 0, pl.pse, 0);
    }
    const int aw = (pl.pse && d.A.dense) ? 1 : 0;
    hipLaunchKernelGGL(k_dual_ratio, dim3(gn + (aw ? tiles_m * pl.awsplits : 0)), dim3(256), 0, s, d, gn, tiles_m,
                       pl.rowpath, ncb, slotw);
    if (pl.fused) {
        if (pl.pse) launch_ftran<2, 1, 1>(s, d, pl, gn, ncb);
        else launch_ftran<1, 1, 0>(s, d, pl, gn, ncb);
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
    hipLaunchKernelGGL(k_dual_commit, dim3(nvb + tiles_m * pl.uchunks), dim3(256), 0, s, d, pl.pse, nvb, tiles_m);
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
