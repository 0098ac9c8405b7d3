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
// Kernel sequence of one pivot (each gated on st->stop):
//   k_dual_top      1 WG   chuzr (:572), rho, reference-space reset
//   k_lgemv_part    grid   trow partials over rows of AT     (eval_trow :655-791)
//   k_trow_finish   grid   trow, max|trow|, PSE vectors, gamma_p partials
//   k_dual_chuzc    1 WG   Harris ratio test (:820-950), gamma_p, h = -N[q]
//   [PSE] A w       grid   (update_gamma :1103-1134)
//   k_lgemv_part    grid   tcol = inv(B) h, u = inv(B)(ys - A w)  (eval_tcol :937)
//   k_lgemv_reduce  grid
//   k_dual_commit   grid   pivot check (:1913), update_bbar/cbar/gamma, rank-1 update of inv(B)
//   k_dual_finish   1 WG   change_basis (:1954-1964), list of dense columns, counters
#include "gk_device.h"
#include <algorithm>

namespace gk {

// ---------------------------------------------------------------------------
// list GEMV partials:
//   part[(s*NRHS + k)*rows + r] = sum over t in chunk s of M[col_t*ld + r] * x_k(t)
// col_t = list[t]; XBYT: x_1(t) = x1[t] (compact values), else x_k(t) = xk[col_t].
// 512 rows per block (2 per lane, 16-byte loads); chunk s = blockIdx.y.
// ---------------------------------------------------------------------------
template <int NRHS, int XBYT>
__global__ void __launch_bounds__(256) k_lgemv_part(const double *__restrict__ M, size_t ld, int rows,
                                                      const int *__restrict__ list, const int *cntp,
                                                      const double *__restrict__ x1, const double *__restrict__ x2,
                                                      double *__restrict__ part, const DState *st)
{
    if (st && st->stop) return;
    const int cnt = *cntp;
    const int splits = gridDim.y;
    const int lps = (cnt + splits - 1) / splits;
    const int t0 = blockIdx.y * lps, t1 = min(cnt, t0 + lps);
    const int r = (blockIdx.x * 256 + threadIdx.x) * 2;
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
    if (r < rows) {
        // r + 1 < ld always (ld is a multiple of 8 and r is even), so the
        // 16-byte load stays inside the allocation even for the last odd row
        int t = t0;
        for (; t + 4 <= t1; t += 4) {
            int c[4];
            double xa[4], xb[4];
            bool any = false;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                c[u] = list[t + u];
                xa[u] = XBYT ? x1[t + u] : x1[c[u]];
                xb[u] = (NRHS == 2) ? x2[c[u]] : 0.0;
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
            const double xa = XBYT ? x1[t] : x1[c];
            const double xb = (NRHS == 2) ? x2[c] : 0.0;
            if (xa == 0.0 && xb == 0.0) continue;
            const double2 v = *(const double2 *)(M + (size_t)c * ld + r);
            a0 += v.x * xa;
            a1 += v.y * xa;
            if (NRHS == 2) {
                b0 += v.x * xb;
                b1 += v.y * xb;
            }
        }
        double *o = part + (size_t)blockIdx.y * NRHS * rows + r;
        o[0] = a0;
        if (r + 1 < rows) o[1] = a1;
        if (NRHS == 2) {
            o[rows] = b0;
            if (r + 1 < rows) o[rows + 1] = b1;
        }
    }
}

// tcol[i] = sum_s part + (unit column of a basic slack at position i) h,
// u[i] likewise with w — inv(B) x = sum over the dense columns + x[head[i]]
// for basic slack head[i].  64 rows per block, 8 waves over the splits,
// combined in a fixed order.
template <int NRHS>
__global__ void __launch_bounds__(512) k_lgemv_reduce(const double *__restrict__ part, int m, int splits,
                                                        const int *__restrict__ head,
                                                        const double *__restrict__ x1, const double *__restrict__ x2,
                                                        double *__restrict__ y1, double *__restrict__ y2,
                                                        const DState *st)
{
    if (st && st->stop) return;
    __shared__ double sh[NRHS][8][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 64 + lane;
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
    if (w == 0 && r < m) {
        double va = sh[0][0][lane], vb = (NRHS == 2) ? sh[NRHS - 1][0][lane] : 0.0;
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            va += sh[0][k][lane];
            if (NRHS == 2) vb += sh[NRHS - 1][k][lane];
        }
        const int kh = head[r];
        if (kh <= m) {
            va += x1[kh - 1];
            if (NRHS == 2) vb += x2[kh - 1];
        }
        y1[r] = va;
        if (NRHS == 2) y2[r] = vb;
    }
}

// ---------------------------------------------------------------------------
// k_dual_top: phase/limit checks, chuzr (glpspx02.js:572) and rho = row p of
// inv(B) (eval_rho :627) from the dense columns plus the unit entry
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(WG) k_dual_top(SpxDev d)
{
    __shared__ int shi[2];
    __shared__ Cand shc[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    if (st->iter_left <= 0 || st->refact_pending) {
        __syncthreads();
        if (threadIdx.x == 0) st->stop = st->refact_pending ? ST_REFACT : ST_BATCH;
        return;
    }
    if (st->pricing == PT_PSE && st->refct == 0) reset_refsp_dev(d, 1);
    if (st->phase == 1) {
        // check_feas (:1296)
        const double tol = st->tol_dj;
        int bad = 0;
        for (int j = threadIdx.x; j < n && !bad; j += blockDim.x) {
            const int k = d.head[m + j];
            const double cb = d.cbar[j];
            const int ot = d.orig_type[k - 1];
            if (cb < -tol && (ot == LO || ot == FR)) bad = 1;
            if (cb > +tol && (ot == UP || ot == FR)) bad = 1;
        }
        if (!block_or(bad, shi)) {
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
    // chuzr: p = argmax r_i^2 / gamma_i over bound violations
    const double tol_bnd = st->tol_bnd;
    Cand c; c.k1 = 0.0; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int k = d.head[i];
        const int t = d.type[k - 1];
        const double bb = d.bbar[i];
        double ri = 0.0;
        if (t == LO || t == DB || t == FX) {
            const double eps = tol_bnd * (1.0 + 0.10 * fabs(d.lb[k - 1]));
            if (bb < d.lb[k - 1] - eps) ri = d.lb[k - 1] - bb;
        }
        if (t == UP || t == DB || t == FX) {
            const double eps = tol_bnd * (1.0 + 0.10 * fabs(d.ub[k - 1]));
            if (bb > d.ub[k - 1] + eps) ri = d.ub[k - 1] - bb;
        }
        if (ri == 0.0) continue;
        double g = d.gamma[i];
        if (g < DBL_EPS) g = DBL_EPS;
        const double temp = (ri * ri) / g;
        Cand e; e.k1 = temp; e.k2 = ri; e.idx = i + 1; e.aux = 0;
        if (temp > 0.0 && better<0>(e, c)) c = e;
    }
    const Cand best = block_best<0>(c, shc);
    if (best.idx == 0) {
        if (threadIdx.x == 0) { st->p = 0; st->stop = ST_P0; }
        return;
    }
    const int p = best.idx;
    for (int l = threadIdx.x; l < m; l += blockDim.x) {
        d.rho[l] = 0.0;
        d.rowp[l] = 0.0;
    }
    __syncthreads();
    const int nr = st->nr;
    for (int t = threadIdx.x; t < nr; t += blockDim.x) {
        const int cc = d.rlist[t];
        const double v = d.Binv[(size_t)(p - 1) + (size_t)cc * d.ldb];
        d.rho[cc] = v;
        d.rowp[cc] = v;
        d.rho_idx[t] = cc;
        d.rho_val[t] = v;
    }
    if (threadIdx.x == 0) {
        const int kp = d.head[p - 1];
        int ns = nr;
        if (kp <= m) {   // the basic slack at position p: unit column of inv(B)
            d.rho[kp - 1] = 1.0;
            d.rowp[kp - 1] = 1.0;
            d.rho_idx[nr] = kp - 1;
            d.rho_val[nr] = 1.0;
            ns++;
        }
        st->p = p;
        st->delta = best.k2;
        st->trow_max_bits = 0ull;
        st->ns = ns;
        st->nw = 0;
    }
}

// ---------------------------------------------------------------------------
// k_trow_finish: structural column c / slack row c of the pivot row.
// FROM_PART: trow from the row-path partials (structurals) and -rho (slacks);
// else trow was written by the column pass.  Also the PSE vectors of
// update_gamma (:1103-1134): wcol[c] / ys[c] = trow of a non-basic variable of
// the reference space, and per-block sums of those trow^2 (gamma_p).
// ---------------------------------------------------------------------------
template <int FROM_PART>
__global__ void __launch_bounds__(256) k_trow_finish(SpxDev d, const double *__restrict__ part, int splits, int pse)
{
    __shared__ double shd[16];
    __shared__ double shm[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    double vmax = 0.0, gsum = 0.0, nwc = 0.0;
    if (idx < n) {
        const int c = idx;
        const int pos = d.bind[m + c];
        double tv = 0.0;
        if (pos > m) {
            const int j = pos - m - 1;
            if (FROM_PART) {
                double acc = 0.0;
#pragma unroll 8
                for (int s = 0; s < splits; ++s) acc += part[(size_t)s * n + c];
                tv = (d.stat[j] == NS) ? 0.0 : acc;
                d.trow[j] = tv;
            } else
                tv = d.trow[j];
            vmax = fabs(tv);
        }
        if (pse) {
            const bool ref = pos > m && d.refsp[m + c];
            const double w = ref ? tv : 0.0;
            d.wcol[c] = w;
            gsum += w * w;
            nwc += (w != 0.0) ? 1.0 : 0.0;
        }
    }
    if (idx < m) {
        const int c = idx;
        const int pos = d.bind[c];
        double tv = 0.0;
        if (pos > m) {
            const int j = pos - m - 1;
            if (FROM_PART) {
                tv = (d.stat[j] == NS) ? 0.0 : -d.rho[c];
                d.trow[j] = tv;
            } else
                tv = d.trow[j];
            vmax = fmax(vmax, fabs(tv));
        }
        if (pse) {
            const double w = (pos > m && d.refsp[c]) ? tv : 0.0;
            d.ys[c] = w;
            gsum += w * w;
        }
    }
    if (FROM_PART) {
        const double b = block_max(vmax, shm);
        if (threadIdx.x == 0 && b > 0.0) atomicMax(&st->trow_max_bits, dbits(b));
    }
    if (pse) {
        const double g = block_sum(gsum, shd);
        const double k = block_sum(nwc, shd);
        if (threadIdx.x == 0) {
            d.gpart[blockIdx.x] = g;
            if (k > 0.0) atomicAdd(&st->nw, (int)k);
        }
    }
}

// ---------------------------------------------------------------------------
// k_dual_chuzc: Harris two-pass ratio test over the pivot row (glpspx02.js
// :820-950, significance filter with tol_bnd as sort_trow :1851), gamma_p
// (update_gamma :1103-1132), h = -N[q] (eval_tcol :937).  One workgroup; for
// n <= 16 * 1024 the row is held in registers across both passes.
// ---------------------------------------------------------------------------
struct RatioCtx {
    double eps, s, rtol;
};

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

constexpr int CHUZC_REG = 16;

__global__ void __launch_bounds__(WG) k_dual_chuzc(SpxDev d, int pse, int gblocks)
{
    __shared__ Cand shc[16];
    __shared__ double shd[16];
    DState *st = d.st;
    if (st->stop) return;
    const int n = d.n;
    const double big = __longlong_as_double((long long)st->trow_max_bits);
    RatioCtx x;
    x.eps = st->tol_bnd * (1.0 + 0.01 * big);
    const double delta = st->delta;
    x.s = (delta > 0.0 ? +1.0 : -1.0);
    x.rtol = (st->rtest == RT_HAR) ? 0.30 * st->tol_dj : 0.0;
    const bool reg = n <= CHUZC_REG * WG;
    double trv[CHUZC_REG], cbv[CHUZC_REG];
    int sjv[CHUZC_REG];
    Cand c; c.k1 = DBL_MAX; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    if (reg) {
#pragma unroll
        for (int r = 0; r < CHUZC_REG; ++r) {
            const int j = threadIdx.x + r * WG;
            trv[r] = (j < n) ? d.trow[j] : 0.0;
            cbv[r] = (j < n) ? d.cbar[j] : 0.0;
            sjv[r] = (j < n) ? d.stat[j] : 0;
        }
#pragma unroll
        for (int r = 0; r < CHUZC_REG; ++r) {
            Cand e;
            if (pass1_cand(x, trv[r], cbv[r], sjv[r], threadIdx.x + r * WG, e) && better<1>(e, c)) c = e;
        }
    } else {
        for (int j = threadIdx.x; j < n; j += WG) {
            Cand e;
            if (pass1_cand(x, d.trow[j], d.cbar[j], d.stat[j], j, e) && better<1>(e, c)) c = e;
        }
    }
    const Cand b1 = block_best<1>(c, shc);
    int q = b1.idx;
    double teta = (q ? b1.k1 : DBL_MAX);
    if (!(x.rtol == 0.0 || q == 0 || teta == 0.0)) {
        const double tmax = teta;
        Cand c2; c2.k1 = 0.0; c2.k2 = 0.0; c2.idx = 0; c2.aux = 0;
        if (reg) {
#pragma unroll
            for (int r = 0; r < CHUZC_REG; ++r) {
                Cand e;
                if (pass2_cand(x, trv[r], cbv[r], sjv[r], threadIdx.x + r * WG, tmax, e) && better<2>(e, c2)) c2 = e;
            }
        } else {
            for (int j = threadIdx.x; j < n; j += WG) {
                Cand e;
                if (pass2_cand(x, d.trow[j], d.cbar[j], d.stat[j], j, tmax, e) && better<2>(e, c2)) c2 = e;
            }
        }
        const Cand b2 = block_best<2>(c2, shc);
        q = b2.idx;
        teta = b2.k1;
    }
    if (q == 0) {
        if (threadIdx.x == 0) { st->q = 0; st->stop = ST_Q0; }
        return;
    }
    const double piv = d.trow[q - 1];
    if (fabs(piv) < 1e-5 * (1.0 + 0.01 * big) && !st->rigorous) {
        __syncthreads();
        if (threadIdx.x == 0) { st->q = q; st->stop = ST_SMALLPIV; }
        return;
    }
    if (pse) {
        double g = 0.0;
        for (int b = threadIdx.x; b < gblocks; b += WG) g += d.gpart[b];
        g = block_sum(g, shd);
        if (threadIdx.x == 0) {
            const double eta = d.refsp[d.head[st->p - 1] - 1] ? 1.0 : 0.0;
            st->eta_pq = eta;
            st->gamma_pq = eta + g;
        }
    }
    build_hq(d, q);
    if (threadIdx.x == 0) {
        st->q = q;
        st->new_dq = x.s * teta;
        st->cbar_q_old = d.cbar[q - 1];
    }
}

// ---------------------------------------------------------------------------
// k_dual_commit: pivot check (:1913-1933), update_bbar (:1042), update_cbar
// (:1020), update_gamma (:1075-1134) in the first `nvb` blocks; the rank-1
// update of the dense columns of inv(B) in the others (product form of the
// basis change: row p := rho / alpha_p, row i -= alpha_i / alpha_p rho).
// A slack leaving the basis turns its unit column dense (virtual list entry
// nr, rho = 1); a slack entering turns its column into exactly e_p.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dual_commit(SpxDev d, int pse, int nvb, int tiles)
{
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
    if ((int)blockIdx.x < nvb) {
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        const double teta = delta / tp;
        const double new_dq = st->new_dq;
        if (i < m) {
            if (i == p - 1) d.bbar[i] = get_xN(d.stat, d.lb, d.ub, kq, q) + teta;
            else if (teta != 0.0) d.bbar[i] += d.tcol[i] * teta;
        }
        if (i < n) {
            if (i == q - 1) d.cbar[i] = new_dq;
            else if (new_dq != 0.0) d.cbar[i] -= d.trow[i] * new_dq;
        }
        if (pse && i < m) {
            const double gamma_p = st->gamma_pq, eta_p = st->eta_pq;
            const double ti = d.tcol[i];
            const int k = d.head[i];
            double g = d.gamma[i];
            if (i == p - 1) {
                if (d.type[kq - 1] == FR) g = 1.0;
                else {
                    g = gamma_p / (tp * tp);
                    if (g < DBL_EPS) g = DBL_EPS;
                }
            } else if (ti != 0.0 && d.type[k - 1] != FR) {
                const double t = ti / tp;
                const double t1 = g + t * t * gamma_p + 2.0 * t * d.u[i];
                const double t2 = (d.refsp[k - 1] ? 1.0 : 0.0) + eta_p * t * t;
                g = (t1 >= t2 ? t1 : t2);
                if (g < DBL_EPS) g = DBL_EPS;
            }
            const int kp = d.head[p - 1];
            if (d.type[kp - 1] == FX && d.refsp[kp - 1] && ti != 0.0) {
                double t = 0.0;
                bool apply = true;
                if (i == p - 1) {
                    if (d.type[kq - 1] == FR) apply = false; else t = 1.0 / tp;
                } else {
                    if (d.type[k - 1] == FR) apply = false; else t = ti / tp;
                }
                if (apply) {
                    g -= t * t;
                    if (g < DBL_EPS) g = DBL_EPS;
                }
            }
            d.gamma[i] = g;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->teta = teta;
            st->pivot = tp;
        }
        return;
    }
    // rank-1 update over the dense columns
    const int b = blockIdx.x - nvb;
    const int tile = b % tiles, chunk = b / tiles, chunks = (gridDim.x - nvb) / tiles;
    const int kp = d.head[p - 1];
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

// change_basis (glpspx02.js:1954-1964) and the list of dense columns
__global__ void k_dual_finish(SpxDev d, int rowpath, double bytes_fixed)
{
    DState *st = d.st;
    if (st->stop || threadIdx.x != 0) return;
    const int m = d.m, n = d.n, p = st->p, q = st->q;
    const int kp = d.head[p - 1];
    const int kq = d.head[m + q - 1];
    const int nr0 = st->nr, ns = st->ns, nw = st->nw;
    if (st->phase == 2) st->obj += (st->cbar_q_old / st->zeta) * (st->delta / st->pivot);
    if (st->pricing == PT_PSE && d.type[kp - 1] == FX && d.refsp[kp - 1]) d.refsp[kp - 1] = 0;
    d.head[p - 1] = kq;
    d.head[m + q - 1] = kp;
    d.bind[kq - 1] = p;
    d.bind[kp - 1] = m + q;
    if (d.type[kp - 1] == FX) d.stat[q - 1] = NS;
    else if (st->delta > 0.0) d.stat[q - 1] = NL;
    else d.stat[q - 1] = NU;
    int nr = nr0;
    if (kq <= m) {               // entering slack: its column is now e_p
        const int c = kq - 1, t = d.rpos[c], last = d.rlist[nr - 1];
        d.rlist[t] = last;
        d.rpos[last] = t;
        d.rpos[c] = -1;
        nr--;
    }
    if (kp <= m) {               // leaving slack: its column became dense
        const int c = kp - 1;
        d.rlist[nr] = c;
        d.rpos[c] = nr;
        nr++;
    }
    st->nr = nr;
    if (st->pricing == PT_PSE && st->refct > 0) st->refct--;
    st->upd_cnt++;
    st->binv_fresh = 0;
    st->cbar_fresh = 0;
    if (st->upd_cnt >= st->upd_lim) st->refact_pending = 1;
    st->it_cnt++;
    st->npiv++;
    st->iter_left--;
    if (st->rigorous > 0) st->rigorous--;
    // algorithmic HBM bytes of this pivot: the pivot row (rows of A in the
    // support of rho, or all of A), A w, inv(B) once for both right-hand
    // sides, read + write of the updated columns, and the O(m + n) vectors
    const double rowb = rowpath ? 8.0 * (double)ns * n : 8.0 * (double)m * n;
    st->bytes += rowb + 8.0 * (double)m * nw + 8.0 * (double)m * (nr0 + 1) +
                 16.0 * (double)m * (nr0 + (kp <= m ? 1 : 0)) + bytes_fixed;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

DualPlan dual_plan(const SpxDev &d, int nr_max, int pse, int rigorous)
{
    const int m = d.m, n = d.n;
    DualPlan pl{};
    pl.pse = pse;
    pl.rigorous = rigorous;
    nr_max = std::min(std::max(nr_max, 0), m);
    const int ns_max = std::min(m, nr_max + 1);
    pl.rowpath = (d.A.dense && d.A.AT && !rigorous && 2 * ns_max <= m) ? 1 : 0;
    const int tiles_t = cdiv(n, 512), tiles_f = cdiv(m, 512);
    pl.tsplits = std::max(1, std::min(2048 / tiles_t, cdiv(ns_max, 8)));
    pl.tsplits = std::max(1, std::min<int>(pl.tsplits, (int)(d.partial_cap / std::max(n, 1))));
    const int nrhs = pse ? 2 : 1;
    pl.fsplits = std::max(1, std::min(2048 / tiles_f, cdiv(std::max(nr_max, 1), 8)));
    pl.fsplits = std::max(1, std::min<int>(pl.fsplits, (int)(d.partial_cap / ((size_t)nrhs * m))));
    pl.uchunks = std::max(1, std::min(2048 / tiles_f, cdiv(nr_max + 1, 4)));
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
    hipLaunchKernelGGL((k_lgemv_part<1, 1>), dim3(cdiv(n, 512), pl.tsplits), dim3(256), 0, s, d.A.AT, (size_t)d.A.ldt,
                       n, d.rho_idx, &d.st->ns, d.rho_val, (const double *)nullptr, d.partial, (const DState *)nullptr);
    return 8.0 * (double)ns * n + 8.0 * (double)pl.tsplits * n + 12.0 * ns;
}

void dual_iteration2(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    const int m = d.m, n = d.n;
    const int gblocks = cdiv(std::max(m, n), 256);
    hipLaunchKernelGGL(k_dual_top, dim3(1), dim3(WG), 0, s, d);
    if (pl.rigorous) refine_rho_dev(s, d);
    if (pl.rowpath) {
        hipLaunchKernelGGL((k_lgemv_part<1, 1>), dim3(cdiv(n, 512), pl.tsplits), dim3(256), 0, s, d.A.AT,
                           (size_t)d.A.ldt, n, d.rho_idx, &d.st->ns, d.rho_val, (const double *)nullptr, d.partial,
                           (const DState *)d.st);
        hipLaunchKernelGGL(k_trow_finish<1>, dim3(gblocks), dim3(256), 0, s, d, d.partial, pl.tsplits, pl.pse);
    } else {
        colpass_gated(s, d.A, CP_TROW, m, n, d.head, d.stat, d.coef, nullptr, d.rho, nullptr, d.trow, nullptr,
                      &d.st->trow_max_bits, d.st, 0);
        if (pl.pse)
            hipLaunchKernelGGL(k_trow_finish<0>, dim3(gblocks), dim3(256), 0, s, d, (const double *)nullptr, 0, 1);
    }
    hipLaunchKernelGGL(k_dual_chuzc, dim3(1), dim3(WG), 0, s, d, pl.pse, gblocks);
    const int tiles_f = cdiv(m, 512);
    if (pl.pse) {
        aprod_neg_gated(s, d.A, d.wcol, d.ys, d.work, d.partial, d.partial_cap, d.st, 0);   // work = ys - A w
        hipLaunchKernelGGL((k_lgemv_part<2, 0>), dim3(tiles_f, pl.fsplits), dim3(256), 0, s, d.Binv, (size_t)d.ldb, m,
                           d.rlist, &d.st->nr, d.h, d.work, d.partial, (const DState *)d.st);
        hipLaunchKernelGGL(k_lgemv_reduce<2>, dim3(cdiv(m, 64)), dim3(512), 0, s, d.partial, m, pl.fsplits, d.head,
                           d.h, d.work, d.tcol, d.u, (const DState *)d.st);
    } else {
        hipLaunchKernelGGL((k_lgemv_part<1, 0>), dim3(tiles_f, pl.fsplits), dim3(256), 0, s, d.Binv, (size_t)d.ldb, m,
                           d.rlist, &d.st->nr, d.h, (const double *)nullptr, d.partial, (const DState *)d.st);
        hipLaunchKernelGGL(k_lgemv_reduce<1>, dim3(cdiv(m, 64)), dim3(512), 0, s, d.partial, m, pl.fsplits, d.head,
                           d.h, (const double *)nullptr, d.tcol, (double *)nullptr, (const DState *)d.st);
    }
    if (pl.rigorous) refine_tcol_dev(s, d, 0);
    const int nvb = gblocks;
    hipLaunchKernelGGL(k_dual_commit, dim3(nvb + tiles_f * pl.uchunks), dim3(256), 0, s, d, pl.pse, nvb, tiles_f);
    const double bytes_fixed = 96.0 * ((double)m + n);
    hipLaunchKernelGGL(k_dual_finish, dim3(1), dim3(64), 0, s, d, pl.rowpath, bytes_fixed);
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
