// HIP kernels of the MI355X simplex core (gfx950, wave64).
//
// Each kernel cites the reference routine whose arithmetic it carries out.
// Pivot-loop kernels take the device state `st` and return at once when a
// previous kernel of the same pivot set st->stop, so a host batch of K pivots
// can be enqueued without synchronisation and drains cheaply after a stop.
//
// Reductions that choose an index reproduce the reference's first-hit scans
// (strict comparisons, glpspx01.js:681, glpspx02.js:617/:865/:921) with a
// lowest-index tie-break; sums are fixed-order (deterministic run to run).
#include "gk_device.h"
#include <cfloat>
#include <cstdio>
#include <algorithm>

namespace gk {


// =====================================================================
// dense GEMV, y = beta*base + alpha * M x (zero x entries skipped)
// =====================================================================
GemvPlan gemv_plan(int rows, int cols, int ld)
{
    GemvPlan p;
    p.rows = rows; p.cols = cols; p.ld = ld;
    p.tiles = (rows + 511) / 512;
    int want = std::max(1, 2048 / std::max(1, p.tiles));
    int maxs = std::max(1, (cols + 7) / 8);
    p.splits = std::min(want, maxs);
    p.cols_per_split = (cols + p.splits - 1) / p.splits;
    p.splits = (cols + p.cols_per_split - 1) / p.cols_per_split;
    if (p.splits < 1) p.splits = 1;
    return p;
}

__global__ void __launch_bounds__(256) k_gemv_n_part(const double *__restrict__ M, int rows, int cols, int ld,
                                                       const double *__restrict__ x, int cps,
                                                       double *__restrict__ part, const DState *st, int need_p)
{
    GATE(st, need_p);
    // the split's multipliers are read once per block, 256 at a time, and
    // the non-zero ones compacted in LDS (ballot + wave prefix), so the
    // column loop touches only columns with x_c != 0, in column order
    __shared__ double sxv[256];
    __shared__ int scol[256];
    __shared__ int swcnt[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = (blockIdx.x * 256 + threadIdx.x) * 2;
    const int c0 = blockIdx.y * cps;
    const int c1 = min(cols, c0 + cps);
    const bool act = r < rows, two = (r + 1 < rows);
    double a0 = 0.0, a1 = 0.0;
    for (int cb = c0; cb < c1; cb += 256) {
        const int c = cb + threadIdx.x;
        const double xv = (c < c1) ? x[c] : 0.0;
        const bool nz = xv != 0.0;
        const unsigned long long bal = __ballot(nz);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) swcnt[w] = __popcll(bal);
        __syncthreads();
        int off = 0, tot = 0;
        for (int k = 0; k < 4; ++k) {
            if (k < w) off += swcnt[k];
            tot += swcnt[k];
        }
        if (nz) {
            sxv[off + below] = xv;
            scol[off + below] = c;
        }
        __syncthreads();
        if (act) {
            int k = 0;
            for (; k + 4 <= tot; k += 4) {
                double2 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double *p0 = M + (size_t)scol[k + u] * ld + r;
                    v[u] = two ? *(const double2 *)p0 : make_double2(p0[0], 0.0);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a0 += v[u].x * sxv[k + u];
                    a1 += v[u].y * sxv[k + u];
                }
            }
            for (; k < tot; ++k) {
                const double *p0 = M + (size_t)scol[k] * ld + r;
                const double2 v = two ? *(const double2 *)p0 : make_double2(p0[0], 0.0);
                a0 += v.x * sxv[k];
                a1 += v.y * sxv[k];
            }
        }
        __syncthreads();
    }
    if (act) {
        double *out = part + (size_t)blockIdx.y * rows + r;
        out[0] = a0;
        if (two) out[1] = a1;
    }
}

// y[r] = beta*base[r] + alpha * sum_s part[s][r]: 64 rows per block, the 8
// waves take splits w, w+8, ... and combine in LDS in a fixed order
__global__ void __launch_bounds__(512) k_gemv_reduce(const double *__restrict__ part, int rows, int splits,
                                                       double *__restrict__ y, double alpha,
                                                       const double *__restrict__ base, double beta,
                                                       const DState *st, int need_p, const double *__restrict__ from)
{
    GATE(st, need_p);
    __shared__ double sh[8][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 64 + lane;
    double acc = 0.0;
    if (r < rows) {
#pragma unroll 4
        for (int s = w; s < splits; s += 8) acc += part[(size_t)s * rows + r];
    }
    sh[w][lane] = acc;
    __syncthreads();
    if (w == 0 && r < rows) {
        double v = sh[0][lane];
#pragma unroll
        for (int k = 1; k < 8; ++k) v += sh[k][lane];
        v *= alpha;
        if (base) v = beta * base[r] + v;
        y[r] = from ? from[r] - v : v;       // (from: y = from - (base - A x), eval_beta's residual)
    }
}

static void gemv_n_gated(hipStream_t s, const double *M, int rows, int cols, int ld, const double *x,
                         double *partial, size_t cap, double *y, double alpha, const double *base, double beta,
                         const DState *st, int need_p, const double *from = nullptr)
{
    if (rows <= 0) return;
    GemvPlan p = gemv_plan(rows, cols, ld);
    if ((size_t)p.splits * rows > cap) {
        p.splits = (int)std::max<size_t>(1, cap / rows);
        p.cols_per_split = (cols + p.splits - 1) / p.splits;
        p.splits = (cols + p.cols_per_split - 1) / p.cols_per_split;
    }
    if (cols > 0) {
        dim3 g(p.tiles, p.splits);
        hipLaunchKernelGGL(k_gemv_n_part, g, dim3(256), 0, s, M, rows, cols, ld, x, p.cols_per_split, partial, st, need_p);
    } else {
        p.splits = 0;
    }
    hipLaunchKernelGGL(k_gemv_reduce, dim3((rows + 63) / 64), dim3(512), 0, s, partial, rows, p.splits, y, alpha,
                       base, beta, st, need_p, from);
}

void gemv_n(hipStream_t s, const double *M, int rows, int cols, int ld, const double *x, double *partial,
            size_t partial_cap, double *y, double alpha, const double *base, double beta)
{
    gemv_n_gated(s, M, rows, cols, ld, x, partial, partial_cap, y, alpha, base, beta, nullptr, 0);
}

// y[l] = alpha * M[:,l] . x — one wave per column, 16-byte loads along the column
__global__ void __launch_bounds__(256) k_gemv_t(const double *__restrict__ M, int rows, int cols, int ld,
                                                  const double *__restrict__ x, double *__restrict__ y, double alpha,
                                                  const DState *st, int need_p)
{
    GATE(st, need_p);
    const int lane = threadIdx.x & 63;
    const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (int c = wv; c < cols; c += nw) {
        const double *col = M + (size_t)c * ld;
        double acc = 0.0;
        int r = lane * 2;
        for (; r + 1 < rows; r += 128) {
            double2 v = *(const double2 *)(col + r);
            acc += v.x * x[r];
            acc += v.y * x[r + 1];
        }
        if (r < rows) acc += col[r] * x[r];
        acc = wsum(acc);
        if (lane == 0) y[c] = alpha * acc;
    }
}

static void gemv_t_gated(hipStream_t s, const double *M, int rows, int cols, int ld, const double *x, double *y,
                         double alpha, const DState *st, int need_p)
{
    if (cols <= 0) return;
    int blocks = std::min((cols + 3) / 4, 4096);
    hipLaunchKernelGGL(k_gemv_t, dim3(blocks), dim3(256), 0, s, M, rows, cols, ld, x, y, alpha, st, need_p);
}

void gemv_t(hipStream_t s, const double *M, int rows, int cols, int ld, const double *x, double *y, double alpha)
{
    gemv_t_gated(s, M, rows, cols, ld, x, y, alpha, nullptr, 0);
}

// =====================================================================
// passes over columns of (I | -A) selected through the basis header
// (eval_trow1 glpspx02.js:655, eval_cost glpspx01.js:531, error_btran
// glpspx01.js:265, update_gamma's N'[j] u glpspx01.js:1231-1241)
// =====================================================================
// returns |out1[i]| for CP_TROW (folded into one atomic max per block)
__device__ __forceinline__ double colpass_emit(int mode, int i, int k, int m, const signed char *stat,
                                               const double *coef, const double *h, double d1, double d2,
                                               double *out1, double *out2)
{
    // d1 = N . x, d2 = N . y
    switch (mode) {
    case CP_TROW: {
        double v = (stat && stat[i] == NS) ? 0.0 : -d1;
        out1[i] = v;
        return fabs(v);
    }
    case CP_CBAR: out1[i] = coef[k - 1] - d1; break;
    case CP_RESID: out1[i] = h[i] - d1; break;
    case CP_TROW_S: {
        bool ns = (stat && stat[i] == NS);
        out1[i] = ns ? 0.0 : -d1;
        out2[i] = ns ? 0.0 : d2;
        break;
    }
    default: out1[i] = d1; break;
    }
    return 0.0;
}

__device__ __forceinline__ void block_atomic_max(double v, unsigned long long *maxbits)
{
    __shared__ double shm[16];
    const double b = block_max(v, shm);
    if (threadIdx.x == 0 && b > 0.0) atomicMax(maxbits, dbits(b));
}

template <int TWO>
__global__ void __launch_bounds__(256) k_colpass_dense(int mode, int m, int off, int cnt, const int *__restrict__ head,
                                                         const signed char *__restrict__ stat, const double *__restrict__ coef,
                                                         const double *__restrict__ h, const double *__restrict__ A, int lda,
                                                         const double *__restrict__ x, const double *__restrict__ y,
                                                         double *out1, double *out2, unsigned long long *maxbits,
                                                         const DState *st, int need_p)
{
    GATE(st, need_p);
    const int lane = threadIdx.x & 63;
    const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    double vmax = 0.0;
    for (int i = wv; i < cnt; i += nw) {
        const int k = head[off + i];
        double d1 = 0.0, d2 = 0.0;
        if (mode == CP_TROW && stat && stat[i] == NS) {
            /* fixed non-basic: no dot needed */
        } else if (k <= m) {
            d1 = x[k - 1];
            if (TWO) d2 = y[k - 1];
        } else {
            const double *col = A + (size_t)(k - m - 1) * lda;
            double a1 = 0.0, a2 = 0.0;
            int r = lane * 2;
            // SEG segments of the column in flight per lane (the pass is bound
            // by the bytes in flight: 8 for one right-hand side — a slice of
            // a sharded pricing pass fills the chip with a quarter of the
            // waves); the same order of accumulation for any SEG
            constexpr int SEG = TWO ? 4 : 16;
            for (; r + (SEG - 1) * 128 + 1 < m; r += SEG * 128) {
                double2 v[SEG], xv[SEG], yv[SEG];
#pragma unroll
                for (int u = 0; u < SEG; ++u) {
                    v[u] = *(const double2 *)(col + r + 128 * u);
                    xv[u] = *(const double2 *)(x + r + 128 * u);
                    if (TWO) yv[u] = *(const double2 *)(y + r + 128 * u);
                }
#pragma unroll
                for (int u = 0; u < SEG; ++u) {
                    a1 += v[u].x * xv[u].x;
                    a1 += v[u].y * xv[u].y;
                    if (TWO) { a2 += v[u].x * yv[u].x; a2 += v[u].y * yv[u].y; }
                }
            }
            for (; r + 1 < m; r += 128) {
                double2 v = *(const double2 *)(col + r);
                a1 += v.x * x[r];
                a1 += v.y * x[r + 1];
                if (TWO) { a2 += v.x * y[r]; a2 += v.y * y[r + 1]; }
            }
            if (r < m) {
                a1 += col[r] * x[r];
                if (TWO) a2 += col[r] * y[r];
            }
            d1 = -wsum(a1);
            if (TWO) d2 = -wsum(a2);
        }
        if (lane == 0) vmax = fmax(vmax, colpass_emit(mode, i, k, m, stat, coef, h, d1, d2, out1, out2));
    }
    if (maxbits) block_atomic_max(vmax, maxbits);
}

// CSC columns with LPC lanes per column (LPC = 1, 8 or 64)
template <int LPC, int TWO>
__global__ void __launch_bounds__(256) k_colpass_csc(int mode, int m, int off, int cnt, const int *__restrict__ head,
                                                       const signed char *__restrict__ stat, const double *__restrict__ coef,
                                                       const double *__restrict__ h, const int *__restrict__ cptr,
                                                       const int *__restrict__ cind, const double *__restrict__ cval,
                                                       const double *__restrict__ x, const double *__restrict__ y,
                                                       double *out1, double *out2, unsigned long long *maxbits,
                                                       const DState *st, int need_p)
{
    GATE(st, need_p);
    const int sub = threadIdx.x % LPC;
    const int grp = (blockIdx.x * blockDim.x + threadIdx.x) / LPC;
    const int ngrp = (gridDim.x * blockDim.x) / LPC;
    const int nit = (cnt + ngrp - 1) / ngrp;      // uniform trip count (shuffles need all lanes)
    double vmax = 0.0;
    for (int it = 0; it < nit; ++it) {
        const int i = grp + it * ngrp;
        const bool act = i < cnt;
        int k = act ? head[off + i] : 0;
        double d1 = 0.0, d2 = 0.0;
        if (act && !(mode == CP_TROW && stat && stat[i] == NS)) {
            if (k <= m) {
                d1 = x[k - 1];
                if (TWO) d2 = y[k - 1];
            } else {
                const int c = k - m - 1;
                double a1 = 0.0, a2 = 0.0;
                for (int t = cptr[c] + sub; t < cptr[c + 1]; t += LPC) {
                    const double v = cval[t];
                    a1 += v * x[cind[t]];
                    if (TWO) a2 += v * y[cind[t]];
                }
                d1 = -a1; d2 = -a2;
            }
        }
        if (LPC > 1) {
            // only structural columns were split across lanes
            const bool structural = act && k > m && !(mode == CP_TROW && stat && stat[i] == NS);
            double s1 = structural ? d1 : 0.0, s2 = structural ? d2 : 0.0;
#pragma unroll
            for (int o = LPC / 2; o > 0; o >>= 1) {
                s1 += __shfl_xor(s1, o);
                if (TWO) s2 += __shfl_xor(s2, o);
            }
            if (structural) { d1 = s1; d2 = s2; }
        }
        if (act && sub == 0) vmax = fmax(vmax, colpass_emit(mode, i, k, m, stat, coef, h, d1, d2, out1, out2));
    }
    if (maxbits) block_atomic_max(vmax, maxbits);
}

void colpass_gated(hipStream_t s, const MatDev &A, int mode, int off, int cnt, const int *head,
                          const signed char *stat, const double *coef, const double *h, const double *x,
                          const double *y, double *out1, double *out2, unsigned long long *maxbits,
                          const DState *st, int need_p)
{
    if (cnt <= 0) return;
    const bool two = (mode == CP_TROW_S);
    if (A.dense) {
        int blocks = std::min((cnt + 3) / 4, 8192);
        if (two)
            hipLaunchKernelGGL(k_colpass_dense<1>, dim3(blocks), dim3(256), 0, s, mode, A.m, off, cnt, head, stat, coef, h,
                               A.A, A.lda, x, y, out1, out2, maxbits, st, need_p);
        else
            hipLaunchKernelGGL(k_colpass_dense<0>, dim3(blocks), dim3(256), 0, s, mode, A.m, off, cnt, head, stat, coef, h,
                               A.A, A.lda, x, y, out1, out2, maxbits, st, need_p);
        return;
    }
    int lpc = A.lpc;
    int per_block = 256 / lpc;
    int blocks = std::min((cnt + per_block - 1) / per_block, 8192);
#define CSC_LAUNCH(L, T) hipLaunchKernelGGL((k_colpass_csc<L, T>), dim3(blocks), dim3(256), 0, s, mode, A.m, off, cnt, head, \
                                            stat, coef, h, A.cptr, A.cind, A.cval, x, y, out1, out2, maxbits, st, need_p)
    if (lpc == 1) { if (two) CSC_LAUNCH(1, 1); else CSC_LAUNCH(1, 0); }
    else if (lpc == 8) { if (two) CSC_LAUNCH(8, 1); else CSC_LAUNCH(8, 0); }
    else { if (two) CSC_LAUNCH(64, 1); else CSC_LAUNCH(64, 0); }
#undef CSC_LAUNCH
}

void colpass(hipStream_t s, const MatDev &A, int mode, int off, int cnt, const int *head, const signed char *stat,
             const double *coef, const double *h, const double *x, const double *y, double *out1, double *out2,
             unsigned long long *maxbits)
{
    colpass_gated(s, A, mode, off, cnt, head, stat, coef, h, x, y, out1, out2, maxbits, nullptr, 0);
}

// y = base - A w over the structural columns (CSR rows for sparse A)
__global__ void __launch_bounds__(256) k_csr_neg(int m, const int *__restrict__ rptr, const int *__restrict__ rcol,
                                                   const double *__restrict__ rval, const double *__restrict__ w,
                                                   const double *__restrict__ base, double *__restrict__ y,
                                                   const DState *st, int need_p)
{
    GATE(st, need_p);
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int rc = min(r, m - 1);
    const int beg = rptr[rc], end = (r < m) ? rptr[rc + 1] : beg;
    const bool lng = end - beg > CSR_LONG;           // the wave sums it (csr_long_rows)
    if (!lng && r < m) {
        double acc = 0.0;
        for (int t = beg; t < end; ++t) {
            const double wv = w[rcol[t]];
            if (wv != 0.0) acc += rval[t] * wv;
        }
        y[r] = (base ? base[r] : 0.0) - acc;
    }
    const int rb = r - (int)(threadIdx.x & 63);
    csr_long_rows(lng, beg, end, rcol, rval, w, [&](int src, double acc) {
        if ((int)(threadIdx.x & 63) == 0) y[rb + src] = (base ? base[rb + src] : 0.0) - acc;
    });
}

void aprod_neg_gated(hipStream_t s, const MatDev &A, const double *w, const double *base, double *y,
                            double *partial, size_t cap, const DState *st, int need_p, const double *from)
{
    if (A.dense)
        gemv_n_gated(s, A.A, A.m, A.n, A.lda, w, partial, cap, y, -1.0, base, 1.0, st, need_p, from);
    else
        hipLaunchKernelGGL(k_csr_neg, dim3((A.m + 255) / 256), dim3(256), 0, s, A.m, A.rptr, A.rcol, A.rval, w, base, y,
                           st, need_p);
}

void aprod_neg(hipStream_t s, const MatDev &A, const double *w, const double *base, double *y, double *partial,
               size_t partial_cap)
{
    aprod_neg_gated(s, A, w, base, y, partial, partial_cap, nullptr, 0);
}

__global__ void k_scatter_pos(int m, int off, int cnt, const int *__restrict__ head, const double *__restrict__ w,
                              double *ys, double *wc, const DState *st, int need_p)
{
    GATE(st, need_p);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    const int k = head[off + i];
    const double v = w[i];
    if (k <= m) ys[k - 1] += v;         // each slack appears once among the positions
    else wc[k - m - 1] = v;
}

void scatter_pos(hipStream_t s, int m, int off, int cnt, const int *head, const double *w, double *ys, double *wc)
{
    if (cnt <= 0) return;
    hipLaunchKernelGGL(k_scatter_pos, dim3((cnt + 255) / 256), dim3(256), 0, s, m, off, cnt, head, w, ys, wc,
                       (const DState *)nullptr, 0);
}

// =====================================================================
// small vector helpers
// =====================================================================
// blockIdx.x = the segment, gridDim.y blocks share it; staged segments are
// 256-byte aligned, destinations are allocation starts (16-byte words, then
// the tail bytes)
__global__ void __launch_bounds__(256) k_scatter_segments(const char *__restrict__ src, const UpSeg *__restrict__ segs)
{
    const UpSeg g = segs[blockIdx.x];
    const char *a = src + g.off;
    char *b = (char *)g.dst;
    const size_t nw = g.bytes / 16;
    const size_t t0 = (size_t)blockIdx.y * blockDim.x + threadIdx.x, st = (size_t)gridDim.y * blockDim.x;
    for (size_t i = t0; i < nw; i += st)
        ((uint4 *)b)[i] = ((const uint4 *)a)[i];
    if (blockIdx.y == 0)
        for (size_t i = nw * 16 + threadIdx.x; i < g.bytes; i += blockDim.x) b[i] = a[i];
}

void scatter_segments(hipStream_t s, const char *src, const UpSeg *segs, int nseg)
{
    // 16 blocks per segment: a segment of a C3 upload is up to 160 KiB
    if (nseg > 0) hipLaunchKernelGGL(k_scatter_segments, dim3(nseg, 16), dim3(256), 0, s, src, segs);
}

__global__ void k_fill(double *x, double v, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) x[i] = v;
}

void fill_d(hipStream_t s, double *x, double v, size_t n)
{
    if (n == 0) return;
    int blocks = (int)std::min<size_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, s, x, v, n);
}

__global__ void k_axpy(double *y, const double *x, double a, int n, const DState *st, int need_p)
{
    GATE(st, need_p);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] += a * x[i];
}

void vec_axpy(hipStream_t s, double *y, const double *x, double a, int n, const DState *st, int need_p)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_axpy, dim3((n + 255) / 256), dim3(256), 0, s, y, x, a, n, st, need_p);
}

__global__ void k_copy(double *y, const double *x, int n, const DState *st, int need_p)
{
    GATE(st, need_p);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i];
}

void vec_copy(hipStream_t s, double *y, const double *x, int n)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, s, y, x, n, (const DState *)nullptr, 0);
}

__global__ void k_gather_row(const double *Binv, int ldb, int m, int p, double *rho)
{
    int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l < m) rho[l] = Binv[(size_t)(p - 1) + (size_t)l * ldb];
}

void gather_row(hipStream_t s, const double *Binv, int ldb, int m, int p, double *rho)
{
    hipLaunchKernelGGL(k_gather_row, dim3((m + 255) / 256), dim3(256), 0, s, Binv, ldb, m, p, rho);
}

__global__ void k_cb(int m, const int *head, const double *coef, double *cB, const DState *st, int need_p)
{
    GATE(st, need_p);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) cB[i] = coef[head[i] - 1];
}

void cb_vector(hipStream_t s, int m, const int *head, const double *coef, double *cB, const DState *st, int need_p)
{
    hipLaunchKernelGGL(k_cb, dim3((m + 255) / 256), dim3(256), 0, s, m, head, coef, cB, st, need_p);
}


// w[j] = -xN[j] for the non-basic positions (eval_beta, glpspx01.js:483-505)
__global__ void k_neg_xn(int m, int n, const int *head, const signed char *stat, const double *lb, const double *ub,
                         double *w)
{
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    int k = head[m + j];
    w[j] = -get_xN(stat, lb, ub, k, j + 1);
}

// eval_beta's two right-hand sides split into the slack part ys[m] and the
// structural weights wc[n] in one gather over the variables (instead of two
// fills and a scatter over the positions): variable k at position pos =
// bind[k] contributes
//   mode 0 (h = -N xN):  -xN(pos - m) when pos > m, else 0
//   mode 1 (B beta):      beta[pos - 1] when pos <= m, else 0
__global__ void k_split_pos(int m, int n, int mode, const int *__restrict__ bind, const signed char *__restrict__ stat,
                            const double *__restrict__ lb, const double *__restrict__ ub,
                            const double *__restrict__ beta, double *__restrict__ ys, double *__restrict__ wc,
                            const DState *st, int need_p)
{
    GATE(st, need_p);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;          // variable k + 1
    if (k >= m + n) return;
    const int pos = bind[k];
    double v = 0.0;
    if (mode == 0) {
        if (pos > m) v = -get_xN(stat, lb, ub, k + 1, pos - m);
    } else if (pos <= m)
        v = beta[pos - 1];
    if (k < m) ys[k] = v;
    else wc[k - m] = v;
}

void split_pos(hipStream_t s, const SpxDev &d, int mode, const double *beta, double *ys, double *wc, const DState *st,
               int need_p)
{
    const int N = d.m + d.n;
    hipLaunchKernelGGL(k_split_pos, dim3((N + 255) / 256), dim3(256), 0, s, d.m, d.n, mode, d.bind, d.stat, d.lb, d.ub,
                       beta, ys, wc, st, need_p);
}

void neg_xn_weights(hipStream_t s, const SpxDev &d, double *w)
{
    hipLaunchKernelGGL(k_neg_xn, dim3((d.n + 255) / 256), dim3(256), 0, s, d.m, d.n, d.head, d.stat, d.lb, d.ub, w);
}


__global__ void __launch_bounds__(WG) k_reset_refsp(SpxDev d, int dual) { reset_refsp_dev(d, dual); }

void launch_reset_refsp(hipStream_t s, const SpxDev &d, int dual)
{
    hipLaunchKernelGGL(k_reset_refsp, dim3(1), dim3(WG), 0, s, d, dual);
}


// =====================================================================
// rank-1 update of inv(B) plus the end-of-pivot bookkeeping
// (update_B + change_basis, glpspx02.js:1954-1964 / glpspx01.js:2035-2055)
// =====================================================================
__device__ void finish_pivot(SpxDev &d, int dual)
{
    DState *st = d.st;
    const int m = d.m, p = st->p, q = st->q;
    if (p > 0) {
        const int kp = d.head[p - 1];
        const int kq = d.head[m + q - 1];
        if (dual && st->pricing == PT_PSE && d.type[kp - 1] == FX && d.refsp[kp - 1]) d.refsp[kp - 1] = 0;
        d.head[p - 1] = kq;
        d.head[m + q - 1] = kp;
        d.bind[kq - 1] = p;
        d.bind[kp - 1] = m + q;
        if (dual) {
            if (d.type[kp - 1] == FX) d.stat[q - 1] = NS;
            else if (st->delta > 0.0) d.stat[q - 1] = NL;
            else d.stat[q - 1] = NU;
        } else {
            d.stat[q - 1] = (signed char)st->p_stat;
        }
        if (st->pricing == PT_PSE && st->refct > 0) st->refct--;
        st->upd_cnt++;
        st->binv_fresh = 0;
        st->cbar_fresh = 0;
        if (st->upd_cnt >= st->upd_lim) st->refact_pending = 1;
    } else {
        // xN[q] goes to its opposite bound
        const int sq = d.stat[q - 1];
        d.stat[q - 1] = (sq == NL) ? NU : NL;
    }
    st->it_cnt++;
    st->npiv++;
    st->iter_left--;
    if (st->rigorous > 0) st->rigorous--;
}

__global__ void __launch_bounds__(256) k_binv_update(SpxDev d, int dual)
{
    DState *st = d.st;
    if (st->stop) return;
    const int p = st->p;
    if (p <= 0) {
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) finish_pivot(d, dual);
        return;
    }
    const int m = d.m;
    const double tp = d.tcol[p - 1];
    const int r = (blockIdx.x * 256 + threadIdx.x) * 2;
    const int cps = (m + gridDim.y - 1) / gridDim.y;
    const int c0 = blockIdx.y * cps, c1 = min(m, c0 + cps);
    if (r < m) {
        const bool two = (r + 1 < m);
        // f_i = tcol_i / tcol_p for i != p, 1 / tcol_p for i == p (row p becomes rho / alpha_p)
        const double f0 = (r == p - 1) ? 1.0 / tp : d.tcol[r] / tp;
        const double f1 = two ? ((r + 1 == p - 1) ? 1.0 / tp : d.tcol[r + 1] / tp) : 0.0;
        const bool z0 = (r == p - 1), z1 = (r + 1 == p - 1);
        const int ce = st->ce;
        for (int c = c0; c < c1; ++c) {
            const double rl = d.rowp[c];
            double *ptr = d.Binv + (size_t)c * d.ldb + r;
            if (c == ce) {            // an entering slack's column is exactly e_p
                ptr[0] = z0 ? 1.0 : 0.0;
                if (two) ptr[1] = z1 ? 1.0 : 0.0;
                continue;
            }
            if (two) {
                double2 v = *(double2 *)ptr;
                v.x = (z0 ? 0.0 : v.x) - f0 * rl;
                v.y = (z1 ? 0.0 : v.y) - f1 * rl;
                *(double2 *)ptr = v;
            } else {
                ptr[0] = (z0 ? 0.0 : ptr[0]) - f0 * rl;
            }
        }
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) finish_pivot(d, dual);
}

static dim3 binv_grid(int m)
{
    int tiles = (m + 511) / 512;
    int chunks = std::max(1, std::min((m + 7) / 8, 2048 / tiles));
    return dim3(tiles, chunks);
}

__global__ void __launch_bounds__(256) k_rank1_plain(double *Binv, int m, int ldb, const double *rho,
                                                       const double *tcol, int p)
{
    const double tp = tcol[p - 1];
    const int r = blockIdx.x * 256 + threadIdx.x;
    const int cps = (m + gridDim.y - 1) / gridDim.y;
    const int c0 = blockIdx.y * cps, c1 = min(m, c0 + cps);
    if (r >= m) return;
    const double f = (r == p - 1) ? 1.0 / tp : tcol[r] / tp;
    for (int c = c0; c < c1; ++c) {
        double *ptr = Binv + (size_t)c * ldb + r;
        *ptr = ((r == p - 1) ? 0.0 : *ptr) - f * rho[c];
    }
}

void binv_rank1(hipStream_t s, double *Binv, int m, int ldb, const double *rho, const double *tcol, int p)
{
    int tiles = (m + 255) / 256;
    int chunks = std::max(1, std::min((m + 7) / 8, 2048 / tiles));
    hipLaunchKernelGGL(k_rank1_plain, dim3(tiles, chunks), dim3(256), 0, s, Binv, m, ldb, rho, tcol, p);
}


// ---- gated helpers for the rigorous-mode refinements ----------------------
__global__ void k_gfill(double *x, double v, int n, const DState *st, int need_p)
{
    GATE(st, need_p);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = v;
}

__global__ void k_unit_p(double *x, int m, const DState *st)
{
    GATE(st, 1);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) x[i] = (i == st->p - 1) ? 1.0 : 0.0;
}

// y = a - y
__global__ void k_rsub(double *y, const double *a, int n, const DState *st, int need_p)
{
    GATE(st, need_p);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = a[i] - y[i];
}

__global__ void k_gscatter(int m, int off, int cnt, const int *__restrict__ head, const double *__restrict__ w,
                           double *ys, double *wc, const DState *st, int need_p)
{
    GATE(st, need_p);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    const int k = head[off + i];
    const double v = w[i];
    if (k <= m) ys[k - 1] += v;
    else wc[k - m - 1] = v;
}

static inline dim3 g1(int n) { return dim3((std::max(n, 1) + 255) / 256); }

// refine_tcol (glpspx01.js:732 / glpspx02.js:979): tcol += inv(B) (h - B tcol)
void refine_tcol_dev(hipStream_t s, const SpxDev &d, int need_p)
{
    const int m = d.m, n = d.n;
    hipLaunchKernelGGL(k_gfill, g1(m), dim3(256), 0, s, d.r1, 0.0, m, d.st, need_p);
    hipLaunchKernelGGL(k_gfill, g1(n), dim3(256), 0, s, d.wcol, 0.0, n, d.st, need_p);
    hipLaunchKernelGGL(k_gscatter, g1(m), dim3(256), 0, s, m, 0, m, d.head, d.tcol, d.r1, d.wcol, d.st, need_p);
    aprod_neg_gated(s, d.A, d.wcol, d.r1, d.r2, d.partial, d.partial_cap, d.st, need_p);   // r2 = B tcol
    hipLaunchKernelGGL(k_rsub, g1(m), dim3(256), 0, s, d.r2, d.h, m, d.st, need_p);          // r2 = h - B tcol
    gemv_n_gated(s, d.Binv, m, m, d.ldb, d.r2, d.partial, d.partial_cap, d.r1, 1.0, nullptr, 0.0, d.st, need_p);
    hipLaunchKernelGGL(k_axpy, g1(m), dim3(256), 0, s, d.tcol, d.r1, 1.0, m, d.st, need_p);
}

// refine_rho (glpspx01.js:1044 / glpspx02.js:641): rho += inv(B') (e_p - B' rho)
void refine_rho_dev(hipStream_t s, const SpxDev &d)
{
    const int m = d.m;
    hipLaunchKernelGGL(k_unit_p, g1(m), dim3(256), 0, s, d.r2, m, d.st);
    colpass_gated(s, d.A, CP_RESID, 0, m, d.head, d.stat, d.coef, d.r2, d.rho, nullptr, d.r1, nullptr, nullptr, d.st, 1);
    gemv_t_gated(s, d.Binv, m, m, d.ldb, d.r1, d.r2, 1.0, d.st, 1);
    hipLaunchKernelGGL(k_axpy, g1(m), dim3(256), 0, s, d.rho, d.r2, 1.0, m, d.st, 1);
}

// =====================================================================
// primal simplex pivot (glpspx01.js main loop :1705-2056)
// =====================================================================
__global__ void __launch_bounds__(WG) k_primal_top(SpxDev d)
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
    if (st->pricing == PT_PSE && st->refct == 0) reset_refsp_dev(d, 0);
    if (st->phase == 1) {
        // check_feas (:1483): still some basic variable violating its bound?
        const double tol = st->tol_bnd;
        int bad = 0;
        for (int i = threadIdx.x; i < m && !bad; i += blockDim.x) {
            const int k = d.head[i];
            const double cf = d.coef[k - 1];
            if (cf < 0.0) {
                const double eps = tol * (1.0 + 0.10 * fabs(d.lb[k - 1]));
                if (d.bbar[i] < d.lb[k - 1] - eps) bad = 1;
            } else if (cf > 0.0) {
                const double eps = tol * (1.0 + 0.10 * fabs(d.ub[k - 1]));
                if (d.bbar[i] > d.ub[k - 1] + eps) bad = 1;
            }
        }
        if (!block_or(bad, shi)) {
            if (threadIdx.x == 0) st->stop = ST_PHASE;
            return;
        }
    }
    // chuzc (:646)
    const double tol_dj = st->tol_dj;
    Cand c; c.k1 = 0.0; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const double dj = d.cbar[j];
        const int sj = d.stat[j];
        if (sj == NL) { if (dj >= -tol_dj) continue; }
        else if (sj == NU) { if (dj <= +tol_dj) continue; }
        else if (sj == NF) { if (-tol_dj <= dj && dj <= +tol_dj) continue; }
        else continue;
        const double temp = (dj * dj) / d.gamma[j];
        Cand e; e.k1 = temp; e.k2 = 0.0; e.idx = j + 1; e.aux = 0;
        if (temp > 0.0 && better<0>(e, c)) c = e;
    }
    Cand best = block_best<0>(c, shc);
    if (best.idx == 0) {
        if (threadIdx.x == 0) { st->q = 0; st->stop = ST_Q0; }
        return;
    }
    build_hq(d, best.idx);
    if (threadIdx.x == 0) {
        st->q = best.idx;
        st->tcol_max_bits = 0ull;
    }
}

// sort_tcol (:773), d1/d2 accuracy check (:1901-1919), chuzr (:808) and the
// set-up of rho and of the PSE vector for the pivot row pass
__global__ void __launch_bounds__(WG) k_primal_chuzr(SpxDev d)
{
    __shared__ double shd[16];
    __shared__ Cand shc[16];
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, q = st->q, phase = st->phase;
    double mx = 0.0, dsum = 0.0;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const double t = d.tcol[i];
        mx = fmax(mx, fabs(t));
        if (t != 0.0) dsum += d.coef[d.head[i] - 1] * t;
    }
    const double big = block_max(mx, shd);
    dsum = block_sum(dsum, shd);
    const int kq = d.head[m + q - 1];
    const double d1 = d.cbar[q - 1];
    const double d2 = d.coef[kq - 1] + dsum;
    if (fabs(d1 - d2) > 1e-5 * (1.0 + fabs(d2)) || !((d1 < 0.0 && d2 < 0.0) || (d1 > 0.0 && d2 > 0.0))) {
        if (!st->cbar_fresh || !st->rigorous) {
            __syncthreads();
            if (threadIdx.x == 0) st->stop = ST_DCHK;
            return;
        }
    }
    const double cq = (d1 > 0.0) ? (d2 > 0.0 ? d2 : +DBL_EPS) : (d2 < 0.0 ? d2 : -DBL_EPS);
    __syncthreads();
    if (threadIdx.x == 0) d.cbar[q - 1] = cq;
    const double eps = st->tol_piv * (1.0 + 0.01 * big);
    const double rtol = (st->rtest == RT_HAR) ? 0.30 * st->tol_bnd : 0.0;
    const double s = (cq > 0.0 ? -1.0 : +1.0);
    // first pass, starting from the opposite bound of xN[q] if it has one
    int p0; double teta0, big0;
    if (d.type[kq - 1] == DB) { p0 = -1; teta0 = d.ub[kq - 1] - d.lb[kq - 1]; big0 = 1.0; }
    else { p0 = 0; teta0 = DBL_MAX; big0 = 0.0; }
    Cand c; c.k1 = DBL_MAX; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const double tv = d.tcol[i];
        if (tv == 0.0 || fabs(tv) < eps) continue;
        const int k = d.head[i];
        const int tk = d.type[k - 1];
        const double ck = d.coef[k - 1];
        const double alfa = s * tv;
        double t; int ist;
        if (alfa > 0.0) {
            if (phase == 1 && ck < 0.0) {
                const double dl = rtol * (1.0 + 0.10 * fabs(d.lb[k - 1]));
                t = ((d.lb[k - 1] + dl) - d.bbar[i]) / alfa; ist = NL;
            } else if (phase == 1 && ck > 0.0) continue;
            else if (tk == UP || tk == DB || tk == FX) {
                const double dl = rtol * (1.0 + 0.10 * fabs(d.ub[k - 1]));
                t = ((d.ub[k - 1] + dl) - d.bbar[i]) / alfa; ist = NU;
            } else continue;
        } else {
            if (phase == 1 && ck > 0.0) {
                const double dl = rtol * (1.0 + 0.10 * fabs(d.ub[k - 1]));
                t = ((d.ub[k - 1] - dl) - d.bbar[i]) / alfa; ist = NU;
            } else if (phase == 1 && ck < 0.0) continue;
            else if (tk == LO || tk == DB || tk == FX) {
                const double dl = rtol * (1.0 + 0.10 * fabs(d.lb[k - 1]));
                t = ((d.lb[k - 1] - dl) - d.bbar[i]) / alfa; ist = NL;
            } else continue;
        }
        if (t < 0.0) t = 0.0;
        Cand e; e.k1 = t; e.k2 = fabs(alfa); e.idx = i + 1; e.aux = ist;
        if (better<1>(e, c)) c = e;
    }
    Cand b1 = block_best<1>(c, shc);
    int p = p0, p_stat = 0;
    double teta = teta0;
    if (b1.idx != 0 && (b1.k1 < teta0 || (b1.k1 == teta0 && b1.k2 > big0))) {
        p = b1.idx; p_stat = b1.aux; teta = b1.k1;
    }
    if (!(rtol == 0.0 || p <= 0 || teta == 0.0)) {
        const double tmax = teta;
        Cand c2; c2.k1 = 0.0; c2.k2 = 0.0; c2.idx = 0; c2.aux = 0;
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            const double tv = d.tcol[i];
            if (tv == 0.0 || fabs(tv) < eps) continue;
            const int k = d.head[i];
            const int tk = d.type[k - 1];
            const double ck = d.coef[k - 1];
            const double alfa = s * tv;
            double t; int ist;
            if (alfa > 0.0) {
                if (phase == 1 && ck < 0.0) { t = (d.lb[k - 1] - d.bbar[i]) / alfa; ist = NL; }
                else if (phase == 1 && ck > 0.0) continue;
                else if (tk == UP || tk == DB || tk == FX) { t = (d.ub[k - 1] - d.bbar[i]) / alfa; ist = NU; }
                else continue;
            } else {
                if (phase == 1 && ck > 0.0) { t = (d.ub[k - 1] - d.bbar[i]) / alfa; ist = NU; }
                else if (phase == 1 && ck < 0.0) continue;
                else if (tk == LO || tk == DB || tk == FX) { t = (d.lb[k - 1] - d.bbar[i]) / alfa; ist = NL; }
                else continue;
            }
            if (t < 0.0) t = 0.0;
            if (!(t <= tmax)) continue;
            Cand e; e.k1 = t; e.k2 = fabs(alfa); e.idx = i + 1; e.aux = ist;
            if (better<2>(e, c2)) c2 = e;
        }
        Cand b2 = block_best<2>(c2, shc);
        p = b2.idx; p_stat = b2.aux; teta = b2.k1;
    }
    if (p == 0) {
        if (threadIdx.x == 0) { st->p = 0; st->stop = ST_P0; }
        return;
    }
    if (p > 0 && d.type[d.head[p - 1] - 1] == FX) p_stat = NS;
    if (p > 0 && fabs(d.tcol[p - 1]) < 1e-5 * (1.0 + 0.01 * big) && !st->rigorous) {
        __syncthreads();
        if (threadIdx.x == 0) { st->p = p; st->stop = ST_SMALLPIV; }
        return;
    }
    if (p > 0) {
        for (int l = threadIdx.x; l < m; l += blockDim.x) {
            const double v = d.Binv[(size_t)(p - 1) + (size_t)l * d.ldb];
            d.rho[l] = v;
            d.rowp[l] = v;
        }
        if (st->pricing == PT_PSE && st->refct > 0) {
            // u := tcol restricted to the reference space (update_gamma, :1208-1218)
            double acc = 0.0;
            for (int i = threadIdx.x; i < m; i += blockDim.x) {
                const double t = d.tcol[i];
                const double w = (t != 0.0 && d.refsp[d.head[i] - 1]) ? t : 0.0;
                d.h[i] = w;
                acc += w * w;
            }
            acc = block_sum(acc, shd);
            if (threadIdx.x == 0) {
                const double dq = d.refsp[kq - 1] ? 1.0 : 0.0;
                st->eta_pq = dq;
                st->gamma_pq = dq + acc;
            }
        } else {
            for (int i = threadIdx.x; i < m; i += blockDim.x) d.h[i] = 0.0;
        }
    }
    if (threadIdx.x == 0) {
        st->p = p;
        st->p_stat = p_stat;
        st->teta = s * teta;
        st->tcol_max = big;
    }
}

__global__ void k_primal_pivot(SpxDev d)
{
    DState *st = d.st;
    if (st->stop || threadIdx.x != 0) return;
    const int m = d.m, p = st->p, q = st->q;
    if (p > 0) {
        const double piv1 = d.tcol[p - 1], piv2 = d.trow[q - 1];
        if (fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) || !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0))) {
            if (!st->binv_fresh || !st->rigorous) { st->stop = ST_PIVCHK; return; }
            d.trow[q - 1] = piv1;
        }
    }
    const int kq = d.head[m + q - 1];
    st->xnq = get_xN(d.stat, d.lb, d.ub, kq, q);
    st->ce = (kq <= m) ? kq - 1 : -1;
    if (p > 0) {
        const double pivot = d.trow[q - 1];
        const double new_dq = d.cbar[q - 1] / pivot;
        st->new_dq = new_dq;
        st->pivot = pivot;
        double cq = new_dq;
        if (st->phase == 1) {
            const int kp = d.head[p - 1];
            cq -= d.coef[kp - 1];
            d.coef[kp - 1] = 0.0;
        }
        st->cbar_q_new = cq;
    }
}

// update_bbar (:1100), update_cbar (:1154), update_gamma (:1178)
__global__ void __launch_bounds__(256) k_primal_update(SpxDev d)
{
    DState *st = d.st;
    if (st->stop) return;
    const int m = d.m, n = d.n, p = st->p, q = st->q;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double teta = st->teta;
    if (i < m) {
        if (p > 0 && i == p - 1) d.bbar[i] = st->xnq + teta;
        else if (teta != 0.0) d.bbar[i] += d.tcol[i] * teta;
    }
    if (p > 0 && i < n) {
        const double tr = d.trow[i];
        if (i == q - 1) d.cbar[i] = st->cbar_q_new;
        else if (tr != 0.0) d.cbar[i] -= tr * st->new_dq;
        if (st->pricing == PT_PSE && st->refct > 0) {
            const double pivot = st->pivot;
            if (i == q - 1) {
                double g;
                if (d.type[d.head[p - 1] - 1] == FX) g = 1.0;
                else {
                    g = st->gamma_pq / (pivot * pivot);
                    if (g < DBL_EPS) g = DBL_EPS;
                }
                d.gamma[i] = g;
            } else if (tr != 0.0) {
                const double t = tr / pivot;
                const int k = d.head[m + i];
                const double t1 = d.gamma[i] + t * t * st->gamma_pq + 2.0 * t * d.s[i];
                const double t2 = (d.refsp[k - 1] ? 1.0 : 0.0) + st->eta_pq * t * t;
                double g = (t1 >= t2 ? t1 : t2);
                if (g < DBL_EPS) g = DBL_EPS;
                d.gamma[i] = g;
            }
        }
    }
}

void primal_iteration(hipStream_t s, const SpxDev &d, int pse, int rigorous)
{
    const int m = d.m, n = d.n;
    hipLaunchKernelGGL(k_primal_top, dim3(1), dim3(WG), 0, s, d);
    gemv_n_gated(s, d.Binv, m, m, d.ldb, d.h, d.partial, d.partial_cap, d.tcol, 1.0, nullptr, 0.0, d.st, 0);
    if (rigorous) refine_tcol_dev(s, d, 0);
    hipLaunchKernelGGL(k_primal_chuzr, dim3(1), dim3(WG), 0, s, d);
    if (rigorous) refine_rho_dev(s, d);
    // u = inv(B') (tcol restricted to refsp) (update_gamma's bfd_btran, :1220)
    if (pse) gemv_t_gated(s, d.Binv, m, m, d.ldb, d.h, d.u, 1.0, d.st, 1);
    // trow = -rho N and s = N' u in one pass over A (eval_trow :1058 + update_gamma :1230-1241)
    colpass_gated(s, d.A, CP_TROW_S, m, n, d.head, d.stat, d.coef, nullptr, d.rho, d.u, d.trow, d.s, nullptr, d.st, 1);
    hipLaunchKernelGGL(k_primal_pivot, dim3(1), dim3(64), 0, s, d);
    int g = (std::max(m, n) + 255) / 256;
    hipLaunchKernelGGL(k_primal_update, dim3(g), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_binv_update, binv_grid(m), dim3(256), 0, s, d, 0);
}

// =====================================================================
// re-inversion: inv(B) from the k x k block C = B[R, J] of the structural
// basic columns and the slack-covered rows S
// =====================================================================
__global__ void k_set_identity(double *M, int m, int ld)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) M[(size_t)i + (size_t)i * ld] = 1.0;
}

void set_identity(hipStream_t s, double *M, int m, int ld)
{
    fill_d(s, M, 0.0, (size_t)ld * m);
    hipLaunchKernelGGL(k_set_identity, dim3((m + 255) / 256), dim3(256), 0, s, M, m, ld);
}

// dense A: C[a + b k] = -A[rowR[a], colJ[b]], BS[s + b ms] = -A[rowS[s], colJ[b]]
__global__ void k_gather_dense(const double *A, int lda, int k, const int *colsJ, const int *rowR, double *C,
                               int ms, const int *rowS, double *BS)
{
    const int b = blockIdx.y;
    const double *col = A + (size_t)(colsJ[b] - 1) * lda;
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < k + ms; a += gridDim.x * blockDim.x) {
        if (a < k) C[(size_t)a + (size_t)b * k] = -col[rowR[a] - 1];
        else BS[(size_t)(a - k) + (size_t)b * ms] = -col[rowS[a - k] - 1];
    }
}

// CSC columns of B (values as in B): scatter into zeroed C / BS through rowmap
__global__ void k_gather_csc(int k, const int *bptr, const int *brow, const double *bval, const int *rowmap,
                             double *C, double *BS, int ms, double sign)
{
    const int b = blockIdx.x;
    for (int t = bptr[b] + threadIdx.x; t < bptr[b + 1]; t += blockDim.x) {
        const int r = brow[t];              // 0-based row
        const int a = rowmap[r];
        const double v = sign * bval[t];
        if (a >= 0) C[(size_t)a + (size_t)b * k] = v;
        else BS[(size_t)(-a - 1) + (size_t)b * ms] = v;
    }
}

void gather_basis_blocks(hipStream_t s, const MatDev &A, int m, int k, const int *colsJ, const int *rowR, double *C,
                         double *BS, int ms, const int *rowS)
{
    (void)m;
    if (k <= 0) return;
    dim3 g(std::max(1, std::min((k + ms + 255) / 256, 64)), k);
    hipLaunchKernelGGL(k_gather_dense, g, dim3(256), 0, s, A.A, A.lda, k, colsJ, rowR, C, ms, rowS, BS);
}

void gather_basis_blocks_csc(hipStream_t s, int m, int k, const int *bptr, const int *brow, const double *bval,
                             const int *rowmap, const int *unused, const int *unused2, double *C, double *BS, int ms)
{
    (void)m; (void)unused; (void)unused2;
    if (k <= 0) return;
    fill_d(s, C, 0.0, (size_t)k * k);
    if (ms > 0) fill_d(s, BS, 0.0, (size_t)ms * k);
    hipLaunchKernelGGL(k_gather_csc, dim3(k), dim3(64), 0, s, k, bptr, brow, bval, rowmap, C, BS, ms, 1.0);
}

// one Gauss–Jordan step on [C | I] (k x 2k, column-major), reading X and
// writing Y; every block finds the same pivot row (partial pivoting over
// rows not pivoted before step t, lowest row on ties)
__global__ void __launch_bounds__(256) k_gj_step(const double *__restrict__ X, double *__restrict__ Y, int k, int t,
                                                   int *piv_step, int *piv, int *flag, double tiny, int cpb)
{
    __shared__ Cand shc[16];
    if (*flag) return;
    const double *colt = X + (size_t)t * k;
    Cand c; c.k1 = 0.0; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    for (int r = threadIdx.x; r < k; r += blockDim.x) {
        if (piv_step[r] < t) continue;
        const double v = fabs(colt[r]);
        Cand e; e.k1 = v; e.k2 = 0.0; e.idx = r + 1; e.aux = 0;
        if (v > 0.0 && better<0>(e, c)) c = e;
    }
    Cand b = block_best<0>(c, shc);
    if (b.idx == 0 || b.k1 <= tiny) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *flag = 1 + t;
        return;
    }
    const int rs = b.idx - 1;
    const double pv = colt[rs];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        piv[t] = rs;
        piv_step[rs] = t;
    }
    const int cbeg = t + blockIdx.x * cpb;
    const int cend = min(2 * k, cbeg + cpb);
    for (int cc = cbeg; cc < cend; ++cc) {
        const double *xc = X + (size_t)cc * k;
        double *yc = Y + (size_t)cc * k;
        const double fr = xc[rs] / pv;
        for (int r = threadIdx.x; r < k; r += blockDim.x) {
            if (r == rs) yc[r] = fr;
            else yc[r] = xc[r] - colt[r] * fr;
        }
    }
}

__global__ void k_gj_init(double *X, const double *C, int k)
{
    size_t n = (size_t)k * 2 * k;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        size_t col = e / k, r = e % k;
        X[e] = (col < (size_t)k) ? C[e] : ((col - k) == r ? 1.0 : 0.0);
    }
}

__global__ void k_int_fill(int *x, int v, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = v;
}

int gauss_jordan(hipStream_t s, double *X, double *Y, int k, int *piv_step, int *piv, int *flag, double tiny,
                 double **result)
{
    // X holds C (k x k) on entry in its first k*k slots; Y is scratch of 2k^2
    hipLaunchKernelGGL(k_gj_init, dim3(std::min<size_t>(((size_t)2 * k * k + 255) / 256, 16384)), dim3(256), 0, s, Y, X, k);
    hipLaunchKernelGGL(k_int_fill, dim3((k + 255) / 256), dim3(256), 0, s, piv_step, 0x7fffffff, k);
    (void)hipMemsetAsync(flag, 0, sizeof(int), s);
    double *in = Y, *out = X;
    const int cpb = 8;
    for (int t = 0; t < k; ++t) {
        int ncols = 2 * k - t;
        int blocks = (ncols + cpb - 1) / cpb;
        hipLaunchKernelGGL(k_gj_step, dim3(blocks), dim3(256), 0, s, in, out, k, t, piv_step, piv, flag, tiny, cpb);
        std::swap(in, out);
    }
    *result = in;   // last written buffer
    return k;
}

// CinvR[b*k + a] = right half row piv[b], column a
__global__ void k_extract_inv(const double *X, int k, const int *piv, double *CinvR)
{
    const int b = blockIdx.y;
    const int r = piv[b];
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < k; a += gridDim.x * blockDim.x)
        CinvR[(size_t)b * k + a] = X[(size_t)r + (size_t)(k + a) * k];
}

void extract_inverse_rowmajor(hipStream_t s, const double *X, int k, const int *piv, double *CinvR)
{
    if (k <= 0) return;
    dim3 g(std::max(1, std::min((k + 255) / 256, 16)), k);
    hipLaunchKernelGGL(k_extract_inv, g, dim3(256), 0, s, X, k, piv, CinvR);
}

// G (ms x k col-major) = BS (ms x k col-major) * CinvR (k x k row-major).
// FMA version: 64x64 tiles, 256 threads x (4 x 4) outputs, K step 16.
__global__ void __launch_bounds__(256) k_gemm_fma(const double *__restrict__ BS, int ms, int k,
                                                    const double *__restrict__ Bm, double *__restrict__ G)
{
    __shared__ double As[16][64 + 1];
    __shared__ double Bs[16][64 + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int row0 = blockIdx.x * 64, col0 = blockIdx.y * 64;
    double acc[4][4] = {};
    for (int kk = 0; kk < k; kk += 16) {
        for (int e = threadIdx.x; e < 16 * 64; e += 256) {
            const int kr = e / 64, rr = e % 64;
            const int gr = row0 + rr, gk = kk + kr, gc = col0 + rr;
            As[kr][rr] = (gr < ms && gk < k) ? BS[(size_t)gr + (size_t)gk * ms] : 0.0;
            Bs[kr][rr] = (gc < k && gk < k) ? Bm[(size_t)gk * k + gc] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            double a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[q][ty * 4 + i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[q][tx * 4 + j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gr = row0 + ty * 4 + i, gc = col0 + tx * 4 + j;
            if (gr < ms && gc < k) G[(size_t)gr + (size_t)gc * ms] = acc[i][j];
        }
}

// MFMA version on v_mfma_f64_16x16x4_f64: one wave computes a 16 x 16 tile,
// four waves per block cover 32 x 32; A/B fragments per lane l:
// A[i = l & 15][kk = l >> 4], B[kk = l >> 4][j = l & 15]; D[(l >> 4) + 4 r][l & 15].
typedef double double4_t __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_gemm_mfma(const double *__restrict__ BS, int ms, int k,
                                                     const double *__restrict__ Bm, double *__restrict__ G)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int row0 = blockIdx.x * 32 + (w & 1) * 16;
    const int col0 = blockIdx.y * 32 + (w >> 1) * 16;
    const int li = lane & 15, lk = lane >> 4;
    double4_t acc = {0.0, 0.0, 0.0, 0.0};
    for (int kk = 0; kk < k; kk += 4) {
        const int gk = kk + lk;
        const int ar = row0 + li, bc = col0 + li;
        const double a = (ar < ms && gk < k) ? BS[(size_t)ar + (size_t)gk * ms] : 0.0;
        const double b = (bc < k && gk < k) ? Bm[(size_t)gk * k + bc] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int gr = row0 + lk + 4 * r, gc = col0 + li;
        if (gr < ms && gc < k) G[(size_t)gr + (size_t)gc * ms] = acc[r];
    }
}

void gemm_bs_cinv(hipStream_t s, const double *BS, int ms, int k, const double *CinvR, double *G, int use_mfma)
{
    if (ms <= 0 || k <= 0) return;
    if (use_mfma) {
        dim3 g((ms + 31) / 32, (k + 31) / 32);
        hipLaunchKernelGGL(k_gemm_mfma, g, dim3(256), 0, s, BS, ms, k, CinvR, G);
    } else {
        dim3 g((ms + 63) / 64, (k + 63) / 64);
        hipLaunchKernelGGL(k_gemm_fma, g, dim3(256), 0, s, BS, ms, k, CinvR, G);
    }
}

// Binv[P_J, R] = inv(C); Binv[P_S, S] = I; Binv[P_S, R] = -G
__global__ void k_assemble_J(double *Binv, int ldb, int k, const int *posJ, const int *rowR, const double *CinvR)
{
    const int b = blockIdx.y;
    const size_t prow = (size_t)(posJ[b] - 1);
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < k; a += gridDim.x * blockDim.x)
        Binv[prow + (size_t)(rowR[a] - 1) * ldb] = CinvR[(size_t)b * k + a];
}

__global__ void k_assemble_S(double *Binv, int ldb, int k, int ms, const int *posS, const int *rowS,
                             const int *rowR, const double *G)
{
    const int sidx = blockIdx.y;
    const size_t prow = (size_t)(posS[sidx] - 1);
    if (blockIdx.x == 0 && threadIdx.x == 0) Binv[prow + (size_t)(rowS[sidx] - 1) * ldb] = 1.0;
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < k; a += gridDim.x * blockDim.x)
        Binv[prow + (size_t)(rowR[a] - 1) * ldb] = -G[(size_t)sidx + (size_t)a * ms];
}

void assemble_binv(hipStream_t s, double *Binv, int m, int ldb, int k, int ms, const int *posJ, const int *rowR,
                   const int *posS, const int *rowS, const double *CinvR, const double *G)
{
    fill_d(s, Binv, 0.0, (size_t)ldb * m);
    if (k > 0) {
        dim3 g(std::max(1, std::min((k + 255) / 256, 16)), k);
        hipLaunchKernelGGL(k_assemble_J, g, dim3(256), 0, s, Binv, ldb, k, posJ, rowR, CinvR);
    }
    if (ms > 0) {
        dim3 g(std::max(1, std::min((k + 255) / 256, 16)), ms);
        hipLaunchKernelGGL(k_assemble_S, g, dim3(256), 0, s, Binv, ldb, k, ms, posS, rowS, rowR, G);
    }
}

}  // namespace gk
