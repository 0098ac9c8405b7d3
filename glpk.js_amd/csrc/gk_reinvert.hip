// Blocked Gauss–Jordan inversion of the structural block C of the basis
// (re-inversion, the device counterpart of bfd_factorize → luf_factorize,
// glpbfd.js:74-103 / glpluf.js:461-812; the reference factorizes B = F·H·V,
// the device keeps inv(B) explicitly).
//
// C (k x k) arrives column-major, i.e. M := C' row-major (M[r * k + c]).
// In-place Gauss–Jordan with partial pivoting on M (rows chosen implicitly,
// never swapped): step t picks the unpivoted row rs with the largest
// |M[rs, t]| (lowest row on ties), and slot t then holds column rs of the
// right half of [M | I], so that at the end
//   inv(M)[b, a] = M[piv[b], piv_step[a]]   (piv_step = inverse of piv).
//
// Blocking (panel of B columns [t0, t0 + b)): one workgroup runs the b steps
// on the panel, k rows held in registers (RPT rows per thread), and leaves
// Q = the transformed panel and R = its pivot rows.  The b steps act on any
// other column x as  x <- x + (Q - E_R) x_R  (every step reads x only at its
// pivot row), so the rest of M takes one rank-b update — an MFMA GEMM
// (v_mfma_f64_16x16x4_f64).  M is double-buffered: the panel kernel and the
// update read M and write M2 (panel columns / the others), so the update
// reads X_R = M[R, :] in place with no race.  2 launches per panel instead
// of one launch per column.
#include "gk_device.h"
#include <cstdlib>
#include <climits>
#include <map>
#include <algorithm>
#include <mutex>
#include <vector>
#include <hip/hip_ext.h>
#include <cstdio>

namespace gk {

constexpr int GJ_NONE = 0x7fffffff;

// The panel: columns [c0, c0 + b) of a row-major buffer with row stride ld
// (M itself, or the outer panel P of the two-level scheme), b = min(B,
// ncols - c0); global step numbers start at tg0.  With xr_cols > 0 the pivot
// rows of the buffer's first xr_cols columns are copied to xr before the
// panel is written back (the inner update's X_R).
template <int NT, int RPT, int B>
__global__ void __launch_bounds__(NT) k_gjb_panel(const double *__restrict__ M, double *__restrict__ M2, int ld,
                                                  int c0, int ncols, double *__restrict__ Qm, int k, int tg0,
                                                  int *__restrict__ piv_step, int *__restrict__ piv,
                                                  int *__restrict__ flag, double tiny, double *__restrict__ xr,
                                                  int xr_cols)
{
    __shared__ Cand shc[NT / 64];
    __shared__ double frs[B];
    __shared__ int rsl[B];
    if (*flag) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int b = min(B, ncols - c0);
    const int t0 = tg0;
    double x[RPT][B];
    bool live[RPT];                      // row owned, and not pivoted yet
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = tid + j * NT;
        live[j] = r < k && piv_step[r] == GJ_NONE;
        const double *row = M + (size_t)r * ld + c0;
#pragma unroll
        for (int c = 0; c < B; ++c) x[j][c] = (r < k && c < b) ? row[c] : 0.0;
    }
    bool dead = false;                   // singular (uniform over the block)
#pragma unroll
    for (int i = 0; i < B; ++i) {
        if (i >= b || dead) continue;
        // pivot row: largest |M[r, t]| over the unpivoted rows, lowest row on ties
        Cand c; c.k1 = 0.0; c.k2 = 0.0; c.idx = 0; c.aux = 0;
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const double v = fabs(x[j][i]);
            if (live[j] && v > 0.0 && (c.idx == 0 || v > c.k1)) {   // rows ascend with j
                c.k1 = v;
                c.idx = tid + j * NT + 1;
            }
        }
        c = wave_best<0>(c);
        if (lane == 0) shc[w] = c;
        __syncthreads();
        Cand e;
        if (lane < NT / 64) e = shc[lane];
        else { e.k1 = 0.0; e.k2 = 0.0; e.idx = 0; e.aux = 0; }
        const Cand best = wave_best<0>(e);
        if (best.idx == 0 || best.k1 <= tiny) {
            if (tid == 0) *flag = 1 + t0 + i;
            dead = true;
            continue;
        }
        const int rs = best.idx - 1;
        // the elementary step: fr = x[rs] / pv (as x[rs] * (1 / pv)),
        // y = x - colt * fr; the new slot i is the right-half column e_rs
        // (fr = 1 / pv).  The owner of row rs publishes fr.
        if (tid == rs % NT) {
            const int jo = rs / NT;
#pragma unroll
            for (int j = 0; j < RPT; ++j)
                if (j == jo) {
                    const double ipv = 1.0 / x[j][i];
#pragma unroll
                    for (int cc = 0; cc < B; ++cc) frs[cc] = (cc == i) ? ipv : x[j][cc] * ipv;
                }
        }
        if (tid == 0) rsl[i] = rs;     // global writes after the loop: a barrier
                                       // would otherwise wait for the stores
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const int r = tid + j * NT;
            if (r == rs) {
#pragma unroll
                for (int cc = 0; cc < B; ++cc) x[j][cc] = frs[cc];
                live[j] = false;
            } else {
                const double colt = x[j][i];
#pragma unroll
                for (int cc = 0; cc < B; ++cc) x[j][cc] = ((cc == i) ? 0.0 : x[j][cc]) - colt * frs[cc];
            }
        }
    }
    if (dead) return;
    if (tid < b) {
        piv[t0 + tid] = rsl[tid];
        piv_step[rsl[tid]] = t0 + tid;
    }
    if (xr_cols > 0) {
        for (int e = tid; e < B * xr_cols; e += NT) {
            const int kk = e / xr_cols, c = e - kk * xr_cols;
            xr[e] = (kk < b) ? M[(size_t)rsl[kk] * ld + c] : 0.0;
        }
        __syncthreads();                 // read before the panel is written back (in place)
    }
    // the panel into M2, Q - E_R for the update
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = tid + j * NT;
        if (r >= k) continue;
        double *row = M2 + (size_t)r * ld + c0;
        double *q = Qm + (size_t)r * B;
#pragma unroll
        for (int c = 0; c < B; ++c) {
            if (c < b) row[c] = x[j][c];
            q[c] = (c < b) ? x[j][c] - (r == rsl[c] ? 1.0 : 0.0) : 0.0;
        }
    }
}

// M2[r, c] = M[r, c] + sum_kk Q[r, kk] M[R[kk], c] for the columns outside
// the panel (R = piv[t0 ..]).
// One block = 64 x 64 outputs, four waves of 32 x 32 (2 x 2 MFMA tiles).
// Fragments of v_mfma_f64_16x16x4_f64 per lane l: A[i = l & 15][kk = l >> 4],
// B[kk = l >> 4][j = l & 15], D[(l >> 4) + 4 r][l & 15].
typedef double gj_double4 __attribute__((ext_vector_type(4)));

template <int B, int SUBE, int QCM = 0>
__global__ void __launch_bounds__(256) k_gjb_update(const double *__restrict__ M, double *__restrict__ M2,
                                                    const double *__restrict__ Qm, int ldq,
                                                    const int *__restrict__ rsl, int k, int t0,
                                                    const int *__restrict__ flag, int cb0, int gap_at, int gap)
{
    if (*flag) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    // column tile: cb0 + blockIdx.x, tiles from gap_at on shifted by gap
    // (the look-ahead schedule updates a column range in two launches)
    int cb = cb0 + (int)blockIdx.x;
    if (cb >= gap_at) cb += gap;
    const int row0 = blockIdx.y * 64 + (w & 1) * 32;
    const int col0 = cb * 64 + (w >> 1) * 32;
    const int b = min(B, k - t0);
    gj_double4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gr = row0 + a * 16 + lk + 4 * r, gc = col0 + bb * 16 + li;
                acc[a][bb][r] = (gr < k && gc < k) ? M[(size_t)gr * k + gc] : 0.0;
            }
#pragma unroll 4
    for (int kk = 0; kk < B; kk += 4) {
        const int gk = kk + lk;
        const int rk = gk < b ? rsl[gk] : -1;
        double av[2], bv[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int gr = row0 + a * 16 + li;
            // Q row-major (ldq >= B) or, QCM, column-major (ldq = k)
            double q = (gr < k && gk < b) ? (QCM ? Qm[(size_t)gk * ldq + gr] : Qm[(size_t)gr * ldq + gk]) : 0.0;
            if (SUBE && gr == rk) q -= 1.0;          // Q - E_R
            av[a] = q;
        }
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int gc = col0 + bb * 16 + li;
            bv[bb] = (gc < k && rk >= 0) ? M[(size_t)rk * k + gc] : 0.0;
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
                acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[bb], acc[a][bb], 0, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gr = row0 + a * 16 + lk + 4 * r, gc = col0 + bb * 16 + li;
                if (gr < k && gc < k && (gc < t0 || gc >= t0 + b)) M2[(size_t)gr * k + gc] = acc[a][bb][r];
            }
}

// ---------------------------------------------------------------------------
// two-level scheme (large k, narrow register panels): an outer panel of
// BO = 64 columns is copied to P (k x 64), factored by inner panels of B
// columns, each followed by a rank-B update of the other columns of P only
// (k_gjb_inner); the rest of M then takes one rank-64 update with
// Q = P - E_R (k_gjb_update<64, 1>): the same arithmetic as the one-level
// scheme regrouped, M streamed k / 64 times instead of k / B.
// ---------------------------------------------------------------------------
constexpr int GJ_BO = 64;

__global__ void __launch_bounds__(256) k_gjb_copy(const double *__restrict__ src, int lds, int cs,
                                                  double *__restrict__ dst, int ldd, int cd, int k, int bo,
                                                  const int *__restrict__ flag)
{
    if (*flag) return;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), c = threadIdx.x & 63;
    if (r < k && c < bo) dst[(size_t)r * ldd + cd + c] = src[(size_t)r * lds + cs + c];
}

// P[r, j] += sum_kk (Q - E_R)[r, kk] X_R[kk, j] for j outside the inner panel [i0, i0 + b)
template <int B>
__global__ void __launch_bounds__(256) k_gjb_inner(double *__restrict__ P, int bo, int i0, const double *__restrict__ Qm,
                                                   const double *__restrict__ xr, int k, const int *__restrict__ flag)
{
    __shared__ double sx[B * GJ_BO];
    if (*flag) return;
    for (int e = threadIdx.x; e < B * bo; e += 256) sx[(e / bo) * GJ_BO + e % bo] = xr[e];
    __syncthreads();
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), j = threadIdx.x & 63;
    if (r >= k || j >= bo || (j >= i0 && j < i0 + B)) return;
    double acc = P[(size_t)r * GJ_BO + j];
    const double *q = Qm + (size_t)r * B;
#pragma unroll
    for (int kk = 0; kk < B; ++kk) acc += q[kk] * sx[kk * GJ_BO + j];
    P[(size_t)r * GJ_BO + j] = acc;
}

template <int NT, int RPT, int B>
static double *gjb_run(hipStream_t s, double *M, double *M2, double *Qm, int k, int *piv_step, int *piv, int *flag,
                       double tiny)
{
    const dim3 g((k + 63) / 64, (k + 63) / 64);
    for (int t0 = 0; t0 < k; t0 += B) {
        hipLaunchKernelGGL((k_gjb_panel<NT, RPT, B>), dim3(1), dim3(NT), 0, s, M, M2, k, t0, k, Qm, k, t0, piv_step,
                           piv, flag, tiny, (double *)nullptr, 0);
        if (k > B)
            hipLaunchKernelGGL((k_gjb_update<B, 0>), g, dim3(256), 0, s, M, M2, Qm, B, piv + t0, k, t0, flag, 0, INT_MAX, 0);
        std::swap(M, M2);
    }
    return M;
}

template <int NT, int RPT, int B>
static double *gjb_run2(hipStream_t s, double *M, double *M2, double *P, double *Qm, double *xr, int k,
                        int *piv_step, int *piv, int *flag, double tiny)
{
    const dim3 g((k + 63) / 64, (k + 63) / 64);
    const dim3 gr((k + 3) / 4);
    for (int T0 = 0; T0 < k; T0 += GJ_BO) {
        const int bo = std::min(GJ_BO, k - T0);
        hipLaunchKernelGGL(k_gjb_copy, gr, dim3(256), 0, s, M, k, T0, P, GJ_BO, 0, k, bo, flag);
        for (int i0 = 0; i0 < bo; i0 += B) {
            hipLaunchKernelGGL((k_gjb_panel<NT, RPT, B>), dim3(1), dim3(NT), 0, s, P, P, GJ_BO, i0, bo, Qm, k,
                               T0 + i0, piv_step, piv, flag, tiny, xr, bo);
            if (bo > B) hipLaunchKernelGGL((k_gjb_inner<B>), gr, dim3(256), 0, s, P, bo, i0, Qm, xr, k, flag);
        }
        if (k > bo)
            hipLaunchKernelGGL((k_gjb_update<GJ_BO, 1>), g, dim3(256), 0, s, M, M2, P, GJ_BO, piv + T0, k, T0, flag, 0, INT_MAX, 0);
        hipLaunchKernelGGL(k_gjb_copy, gr, dim3(256), 0, s, P, GJ_BO, 0, M2, k, T0, k, bo, flag);
        std::swap(M, M2);
    }
    return M;
}

// ---------------------------------------------------------------------------
// two-level scheme with a column-major outer panel (k > 256): P[c * k + r],
// so every panel load / store and the inner updates are coalesced over rows
// (the row-major panel read 64 scattered lines per wave instruction: one
// workgroup spent 67 us per 8-column panel at k = 4096, 34 ms per
// re-inversion).  Q = the transformed inner panel minus E_R, column-major
// (Q[c * k + r]); X_R = the pivot rows of P's bo columns (B x bo).
// ---------------------------------------------------------------------------
template <int NT, int RPT, int B>
__global__ void __launch_bounds__(NT) k_gjc_panel(double *__restrict__ P, int k, int c0, int bo, int tg0,
                                                  int *__restrict__ piv_step, int *__restrict__ piv,
                                                  int *__restrict__ flag, double tiny, double *__restrict__ xr)
{
    constexpr int NW = NT / 64;
    // per step and wave: the wave's best key and its row's B values,
    // double-buffered by step parity (one barrier per step)
    __shared__ unsigned long long shk[2][NW];
    __shared__ double shr[2][NW][B];
    __shared__ int rsl[B];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int b = min(B, bo - c0);
    // the panel loads go out before the singularity flag of an earlier panel
    // is read (a load tested before the others costs a memory round trip)
    double x[RPT][B];
    bool live[RPT];                      // row owned, and not pivoted yet
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = tid + j * NT;
        const int rc = min(r, k - 1);
        live[j] = r < k && piv_step[rc] == GJ_NONE;
#pragma unroll
        for (int c = 0; c < B; ++c) x[j][c] = (r < k && c < b) ? P[(size_t)(c0 + c) * k + rc] : 0.0;
    }
    if (*flag) return;
    // B steps, the active column always in slot 0: after a step the columns
    // rotate left by one (the transformed pivot column goes to slot B - 1),
    // so after B steps every column is back in its slot (static register
    // indices, the step body a loop).  The candidate of a row is one 64-bit
    // key: the bits of |x| with the low 13 mantissa bits replaced by
    // 8191 - row (k <= 8192), so one unsigned max picks the largest |x| and
    // the lowest row among values equal to 2^-39 relative — partial pivoting
    // up to a tie margin far below any pivot tolerance.  A step: every wave
    // reduces its keys (DPP), its winning lane stores its row's B values in
    // LDS; after the barrier every wave scans the NW keys and forms the
    // multipliers itself.  Per-step cost is instruction issue (every wave
    // repeats the choice), so the panel runs 8 waves, not 16 (tools/
    // ubench_gjpanel.hip: 1.7 us per step at 8 waves x 8 rows against 2.6 us
    // for 16 waves x 4 rows with shuffled row values).
#pragma unroll 1
    for (int i = 0; i < B; ++i) {
        const int par = i & 1;
        if (i >= b) {
            // inactive step (narrow last panel): rotate only
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const double t0 = x[j][0];
#pragma unroll
                for (int cc = 1; cc < B; ++cc) x[j][cc - 1] = x[j][cc];
                x[j][B - 1] = t0;
            }
            continue;
        }
        unsigned long long key = 0;
        int jb = 0;
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const double v = fabs(x[j][0]);
            const unsigned long long kk =
                (live[j] && v > 0.0) ? ((dbits(v) & ~0x1fffull) | (unsigned long long)(0x1fff - (tid + j * NT))) : 0ull;
            if (kk > key) { key = kk; jb = j; }
        }
        const unsigned long long wk = __ockl_wfred_max_u64(key);
        const bool win = wk != 0 && key == wk;           // unique: the key holds the row
#pragma unroll
        for (int j = 0; j < RPT; ++j)
            if (win && j == jb) {
#pragma unroll
                for (int cc = 0; cc < B; ++cc) shr[par][w][cc] = x[j][cc];
            }
        if (lane == 0) shk[par][w] = wk;
        __syncthreads();
        unsigned long long bk = 0;
        int ws = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            const unsigned long long e = shk[par][q];
            if (e > bk) { bk = e; ws = q; }
        }
        const double pv = shr[par][ws][0];
        if (bk == 0 || fabs(pv) <= tiny) {
            if (tid == 0) *flag = 1 + tg0 + i;
            return;                      // uniform: every thread saw the same keys
        }
        const int rs = 0x1fff - (int)(bk & 0x1fff);
        if (tid == 0) rsl[i] = rs;
        const double ipv = 1.0 / pv;
        // the update, rotating left in place: slot 0 (the step's column)
        // goes to slot B - 1; the pivot row is overwritten afterwards by its
        // owner (no per-element select)
        double fr[B];
        fr[0] = ipv;
#pragma unroll
        for (int cc = 1; cc < B; ++cc) fr[cc] = shr[par][ws][cc] * ipv;
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const double colt = x[j][0];
#pragma unroll
            for (int cc = 1; cc < B; ++cc) x[j][cc - 1] = x[j][cc] - colt * fr[cc];
            x[j][B - 1] = -colt * fr[0];
        }
        if ((rs % NT) == tid) {
            const int jo = rs / NT;
#pragma unroll
            for (int j = 0; j < RPT; ++j)
                if (j == jo) {
#pragma unroll
                    for (int cc = 1; cc < B; ++cc) x[j][cc - 1] = fr[cc];
                    x[j][B - 1] = fr[0];
                    live[j] = false;
                }
        }
    }
    __syncthreads();                     // rsl complete
    if (tid < b) {
        piv[tg0 + tid] = rsl[tid];
        piv_step[rsl[tid]] = tg0 + tid;
    }
    // X_R of the columns outside this panel (unchanged by it; a panel column
    // read here races with the write-back below and is never used)
    for (int e = tid; e < B * bo; e += NT) {
        const int kk = e / bo, c = e - kk * bo;
        xr[e] = (kk < b) ? P[(size_t)c * k + rsl[kk]] : 0.0;
    }
    // the panel back into P (k_gjc_inner forms Q = panel - E_R from it)
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = tid + j * NT;
        if (r >= k) continue;
#pragma unroll
        for (int c = 0; c < B; ++c)
            if (c < b) P[(size_t)(c0 + c) * k + r] = x[j][c];
    }
}

// P[j, r] += sum_kk Q[kk, r] X_R[kk, j] for the columns j < bo outside the
// inner panel [i0, i0 + B); one row per thread
template <int B>
__global__ void __launch_bounds__(256) k_gjc_inner(double *__restrict__ P, int bo, int i0,
                                                   const int *__restrict__ pivp, const double *__restrict__ xr, int k,
                                                   const int *__restrict__ flag)
{
    __shared__ double sx[B * GJ_BO];
    if (*flag) return;
    for (int e = threadIdx.x; e < B * bo; e += 256) sx[e] = xr[e];
    const int r = blockIdx.x * 256 + threadIdx.x;
    const int rc = min(r, k - 1);
    const int bi = min(B, bo - i0);
    // Q = the transformed panel columns minus E_R (the unit at the step's
    // pivot row); a column past the panel's width contributes nothing
    double q[B];
#pragma unroll
    for (int kk = 0; kk < B; ++kk) {
        const double pk = P[(size_t)(i0 + min(kk, bi - 1)) * k + rc];
        const int rp = pivp[min(kk, bi - 1)];
        q[kk] = kk < bi ? pk - (rc == rp ? 1.0 : 0.0) : 0.0;
    }
    __syncthreads();
    // 8 columns per thread (blockIdx.y), their loads issued together: one
    // memory round trip per thread
    {
        const int j0 = blockIdx.y * 8;
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = (j0 + u < bo) ? P[(size_t)(j0 + u) * k + rc] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u;
            double acc = a[u];
#pragma unroll
            for (int kk = 0; kk < B; ++kk) acc += q[kk] * sx[kk * bo + min(j, bo - 1)];
            if (r < k && j < bo && !(j >= i0 && j < i0 + B)) P[(size_t)j * k + r] = acc;
        }
    }
}

// the outer panel between M (row-major k x k, columns [T0, T0 + bo)) and P
// (column-major k x bo): 64 x 64 tiles transposed through LDS
template <int IN>
__global__ void __launch_bounds__(256) k_gjc_copy(const double *__restrict__ src, double *__restrict__ dst, int k,
                                                  int T0, int bo, const int *__restrict__ flag)
{
    __shared__ double t[64][65];
    if (*flag) return;
    const int r0 = blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    if (IN) {
        // read rows of M (coalesced over columns), write columns of P
        for (int y = ty; y < 64; y += 4) {
            const int r = r0 + y;
            t[y][tx] = (r < k && tx < bo) ? src[(size_t)r * k + T0 + tx] : 0.0;
        }
        __syncthreads();
        for (int c = ty; c < bo; c += 4) {
            const int r = r0 + tx;
            if (r < k) dst[(size_t)c * k + r] = t[tx][c];
        }
    } else {
        // read columns of P (coalesced over rows), write rows of M
        for (int c = ty; c < 64; c += 4) {
            const int r = r0 + tx;
            t[tx][c] = (r < k && c < bo) ? src[(size_t)c * k + r] : 0.0;
        }
        __syncthreads();
        for (int y = ty; y < 64; y += 4) {
            const int r = r0 + y;
            if (r < k && tx < bo) dst[(size_t)r * k + T0 + tx] = t[y][tx];
        }
    }
}

template <int NT, int RPT, int B>
static double *gjc_run(hipStream_t s, double *M, double *M2, double *P, double *Qm, double *xr, int k,
                       int *piv_step, int *piv, int *flag, double tiny)
{
    const dim3 g((k + 63) / 64, (k + 63) / 64);
    const dim3 gt((k + 63) / 64), gr((k + 255) / 256);
    for (int T0 = 0; T0 < k; T0 += GJ_BO) {
        const int bo = std::min(GJ_BO, k - T0);
        hipLaunchKernelGGL(k_gjc_copy<1>, gt, dim3(256), 0, s, M, P, k, T0, bo, flag);
        for (int i0 = 0; i0 < bo; i0 += B) {
            hipLaunchKernelGGL((k_gjc_panel<NT, RPT, B>), dim3(1), dim3(NT), 0, s, P, k, i0, bo, T0 + i0, piv_step,
                               piv, flag, tiny, xr);
            if (bo > B)
                hipLaunchKernelGGL((k_gjc_inner<B>), dim3(gr.x, (bo + 7) / 8), dim3(256), 0, s, P, bo, i0,
                                   piv + T0 + i0, xr, k, flag);
        }
        if (k > bo)
            hipLaunchKernelGGL((k_gjb_update<GJ_BO, 1, 1>), g, dim3(256), 0, s, M, M2, P, k, piv + T0, k, T0, flag, 0, INT_MAX, 0);
        hipLaunchKernelGGL(k_gjc_copy<0>, gt, dim3(256), 0, s, P, M2, k, T0, bo, flag);
        std::swap(M, M2);
    }
    return M;
}

// The same arithmetic with look-ahead: the one-workgroup panels are the
// critical path, so outer panel T0's rank-64 update is split.  The next
// outer panel's 64 columns are updated first, on s, and copied into the
// other P buffer; the rest of M (every other column, all rows) and the
// write-back of P run on a side stream under the next panel's Gauss–Jordan
// steps.  Every element sees the same operations in the same order as in
// gjc_run, so the inverse is bit-identical.  Hazards: outer panel T0 + 64's
// own next-columns update reads columns written by T0's rest update and
// writes the buffer that update reads, and its copy-in overwrites the P that
// T0's write-back reads, so s waits for the side stream's event of T0 before
// them.
// the critical-path stream (the panels, on GK_GJ_CRIT_CUS compute units,
// default 64) and the side stream (the other CUs), disjoint CU masks so the
// big updates do not share a CU with the one-workgroup panel; three events.
// Owned by the context that re-inverts (gk_ctx, created on its first
// look-ahead re-inversion, destroyed with it) and, until then, recorded in
// a registry that an atexit handler drains: the handles are never left to
// the runtime's own teardown (a process that left CU-masked streams alive
// died in its exit handlers under rocprofv3).
static std::mutex g_side_mu;
static std::vector<GjSide *> *g_sides = nullptr;     // live handles (never freed itself: outlives exit)

static void gj_side_release(GjSide *g)
{
    if (g->crit) (void)hipStreamSynchronize(g->crit);
    if (g->side) (void)hipStreamSynchronize(g->side);
    if (g->ev_in) (void)hipEventDestroy(g->ev_in);
    if (g->ev_main) (void)hipEventDestroy(g->ev_main);
    if (g->ev_side) (void)hipEventDestroy(g->ev_side);
    if (g->crit) (void)hipStreamDestroy(g->crit);
    if (g->side) (void)hipStreamDestroy(g->side);
    *g = GjSide{};
}

static void gj_side_atexit()
{
    std::lock_guard<std::mutex> lk(g_side_mu);
    if (!g_sides) return;
    for (GjSide *g : *g_sides) {
        gj_side_release(g);
        delete g;
    }
    g_sides->clear();
}

GjSide *gj_side_create(int dev)
{
    static const int crit_cus = [] {
        const char *e = std::getenv("GK_GJ_CRIT_CUS");
        return e ? std::atoi(e) : 64;
    }();
    int ncu = 0;
    if (hipSetDevice(dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return nullptr;
    GjSide *g = new GjSide;
    bool ok;
    if (crit_cus > 0 && crit_cus < ncu) {
        const int words = (ncu + 31) / 32;
        std::vector<uint32_t> mc(words, 0u), ms(words, 0u);
        for (int c = 0; c < ncu; ++c) (c < crit_cus ? mc : ms)[c / 32] |= 1u << (c % 32);
        ok = hipExtStreamCreateWithCUMask(&g->crit, words, mc.data()) == hipSuccess &&
             hipExtStreamCreateWithCUMask(&g->side, words, ms.data()) == hipSuccess;
    } else {
        ok = hipStreamCreateWithFlags(&g->crit, hipStreamNonBlocking) == hipSuccess &&
             hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking) == hipSuccess;
    }
    ok = ok && hipEventCreateWithFlags(&g->ev_in, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&g->ev_main, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&g->ev_side, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        fprintf(stderr, "gk re-inversion: look-ahead streams unavailable, single stream\n");
        gj_side_release(g);
        delete g;
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_side_mu);
    if (!g_sides) {
        g_sides = new std::vector<GjSide *>;
        std::atexit(gj_side_atexit);
    }
    g_sides->push_back(g);
    return g;
}

void gj_side_destroy(GjSide *g)
{
    if (!g) return;
    {
        std::lock_guard<std::mutex> lk(g_side_mu);
        if (g_sides) g_sides->erase(std::remove(g_sides->begin(), g_sides->end(), g), g_sides->end());
    }
    gj_side_release(g);
    delete g;
}

// event record / wait on valid handles; a failure is reported, never ignored
#define GJCHK(x)                                                                              \
    do {                                                                                      \
        hipError_t e__ = (x);                                                                 \
        if (e__ != hipSuccess) {                                                              \
            fprintf(stderr, "gk re-inversion: %s failed: %s\n", #x, hipGetErrorString(e__));   \
            abort();                                                                          \
        }                                                                                     \
    } while (0)

template <int NT, int RPT, int B>
static double *gjc_run_la(GjSide &gs, hipStream_t s, double *M, double *M2, double *P0, double *P1, double *xr,
                          int k, int *piv_step, int *piv, int *flag, double tiny)
{
    const hipStream_t s_in = s;
    GJCHK(hipEventRecord(gs.ev_in, s_in));
    s = gs.crit;
    GJCHK(hipStreamWaitEvent(s, gs.ev_in, 0));
    const int nb = (k + 63) / 64;                       // column (and row) tiles
    const dim3 gt(nb), gr((k + 255) / 256);
    double *P[2] = {P0, P1};
    int cur = 0;
    bool side_busy = false;
    hipLaunchKernelGGL(k_gjc_copy<1>, gt, dim3(256), 0, s, M, P[cur], k, 0, std::min(GJ_BO, k), flag);
    for (int T0 = 0; T0 < k; T0 += GJ_BO) {
        const int bo = std::min(GJ_BO, k - T0);
        double *Pc = P[cur];
        for (int i0 = 0; i0 < bo; i0 += B) {
            hipLaunchKernelGGL((k_gjc_panel<NT, RPT, B>), dim3(1), dim3(NT), 0, s, Pc, k, i0, bo, T0 + i0, piv_step,
                               piv, flag, tiny, xr);
            if (bo > B)
                hipLaunchKernelGGL((k_gjc_inner<B>), dim3(gr.x, (bo + 7) / 8), dim3(256), 0, s, Pc, bo, i0,
                                   piv + T0 + i0, xr, k, flag);
        }
        const int tb = T0 / 64;                         // this panel's tile
        if (side_busy) GJCHK(hipStreamWaitEvent(s, gs.ev_side, 0));
        side_busy = false;
        if (T0 + GJ_BO < k) {
            // the next panel's columns first, then its copy into the other P
            hipLaunchKernelGGL((k_gjb_update<GJ_BO, 1, 1>), dim3(1, nb), dim3(256), 0, s, M, M2, Pc, k, piv + T0, k,
                               T0, flag, tb + 1, INT_MAX, 0);
            hipLaunchKernelGGL(k_gjc_copy<1>, gt, dim3(256), 0, s, M2, P[cur ^ 1], k, T0 + GJ_BO,
                               std::min(GJ_BO, k - T0 - GJ_BO), flag);
            // the rest on the side stream: tiles [0, tb) and [tb + 2, nb)
            GJCHK(hipEventRecord(gs.ev_main, s));
            GJCHK(hipStreamWaitEvent(gs.side, gs.ev_main, 0));
            if (nb - 2 > 0)
                hipLaunchKernelGGL((k_gjb_update<GJ_BO, 1, 1>), dim3(nb - 2, nb), dim3(256), 0, gs.side, M, M2, Pc, k,
                                   piv + T0, k, T0, flag, 0, tb, 2);
            hipLaunchKernelGGL(k_gjc_copy<0>, gt, dim3(256), 0, gs.side, Pc, M2, k, T0, bo, flag);
            GJCHK(hipEventRecord(gs.ev_side, gs.side));
            side_busy = true;
        } else {
            // last panel: the other tiles (all before it) and the write-back on s
            if (tb > 0)
                hipLaunchKernelGGL((k_gjb_update<GJ_BO, 1, 1>), dim3(tb, nb), dim3(256), 0, s, M, M2, Pc, k, piv + T0,
                                   k, T0, flag, 0, INT_MAX, 0);
            hipLaunchKernelGGL(k_gjc_copy<0>, gt, dim3(256), 0, s, Pc, M2, k, T0, bo, flag);
        }
        std::swap(M, M2);
        cur ^= 1;
    }
    if (side_busy) GJCHK(hipStreamWaitEvent(s_in, gs.ev_side, 0));
    GJCHK(hipEventRecord(gs.ev_main, s));
    GJCHK(hipStreamWaitEvent(s_in, gs.ev_main, 0));
    return M;
}

__global__ void k_gjb_init(int *piv_step, int k, int *flag)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x) piv_step[i] = GJ_NONE;
    if (blockIdx.x == 0 && threadIdx.x == 0) *flag = 0;
}

int gj_blocked_max() { return 8192; }

// whether a re-inversion of order k runs the look-ahead schedule:
// GK_GJ_LOOKAHEAD=0 never, 2 every k, default (1) k > 2048
bool gj_lookahead(int k)
{
    static const int la = [] {
        const char *e = std::getenv("GK_GJ_LOOKAHEAD");
        return e ? std::atoi(e) : 1;
    }();
    return la > 1 || (la == 1 && k > 2048);
}

size_t gj_blocked_scratch(int k)
{
    // Q (k x B, B <= 32), the outer panel P (k x 64), X_R (32 x 64), the
    // look-ahead's second outer panel (k x 64)
    return (size_t)32 * k + (size_t)GJ_BO * k + 32 * GJ_BO + (size_t)GJ_BO * k;
}

// inverse of C (k x k, column-major in X[0, k^2)) by the blocked scheme
// above; X must hold 2 k^2 doubles (the second buffer of M), scratch
// gj_blocked_scratch(k); returns the buffer holding the result.  BFD_ESING
// is reported through *flag (1 + step).
double *gauss_jordan_blocked(hipStream_t s, double *X, double *scratch, int k, int *piv_step, int *piv, int *flag,
                             double tiny, GjSide *side)
{
    if (k <= 0) return X;
    hipLaunchKernelGGL(k_gjb_init, dim3(std::min((k + 255) / 256, 64)), dim3(256), 0, s, piv_step, k, flag);
    double *M2 = X + (size_t)k * k, *Qm = scratch, *P = scratch + (size_t)32 * k, *xr = P + (size_t)GJ_BO * k;
    // registers: RPT * B doubles of the panel per thread (1 / 2 / 4 waves per
    // SIMD); beyond 1024 the two-level scheme streams M once per 64 columns
    static const int rowmajor = [] {
        const char *e = std::getenv("GK_GJ_ROWMAJOR");   // the row-major two-level panels (experiments)
        return e ? std::atoi(e) : 0;
    }();
    if (k <= 256) return gjb_run<256, 1, 16>(s, X, M2, Qm, k, piv_step, piv, flag, tiny);
    if (rowmajor) {
        if (k <= 512) return gjb_run<256, 2, 16>(s, X, M2, Qm, k, piv_step, piv, flag, tiny);
        if (k <= 1024) return gjb_run<512, 2, 16>(s, X, M2, Qm, k, piv_step, piv, flag, tiny);
        if (k <= 2048) return gjb_run2<1024, 2, 16>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
        if (k <= 4096) return gjb_run2<1024, 4, 8>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
        return gjb_run2<1024, 8, 4>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
    }
    // look-ahead when the caller passes the side streams (gj_lookahead:
    // k > 2048 by default; k = 4096: 21.3 -> 19.8 ms; k = 2048: no gain, the
    // panels slow down by what the hidden updates save)
    double *P1 = xr + 32 * GJ_BO;
    if (side) {
        if (k <= 1024) return gjc_run_la<512, 2, 16>(*side, s, X, M2, P, P1, xr, k, piv_step, piv, flag, tiny);
        if (k <= 2048) return gjc_run_la<512, 4, 16>(*side, s, X, M2, P, P1, xr, k, piv_step, piv, flag, tiny);
        if (k <= 4096) return gjc_run_la<512, 8, 8>(*side, s, X, M2, P, P1, xr, k, piv_step, piv, flag, tiny);
        return gjc_run_la<1024, 8, 4>(*side, s, X, M2, P, P1, xr, k, piv_step, piv, flag, tiny);
    }
    if (k <= 1024) return gjc_run<512, 2, 16>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
    if (k <= 2048) return gjc_run<512, 4, 16>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
    if (k <= 4096) return gjc_run<512, 8, 8>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
    return gjc_run<1024, 8, 4>(s, X, M2, P, Qm, xr, k, piv_step, piv, flag, tiny);
}

// CinvR (row-major inv(C)): with M = C' inverted in place,
// inv(C)[a, b] = inv(M)[b, a] = M[piv[b], piv_step[a]]
__global__ void k_gjb_extract(const double *__restrict__ M, int k, const int *__restrict__ piv,
                              const int *__restrict__ piv_step, double *__restrict__ CinvR)
{
    const int a = blockIdx.y;
    const size_t col = (size_t)piv_step[a];
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < k; b += gridDim.x * blockDim.x)
        CinvR[(size_t)a * k + b] = M[(size_t)piv[b] * k + col];
}

void extract_inverse_blocked(hipStream_t s, const double *M, int k, const int *piv, const int *piv_step,
                             double *CinvR)
{
    if (k <= 0) return;
    dim3 g(std::max(1, std::min((k + 255) / 256, 16)), k);
    hipLaunchKernelGGL(k_gjb_extract, g, dim3(256), 0, s, M, k, piv, piv_step, CinvR);
}

}  // namespace gk
