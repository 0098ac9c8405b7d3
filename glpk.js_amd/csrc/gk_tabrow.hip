// glp_eval_tab_row (glpapi12.js:401-451) for a batch of basic variables:
// row i_t of the simplex tableau for each requested x[k_t] (i_t its basis
// position),
//   alfa[t, j]  = (rho_t' A)_j          structural j non-basic,
//   alfa[t, k]  = -rho_t[k]             auxiliary k non-basic,
// with rho_t = glp_btran(e_{i_t}) (glpapi12.js:222: R inv(B")' SB e_i).  In
// terms of the device factor inv(B") of the scaled basis and the scaled
// matrix A" = R A S the engine keeps:
//   alfa[t, j] = d_t / s_j  (G A")[t, j],   alfa[t, k] = -d_t r_k G[t, k],
// where G = the rows i_t of inv(B") and d_t = 1 / r_k (k <= m) or s_{k-m}
// (the SB entry of position i_t).  The batch is one GEMM G (nk x m) times
// A" (m x n): on dense A it runs on the matrix cores
// (v_mfma_f64_16x16x4_f64, k_tab_mfma); the per-row path the tests compare
// it with is one thread per (row, column), down the dense column
// (k_tab_dense) or over the CSC entries of a sparse A" (k_tab_csc).
#include "gk_internal.h"
#include <cstdlib>

namespace gk {

// G[t * m + c] = inv(B")[pos_t, c] (column-major inv(B"), ldb)
__global__ void __launch_bounds__(256) k_tab_gather(const double *__restrict__ Binv, int ldb, int m,
                                                     const int *__restrict__ pos, double *__restrict__ G)
{
    const int t = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < m) G[(size_t)t * m + c] = Binv[(size_t)c * ldb + pos[t]];
}

// the auxiliary part: out[t, k] = G[t, k] * aux[k] * rs[t], aux[k] = -r_k
// for a non-basic row, 0 for a basic one
__global__ void __launch_bounds__(256) k_tab_aux(const double *__restrict__ G, int m, const double *__restrict__ aux,
                                                  const double *__restrict__ rs, double *__restrict__ out, size_t ldo)
{
    const int t = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k < m) out[(size_t)t * ldo + k] = G[(size_t)t * m + k] * aux[k] * rs[t];
}

// the structural part, per-row path: one thread per (t, j) over the CSC
// entries of column j (A" by columns, 0-based rows)
__global__ void __launch_bounds__(256) k_tab_csc(const double *__restrict__ G, int m, int n,
                                                  const int *__restrict__ cptr, const int *__restrict__ cind,
                                                  const double *__restrict__ cval, const double *__restrict__ cs,
                                                  const double *__restrict__ rs, double *__restrict__ out, size_t ldo)
{
    const int t = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const double *g = G + (size_t)t * m;
    double acc = 0.0;
    for (int p = cptr[j]; p < cptr[j + 1]; p++) acc += g[cind[p]] * cval[p];
    out[(size_t)t * ldo + m + j] = acc * cs[j] * rs[t];
}

// the same on dense A" (column-major, lda; the engine keeps no CSC values
// for a dense problem): one thread per (t, j), down column j
__global__ void __launch_bounds__(256) k_tab_dense(const double *__restrict__ G, int m, int n,
                                                    const double *__restrict__ A, int lda, const double *__restrict__ cs,
                                                    const double *__restrict__ rs, double *__restrict__ out, size_t ldo)
{
    const int t = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const double *g = G + (size_t)t * m;
    const double *a = A + (size_t)j * lda;
    double acc = 0.0;
    for (int r = 0; r < m; r++) acc += g[r] * a[r];
    out[(size_t)t * ldo + m + j] = acc * cs[j] * rs[t];
}

// the structural part on dense A" (column-major, lda): T = G A" on
// v_mfma_f64_16x16x4_f64.  A block of 4 waves owns 64 columns (16 per wave)
// and RT x 16 rows of the batch; the inner dimension m streams through LDS in
// chunks of 32 — A" in coalesced 256-byte column segments, G likewise — so
// every entry of A" is read from HBM once per RT x 16 rows.  Fragments (lane
// l): A-operand G[i = l & 15][kk = l >> 4], B-operand A"[kk = l >> 4][j =
// l & 15], result D[(l >> 4) + 4 r][l & 15].
typedef double tab_d4 __attribute__((ext_vector_type(4)));
template <int RT>
__global__ void __launch_bounds__(256) k_tab_mfma(const double *__restrict__ G, int nk, int m,
                                                   const double *__restrict__ A, int lda, int n,
                                                   const double *__restrict__ cs, const double *__restrict__ rs,
                                                   double *__restrict__ out, size_t ldo)
{
    constexpr int KC = 32, NC = 64, NR = RT * 16;
    __shared__ double As[KC][NC + 1];
    __shared__ double Gs[NR][KC + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int c0 = blockIdx.x * NC, r0 = blockIdx.y * NR;
    tab_d4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = tab_d4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < m; k0 += KC) {
        // A" chunk: 64 columns x 32 rows, 32 consecutive rows per 32 lanes
#pragma unroll
        for (int q = 0; q < (KC * NC) / 256; ++q) {
            const int e = tid + 256 * q, rr = e & (KC - 1), cc = e / KC;
            const int r = k0 + rr, c = c0 + cc;
            As[rr][cc] = (r < m && c < n) ? A[(size_t)c * lda + r] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < (KC * NR + 255) / 256; ++q) {
            const int e = tid + 256 * q;
            if (e < KC * NR) {
                const int rr = e & (KC - 1), row = e / KC;
                const int r = k0 + rr, t = r0 + row;
                Gs[row][rr] = (r < m && t < nk) ? G[(size_t)t * m + r] : 0.0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KC / 4; ++ks) {
            const double b = As[ks * 4 + lk][w * 16 + li];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const double a = Gs[rt * 16 + li][ks * 4 + lk];
                acc[rt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[rt], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    const int j = c0 + w * 16 + li;
    if (j >= n) return;
    const double sj = cs[j];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = r0 + rt * 16 + lk + 4 * r;
            if (t < nk) out[(size_t)t * ldo + m + j] = acc[rt][r] * sj * rs[t];
        }
}

// batches of 17..64 rows: 32 columns per block (twice the blocks of
// k_tab_mfma, two per CU on C3), each wave one 16-column tile and RT / 2 row
// tiles, and the next chunk of A" and G loaded into registers while the
// matrix cores work on the current one (one LDS buffer, two barriers per
// chunk; the loads of chunk k + 1 are in flight during chunk k's MFMAs)
template <int RT>
__global__ void __launch_bounds__(256) k_tab_mfma2(const double *__restrict__ G, int nk, int m,
                                                    const double *__restrict__ A, int lda, int n,
                                                    const double *__restrict__ cs, const double *__restrict__ rs,
                                                    double *__restrict__ out, size_t ldo)
{
    constexpr int KC = 32, NC = 32, NR = RT * 16, RW = RT / 2;
    constexpr int QA = (KC * NC) / 256, QG = (KC * NR) / 256;
    __shared__ double As[KC][NC + 1];
    __shared__ double Gs[NR][KC + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int ct = w & 1, rt0 = (w >> 1) * RW;
    const int c0 = blockIdx.x * NC, r0 = blockIdx.y * NR;
    tab_d4 acc[RW];
#pragma unroll
    for (int q = 0; q < RW; ++q) acc[q] = tab_d4{0.0, 0.0, 0.0, 0.0};
    double ra[QA], rg[QG];
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = tid + 256 * q, rr = e & (KC - 1), cc = e / KC;
            const int r = k0 + rr, c = c0 + cc;
            ra[q] = (r < m && c < n) ? A[(size_t)c * lda + r] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const int e = tid + 256 * q, rr = e & (KC - 1), row = e / KC;
            const int r = k0 + rr, t = r0 + row;
            rg[q] = (r < m && t < nk) ? G[(size_t)t * m + r] : 0.0;
        }
    };
    load(0);
    for (int k0 = 0; k0 < m; k0 += KC) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = tid + 256 * q;
            As[e & (KC - 1)][e / KC] = ra[q];
        }
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const int e = tid + 256 * q;
            Gs[e / KC][e & (KC - 1)] = rg[q];
        }
        __syncthreads();
        if (k0 + KC < m) load(k0 + KC);
#pragma unroll
        for (int ks = 0; ks < KC / 4; ++ks) {
            const double b = As[ks * 4 + lk][ct * 16 + li];
#pragma unroll
            for (int q = 0; q < RW; ++q) {
                const double a = Gs[(rt0 + q) * 16 + li][ks * 4 + lk];
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    const int j = c0 + ct * 16 + li;
    if (j >= n) return;
    const double sj = cs[j];
#pragma unroll
    for (int q = 0; q < RW; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = r0 + (rt0 + q) * 16 + lk + 4 * r;
            if (t < nk) out[(size_t)t * ldo + m + j] = acc[q][r] * sj * rs[t];
        }
}

void tab_rows(hipStream_t s, const double *Binv, int ldb, const MatDev &A, int nk, const int *pos, double *G,
              const double *aux, const double *cs, const double *rs, double *out, int use_mfma)
{
    const int m = A.m, n = A.n;
    const size_t ldo = (size_t)m + n;
    if (nk <= 0) return;
    // (Binv null: G holds the rows of inv(B) already — the sparse factor's BTRANs)
    if (Binv) hipLaunchKernelGGL(k_tab_gather, dim3((m + 255) / 256, nk), dim3(256), 0, s, Binv, ldb, m, pos, G);
    hipLaunchKernelGGL(k_tab_aux, dim3((m + 255) / 256, nk), dim3(256), 0, s, G, m, aux, rs, out, ldo);
    if (A.dense) {
        if (!use_mfma) {
            hipLaunchKernelGGL(k_tab_dense, dim3((n + 255) / 256, nk), dim3(256), 0, s, G, m, n, A.A, A.lda, cs, rs,
                               out, ldo);
            return;
        }
        static const int v1 = std::getenv("GK_TAB_V1") != nullptr;   // the one-buffer 64-column kernel (experiments)
        if (nk <= 16 || v1) {
            const int gx = (n + 63) / 64;
            if (nk <= 16)
                hipLaunchKernelGGL(k_tab_mfma<1>, dim3(gx, 1), dim3(256), 0, s, G, nk, m, A.A, A.lda, n, cs, rs, out,
                                   ldo);
            else
                hipLaunchKernelGGL(k_tab_mfma<4>, dim3(gx, (nk + 63) / 64), dim3(256), 0, s, G, nk, m, A.A, A.lda, n,
                                   cs, rs, out, ldo);
        } else {
            const int gx = (n + 31) / 32;
            if (nk <= 32)
                hipLaunchKernelGGL(k_tab_mfma2<2>, dim3(gx, 1), dim3(256), 0, s, G, nk, m, A.A, A.lda, n, cs, rs, out,
                                   ldo);
            else
                hipLaunchKernelGGL(k_tab_mfma2<4>, dim3(gx, (nk + 63) / 64), dim3(256), 0, s, G, nk, m, A.A, A.lda, n,
                                   cs, rs, out, ldo);
        }
    } else {
        // sparse A": the CSC entries (0-based rows)
        hipLaunchKernelGGL(k_tab_csc, dim3((n + 255) / 256, nk), dim3(256), 0, s, G, m, n, A.cptr, A.cind, A.cval, cs,
                           rs, out, ldo);
    }
}

}  // namespace gk
