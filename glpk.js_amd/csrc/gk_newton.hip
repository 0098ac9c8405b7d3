// Re-inversion by Newton refinement of the updated inverse (the scheduled
// re-inversion of a large structural block on the matrix cores).
//
// The reference refactorizes after nfs_max Forrest-Tomlin updates
// (glpfhv.js:182-187 -> bfd_factorize, glpbfd.js:74-103) to bound the error
// the update chain accumulates.  On the device, at that point, the factor
// holds inv(B) of the *current* basis, kept by product-form updates, and is
// off only by the chain's rounding.  The structural block of the new inverse,
// inv(C) with C = B[R, J] (gk_engine.hip BasisSplit), is then one Newton step
// away (Newton-Schulz):
//   X0 = inv(B)[J, R]              (the updated inverse, gathered)
//   R0 = I - C X0                  (one k x k x k GEMM; r0 = max |R0|)
//   X1 = X0 + X0 R0                (a second GEMM), ||I - C X1|| <= ||R0||^2
// Two dependent MFMA GEMMs (v_mfma_f64_16x16x4_f64) replace the k / 8
// dependent one-workgroup panels of the blocked Gauss-Jordan (gk_reinvert.hip),
// whose chain is the limit at k = 4096.  The rest of the factor (the rows of
// the basic slacks, G = BS inv(C)) is assembled from X1 exactly as after
// Gauss-Jordan.  The iteration is taken only when it provably converges
// (k * r < 1/2, the infinity norm of R bounded by k max |R|), and is repeated
// until that bound, squared, is below k eps; anything else — a NaN, a residual that does not
// shrink, three steps — hands the block back to Gauss-Jordan (the caller
// still holds C untouched).  Size threshold k >= GK_NEWTON_MIN_K (512).
// Only the engine's scheduled re-inversions (update
// count reached, no growth-check failure since the last one) use it: the
// factor's own entry point (gk_bfd_factorize) and every recovery re-inversion
// (check_stab, pivot checks, growth) stay with Gauss-Jordan from C.
#include "gk_internal.h"
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace gk {

typedef double nwt_d4 __attribute__((ext_vector_type(4)));

// X[b * k + a] = inv(B)[posJ[b] - 1, rowR[a] - 1] (the layout of CinvR) and
// its column-major copy Xc[b + a * k] (the A operand of the update GEMM):
// 64 x 64 tiles through LDS — the column of inv(B) is read down its rows and
// Xc written from the same registers, the row of X written along a
__global__ void __launch_bounds__(256) k_nwt_gather(const double *__restrict__ Binv, int ldb, int k,
                                                    const int *__restrict__ posJ, const int *__restrict__ rowR,
                                                    double *__restrict__ X, double *__restrict__ Xc)
{
    __shared__ double t[64][65];
    const int a0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int lane = threadIdx.x & 63, q0 = threadIdx.x >> 6;
    const int b = b0 + lane;
    const int prow = (b < k) ? posJ[b] - 1 : 0;
    for (int q = q0; q < 64; q += 4) {
        const int a = a0 + q;
        if (a < k && b < k) {
            const double v = Binv[(size_t)prow + (size_t)(rowR[a] - 1) * ldb];
            t[q][lane] = v;
            Xc[(size_t)b + (size_t)a * k] = v;
        }
    }
    __syncthreads();
    const int a = a0 + lane;
    for (int q = q0; q < 64; q += 4) {
        const int bb = b0 + q;
        if (a < k && bb < k) X[(size_t)bb * k + a] = t[lane][q];
    }
}

// Xc[b + a * k] = X[b * k + a] (a later step's A operand)
__global__ void __launch_bounds__(256) k_nwt_transpose(const double *__restrict__ X, int k, double *__restrict__ Xc)
{
    __shared__ double t[64][65];
    const int a0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int lane = threadIdx.x & 63, q0 = threadIdx.x >> 6;
    for (int q = q0; q < 64; q += 4) {
        const int b = b0 + q, a = a0 + lane;
        if (a < k && b < k) t[q][lane] = X[(size_t)b * k + a];
    }
    __syncthreads();
    for (int q = q0; q < 64; q += 4) {
        const int a = a0 + q, b = b0 + lane;
        if (a < k && b < k) Xc[(size_t)b + (size_t)a * k] = t[lane][q];
    }
}

// D = I - A B (MODE 0, max |D| into *rmax as ordered bits) or D = E + A B
// (MODE 1), all k x k with leading dimension k:
//   A(i, l) = A_IC ? A[i + l k] : A[i k + l]
//   B(l, j) = B_JC ? B[l k + j] : B[l + j k]
//   D(i, j), E(i, j) = D_CM ? [i + j k] : [i k + j]
// A block owns a 128 x 128 tile of D, four waves of 64 x 64 (4 x 4 MFMA
// tiles of 16 x 16); the inner dimension streams through LDS in chunks of 16,
// the next chunk held in registers while the matrix cores work on the
// current one.  Tiles are dealt so that each XCD (blocks b, b + 8, ...) gets
// a contiguous run of row bands and shares their rows of A in its own L2.
constexpr int NW_T = 128, NW_KC = 16, NW_LD = NW_T + 16;   // LDS row stride: 288 dwords = 32 mod 64 banks

template <bool A_IC, bool B_JC, bool D_CM, int MODE>
__global__ void __launch_bounds__(256, 2) k_nwt_gemm(int k, const double *__restrict__ A, const double *__restrict__ B,
                                                  double *__restrict__ D, const double *__restrict__ E,
                                                  unsigned long long *__restrict__ rmax)
{
    __shared__ double As[NW_KC][NW_LD];
    __shared__ double Bs[NW_KC][NW_LD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int wr = w >> 1, wc = w & 1;
    const int gt = (k + NW_T - 1) / NW_T, nt = gt * gt;
    int tile = blockIdx.x;
    if ((nt & 7) == 0) tile = (tile & 7) * (nt >> 3) + (tile >> 3);   // XCD-contiguous runs
    const int i0 = (tile / gt) * NW_T, j0 = (tile % gt) * NW_T;
    const size_t K = (size_t)k;
    double ra[8], rb[8];
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            int i, l;
            if (A_IC) { i = e & (NW_T - 1); l = e >> 7; }
            else { l = e & (NW_KC - 1); i = e >> 4; }
            const int gi = i0 + i, gl = k0 + l;
            ra[q] = (gi < k && gl < k) ? (A_IC ? A[gi + gl * K] : A[gi * K + gl]) : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            int j, l;
            if (B_JC) { j = e & (NW_T - 1); l = e >> 7; }
            else { l = e & (NW_KC - 1); j = e >> 4; }
            const int gj = j0 + j, gl = k0 + l;
            rb[q] = (gj < k && gl < k) ? (B_JC ? B[gl * K + gj] : B[gl + gj * K]) : 0.0;
        }
    };
    nwt_d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = nwt_d4{0.0, 0.0, 0.0, 0.0};
    load(0);
    for (int k0 = 0; k0 < k; k0 += NW_KC) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            if (A_IC) As[e >> 7][e & (NW_T - 1)] = ra[q];
            else As[e & (NW_KC - 1)][e >> 4] = ra[q];
            if (B_JC) Bs[e >> 7][e & (NW_T - 1)] = rb[q];
            else Bs[e & (NW_KC - 1)][e >> 4] = rb[q];
        }
        __syncthreads();
        if (k0 + NW_KC < k) load(k0 + NW_KC);
#pragma unroll
        for (int ks = 0; ks < NW_KC / 4; ++ks) {
            double fa[4], fb[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                fa[t] = As[ks * 4 + lk][wr * 64 + t * 16 + li];
                fb[t] = Bs[ks * 4 + lk][wc * 64 + t * 16 + li];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    double vmax = 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wr * 64 + a * 16 + lk + 4 * r;
                const int j = j0 + wc * 64 + b * 16 + li;
                if (i >= k || j >= k) continue;
                const size_t o = D_CM ? (size_t)i + (size_t)j * K : (size_t)i * K + j;
                double v;
                if (MODE == 0) {
                    v = (i == j ? 1.0 : 0.0) - acc[a][b][r];
                    double av = fabs(v);
                    if (!(av <= 1e300)) av = 1e300;           // NaN / Inf: report as huge
                    vmax = fmax(vmax, av);
                } else
                    v = E[o] + acc[a][b][r];
                D[o] = v;
            }
    if (MODE == 0) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) vmax = fmax(vmax, __shfl_xor(vmax, o));
        if (lane == 0) atomicMax(rmax, (unsigned long long)__double_as_longlong(vmax));
    }
}

static double nwt_residual(hipStream_t s, int k, const double *C, const double *X, double *R,
                           unsigned long long *rbits)
{
    // a HIP error reads as "no convergence": the caller's Gauss-Jordan path
    // then meets it again and reports it
    if (hipMemsetAsync(rbits, 0, sizeof(unsigned long long), s) != hipSuccess) return 1e300;
    const int gt = (k + NW_T - 1) / NW_T;
    // R(a, a') = delta - sum_b C(a, b) X(b, a'): C column-major, X = CinvR layout (row-major in b),
    // R row-major (the update's B operand, contiguous along a')
    hipLaunchKernelGGL((k_nwt_gemm<true, true, false, 0>), dim3(gt * gt), dim3(256), 0, s, k, C, X, R,
                       (const double *)nullptr, rbits);
    unsigned long long bits = 0;
    if (hipMemcpyAsync(&bits, rbits, sizeof(bits), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return 1e300;
    double r;
    std::memcpy(&r, &bits, sizeof(r));
    return r;
}

static void nwt_update(hipStream_t s, int k, const double *X, const double *Xc, const double *R, double *Xn)
{
    const int gt = (k + NW_T - 1) / NW_T;
    // Xn(b, a') = X(b, a') + sum_a X(b, a) R(a, a'): A = the column-major copy Xc
    // (A(i, l) = Xc[i + l k]), B = R row-major (B(l, j) = R[l k + j]), Xn row-major;
    // both operands load along their contiguous dimension (the row-major X as A
    // operand measured 3.48 ms against 2.47 ms at k = 4096)
    hipLaunchKernelGGL((k_nwt_gemm<true, true, false, 1>), dim3(gt * gt), dim3(256), 0, s, k, Xc, R, Xn, X,
                       (unsigned long long *)nullptr);
}

// read at every re-inversion (tests change it between solves); 0: off
int newton_min_k()
{
    const char *e = std::getenv("GK_NEWTON_MIN_K");
    return e ? std::atoi(e) : 512;
}

const double *newton_refine(hipStream_t s, int k, const double *C, const double *Binv, int ldb, const int *posJ,
                            const int *rowR, double *X0, double *R, double *X1, double *Xc,
                            unsigned long long *rbits, NewtonInfo *info)
{
    info->steps = 0;
    info->resid = 0.0;
    const int g = (k + 63) / 64;
    hipLaunchKernelGGL(k_nwt_gather, dim3(g, g), dim3(256), 0, s, Binv, ldb, k, posJ, rowR, X0, Xc);
    double *x = X0, *xn = X1;
    double prev = 1e300;
    for (int it = 0; it < 3; ++it) {
        const double r = nwt_residual(s, k, C, x, R, rbits);
        if (it == 0) info->resid = r;
        const double kr = (double)k * r;
        if (!(kr < 0.5) || r > 0.5 * prev) return nullptr;    // no convergence guarantee: Gauss-Jordan
        if (it > 0) hipLaunchKernelGGL(k_nwt_transpose, dim3(g, g), dim3(256), 0, s, x, k, Xc);
        nwt_update(s, k, x, Xc, R, xn);
        info->steps++;
        std::swap(x, xn);
        // the remaining residual is bounded by (k r)^2; below k eps — the
        // worst-case rounding of one GEMM (or Gauss-Jordan step) on this
        // block — a further step cannot improve it
        if (kr * kr <= (double)k * 1.1102230246251565e-16) {
            info->final_bound = kr * kr;
            return x;
        }
        prev = r;
    }
    return nullptr;
}

}  // namespace gk
