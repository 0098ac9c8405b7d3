// gk_scale.hip — glp_scale_prob (glpscl.js:1-225) on the device.
//
// SURVEY.md §8(f) #2.  The reference scales the problem before the simplex
// on its presolve paths (glpapi06.js:115 with GLP_SF_AUTO, glpapi09.js:204
// with GM | EQ | 2N | SKIP) and on request.  Every quantity it forms is a
// min / max over a row or a column of |a_ij| * (r_i * s_j), a product or
// quotient of two of them, or a square root — all exactly rounded and, for
// min / max, independent of the order of the entries — so the device result
// is the reference's bit for bit (tests/test_scale.py against the
// reference's own factors, tests/golden/scale_*.json).
//
// Layout: A arrives by columns (the boundary's CSC); the row sweeps need it
// by rows, so a row copy is built once on the device (counts, one scan,
// scatter — entry order inside a row is free because only min / max are
// taken).  A sweep is one kernel, one wave per row (or column): it streams
// the row's values and indices once (12 bytes per entry) and gathers s_j
// (or r_i) from L2.  The iteration control of gm_iterate (≤ 15 sweeps, stop
// when the ratio improves by less than 10 %) needs two scalars per sweep and
// stays on the host; each statistics pass returns them through one 32-byte
// copy.
#include "gk_internal.h"
#include "gk_device.h"
#include "../../include/glpk_mi355x.h"
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <algorithm>
#include <vector>

namespace gk {

void set_err(const char *fmt, ...);

namespace {

enum : int { SC_STAT = 0, SC_GM = 1, SC_EQ = 2 };

// acc[0] min over rows of the row minimum, acc[1] max of the row maximum,
// acc[2] max row ratio, acc[3] max column ratio: bit patterns of
// non-negative doubles, which order like the doubles
__global__ void k_scl_acc_init(unsigned long long *acc)
{
    if (threadIdx.x == 0) {
        acc[0] = (unsigned long long)__double_as_longlong(DBL_MAX * 2.0);   // +inf
        acc[1] = 0ull;
        acc[2] = 0ull;
        acc[3] = 0ull;
    }
}

__device__ __forceinline__ double wmin_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ double wmax_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// one wave per line (row of the row copy, or column of A): min / max of
// |a| * (r_i * s_j) over its entries (1, 1 when it has none), then
//   SC_STAT  the matrix and ratio accumulators (rows: acc 0-2, columns: acc 3)
//   SC_GM    own /= sqrt(min * max)   (gm_scaling, glpscl.js:98-117)
//   SC_EQ    own /= max               (eq_scaling, glpscl.js:82-96)
// `own` is r (rows) or s (columns); `other` is indexed by the entry's index.
template <int ROWS>
__global__ void __launch_bounds__(1024) k_scl_sweep(int lines, const int *__restrict__ ptr,
                                                   const int *__restrict__ idx, const double *__restrict__ val,
                                                   double *__restrict__ own, const double *__restrict__ other,
                                                   int mode, unsigned long long *acc)
{
    const int line = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (line >= lines) return;                          // wave-uniform
    const int beg = ptr[line], end = ptr[line + 1];
    const double o = own[line];
    double lo = DBL_MAX * 2.0, hi = 0.0;
    // software-pipelined: the next group's values and indices load while
    // this group's gathers of the other factor are in flight
    constexpr int U = 8;
    if (end > beg) {
        const int last = end - 1;
        double v[U];
        int c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int tt = min(beg + lane + 64 * u, last);
            v[u] = __builtin_nontemporal_load(val + tt);      // streamed once per sweep
            c[u] = __builtin_nontemporal_load(idx + tt);
        }
        for (int t = beg + lane; t - lane < end; t += 64 * U) {
            double g[U], v2[U];
            int c2[U];
#pragma unroll
            for (int u = 0; u < U; ++u) g[u] = other[ROWS ? c[u] : c[u] - 1];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int tt = min(t + 64 * (U + u), last);
                v2[u] = __builtin_nontemporal_load(val + tt);
                c2[u] = __builtin_nontemporal_load(idx + tt);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // rows: |a| (r_i s_j); columns: |a| (r_i s_j) with own = s_j
                const double temp = ROWS ? fabs(v[u]) * (o * g[u]) : fabs(v[u]) * (g[u] * o);
                if (t + 64 * u < end) {
                    lo = fmin(lo, temp);
                    hi = fmax(hi, temp);
                }
                v[u] = v2[u];
                c[u] = c2[u];
            }
        }
    }
    lo = wmin_d(lo);
    hi = wmax_d(hi);
    if (end == beg) lo = hi = 1.0;
    if (lane != 0) return;
    if (mode == SC_STAT) {
        const double ratio = hi / lo;
        if (ROWS) {
            atomicMin(&acc[0], (unsigned long long)__double_as_longlong(lo));
            atomicMax(&acc[1], (unsigned long long)__double_as_longlong(hi));
            atomicMax(&acc[2], (unsigned long long)__double_as_longlong(ratio));
        } else {
            atomicMax(&acc[3], (unsigned long long)__double_as_longlong(ratio));
        }
    } else if (mode == SC_GM) {
        own[line] = o / sqrt(lo * hi);
    } else {
        own[line] = o / hi;
    }
}

// round2n (glplib03.js:26): the nearest power of two, f = 0.75 rounding down
__global__ void k_scl_round2n(double *x, int cnt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    int e;
    const double f = frexp(x[i], &e);
    x[i] = ldexp(1.0, f <= 0.75 ? e - 1 : e);
}

__global__ void k_scl_fill1(double *x, int cnt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cnt) x[i] = 1.0;
}

// row copy of A: counts per row
__global__ void k_scl_count(const int *__restrict__ ind, long long nnz, int *__restrict__ cnt)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nnz) atomicAdd(&cnt[ind[t] - 1], 1);
}

// exclusive scan of cnt[0..m) into ptr[0..m] by one workgroup
__global__ void __launch_bounds__(1024) k_scl_scan(const int *__restrict__ cnt, int m, int *__restrict__ ptr)
{
    __shared__ int part[1024];
    const int per = (m + 1023) / 1024;
    const int b = threadIdx.x * per, e = min(m, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = part[threadIdx.x] - s;
    for (int i = b; i < e; ++i) {
        ptr[i] = run;
        run += cnt[i];
    }
    if (threadIdx.x == 1023) ptr[m] = part[1023];
}

// scatter: one wave per column; fill[] starts as the row pointers
__global__ void __launch_bounds__(256) k_scl_scatter(int n, const int *__restrict__ cptr, const int *__restrict__ ind,
                                                     const double *__restrict__ val, int *__restrict__ fill,
                                                     int *__restrict__ rcol, double *__restrict__ rval)
{
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    for (int t = cptr[j] + (threadIdx.x & 63); t < cptr[j + 1]; t += 64) {
        const int p = atomicAdd(&fill[ind[t] - 1], 1);
        rcol[p] = j;
        rval[p] = val[t];
    }
}

// Row statistics without a row copy (m <= ROWPART_MAX): block b takes a
// contiguous range of columns and keeps per-row min / max of its entries in
// LDS (bit patterns of non-negative doubles, ds_min_u64 / ds_max_u64); the
// block's m pairs go to partials[b], and k_scl_rowfin reduces them per row.
constexpr int ROWPART_MAX = 8192;
constexpr int ROWPART_TILES = 256;

template <bool COLSTAT>
__global__ void __launch_bounds__(1024) k_scl_rowpart(int n, int m, int cols_per_block, const int *__restrict__ cptr,
                                                     const int *__restrict__ ind, const double *__restrict__ val,
                                                     const double *__restrict__ r, const double *__restrict__ sj,
                                                     unsigned long long *__restrict__ plo,
                                                     unsigned long long *__restrict__ phi, unsigned long long *colacc)
{
    extern __shared__ unsigned long long lds[];
    unsigned long long *lo = lds, *hi = lds + m;
    const unsigned long long INF = (unsigned long long)__double_as_longlong(DBL_MAX * 2.0);
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        lo[i] = INF;
        hi[i] = 0ull;
    }
    __syncthreads();
    const int j0 = blockIdx.x * cols_per_block, j1 = min(n, j0 + cols_per_block);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    __shared__ unsigned long long wr[16];             // per-wave max column ratio
    double cmax = 0.0;
    for (int j = j0 + w; j < j1; j += nw) {
        const int beg = cptr[j], end = cptr[j + 1];
        const double o = sj[j];
        double clo = DBL_MAX * 2.0, chi = 0.0;          // the column's own min / max (colacc)
        constexpr int U = 8;
        for (int t0 = beg; t0 < end; t0 += 64 * U) {
            double v[U], g[U];
            int c[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int tt = min(t0 + lane + 64 * u, end - 1);
                v[u] = __builtin_nontemporal_load(val + tt);
                c[u] = __builtin_nontemporal_load(ind + tt) - 1;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) g[u] = r[c[u]];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (t0 + lane + 64 * u < end) {
                    const double temp = fabs(v[u]) * (g[u] * o);        // |a| (r_i s_j)
                    const unsigned long long b = (unsigned long long)__double_as_longlong(temp);
                    atomicMin(&lo[c[u]], b);        // (a read-compare first measured slower)
                    atomicMax(&hi[c[u]], b);
                    if (COLSTAT) {
                        clo = fmin(clo, temp);
                        chi = fmax(chi, temp);
                    }
                }
        }
        // column statistics of the same pass (k_scl_sweep<0>'s SC_STAT epilogue:
        // the same |a| (r_i s_j) products, an empty column counts as 1, 1)
        if (COLSTAT) {
            clo = wmin_d(clo);
            chi = wmax_d(chi);
            if (end == beg) clo = chi = 1.0;
            cmax = fmax(cmax, chi / clo);
        }
    }
    if (COLSTAT && lane == 0) wr[w] = (unsigned long long)__double_as_longlong(cmax);
    __syncthreads();
    // one atomic per workgroup (one per column serialised on a single L2 line)
    if (COLSTAT && threadIdx.x == 0) {
        unsigned long long b = 0ull;
        for (int k = 0; k < nw; ++k) b = wr[k] > b ? wr[k] : b;
        atomicMax(colacc, b);
    }
    unsigned long long *ql = plo + (size_t)blockIdx.x * m, *qh = phi + (size_t)blockIdx.x * m;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        ql[i] = lo[i];
        qh[i] = hi[i];
    }
}

// per row: min / max over the tiles' partials (an empty row: 1, 1), then the
// epilogue of k_scl_sweep<1>.  64 rows per block (lanes), the 16 waves split
// the tiles (8 loads in flight each) and meet in LDS.
__global__ void __launch_bounds__(1024) k_scl_rowfin(int m, int tiles, const unsigned long long *__restrict__ plo,
                                                     const unsigned long long *__restrict__ phi,
                                                     double *__restrict__ r, int mode, unsigned long long *acc)
{
    __shared__ unsigned long long sl[16][64], sh[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    const int ii = min(i, m - 1);
    const unsigned long long INF = (unsigned long long)__double_as_longlong(DBL_MAX * 2.0);
    unsigned long long a = INF, b = 0ull;
    for (int t0 = w; t0 < tiles; t0 += 8 * nw) {
        unsigned long long x[8], y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = min(t0 + u * nw, tiles - 1);
            x[u] = plo[(size_t)t * m + ii];
            y[u] = phi[(size_t)t * m + ii];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a = x[u] < a ? x[u] : a;                  // repeated tiles (clamped) change nothing
            b = y[u] > b ? y[u] : b;
        }
    }
    sl[w][lane] = a;
    sh[w][lane] = b;
    __syncthreads();
    if (w != 0) return;
    for (int k = 1; k < nw; ++k) {
        a = sl[k][lane] < a ? sl[k][lane] : a;
        b = sh[k][lane] > b ? sh[k][lane] : b;
    }
    double lo = __longlong_as_double((long long)a), hi = __longlong_as_double((long long)b);
    if (a == INF) lo = hi = 1.0;                      // no entries
    if (mode == SC_STAT) {
        double l = i < m ? lo : DBL_MAX * 2.0, h = i < m ? hi : 0.0, q = i < m ? hi / lo : 0.0;
        l = wmin_d(l);
        h = wmax_d(h);
        q = wmax_d(q);
        if (lane == 0) {
            atomicMin(&acc[0], (unsigned long long)__double_as_longlong(l));
            atomicMax(&acc[1], (unsigned long long)__double_as_longlong(h));
            atomicMax(&acc[2], (unsigned long long)__double_as_longlong(q));
        }
    } else if (i < m) {
        r[i] = (mode == SC_GM) ? r[i] / sqrt(lo * hi) : r[i] / hi;
    }
}

template <class T>
struct DevBuf {
    T *p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t n) { return hipMalloc((void **)&p, std::max<size_t>(n, 1) * sizeof(T)); }
};

#define SCHK(x)                                                                                                 \
    do {                                                                                                        \
        hipError_t e__ = (x);                                                                                   \
        if (e__ != hipSuccess) {                                                                                \
            set_err("gk_scale_prob: HIP error %s at %s", hipGetErrorString(e__), #x);                           \
            return GK_EABI;                                                                                     \
        }                                                                                                       \
    } while (0)

}  // namespace

int scale_prob_dev(hipStream_t s, int m, int n, const int *ptr, const int *ind, const double *val, int flags,
                   double *rii, double *sjj, double *report, double *sweep_ms, double *sweep_bytes)
{
    const int SF_GM = 0x01, SF_EQ = 0x10, SF_2N = 0x20, SF_SKIP = 0x40, SF_AUTO = 0x80;
    if (flags & ~(SF_GM | SF_EQ | SF_2N | SF_SKIP | SF_AUTO)) return 1;
    if (flags & SF_AUTO) flags = SF_GM | SF_EQ | SF_SKIP;
    const long long nnz = n > 0 ? ptr[n] : 0;
    DevBuf<int> d_cptr, d_ind, d_rptr, d_fill, d_rcol;
    DevBuf<double> d_val, d_rval, d_r, d_s;
    DevBuf<unsigned long long> d_acc;
    SCHK(d_cptr.alloc(n + 1));
    SCHK(d_ind.alloc(nnz));
    SCHK(d_val.alloc(nnz));
    // rows by LDS partials when m fits, else a row copy of A
    const bool part = m > 0 && m <= ROWPART_MAX && n > 0 && std::getenv("GK_SCALE_ROWCOPY") == nullptr;
    const int tiles = part ? std::min(ROWPART_TILES, n) : 0;
    const int cpb = part ? cdiv(n, tiles) : 0;
    DevBuf<unsigned long long> d_plo, d_phi;
    if (part) {
        SCHK(d_plo.alloc((size_t)tiles * m));
        SCHK(d_phi.alloc((size_t)tiles * m));
    } else {
        SCHK(d_rptr.alloc(m + 1));
        SCHK(d_fill.alloc(m + 1));
        SCHK(d_rcol.alloc(nnz));
        SCHK(d_rval.alloc(nnz));
    }
    SCHK(d_r.alloc(m));
    SCHK(d_s.alloc(n));
    SCHK(d_acc.alloc(4));
    SCHK(hipMemcpyAsync(d_cptr.p, ptr, sizeof(int) * (n + 1), hipMemcpyHostToDevice, s));
    if (nnz) {
        SCHK(hipMemcpyAsync(d_ind.p, ind, sizeof(int) * nnz, hipMemcpyHostToDevice, s));
        SCHK(hipMemcpyAsync(d_val.p, val, sizeof(double) * nnz, hipMemcpyHostToDevice, s));
    }
    hipEvent_t b0, b1;
    SCHK(hipEventCreate(&b0));
    SCHK(hipEventCreate(&b1));
    SCHK(hipEventRecord(b0, s));
    if (!part) {
        // the row copy
        SCHK(hipMemsetAsync(d_fill.p, 0, sizeof(int) * (m + 1), s));
        if (nnz)
            hipLaunchKernelGGL(k_scl_count, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_ind.p, nnz, d_fill.p);
        if (m) hipLaunchKernelGGL(k_scl_scan, dim3(1), dim3(1024), 0, s, d_fill.p, m, d_rptr.p);
        SCHK(hipMemcpyAsync(d_fill.p, d_rptr.p, sizeof(int) * (m + 1), hipMemcpyDeviceToDevice, s));
        if (n)
            hipLaunchKernelGGL(k_scl_scatter, dim3(cdiv(n, 4)), dim3(256), 0, s, n, d_cptr.p, d_ind.p, d_val.p,
                               d_fill.p, d_rcol.p, d_rval.p);
    }
    // glp_unscale_prob
    if (m) hipLaunchKernelGGL(k_scl_fill1, dim3(cdiv(m, 256)), dim3(256), 0, s, d_r.p, m);
    if (n) hipLaunchKernelGGL(k_scl_fill1, dim3(cdiv(n, 256)), dim3(256), 0, s, d_s.p, n);
    SCHK(hipGetLastError());
    SCHK(hipEventRecord(b1, s));
    SCHK(hipEventSynchronize(b1));
    float build_ms = 0.f;
    (void)hipEventElapsedTime(&build_ms, b0, b1);
    (void)hipEventDestroy(b0);
    (void)hipEventDestroy(b1);

    hipEvent_t e0, e1;
    SCHK(hipEventCreate(&e0));
    SCHK(hipEventCreate(&e1));
    // device time of the scaling work: the row copy (when built) plus every
    // sweep (the host's stage decisions between sweeps are not counted)
    double ms_total = build_ms, bytes_total = 0.0;
    // colstat: a row statistics pass by partials also forms the column ratio
    // (acc 3) from the same entries, so stats(true) streams A once
    auto sweep = [&](bool rows, int mode, bool colstat = false) -> hipError_t {
        if (rows ? m == 0 : n == 0) return hipSuccess;
        hipError_t e = hipEventRecord(e0, s);
        if (e != hipSuccess) return e;
        if (rows && part) {
            if (colstat)
                hipLaunchKernelGGL(k_scl_rowpart<true>, dim3(tiles), dim3(1024), (size_t)16 * m, s, n, m, cpb, d_cptr.p,
                                   d_ind.p, d_val.p, d_r.p, d_s.p, d_plo.p, d_phi.p, d_acc.p + 3);
            else
                hipLaunchKernelGGL(k_scl_rowpart<false>, dim3(tiles), dim3(1024), (size_t)16 * m, s, n, m, cpb, d_cptr.p,
                                   d_ind.p, d_val.p, d_r.p, d_s.p, d_plo.p, d_phi.p, nullptr);
            hipLaunchKernelGGL(k_scl_rowfin, dim3(cdiv(m, 64)), dim3(1024), 0, s, m, tiles, d_plo.p, d_phi.p, d_r.p,
                               mode, d_acc.p);
        } else if (rows)
            hipLaunchKernelGGL(k_scl_sweep<1>, dim3(cdiv(m, 16)), dim3(1024), 0, s, m, d_rptr.p, d_rcol.p, d_rval.p, d_r.p,
                               d_s.p, mode, d_acc.p);
        else
            hipLaunchKernelGGL(k_scl_sweep<0>, dim3(cdiv(n, 16)), dim3(1024), 0, s, n, d_cptr.p, d_ind.p, d_val.p, d_s.p,
                               d_r.p, mode, d_acc.p);
        if ((e = hipEventRecord(e1, s)) != hipSuccess) return e;
        if ((e = hipEventSynchronize(e1)) != hipSuccess) return e;
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms_total += ms;
        // algorithmic: the 12-byte entries once, the line's own factor (read,
        // and written by GM / EQ), its pointers
        bytes_total += 12.0 * (double)nnz + 8.0 * (rows ? m : n) * (mode == SC_STAT ? 1 : 2) + 4.0 * ((rows ? m : n) + 1);
        if (colstat) bytes_total += 8.0 * n + 4.0 * (n + 1);   // the column factors and pointers
        return hipGetLastError();
    };
    // statistics with the current factors: (mat min, mat max, row ratio, col ratio)
    auto stats = [&](bool cols, double *q) -> int {
        hipLaunchKernelGGL(k_scl_acc_init, dim3(1), dim3(64), 0, s, d_acc.p);
        const bool fused = cols && part;
        SCHK(sweep(true, SC_STAT, fused));
        if (cols && !fused) SCHK(sweep(false, SC_STAT));
        unsigned long long a[4];
        SCHK(hipMemcpyAsync(a, d_acc.p, sizeof a, hipMemcpyDeviceToHost, s));
        SCHK(hipStreamSynchronize(s));
        for (int k = 0; k < 4; ++k) q[k] = __builtin_bit_cast(double, a[k]);
        if (m == 0) q[0] = q[1] = q[2] = 1.0;
        if (n == 0) q[3] = 1.0;
        return 0;
    };
    auto gm_or_eq = [&](int flag, int mode) -> int {
        // rows first when flag == 0, columns first when flag == 1
        for (int pass = 0; pass <= 1; ++pass) SCHK(sweep(pass == flag, mode));
        return 0;
    };
    auto stage = [&](double *rep) -> int {
        double q[4];
        if (stats(false, q)) return GK_EABI;
        rep[0] = q[0];
        rep[1] = q[1];
        rep[2] = q[1] / q[0];
        return 0;
    };
    int rc = 0, bits = 0;
    for (int k = 0; k < 13; ++k) report[k] = 0.0;
    do {
        if ((rc = stage(report))) break;
        if (report[0] >= 0.10 && report[1] <= 10.0) {
            bits |= 1;
            if (flags & SF_SKIP) {
                bits |= 16;
                break;
            }
        }
        if (flags & SF_GM) {
            // gm_iterate (glpscl.js:143-160): it_max 15, tau 0.90
            double q[4];
            if ((rc = stats(true, q))) break;
            const int flag = q[2] > q[3];
            double ratio = 0.0;
            for (int k = 1; k <= 15; ++k) {
                const double r_old = ratio;
                if (k > 1 && (rc = stats(false, q))) break;
                ratio = q[1] / q[0];
                if (k > 1 && ratio > 0.90 * r_old) break;
                if ((rc = gm_or_eq(flag, SC_GM))) break;
            }
            if (rc || (rc = stage(report + 3))) break;
            bits |= 2;
        }
        if (flags & SF_EQ) {
            double q[4];
            if ((rc = stats(true, q))) break;
            if ((rc = gm_or_eq(q[2] > q[3], SC_EQ))) break;
            if ((rc = stage(report + 6))) break;
            bits |= 4;
        }
        if (flags & SF_2N) {
            if (m) hipLaunchKernelGGL(k_scl_round2n, dim3(cdiv(m, 256)), dim3(256), 0, s, d_r.p, m);
            if (n) hipLaunchKernelGGL(k_scl_round2n, dim3(cdiv(n, 256)), dim3(256), 0, s, d_s.p, n);
            if ((rc = stage(report + 9))) break;
            bits |= 8;
        }
    } while (0);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    report[12] = bits;
    if (m) SCHK(hipMemcpyAsync(rii, d_r.p, sizeof(double) * m, hipMemcpyDeviceToHost, s));
    if (n) SCHK(hipMemcpyAsync(sjj, d_s.p, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    SCHK(hipStreamSynchronize(s));
    if (sweep_ms) *sweep_ms = ms_total;
    if (sweep_bytes) *sweep_bytes = bytes_total;
    return 0;
}

}  // namespace gk

int gk_ctx_device(gk_ctx *);
hipStream_t gk_ctx_stream(gk_ctx *);

extern "C" int gk_scale_prob(gk_ctx *ctx, int m, int n, const int *ptr, const int *ind, const double *val, int flags,
                             double *rii, double *sjj, double *report)
{
    if (!ctx || m < 0 || n < 0 || !ptr || !rii || !sjj || !report) {
        gk::set_err("gk_scale_prob: invalid argument");
        return GK_EABI;
    }
    if (hipSetDevice(gk_ctx_device(ctx)) != hipSuccess) {
        gk::set_err("gk_scale_prob: hipSetDevice failed");
        return GK_EABI;
    }
    return gk::scale_prob_dev(gk_ctx_stream(ctx), m, n, ptr, ind, val, flags, rii, sjj, report, nullptr, nullptr);
}

extern "C" int gk_scale_prob_timed(gk_ctx *ctx, int m, int n, const int *ptr, const int *ind, const double *val,
                                   int flags, double *rii, double *sjj, double *report, double *sweep_ms,
                                   double *sweep_bytes)
{
    if (!ctx || m < 0 || n < 0 || !ptr || !rii || !sjj || !report) {
        gk::set_err("gk_scale_prob: invalid argument");
        return GK_EABI;
    }
    if (hipSetDevice(gk_ctx_device(ctx)) != hipSuccess) {
        gk::set_err("gk_scale_prob: hipSetDevice failed");
        return GK_EABI;
    }
    return gk::scale_prob_dev(gk_ctx_stream(ctx), m, n, ptr, ind, val, flags, rii, sjj, report, sweep_ms,
                              sweep_bytes);
}
