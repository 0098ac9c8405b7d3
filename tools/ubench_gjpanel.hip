// Microbenchmark: the one-workgroup Gauss-Jordan panel of the re-inversion
// (k_gjc_panel, gk_reinvert.hip) in isolation, with device wall-clock stamps
// (s_memrealtime, 100 MHz) at entry, after the panel load, after every step
// and at exit, for variants of the per-step choice:
//   MODE 0  as the library: per-wave wave_best, the winner's row values
//           moved by shuffles, cross-wave choice by a second wave_best
//   MODE 1  the winning lane stores its row values to LDS itself
//   MODE 2  MODE 1 + the cross-wave choice by a serial scan of the NW
//           published candidates (every lane, LDS broadcast reads)
//   MODE 3  MODE 2 + the per-wave choice as one u64 max over packed keys
//           (|x| bits with the low 13 mantissa bits replaced by 8191 - row)
// Prints per-phase times and checks every variant's pivots and panel against
// MODE 0.  Build: hipcc --offload-arch=gfx950 -O3 -I glpk.js_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
#include "gk_device.h"
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

using namespace gk;
constexpr int NONE = 0x7fffffff;

__device__ __forceinline__ unsigned long long stamp() { return __builtin_amdgcn_s_memrealtime(); }

template <int NT, int RPT, int B, int MODE>
__global__ void __launch_bounds__(NT) k_panel(double *__restrict__ P, int k, int c0, int bo, double *__restrict__ Qm,
                                              int tg0, int *__restrict__ piv_step, int *__restrict__ piv,
                                              int *__restrict__ flag, double tiny, unsigned long long *__restrict__ ts)
{
    constexpr int NW = NT / 64;
    __shared__ Cand shc[2][NW];
    __shared__ unsigned long long shk[2][NW];
    __shared__ double shr[2][NW][B];
    __shared__ int rsl[B];
    const unsigned long long t0 = stamp();
    const unsigned long long c0c = clock64();
    if (MODE < 4 && *flag) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int b = min(B, bo - c0);
    double x[RPT][B];
    bool live[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = tid + j * NT;
        const int rc = min(r, k - 1);
        live[j] = r < k && piv_step[rc] == NONE;
#pragma unroll
        for (int c = 0; c < B; ++c) x[j][c] = (r < k && c < b) ? P[(size_t)(c0 + c) * k + rc] : 0.0;
    }
    // force the loads to complete before the stamp
    double sink = 0.0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) sink += x[j][0];
    if (sink == 12345.678) flag[1] = 1;
    __syncthreads();
    if (tid == 0) ts[0] = stamp() - t0;
#pragma unroll 1
    for (int i = 0; i < B; ++i) {
        const int par = i & 1;
        int rs;
        double ipv;
        double fr[B];
        if (MODE >= 3) {
            unsigned long long key = 0;
            int jb = 0;
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const double v = fabs(x[j][0]);
                const unsigned long long kk = (live[j] && v > 0.0)
                    ? ((dbits(v) & ~0x1fffull) | (unsigned long long)(0x1fff - (tid + j * NT))) : 0ull;
                if (kk > key) { key = kk; jb = j; }
            }
            const unsigned long long wk = __ockl_wfred_max_u64(key);
            if (MODE >= 4) {
                const bool win = wk != 0 && key == wk;
#pragma unroll
                for (int j = 0; j < RPT; ++j)
                    if (win && j == jb) {
#pragma unroll
                        for (int cc = 0; cc < B; ++cc) shr[par][w][cc] = x[j][cc];
                    }
            } else if (wk != 0 && key == wk) {          // the winning lane (unique key)
#pragma unroll
                for (int cc = 0; cc < B; ++cc) {
                    double mine = 0.0;
#pragma unroll
                    for (int j = 0; j < RPT; ++j) if (j == jb) mine = x[j][cc];
                    shr[par][w][cc] = mine;
                }
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
            if (bk == 0) { if (tid == 0) *flag = 1 + tg0 + i; return; }
            rs = 0x1fff - (int)(bk & 0x1fff);
            const double pv = shr[par][ws][0];
            if (fabs(pv) <= tiny) { if (tid == 0) *flag = 1 + tg0 + i; return; }
            ipv = 1.0 / pv;
            fr[0] = ipv;
#pragma unroll
            for (int cc = 1; cc < B; ++cc) fr[cc] = shr[par][ws][cc] * ipv;
        } else {
            Cand c; c.k1 = 0.0; c.k2 = 0.0; c.idx = 0; c.aux = 0;
            int jb = 0;
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const double v = fabs(x[j][0]);
                if (live[j] && v > 0.0 && (c.idx == 0 || v > c.k1)) { c.k1 = v; c.idx = tid + j * NT + 1; jb = j; }
            }
            const Cand wb = wave_best<0>(c);
            if (MODE == 0) {
                const int src = wb.idx ? ((wb.idx - 1) & 63) : 0;
                double rowv[B];
#pragma unroll
                for (int cc = 0; cc < B; ++cc) {
                    double mine = 0.0;
#pragma unroll
                    for (int j = 0; j < RPT; ++j) if (j == jb) mine = x[j][cc];
                    rowv[cc] = __shfl(mine, src);
                }
                if (lane == 0) {
                    shc[par][w] = wb;
#pragma unroll
                    for (int cc = 0; cc < B; ++cc) shr[par][w][cc] = rowv[cc];
                }
            } else {
                if (wb.idx != 0 && c.idx == wb.idx) {
#pragma unroll
                    for (int cc = 0; cc < B; ++cc) {
                        double mine = 0.0;
#pragma unroll
                        for (int j = 0; j < RPT; ++j) if (j == jb) mine = x[j][cc];
                        shr[par][w][cc] = mine;
                    }
                }
                if (lane == 0) shc[par][w] = wb;
            }
            __syncthreads();
            Cand best;
            if (MODE == 2) {
                best.k1 = 0.0; best.k2 = 0.0; best.idx = 0; best.aux = 0;
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    const Cand e = shc[par][q];
                    if (e.idx != 0 && (best.idx == 0 || e.k1 > best.k1)) best = e;   // waves ascend in row
                }
            } else {
                Cand e;
                if (lane < NW) e = shc[par][lane];
                else { e.k1 = 0.0; e.k2 = 0.0; e.idx = 0; e.aux = 0; }
                best = wave_best<0>(e);
            }
            if (best.idx == 0 || best.k1 <= tiny) { if (tid == 0) *flag = 1 + tg0 + i; return; }
            rs = best.idx - 1;
            const int ws = (rs % NT) >> 6;
            ipv = 1.0 / shr[par][ws][0];
            fr[0] = ipv;
#pragma unroll
            for (int cc = 1; cc < B; ++cc) fr[cc] = shr[par][ws][cc] * ipv;
        }
        if (tid == 0) rsl[i] = rs;
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
        if (tid == 0) ts[1 + i] = stamp() - t0;
    }
    __syncthreads();
    if (tid < b) {
        piv[tg0 + tid] = rsl[tid];
        piv_step[rsl[tid]] = tg0 + tid;
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = tid + j * NT;
        if (r >= k) continue;
#pragma unroll
        for (int c = 0; c < B; ++c) {
            if (c < b) P[(size_t)(c0 + c) * k + r] = x[j][c];
            if (MODE < 4) Qm[(size_t)c * k + r] = (c < b) ? x[j][c] - (r == rsl[c] ? 1.0 : 0.0) : 0.0;
        }
    }
    __syncthreads();
    if (tid == 0) {
        ts[1 + B] = stamp() - t0;
        ts[2 + B] = clock64() - c0c;
    }
}

template <int NT, int RPT, int B, int MODE>
int run(int k, const std::vector<double> &h, std::vector<double> &outP, std::vector<int> &outPiv, const char *name)
{
    const int bo = 64;
    double *P, *Q; int *ps, *pv, *fl; unsigned long long *ts;
    CHK(hipMalloc(&P, sizeof(double) * k * bo)); CHK(hipMalloc(&Q, sizeof(double) * k * B));
    CHK(hipMalloc(&ps, sizeof(int) * k)); CHK(hipMalloc(&pv, sizeof(int) * bo)); CHK(hipMalloc(&fl, 8));
    CHK(hipMalloc(&ts, sizeof(unsigned long long) * 64 * 16));
    std::vector<int> none(k, NONE);
    double best = 1e30, cyc = 0.0; std::vector<double> acc(B + 2, 0.0); int reps = 20;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < reps + 2; ++rep) {
        CHK(hipMemcpy(P, h.data(), sizeof(double) * k * bo, hipMemcpyHostToDevice));
        CHK(hipMemcpy(ps, none.data(), sizeof(int) * k, hipMemcpyHostToDevice));
        CHK(hipMemset(fl, 0, 8));
        hipEventRecord(e0);
        for (int i0 = 0; i0 < bo; i0 += B)
            hipLaunchKernelGGL((k_panel<NT, RPT, B, MODE>), dim3(1), dim3(NT), 0, 0, P, k, i0, bo, Q, i0, ps, pv, fl,
                               1e-300, ts + (i0 / B) * 16);
        hipEventRecord(e1);
        CHK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (rep >= 2) {
            best = std::min(best, (double)ms);
            std::vector<unsigned long long> t(64 * 16);
            CHK(hipMemcpy(t.data(), ts, t.size() * 8, hipMemcpyDeviceToHost));
            for (int p = 0; p < bo / B; ++p) {
                for (int q = 0; q < B + 2; ++q) acc[q] += t[p * 16 + q] * 10e-3 / (reps * (bo / B));
                cyc += (double)t[p * 16 + B + 2] / (reps * (bo / B));
            }
        }
    }
    int f = 0; CHK(hipMemcpy(&f, fl, 4, hipMemcpyDeviceToHost));
    outP.resize((size_t)k * bo); outPiv.resize(bo);
    CHK(hipMemcpy(outP.data(), P, sizeof(double) * k * bo, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(outPiv.data(), pv, sizeof(int) * bo, hipMemcpyDeviceToHost));
    printf("%-28s k=%d flag=%d  64 columns: %.1f us (%.2f us/panel)  load %.2f us, steps", name, k, f, best * 1e3,
           best * 1e3 / (bo / B), acc[0]);
    for (int q = 1; q <= B; ++q) printf(" %.2f", acc[q] - acc[q - 1]);
    printf(", store %.2f us; %.0f shader clocks per panel = %.2f GHz\n", acc[B + 1] - acc[B], cyc,
           cyc / (acc[B + 1] * 1e3));
    hipFree(P); hipFree(Q); hipFree(ps); hipFree(pv); hipFree(fl); hipFree(ts);
    return 0;
}

int main(int argc, char **argv)
{
    const int k = argc > 1 ? atoi(argv[1]) : 4096;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::vector<double> h((size_t)k * 64);
    for (auto &v : h) v = u(g);
    std::vector<double> P0, P1; std::vector<int> v0, v1;
    auto cmp = [&](const char *n) {
        int dp = 0; double dm = 0;
        for (int i = 0; i < 64; ++i) dp += v0[i] != v1[i];
        for (size_t i = 0; i < P0.size(); ++i) dm = std::max(dm, std::fabs(P0[i] - P1[i]));
        printf("   %s vs mode 0: %d pivots differ, max |dP| %.3g\n", n, dp, dm);
    };
    if (run<1024, 4, 8, 0>(k, h, P0, v0, "NT1024 RPT4 B8 mode0")) return 1;
    run<1024, 4, 8, 1>(k, h, P1, v1, "NT1024 RPT4 B8 mode1"); cmp("mode1");
    run<1024, 4, 8, 2>(k, h, P1, v1, "NT1024 RPT4 B8 mode2"); cmp("mode2");
    run<1024, 4, 8, 3>(k, h, P1, v1, "NT1024 RPT4 B8 mode3"); cmp("mode3");
    run<512, 8, 8, 2>(k, h, P1, v1, "NT512 RPT8 B8 mode2"); cmp("512/2");
    run<512, 8, 8, 3>(k, h, P1, v1, "NT512 RPT8 B8 mode3"); cmp("512/3");
    run<256, 16, 8, 3>(k, h, P1, v1, "NT256 RPT16 B8 mode3"); cmp("256/3");
    run<512, 8, 8, 4>(k, h, P1, v1, "NT512 RPT8 B8 mode4"); cmp("512/4");
    run<1024, 4, 8, 4>(k, h, P1, v1, "NT1024 RPT4 B8 mode4"); cmp("1024/4");
    run<512, 8, 4, 4>(k, h, P1, v1, "NT512 RPT8 B4 mode4");
    run<512, 4, 16, 4>(k, h, P1, v1, "NT512 RPT4 B16 mode4 (k<=2048)");
    return 0;
}
