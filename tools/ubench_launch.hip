// Microbenchmark: per-kernel cost of short dependent kernels replayed from a
// HIP graph (the dual pivot pipeline is a chain of such kernels).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_empty(int *x) { if (x == nullptr) x[0] = 1; }
__global__ void k_load1(const int *a, int *b, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) b[i] = a[i] + 1; }
__global__ void k_load3(const int *a, const int *c, int *b, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { int k = a[i]; int v = c[k]; b[i] = a[v] + 1; }
}
__device__ double bsum(double v, double *sh)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0;
    if (w == 0) { r = lane < nw ? sh[lane] : 0; for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o); if (lane == 0) sh[0] = r; }
    __syncthreads();
    r = sh[0];
    __syncthreads();
    return r;
}
__global__ void k_red(const double *a, double *b, int n)
{
    __shared__ double sh[16];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    double v = i < n ? a[i] : 0;
    v = bsum(v, sh); v = bsum(v * 0.5, sh); v = bsum(v * 0.25, sh);
    if (threadIdx.x == 0) b[blockIdx.x] = v;
}
__global__ void k_atomic(const double *a, unsigned long long *mx, int n)
{
    __shared__ double sh[16];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    double v = i < n ? a[i] : 0;
    v = bsum(v, sh);
    if (threadIdx.x == 0) atomicMax(mx, (unsigned long long)__double_as_longlong(v));
}
__global__ void k_onewg(const double *a, double *b, int n)
{
    __shared__ double sh[16];
    double v = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) v += a[i];
    v = bsum(v, sh);
    if (threadIdx.x == 0) b[0] = v;
}

int main()
{
    const int n = 16384, reps = 200;
    int *ia, *ib, *ic; double *da, *db; unsigned long long *mx;
    CHK(hipMalloc(&ia, n * 4)); CHK(hipMalloc(&ib, n * 4)); CHK(hipMalloc(&ic, n * 4));
    CHK(hipMalloc(&da, n * 8)); CHK(hipMalloc(&db, n * 8)); CHK(hipMalloc(&mx, 8));
    CHK(hipMemset(ia, 0, n * 4)); CHK(hipMemset(ic, 0, n * 4)); CHK(hipMemset(da, 0, n * 8));
    hipStream_t s; CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const char *names[] = {"empty 64x256", "load1 64x256", "load3 64x256", "3x blocksum 64x256", "blocksum+atomicMax 64x256",
                           "one WG 1024 reduce 16K", "one WG 256 reduce 16K", "empty 2048x256", "load1 2048x256 (n=512K?)"};
    for (int kind = 0; kind < 8; ++kind) {
        hipGraph_t g; hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < reps; ++r) {
            switch (kind) {
            case 0: hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, ib); break;
            case 1: hipLaunchKernelGGL(k_load1, dim3(64), dim3(256), 0, s, ia, ib, n); break;
            case 2: hipLaunchKernelGGL(k_load3, dim3(64), dim3(256), 0, s, ia, ic, ib, n); break;
            case 3: hipLaunchKernelGGL(k_red, dim3(64), dim3(256), 0, s, da, db, n); break;
            case 4: hipLaunchKernelGGL(k_atomic, dim3(64), dim3(256), 0, s, da, mx, n); break;
            case 5: hipLaunchKernelGGL(k_onewg, dim3(1), dim3(1024), 0, s, da, db, n); break;
            case 6: hipLaunchKernelGGL(k_onewg, dim3(1), dim3(256), 0, s, da, db, n); break;
            case 7: hipLaunchKernelGGL(k_empty, dim3(2048), dim3(256), 0, s, ib); break;
            }
        }
        CHK(hipStreamEndCapture(s, &g));
        CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CHK(hipGraphLaunch(ge, s)); CHK(hipStreamSynchronize(s));
        hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
        CHK(hipEventRecord(e0, s)); CHK(hipGraphLaunch(ge, s)); CHK(hipEventRecord(e1, s)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-32s %7.2f us/kernel\n", names[kind], 1000.0 * ms / reps);
        hipGraphExecDestroy(ge); hipGraphDestroy(g);
    }
    return 0;
}
