// Microbenchmark: cost model of the short dependent kernels of the dual
// pivot pipeline, replayed from a HIP graph.  Each variant is one kernel
// shape (blocks x threads) doing D dependent global-load trips (index
// chains through a 16K-entry table, L2-resident after the first replay) and
// R block reductions; the per-kernel time separates launch cost, trip
// latency and reduction cost.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ double bsum(double v, double *sh)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0;
    for (int k = 0; k < nw; ++k) r += sh[k];
    __syncthreads();
    return r;
}

// D dependent trips, R block reductions
template <int D, int R>
__global__ void k_chain(const int *__restrict__ idx, const double *__restrict__ val, double *out, int n)
{
    __shared__ double sh[16];
    int i = (blockIdx.x * blockDim.x + threadIdx.x) & (n - 1);
#pragma unroll
    for (int d = 0; d < D; ++d) i = idx[i];
    double v = val[i];
#pragma unroll
    for (int r = 0; r < R; ++r) v = bsum(v, sh) * 1e-3;
    if (threadIdx.x == 0) out[blockIdx.x] = v;
}

// D dependent trips with 8 independent loads per trip per thread
template <int D>
__global__ void k_chain8(const int *__restrict__ idx, const double *__restrict__ val, double *out, int n)
{
    int i[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) i[u] = (blockIdx.x * blockDim.x + threadIdx.x + u * 4099) & (n - 1);
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int u = 0; u < 8; ++u) i[u] = idx[i[u]];
    double v = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) v += val[i[u]];
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

// producer: rewrites the index table (a permutation step) so that the
// consumer's loads find fresh data written by another kernel (other XCDs)
__global__ void k_produce(int *idx, int n, int salt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) idx[i] = (int)(((unsigned)i * 2654435761u + (unsigned)salt * 40503u) & (unsigned)(n - 1));
}

struct V {
    const char *name;
    void (*fn)(const int *, const double *, double *, int);
    int blocks, threads;
};

int main()
{
    const int n = 1 << 14, reps = 200;
    int *idx; double *val, *out;
    CHK(hipMalloc(&idx, n * 4)); CHK(hipMalloc(&val, n * 8)); CHK(hipMalloc(&out, (1 << 20) * 8));
    std::vector<int> h(n);
    for (int i = 0; i < n; ++i) h[i] = (int)((i * 2654435761u) & (n - 1));
    CHK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
    CHK(hipMemset(val, 0, n * 8));
    hipStream_t s; CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    V vs[] = {
        {"D0 R0  96x256", k_chain<0, 0>, 96, 256},
        {"D1 R0  96x256", k_chain<1, 0>, 96, 256},
        {"D2 R0  96x256", k_chain<2, 0>, 96, 256},
        {"D4 R0  96x256", k_chain<4, 0>, 96, 256},
        {"D1 R1  96x256", k_chain<1, 1>, 96, 256},
        {"D1 R3  96x256", k_chain<1, 3>, 96, 256},
        {"D1 R0   1x1024", k_chain<1, 0>, 1, 1024},
        {"D4 R0   1x1024", k_chain<4, 0>, 1, 1024},
        {"D1 R3   1x1024", k_chain<1, 3>, 1, 1024},
        {"D1 R0 256x1024", k_chain<1, 0>, 256, 1024},
        {"D2 R0 256x1024", k_chain<2, 0>, 256, 1024},
        {"D1 R1 256x1024", k_chain<1, 1>, 256, 1024},
        {"D1 R0  64x1024", k_chain<1, 0>, 64, 1024},
        {"D1 R0 712x256", k_chain<1, 0>, 712, 256},
        {"D2 R1 712x256", k_chain<2, 1>, 712, 256},
        {"8x D1 256x1024", k_chain8<1>, 256, 1024},
        {"8x D2 256x1024", k_chain8<2>, 256, 1024},
    };
    for (const V &v : vs) {
        hipGraph_t g; hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(v.fn, dim3(v.blocks), dim3(v.threads), 0, s, idx, val, out, n);
        CHK(hipStreamEndCapture(s, &g));
        CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CHK(hipGraphLaunch(ge, s)); CHK(hipStreamSynchronize(s));
        hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
        float best = 1e30f;
        for (int k = 0; k < 3; ++k) {
            CHK(hipEventRecord(e0, s)); CHK(hipGraphLaunch(ge, s)); CHK(hipEventRecord(e1, s)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-20s %7.2f us/kernel\n", v.name, 1000.0 * best / reps);
        (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    }
    // producer / consumer pairs: D dependent trips over data the previous
    // kernel wrote
    struct P { const char *name; void (*fn)(const int *, const double *, double *, int); int blocks, threads; };
    P ps[] = {
        {"pair D0  96x256", k_chain<0, 0>, 96, 256},
        {"pair D1  96x256", k_chain<1, 0>, 96, 256},
        {"pair D2  96x256", k_chain<2, 0>, 96, 256},
        {"pair D4  96x256", k_chain<4, 0>, 96, 256},
        {"pair D1   1x256", k_chain<1, 0>, 1, 256},
        {"pair D4   1x256", k_chain<4, 0>, 1, 256},
    };
    for (const P &v : ps) {
        hipGraph_t g; hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_produce, dim3(n / 256), dim3(256), 0, s, idx, n, r);
            hipLaunchKernelGGL(v.fn, dim3(v.blocks), dim3(v.threads), 0, s, idx, val, out, n);
        }
        CHK(hipStreamEndCapture(s, &g));
        CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CHK(hipGraphLaunch(ge, s)); CHK(hipStreamSynchronize(s));
        hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
        float best = 1e30f;
        for (int k = 0; k < 3; ++k) {
            CHK(hipEventRecord(e0, s)); CHK(hipGraphLaunch(ge, s)); CHK(hipEventRecord(e1, s)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-20s %7.2f us/pair\n", v.name, 1000.0 * best / reps);
        (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    }
    return 0;
}
