// Microbenchmark: dependent-load latency over a compact table versus the
// same chain spread over a large allocation (one entry per 128 KiB, like the
// rows of AT touched by the pivot row), cold per kernel (the producer
// rewrites the chain between consumers).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int D>
__global__ void k_walk(const long long *__restrict__ big, size_t stride, int n, double *out)
{
    long long i = (blockIdx.x * 64 + threadIdx.x) % n;
#pragma unroll
    for (int d = 0; d < D; ++d) i = big[(size_t)i * stride];
    if (threadIdx.x == 0) out[blockIdx.x] = (double)i;
}

__global__ void k_fill(long long *big, size_t stride, int n, int salt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) big[(size_t)i * stride] = (long long)(((unsigned)i * 2654435761u + (unsigned)salt * 97u) % (unsigned)n);
}

int main()
{
    const int n = 4096, reps = 200;
    long long *big; double *out;
    const size_t span = (size_t)n * 16384 * 8;      // 512 MiB
    CHK(hipMalloc(&big, span)); CHK(hipMalloc(&out, 1 << 20));
    hipStream_t s; CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct V { const char *name; size_t stride; int blocks; void (*fn)(const long long *, size_t, int, double *); };
    V vs[] = {
        {"compact 128B  D1", 16, 64, k_walk<1>},  {"compact 128B  D4", 16, 64, k_walk<4>},
        {"spread 128KiB D1", 16384, 64, k_walk<1>}, {"spread 128KiB D4", 16384, 64, k_walk<4>},
        {"spread 32KiB  D4", 4096, 64, k_walk<4>},
    };
    for (const V &v : vs) {
        hipGraph_t g; hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, s, big, v.stride, n, r);
            hipLaunchKernelGGL(v.fn, dim3(v.blocks), dim3(64), 0, s, big, v.stride, n, out);
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
