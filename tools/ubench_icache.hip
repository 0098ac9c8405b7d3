// Microbenchmark: what straight-line code costs a short kernel replayed from a
// HIP graph (instruction fetch after each dispatch).  Every variant executes
// the same N scalar no-ops (s_nop 0, 4 bytes each, one per clock per wave):
// "unrolled" as N straight-line instructions (4N bytes of code), "rolled" as
// a 64-instruction loop body (256 bytes) run N/64 times.  256 blocks of 1024
// or 64 threads, launched alternately with a second kernel of the same shape
// (another code address); per-launch time from events around the replay.
// Result (MI355X, profiles/r03_ubench_icache.txt): see DESIGN.md §4.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int N, int ROLL, int TAG>
__global__ void __launch_bounds__(1024) k_code(int *out)
{
    if (ROLL) {
#pragma unroll 1
        for (int i = 0; i < N / 64; ++i) {
            asm volatile(".rept 64\n s_nop 0\n .endr" ::: "memory");
        }
    } else {
        asm volatile(".rept %0\n s_nop 0\n .endr" ::"i"(N) : "memory");
    }
    if (out == nullptr) out[TAG] = 1;
}

template <int N, int ROLL>
static int run(hipStream_t s, int *out, int threads, const char *name)
{
    const int reps = 200;
    hipGraph_t g; hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < reps; ++r) {
        if (r & 1) hipLaunchKernelGGL((k_code<N, ROLL, 1>), dim3(256), dim3(threads), 0, s, out);
        else hipLaunchKernelGGL((k_code<N, ROLL, 0>), dim3(256), dim3(threads), 0, s, out);
    }
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, s)); CHK(hipStreamSynchronize(s));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
        CHK(hipEventRecord(e0, s)); CHK(hipGraphLaunch(ge, s)); CHK(hipEventRecord(e1, s)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    printf("%-9s %4d threads  N=%5d (%6d B of code)  %8.2f us/kernel\n", name, threads, N, ROLL ? 256 : 4 * N,
           1000.0 * best / reps);
    (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    return 0;
}

template <int N>
static int pair(hipStream_t s, int *out)
{
    for (int th : {1024, 64})
        if (run<N, 0>(s, out, th, "unrolled") || run<N, 1>(s, out, th, "rolled")) return 1;
    return 0;
}

int main()
{
    int *out; CHK(hipMalloc(&out, 64));
    hipStream_t s; CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (pair<64>(s, out) || pair<256>(s, out) || pair<1024>(s, out) || pair<2048>(s, out) || pair<4096>(s, out) ||
        pair<8192>(s, out))
        return 1;
    return 0;
}
