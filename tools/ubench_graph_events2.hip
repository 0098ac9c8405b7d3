#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k_spin(double *x, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) x[i] = x[i] * 1.0001 + 1.0; }
int main()
{
    double *x; (void)hipMalloc(&x, 1 << 24);
    hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int variant = 0; variant < 3; ++variant) {
        std::vector<hipEvent_t> ev(16);
        for (auto &e : ev) (void)hipEventCreate(&e);
        hipGraph_t g; hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int t = 0; t < 8; ++t) {
            hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, x, 1 << 14);
            (void)hipEventRecordWithFlags(ev[2 * t], s, hipEventRecordExternal);
            hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, x, 1 << 14);
            (void)hipEventRecordWithFlags(ev[2 * t + 1], s, hipEventRecordExternal);
            if (variant >= 1) hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, x, 1 << 14);
        }
        if (variant == 2) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, x, 1);
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipGraphLaunch(ge, s);
            (void)hipStreamSynchronize(s);
            for (int t = 0; t < 8; ++t) {
                float ms = -1; hipError_t e = hipEventElapsedTime(&ms, ev[2 * t], ev[2 * t + 1]);
                printf("variant %d rep %d t %d: %s %.4f\n", variant, rep, t, hipGetErrorName(e), ms);
            }
        }
    }
    return 0;
}
