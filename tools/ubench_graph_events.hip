// Does hipEventElapsedTime work on events recorded inside a captured graph?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_spin(double *x, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) x[i] = x[i] * 1.0001 + 1.0; }
int main()
{
    double *x; (void)hipMalloc(&x, 1 << 24);
    hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 3; ++mode) {
        hipGraph_t g; hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        hipLaunchKernelGGL(k_spin, dim3(4096), dim3(256), 0, s, x, 1 << 20);
        hipError_t r0 = mode == 0 ? hipEventRecord(e0, s) : hipEventRecordWithFlags(e0, s, hipEventRecordExternal);
        for (int k = 0; k < 10; ++k) hipLaunchKernelGGL(k_spin, dim3(4096), dim3(256), 0, s, x, 1 << 20);
        hipError_t r1 = mode == 0 ? hipEventRecord(e1, s) : hipEventRecordWithFlags(e1, s, hipEventRecordExternal);
        hipError_t rc = hipStreamEndCapture(s, &g);
        hipError_t ri = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipError_t rl = hipGraphLaunch(ge, s);
        hipError_t rs = hipStreamSynchronize(s);
        float ms = -1; hipError_t re = hipEventElapsedTime(&ms, e0, e1);
        hipError_t q0 = hipEventQuery(e0);
        printf("mode %d: rec %s/%s cap %s inst %s launch %s sync %s elapsed %s (%f ms) query %s\n", mode,
               hipGetErrorName(r0), hipGetErrorName(r1), hipGetErrorName(rc), hipGetErrorName(ri), hipGetErrorName(rl),
               hipGetErrorName(rs), hipGetErrorName(re), ms, hipGetErrorName(q0));
        if (mode == 2) {   // manual event-record nodes
            hipGraph_t g2; (void)hipGraphCreate(&g2, 0);
            hipGraphNode_t n0, n1, nk;
            (void)hipGraphAddEventRecordNode(&n0, g2, nullptr, 0, e0);
            hipKernelNodeParams kp{}; void *args[] = {&x, nullptr}; int nn = 1 << 20; args[1] = &nn;
            kp.func = (void *)k_spin; kp.gridDim = dim3(4096); kp.blockDim = dim3(256); kp.kernelParams = args;
            (void)hipGraphAddKernelNode(&nk, g2, &n0, 1, &kp);
            (void)hipGraphAddEventRecordNode(&n1, g2, &nk, 1, e1);
            hipGraphExec_t ge2; hipError_t i2 = hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0);
            hipError_t l2 = hipGraphLaunch(ge2, s); (void)hipStreamSynchronize(s);
            float ms2 = -1; hipError_t e2 = hipEventElapsedTime(&ms2, e0, e1);
            printf("manual nodes: inst %s launch %s elapsed %s (%f ms)\n", hipGetErrorName(i2), hipGetErrorName(l2), hipGetErrorName(e2), ms2);
        }
    }
    return 0;
}
