// which __ockl_wfred_* primitives reduce over all 64 lanes on gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
extern "C" __device__ double __ockl_wfred_add_f64(double);
extern "C" __device__ double __ockl_wfred_max_f64(double);
extern "C" __device__ unsigned long long __ockl_wfred_min_u64(unsigned long long);
extern "C" __device__ unsigned long long __ockl_wfred_max_u64(unsigned long long);
extern "C" __device__ unsigned int __ockl_wfred_min_u32(unsigned int);
extern "C" __device__ unsigned int __ockl_wfred_max_u32(unsigned int);
__global__ void k(double *o)
{
    const int l = threadIdx.x;
    const unsigned long long v = (unsigned long long)((l * 37) % 64) << 33 | (unsigned long long)((l * 11) % 64);
    double r[8];
    r[0] = __ockl_wfred_add_f64((double)l);
    r[1] = __ockl_wfred_max_f64((double)((l * 37) % 64));
    r[2] = (double)(__ockl_wfred_min_u64(v + 5) >> 33);
    r[3] = (double)(__ockl_wfred_max_u64(v) >> 33);
    r[4] = (double)__ockl_wfred_min_u32(100u + (unsigned)((l * 37) % 64));
    r[5] = (double)__ockl_wfred_max_u32((unsigned)((l * 37) % 64));
    r[6] = (double)(__ockl_wfred_max_u64(v) & 0xffffffffull);
    r[7] = (double)(__ockl_wfred_min_u64(v + 5) & 0xffffffffull);
    for (int i = 0; i < 8; ++i) o[l * 8 + i] = r[i];
}
int main()
{
    double *d; hipMalloc(&d, 64 * 8 * 8);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    double h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *nm[8] = {"add_f64 (2016)", "max_f64 (63)", "min_u64 hi (0)", "max_u64 hi (63)", "min_u32 (100)", "max_u32 (63)", "max_u64 lo", "min_u64 lo (5)"};
    for (int i = 0; i < 8; ++i) printf("%-18s lane0 %g lane63 %g\n", nm[i], h[i], h[63 * 8 + i]);
    return 0;
}
