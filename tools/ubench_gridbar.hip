// Microbenchmark: cost of a grid-wide barrier inside one persistent
// (cooperatively launched) kernel, against the kernel-boundary cost of a
// chain of graph-replayed launches (tools/ubench_launch.hip).  Decides
// whether the dual pivot pipeline (7 dependent kernels per pivot) is worth
// folding into one kernel with grid barriers.
// Every spin loop is bounded: a barrier that never completes sets *err and
// the kernel drains.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
#include <vector>
namespace cg = cooperative_groups;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Bar {
    unsigned *count;
    unsigned *gen;
    int *err;
};

__device__ __forceinline__ void grid_bar(const Bar &b, unsigned nblocks, unsigned &local_gen)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = local_gen;
        __threadfence();
        const unsigned a = __hip_atomic_fetch_add(b.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (a == nblocks - 1) {
            __hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            long spins = 0;
            while (__hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > (1L << 26)) { atomicExch(b.err, 1); break; }
            }
        }
        local_gen = g + 1;
    }
    __syncthreads();
}

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

// nbar barriers, nothing else
__global__ void k_bars(Bar b, int nbar)
{
    unsigned lg = 0;
    for (int r = 0; r < nbar; ++r) {
        grid_bar(b, gridDim.x, lg);
        if (*(volatile int *)b.err) return;
    }
}

__global__ void k_cgbars(int nbar)
{
    cg::grid_group g = cg::this_grid();
    for (int r = 0; r < nbar; ++r) g.sync();
}

// phase work: each block reads a chunk, block-reduces, publishes a partial;
// after the barrier every block reads all partials (a broadcast)
__global__ void k_phases(Bar b, int nphase, const double *a, double *part, int n)
{
    __shared__ double sh[16];
    unsigned lg = 0;
    double acc = 0.0;
    for (int r = 0; r < nphase; ++r) {
        double v = 0.0;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v += a[i] * (1.0 + acc * 1e-30);
        v = bsum(v, sh);
        if (threadIdx.x == 0) part[(r & 1) * gridDim.x + blockIdx.x] = v;
        grid_bar(b, gridDim.x, lg);
        if (*(volatile int *)b.err) return;
        double s = 0.0;
        for (int k = threadIdx.x; k < (int)gridDim.x; k += blockDim.x) s += part[(r & 1) * gridDim.x + k];
        acc = bsum(s, sh);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) part[2 * gridDim.x] = acc;
}

__global__ void k_phase1(const double *a, double *part, int n, int r)
{
    __shared__ double sh[16];
    double s = 0.0;
    if (r > 0)
        for (int k = threadIdx.x; k < (int)gridDim.x; k += blockDim.x) s += part[((r - 1) & 1) * gridDim.x + k];
    const double acc = bsum(s, sh);
    double v = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v += a[i] * (1.0 + acc * 1e-30);
    v = bsum(v, sh);
    if (threadIdx.x == 0) part[(r & 1) * gridDim.x + blockIdx.x] = v;
}

int main()
{
    int dev = 0, ncu = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_phases, 256, 0));
    printf("CUs %d, k_phases blocks/CU %d\n", ncu, occ);
    Bar b;
    CHK(hipMalloc(&b.count, 4)); CHK(hipMalloc(&b.gen, 4)); CHK(hipMalloc(&b.err, 4));
    const int n = 1 << 20;
    double *a, *part;
    CHK(hipMalloc(&a, n * 8)); CHK(hipMalloc(&part, 8 * 8192));
    CHK(hipMemset(a, 0, n * 8));
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const int nbar = 2000;
    for (int nb : {64, 128, 256, 512, 1024}) {
        if (nb > ncu * occ) continue;
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipMemset(b.count, 0, 4)); CHK(hipMemset(b.gen, 0, 4)); CHK(hipMemset(b.err, 0, 4));
            int nbar_ = nbar;
            void *args[] = {&b, &nbar_};
            CHK(hipEventRecord(e0, s));
            CHK(hipLaunchCooperativeKernel((void *)k_bars, dim3(nb), dim3(256), args, 0, s));
            CHK(hipEventRecord(e1, s));
            CHK(hipStreamSynchronize(s));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            int err; CHK(hipMemcpy(&err, b.err, 4, hipMemcpyDeviceToHost));
            if (rep) printf("custom barrier  blocks %4d: %.3f us/barrier (err %d)\n", nb, ms * 1000.0 / nbar, err);
        }
        for (int rep = 0; rep < 2; ++rep) {
            int nbar_ = nbar;
            void *args[] = {&nbar_};
            CHK(hipEventRecord(e0, s));
            CHK(hipLaunchCooperativeKernel((void *)k_cgbars, dim3(nb), dim3(256), args, 0, s));
            CHK(hipEventRecord(e1, s));
            CHK(hipStreamSynchronize(s));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) printf("cg grid.sync    blocks %4d: %.3f us/barrier\n", nb, ms * 1000.0 / nbar);
        }
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipMemset(b.count, 0, 4)); CHK(hipMemset(b.gen, 0, 4)); CHK(hipMemset(b.err, 0, 4));
            int np = nbar, nn = 65536;
            void *args[] = {&b, &np, &a, &part, &nn};
            CHK(hipEventRecord(e0, s));
            CHK(hipLaunchCooperativeKernel((void *)k_phases, dim3(nb), dim3(256), args, 0, s));
            CHK(hipEventRecord(e1, s));
            CHK(hipStreamSynchronize(s));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            int err; CHK(hipMemcpy(&err, b.err, 4, hipMemcpyDeviceToHost));
            if (rep) printf("persistent phase blocks %4d: %.3f us/phase (err %d)\n", nb, ms * 1000.0 / np, err);
        }
        // same phases as a graph of separate kernels
        {
            const int np = 200, nn = 65536;
            hipGraph_t g; hipGraphExec_t ge;
            CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (int r = 0; r < np; ++r) hipLaunchKernelGGL(k_phase1, dim3(nb), dim3(256), 0, s, a, part, nn, r);
            CHK(hipStreamEndCapture(s, &g));
            CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CHK(hipGraphLaunch(ge, s));
            CHK(hipStreamSynchronize(s));
            CHK(hipEventRecord(e0, s));
            for (int k = 0; k < 5; ++k) CHK(hipGraphLaunch(ge, s));
            CHK(hipEventRecord(e1, s));
            CHK(hipStreamSynchronize(s));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            printf("graph kernels   blocks %4d: %.3f us/phase\n", nb, ms * 1000.0 / (5 * np));
            CHK(hipGraphExecDestroy(ge)); CHK(hipGraphDestroy(g));
        }
    }
    return 0;
}
