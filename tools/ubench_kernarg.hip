// Microbenchmark: a short dependent kernel whose pointers come (a) from
// small kernel arguments, (b) from a ~600-byte struct passed by value (like
// SpxDev), (c) from the same struct resident in device memory (one pointer
// argument).  Graph-replayed producer/consumer pairs.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Big {
    const int *idx;
    const double *val;
    double *out;
    int n;
    double pad[72];
};

__global__ void k_small(const int *__restrict__ idx, const double *__restrict__ val, double *out, int n)
{
    int i = (blockIdx.x * blockDim.x + threadIdx.x) & (n - 1);
    i = idx[i];
    i = idx[i];
    if (threadIdx.x == 0) out[blockIdx.x] = val[i];
}
__global__ void k_byval(Big b)
{
    int i = (blockIdx.x * blockDim.x + threadIdx.x) & (b.n - 1);
    i = b.idx[i];
    i = b.idx[i];
    if (threadIdx.x == 0) b.out[blockIdx.x] = b.val[i] + b.pad[(i & 7) + 40];
}
__global__ void k_byptr(const Big *__restrict__ pb)
{
    const Big &b = *pb;
    int i = (blockIdx.x * blockDim.x + threadIdx.x) & (b.n - 1);
    i = b.idx[i];
    i = b.idx[i];
    if (threadIdx.x == 0) b.out[blockIdx.x] = b.val[i] + b.pad[(i & 7) + 40];
}
__global__ void k_produce(int *idx, int n, int salt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) idx[i] = (int)(((unsigned)i * 2654435761u + (unsigned)salt * 40503u) & (unsigned)(n - 1));
}

int main()
{
    const int n = 1 << 14, reps = 200;
    int *idx; double *val, *out; Big *db;
    CHK(hipMalloc(&idx, n * 4)); CHK(hipMalloc(&val, n * 8)); CHK(hipMalloc(&out, 1 << 20)); CHK(hipMalloc(&db, sizeof(Big)));
    CHK(hipMemset(val, 0, n * 8)); CHK(hipMemset(idx, 0, n * 4));
    Big hb{};
    hb.idx = idx; hb.val = val; hb.out = out; hb.n = n;
    CHK(hipMemcpy(db, &hb, sizeof(Big), hipMemcpyHostToDevice));
    hipStream_t s; CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    printf("sizeof(Big) = %zu\n", sizeof(Big));
    for (int kind = 0; kind < 3; ++kind) {
        hipGraph_t g; hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_produce, dim3(n / 256), dim3(256), 0, s, idx, n, r);
            if (kind == 0) hipLaunchKernelGGL(k_small, dim3(96), dim3(256), 0, s, idx, val, out, n);
            if (kind == 1) hipLaunchKernelGGL(k_byval, dim3(96), dim3(256), 0, s, hb);
            if (kind == 2) hipLaunchKernelGGL(k_byptr, dim3(96), dim3(256), 0, s, db);
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
        const char *nm[] = {"small args", "600-byte struct by value", "struct in device memory"};
        printf("%-28s %7.2f us/pair\n", nm[kind], 1000.0 * best / reps);
        (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    }
    return 0;
}
