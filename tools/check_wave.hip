// Device check of the wave-reduction helpers of gk_device.h against naive
// references (random candidates, all three modes, partial activity).
#include "../glpk.js_amd/csrc/gk_device.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace gk;

__global__ void k_check(const Cand *in, Cand *out, double *sums, int active)
{
    const int lane = threadIdx.x;
    Cand c = in[blockIdx.x * 64 + lane];
    if (lane < active) {
        Cand b0 = wave_best<0>(c), b1 = wave_best<1>(c), b2 = wave_best<2>(c);
        double s = wsum(c.k1), mx = wmax(c.k2);
        if (lane == 0) {
            out[blockIdx.x * 3 + 0] = b0;
            out[blockIdx.x * 3 + 1] = b1;
            out[blockIdx.x * 3 + 2] = b2;
            sums[blockIdx.x * 2] = s;
            sums[blockIdx.x * 2 + 1] = mx;
        }
    }
}

template <int MODE>
static bool better_h(const Cand &a, const Cand &b)
{
    if (a.idx == 0) return false;
    if (b.idx == 0) return true;
    if (MODE == 0) { if (a.k1 != b.k1) return a.k1 > b.k1; }
    else if (MODE == 1) { if (a.k1 != b.k1) return a.k1 < b.k1; if (a.k2 != b.k2) return a.k2 > b.k2; }
    else { if (a.k2 != b.k2) return a.k2 > b.k2; }
    return a.idx < b.idx;
}

int main()
{
    const int B = 4096;
    std::vector<Cand> h(B * 64);
    srand(7);
    for (int b = 0; b < B; ++b)
        for (int l = 0; l < 64; ++l) {
            Cand &c = h[b * 64 + l];
            const int kind = rand() % 4;
            c.k1 = (kind == 0) ? 0.0 : (double)(rand() % 7) * 0.5;
            c.k2 = (double)(rand() % 5);
            c.idx = (rand() % 3 == 0) ? 0 : 1 + (b * 64 + l) * 3 % 1000 + l;
            c.aux = rand();
        }
    Cand *din, *dout; double *ds;
    hipMalloc(&din, h.size() * sizeof(Cand)); hipMalloc(&dout, B * 3 * sizeof(Cand)); hipMalloc(&ds, B * 2 * 8);
    hipMemcpy(din, h.data(), h.size() * sizeof(Cand), hipMemcpyHostToDevice);
    int bad = 0;
    for (int active : {64, 37}) {
        hipLaunchKernelGGL(k_check, dim3(B), dim3(64), 0, 0, din, dout, ds, active);
        std::vector<Cand> o(B * 3); std::vector<double> s(B * 2);
        hipMemcpy(o.data(), dout, o.size() * sizeof(Cand), hipMemcpyDeviceToHost);
        hipMemcpy(s.data(), ds, s.size() * 8, hipMemcpyDeviceToHost);
        for (int b = 0; b < B; ++b) {
            Cand r[3]; for (auto &x : r) { x.k1 = x.k2 = 0; x.idx = 0; x.aux = 0; }
            double sum = 0, mx = -1e300;
            for (int l = 0; l < active; ++l) {
                const Cand &c = h[b * 64 + l];
                if (better_h<0>(c, r[0])) r[0] = c;
                if (better_h<1>(c, r[1])) r[1] = c;
                if (better_h<2>(c, r[2])) r[2] = c;
                sum += c.k1; mx = mx > c.k2 ? mx : c.k2;
            }
            for (int k = 0; k < 3; ++k)
                if (o[b * 3 + k].idx != r[k].idx || (r[k].idx && (o[b * 3 + k].aux != r[k].aux || o[b * 3 + k].k1 != r[k].k1))) {
                    if (bad < 10) printf("active %d block %d mode %d: got idx %d aux %d k1 %g, want idx %d aux %d k1 %g\n",
                                         active, b, k, o[b * 3 + k].idx, o[b * 3 + k].aux, o[b * 3 + k].k1, r[k].idx, r[k].aux, r[k].k1);
                    bad++;
                }
            if (s[b * 2] != sum || s[b * 2 + 1] != mx) {
                if (bad < 10) printf("active %d block %d: sum %g/%g max %g/%g\n", active, b, s[b * 2], sum, s[b * 2 + 1], mx);
                bad++;
            }
        }
    }
    printf("%s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
    return bad ? 1 : 0;
}
