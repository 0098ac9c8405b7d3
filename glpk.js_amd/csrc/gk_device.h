// Device-side helpers shared by the kernel translation units (wave64
// reductions, deterministic candidate selection, small accessors).
#pragma once
#include "gk_internal.h"
#include <cfloat>

namespace gk {
// need_p == EPI_GATE: the end-of-call epilogue enqueued behind a batch runs
// only when that batch used its whole budget (stop is ST_RUN or ST_BATCH)
#define GATE(st, need_p)                                                   \
    if ((st) != nullptr) {                                                 \
        if ((need_p) == EPI_GATE) {                                        \
            if ((st)->stop > ST_BATCH) return;                             \
        } else {                                                           \
            if ((st)->stop) return;                                        \
            if ((need_p) && (st)->p <= 0) return;                          \
        }                                                                  \
    }

constexpr int WG = 1024;       // single-workgroup control kernels
constexpr double DBL_EPS = 2.220446049250313e-16;   // glpapi.js:7

// wave-wide reductions of the device library (DPP sequences, not LDS
// permutes); all lanes of the wave must be active
extern "C" __device__ __attribute__((const)) double __ockl_wfred_add_f64(double);
extern "C" __device__ __attribute__((const)) double __ockl_wfred_max_f64(double);
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_min_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_max_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_min_u32(unsigned int);

// sum over the wave in a fixed order (deterministic)
__device__ __forceinline__ double wsum(double v) { return __ockl_wfred_add_f64(v); }

// rows of a CSR matrix longer than CSR_LONG entries are summed by the whole
// wave (lanes stride the entries, a fixed-order wave reduction) instead of
// by their own thread: a dense row (a linking row of a block-angular LP has
// thousands of entries) would otherwise be a serial chain of dependent
// loads.  Call with every lane of the wave; lanes flag their long rows.
template <typename F>
__device__ __forceinline__ void csr_long_rows(bool is_long, int beg, int end, const int *__restrict__ rcol,
                                              const double *__restrict__ rval, const double *__restrict__ x, F &&done)
{
    const int lane = threadIdx.x & 63;
    unsigned long long mask = __ballot(is_long);
    while (mask) {
        const int src = __ffsll((long long)mask) - 1;
        mask &= mask - 1;
        const int b = __shfl(beg, src), e = __shfl(end, src);
        double acc = 0.0;
        int t = b + lane;
        for (; t + 192 < e; t += 256) {
            const int c0 = rcol[t], c1 = rcol[t + 64], c2 = rcol[t + 128], c3 = rcol[t + 192];
            const double v0 = rval[t], v1 = rval[t + 64], v2 = rval[t + 128], v3 = rval[t + 192];
            acc += v0 * x[c0];
            acc += v1 * x[c1];
            acc += v2 * x[c2];
            acc += v3 * x[c3];
        }
        for (; t < e; t += 64) acc += rval[t] * x[rcol[t]];
        acc = wsum(acc);
        done(src, acc);
    }
}

__device__ __forceinline__ double wmax(double v) { return __ockl_wfred_max_f64(v); }

// block-wide reductions for blockDim.x <= 1024 (16 waves)
static __device__ double block_sum(double v, double *sh)
{
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wsum(v);
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (w == 0) {
        r = lane < nw ? sh[lane] : 0.0;
        r = wsum(r);
        if (lane == 0) sh[0] = r;
    }
    __syncthreads();
    r = sh[0];
    __syncthreads();
    return r;
}

static __device__ double block_max(double v, double *sh)
{
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wmax(v);
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (w == 0) {
        r = lane < nw ? sh[lane] : 0.0;
        r = wmax(r);
        if (lane == 0) sh[0] = r;
    }
    __syncthreads();
    r = sh[0];
    __syncthreads();
    return r;
}

static __device__ int block_or(int v, int *sh)
{
    __syncthreads();
    if (threadIdx.x == 0) sh[0] = 0;
    __syncthreads();
    if (v) sh[0] = 1;
    __syncthreads();
    int r = sh[0];
    __syncthreads();
    return r;
}

__device__ __forceinline__ unsigned long long dbits(double v) { return (unsigned long long)__double_as_longlong(v); }

// ---- the entry gate of a multi-block pivot kernel ---------------------------
// Every block of a pivot kernel reads the scalar state (DState) and the
// basis header at entry, and one block (the writer) rewrites some of it for
// the kernels that follow.  The blocks of a launch start on the 8 XCDs
// independently, so a block can issue its entry loads after the writer has
// finished and would then read the next pivot's state: the same solve took
// different pivot paths from run to run (round 4, tools/det_probe.py).  So
// every block passes gate_arrive once its entry loads have returned, and the
// writer's stores to anything another block reads at entry wait in
// gate_wait until every block of the launch has arrived.  Eight arrival words
// (blockIdx & 7, one per XCD) keep the atomics off a single address.  Only
// the writer waits, and the other blocks never wait on anything, so the
// launch drains however its blocks are scheduled.
//
// gate_arrive: every thread of the block (a block barrier inside); the
// s_waitcnt makes each wave's outstanding loads complete before the barrier
__device__ __forceinline__ void gate_arrive(DState *st)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&st->gate[blockIdx.x & 7], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same gate without a waiting writer, for state every block can compute
// itself: each block arrives with a returning add (thread 0, after the
// s_waitcnt and the block barrier, as gate_arrive), and the block whose add
// completes the count — the last of its XCD slot, then the last of the slots
// on gate_top — is the one that stores the state (its own entry loads and
// every other block's are done by then) and clears the words.  The add's
// round trip overlaps the block's remaining work: gate_last is called at its
// end.  gate_arrive_ret: every thread; returns the slot count before the add
// in thread 0.
__device__ __forceinline__ int gate_arrive_ret(DState *st)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int a = 0;
    if (threadIdx.x == 0) a = __hip_atomic_fetch_add(&st->gate[blockIdx.x & 7], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return a;
}

// thread 0 of every block, with gate_arrive_ret's value: true in the last block
__device__ __forceinline__ bool gate_last(DState *st, int a)
{
    const int blocks = (int)gridDim.x, x = (int)(blockIdx.x & 7);
    if (a != ((blocks - x + 7) >> 3) - 1) return false;
    const int slots = blocks < 8 ? blocks : 8;
    if (__hip_atomic_fetch_add(&st->gate_top, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != slots - 1) return false;
#pragma unroll
    for (int y = 0; y < 8; ++y) __hip_atomic_store(&st->gate[y], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->gate_top, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::: "memory");
    return true;
}

// gate_wait: ONE thread of the writer block, after its own block arrived;
// resets the words for the next launch
__device__ __forceinline__ void gate_wait(DState *st)
{
    const int blocks = (int)gridDim.x;
    // the eight words polled together (one memory round trip per poll, not
    // eight dependent ones)
    for (;;) {
        int v[8];
#pragma unroll
        for (int x = 0; x < 8; ++x) v[x] = __hip_atomic_load(&st->gate[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool all = true;
#pragma unroll
        for (int x = 0; x < 8; ++x) all = all && v[x] >= ((blocks - x + 7) >> 3);
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
    }
    for (int x = 0; x < 8; ++x) __hip_atomic_store(&st->gate[x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::: "memory");           // the writer's stores stay after the wait
}

// candidate of an index-choosing scan: key1 (primary), key2 (secondary), idx
struct Cand {
    double k1, k2;
    int idx, aux;
};

// mode 0: max k1, tie lowest idx                   (chuzr dual / chuzc primal)
// mode 1: min k1, then max k2, tie lowest idx       (Harris pass 1)
// mode 2: max k2, tie lowest idx                    (Harris pass 2)
template <int MODE>
__device__ __forceinline__ bool better(const Cand &a, const Cand &b)
{
    if (a.idx == 0) return false;
    if (b.idx == 0) return true;
    if (MODE == 0) {
        if (a.k1 != b.k1) return a.k1 > b.k1;
    } else if (MODE == 1) {
        if (a.k1 != b.k1) return a.k1 < b.k1;
        if (a.k2 != b.k2) return a.k2 > b.k2;
    } else {
        if (a.k2 != b.k2) return a.k2 > b.k2;
    }
    return a.idx < b.idx;
}

template <int MODE>
static __device__ Cand block_best(Cand c, Cand *sh)
{
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        Cand d;
        d.k1 = __shfl_xor(c.k1, o);
        d.k2 = __shfl_xor(c.k2, o);
        d.idx = __shfl_xor(c.idx, o);
        d.aux = __shfl_xor(c.aux, o);
        if (better<MODE>(d, c)) c = d;
    }
    __syncthreads();
    if (lane == 0) sh[w] = c;
    __syncthreads();
    if (w == 0) {
        Cand r;
        if (lane < nw) r = sh[lane];
        else { r.k1 = 0; r.k2 = 0; r.idx = 0; r.aux = 0; }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            Cand d;
            d.k1 = __shfl_xor(r.k1, o);
            d.k2 = __shfl_xor(r.k2, o);
            d.idx = __shfl_xor(r.idx, o);
            d.aux = __shfl_xor(r.aux, o);
            if (better<MODE>(d, r)) r = d;
        }
        if (lane == 0) sh[0] = r;
    }
    __syncthreads();
    Cand r = sh[0];
    __syncthreads();
    return r;
}

// the same within one wave (no block synchronisation); every lane gets it.
// The keys are non-negative doubles (ratios, |alfa|, r^2 / gamma), whose
// bit patterns order like the values once -0 is folded into +0, so the
// choice is three exact wave reductions (key, secondary key, index) and a
// ballot for the winning lane; identical to better<MODE> for distinct
// indices.
template <int MODE>
__device__ __forceinline__ Cand wave_best(Cand c)
{
    // every reduction is called by every lane (no short-circuit: the
    // reductions run over the active lanes)
    const bool valid = c.idx != 0;
    bool tie;
    if (MODE == 1) {
        const unsigned long long k = valid ? dbits(fabs(c.k1)) : ~0ull;
        const unsigned long long mk = __ockl_wfred_min_u64(k);
        tie = valid & (k == mk);
        const unsigned long long k2 = tie ? dbits(fabs(c.k2)) + 1ull : 0ull;
        const unsigned long long m2 = __ockl_wfred_max_u64(k2);
        tie = tie & (k2 == m2);
    } else {
        const double kk = (MODE == 0) ? c.k1 : c.k2;
        const unsigned long long k = valid ? dbits(fabs(kk)) + 1ull : 0ull;
        const unsigned long long mk = __ockl_wfred_max_u64(k);
        tie = valid & (k == mk);
    }
    const unsigned int ii = tie ? (unsigned int)c.idx : 0xffffffffu;
    const unsigned int mi = __ockl_wfred_min_u32(ii);
    Cand r;
    if (mi == 0xffffffffu) {
        r.k1 = 0.0; r.k2 = 0.0; r.idx = 0; r.aux = 0;
        return r;
    }
    const unsigned long long bal = __ballot(tie & ((unsigned int)c.idx == mi));
    const int src = __builtin_amdgcn_readfirstlane(__ffsll((long long)bal) - 1);
    r.k1 = __shfl(c.k1, src);
    r.k2 = __shfl(c.k2, src);
    r.idx = (int)mi;
    r.aux = __shfl(c.aux, src);
    return r;
}


__device__ __forceinline__ double get_xN(const signed char *stat, const double *lb, const double *ub, int k, int j)
{
    // glpspx01.js:442
    switch (stat[j - 1]) {
    case NL: return lb[k - 1];
    case NU: return ub[k - 1];
    case NF: return 0.0;
    default: return lb[k - 1];
    }
}

// reset_refsp (glpspx01.js:586 / glpspx02.js:497)
static __device__ void reset_refsp_dev(const SpxDev &d, int dual, bool set_refct = true)
{
    const int m = d.m, n = d.n;
    for (int k = threadIdx.x; k < m + n; k += blockDim.x) d.refsp[k] = 0;
    __syncthreads();
    if (dual) {
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            d.refsp[d.head[i] - 1] = 1;
            d.gamma[i] = 1.0;
        }
    } else {
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            d.refsp[d.head[m + j] - 1] = 1;
            d.gamma[j] = 1.0;
        }
    }
    __syncthreads();
    // (a gated multi-block kernel stores refct with its other scalars, after
    // gate_wait: set_refct false)
    if (set_refct && threadIdx.x == 0) d.st->refct = 1000;
    __syncthreads();
}

// h = -N[q] (eval_tcol, glpspx01.js:702-719); runs inside a single workgroup
static __device__ void build_hq(const SpxDev &d, int q, bool zeroed = false)
{
    const int m = d.m;
    const int k = d.head[m + q - 1];
    if (!zeroed) {                      // (the dual on the sparse factor: zeroed by k_trow_finish)
        for (int i = threadIdx.x; i < m; i += blockDim.x) d.h[i] = 0.0;
        __syncthreads();
    }
    if (k <= m) {
        if (threadIdx.x == 0) d.h[k - 1] = -1.0;
    } else {
        const int c = k - m - 1;
        if (d.A.dense) {
            const double *col = d.A.A + (size_t)c * d.A.lda;
            for (int i = threadIdx.x; i < m; i += blockDim.x) d.h[i] = col[i];
        } else {
            for (int t = d.A.cptr[c] + threadIdx.x; t < d.A.cptr[c + 1]; t += blockDim.x) d.h[d.A.cind[t]] = d.A.cval[t];
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// per-wave candidate buffers and profiling stamps shared by the pivot
// pipelines (gk_dual.hip, gk_primal.hip)
// ---------------------------------------------------------------------------
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__device__ __forceinline__ int gv_of(int m, int n) { return (max(m, n) + 255) / 256; }
__device__ __forceinline__ Cand *cand_chuzr(const SpxDev &d) { return (Cand *)d.cand; }

// the pricing panel's pick for the leaving row p (gk_panel.hip): a hit sets
// pcur to p's slot; a miss (or a panel older than age_max updates) ranks the
// chuzr candidates by better<0> and fills the panel's positions, p first.
// Called by every thread of one 256-thread block (k_panel_pick, or block 0
// of k_dual_top_grid with the chuzr choice in hand).
__device__ __forceinline__ void panel_pick_dev(const SpxDev &d, int gm, int cap, int age_max, int p)
{
    __shared__ Cand cs[1024];
    __shared__ int nval;
    DState *st = d.st;
    const int valid = st->pvalid, pk = st->pk, age = st->page;
    const int sl = d.pslot[p - 1];
    const bool hit = valid && age < age_max && sl >= 0 && sl < pk && d.ppos[sl] == p;
    if (hit) {
        if (threadIdx.x == 0) {
            st->pcur = sl;
            st->pmiss = 0;
            st->phits += 1.0;
        }
        return;
    }
    if (threadIdx.x == 0) nval = 0;
    for (int b = threadIdx.x; b < gm; b += blockDim.x) cs[b] = cand_chuzr(d)[b];
    __syncthreads();
    int mine = 0;
    for (int b = threadIdx.x; b < gm; b += blockDim.x) {
        const Cand c = cs[b];
        if (c.idx == 0 || c.idx == p) continue;
        mine++;
        int r = 0;
        for (int u = 0; u < gm; ++u) {
            const Cand e = cs[u];
            if (e.idx != 0 && e.idx != p && better<0>(e, c)) r++;
        }
        if (r < cap - 1) {
            d.ppos[1 + r] = c.idx;
            d.pslot[c.idx - 1] = 1 + r;
        }
    }
    if (mine) atomicAdd(&nval, mine);
    __syncthreads();
    if (threadIdx.x == 0) {
        d.ppos[0] = p;
        d.pslot[p - 1] = 0;
        st->pk = 1 + min(nval, cap - 1);
        st->page = 0;
        st->pcur = 0;
        st->pmiss = 1;
        st->pvalid = 1;
        st->pmisses += 1.0;
    }
}

__device__ __forceinline__ Cand no_cand(double k1)
{
    Cand c; c.k1 = k1; c.k2 = 0.0; c.idx = 0; c.aux = 0;
    return c;
}

// Per-wave outputs, 4 gv entries each, so that no producer needs a block
// barrier and every consumer wave reduces them on its own: chuzr candidates
// (one per wave of k_dual_commit / k_dual_prep), pass-1 candidates (one per
// 64-slot group of the pivot row), pass-2 candidates (one per wave of
// k_dual_ratio).  gpart: gamma_p sums of the 64-slot groups [4 gv), then
// their max |trow| [4 gv).
__device__ __forceinline__ Cand *cand_pass1(const SpxDev &d) { return (Cand *)d.cand + 4 * gv_of(d.m, d.n); }
__device__ __forceinline__ Cand *cand_pass2(const SpxDev &d) { return (Cand *)d.cand + 8 * gv_of(d.m, d.n); }
__device__ __forceinline__ double *tmax_part(const SpxDev &d) { return d.gpart + 4 * gv_of(d.m, d.n); }

// the choice over cnt stored candidates, made by one wave (lane-strided scan,
// then the butterfly): the same result in every wave that calls it
template <int MODE>
__device__ __forceinline__ Cand wave_scan(const Cand *a, int cnt)
{
    Cand c = no_cand(0.0);
    for (int b = (int)(threadIdx.x & 63); b < cnt; b += 64) {
        const Cand e = a[b];
        if (better<MODE>(e, c)) c = e;
    }
    return wave_best<MODE>(c);
}

__device__ __forceinline__ unsigned long long wmax_u64(unsigned long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long u = __shfl_xor(v, o);
        v = u > v ? u : v;
    }
    return v;
}

// profiling (gk_bfd_profile(bfd, 2), eager launches): device clock at block
// entry (thread 0) and the latest wave exit of the block
struct TraceScope {
    unsigned long long *p;
    __device__ __forceinline__ TraceScope(const SpxDev &d, int kid)
        : p((d.trace && blockIdx.x < (unsigned)TRACE_BLOCKS) ? d.trace + ((size_t)kid * TRACE_BLOCKS + blockIdx.x) * 2
                                                              : nullptr)
    {
        if (p && threadIdx.x == 0) p[0] = wall_clock64();
    }
    __device__ __forceinline__ ~TraceScope()
    {
        if (p && (threadIdx.x & 63) == 0) atomicMax(p + 1, wall_clock64());
    }
};

// exit stamp of a block (the latest wave exit; atomicMax over the waves —
// the stamps only grow, so the slot needs no reset between pivots)
struct ExitStamp {
    unsigned long long *p;
    __device__ __forceinline__ ExitStamp(unsigned long long *slots, unsigned b) : p(slots ? slots + b : nullptr) {}
    __device__ __forceinline__ ~ExitStamp()
    {
        if (p && (threadIdx.x & 63) == 0) atomicMax(p, wall_clock64());
    }
};

// phase stamp of wave 0 (profiling only)
#define TPH(kid, ph)                                                                                              \
    do {                                                                                                          \
        if (d.trace && threadIdx.x == 0 && blockIdx.x < (unsigned)TRACE_BLOCKS)                                   \
            d.trace[(size_t)TRACE_KERNELS * TRACE_BLOCKS * 2 + ((size_t)(kid) * TRACE_BLOCKS + blockIdx.x) * 8 + \
                    (ph)] = wall_clock64();                                                                       \
    } while (0)


}  // namespace gk
