// MFMA panel pricing: the dual simplex's pivot row (eval_trow,
// glpspx02.js:655-791) in the HBM-bound regime — dense A and rho too dense
// for the row path, where the pivot row is otherwise a pass over all of A
// (8 m n bytes, 537 MB on C3) for ONE row.
//
// The panel holds up to PANEL_MAX rows of the current simplex tableau over the
// structural columns,
//     G[t, j] = (inv(B)[pos_t, :] A)_j,
// for the basis positions pos_t of the best chuzr candidates at the time it
// was filled.  A tableau row follows a change of basis exactly as the row of
// inv(B) it comes from (the product-form update of k_dual_commit): for the
// pivot (p, q) with alpha = tcol[p],
//     G[t] -= (tcol[pos_t] / alpha) G[p]   (pos_t != p),   G[p] := -G[p] / alpha,
// so the panel stays a set of rows of the current tableau as long as it is
// kept, and a later pivot whose chosen row is in it reads one panel row
// instead of making a pass over A.  The choice itself is untouched: chuzr
// (glpspx02.js:572-626) picks p by the reference's rule in k_dual_top_grid;
// the panel only serves the row of p.
//   * k_panel_pick:   p in the panel -> hit.  Otherwise (a miss, or an
//                     emptied panel) the slots are refilled with p and the
//                     next best of the per-wave chuzr candidates;
//   * k_panel_gather: the rows of inv(B) at those positions (the unit entry
//                     of a basic slack's column made exact, as k_dual_top_grid
//                     forms rho);
//   * k_panel_mfma:   times A on v_mfma_f64_16x16x4_f64 — one pass over A for
//                     up to 32 rows (the batch of candidate rows packed into a
//                     dense panel, the MFMA operand);
//   * trow (k_trow_finish with panel = 1): every non-basic position, as the column pass
//                     CP_TROW writes it: the panel row of p at a structural,
//                     -rho at an auxiliary, 0 at a fixed variable;
//   * after the commit, the update above (PK rows, n columns): k_dual_commit's
//     extra blocks for the rows t != pcur, then k_panel_update_cur.
// Pick, gather and MFMA are in every pivot of the captured graph and gate
// themselves on the device flags.  A tableau row is a property of the basis,
// not of the factor, so the panel survives batch boundaries; it is emptied
// by a re-inversion (its rows are then re-formed from the fresh inverse: the
// product-form drift is bounded as the inverse's own), by a batch that pivots
// without maintaining it (k_dual_prep) and at every gk_spx_* call.
#include "gk_device.h"
#include <cstdlib>

namespace gk {

// the slots for this pivot: a hit, or a refill with p in slot 0 and the
// next best per-wave chuzr candidates (better<0>: r^2 / gamma, ties by
// position) in slots 1.., ranked by counting (gm <= 1024 candidates in LDS).
// A panel whose rows went through `age_max` product-form updates is refilled
// whatever the hit: its rows are then no older than the rows of a
// Forrest-Tomlin factor refreshed every nfs_max = 100 updates (glpspx02's
// default), so the drift of a served row stays that of a freshly formed one
__global__ void __launch_bounds__(256) k_panel_pick(SpxDev d, int gm, int cap, int age_max)
{
    const DState *st = d.st;
    if (st->stop || st->p <= 0) return;
    panel_pick_dev(d, gm, cap, age_max, st->p);
}

// pnl_src[t * m + i] = inv(B)[pos_t, i] for a dense column i of inv(B); for a
// basic slack's column (a unit vector) 1 exactly at the slack's own position
__global__ void __launch_bounds__(256) k_panel_gather(SpxDev d)
{
    const DState *st = d.st;
    if (st->stop || !st->pmiss) return;
    const int t = blockIdx.y;
    if (t >= st->pk) return;
    const int m = d.m;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int pos = d.ppos[t];
    const int kb = d.head[pos - 1];
    const int rp = d.rpos[i];
    const double v = (rp >= 0) ? d.Binv[(size_t)i * d.ldb + (pos - 1)] : (i == kb - 1 ? 1.0 : 0.0);
    d.pnl_src[(size_t)t * m + i] = v;
}

// G (pk x n) = pnl_src (pk x m) A (m x n, column-major, lda) on the matrix
// cores.  A block of 4 waves owns 32 columns and the 32 panel rows (one
// 16 x 16 tile per wave); the inner dimension streams in chunks of 32 (A in
// 256-byte column segments, the source rows likewise), the next chunk loaded
// into registers while the MFMAs run on the current one.  Fragments (lane l):
// A-operand src[l & 15][kk = l >> 4], B-operand A[kk = l >> 4][l & 15],
// result D[(l >> 4) + 4 r][l & 15].
typedef double pnl_d4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_panel_mfma(SpxDev d)
{
    constexpr int KC = 32, NC = 32, NR = 32;
    constexpr int QA = (KC * NC) / 256, QG = (KC * NR) / 256;
    __shared__ double As[KC][NC + 1];
    __shared__ double Gs[NR][KC + 1];
    const DState *st = d.st;
    if (st->stop || !st->pmiss) return;
    const int nk = st->pk;
    const int m = d.m, n = d.n, lda = d.A.lda;
    const double *__restrict__ A = d.A.A;
    const double *__restrict__ G = d.pnl_src;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int ct = w & 1, rt = w >> 1;
    const int c0 = blockIdx.x * NC;
    pnl_d4 acc = pnl_d4{0.0, 0.0, 0.0, 0.0};
    double ra[QA], rg[QG];
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = tid + 256 * q, rr = e & (KC - 1), cc = e / KC;
            const int r = k0 + rr, c = c0 + cc;
            ra[q] = (r < m && c < n) ? A[(size_t)c * lda + r] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const int e = tid + 256 * q, rr = e & (KC - 1), row = e / KC;
            const int r = k0 + rr;
            rg[q] = (r < m && row < nk) ? G[(size_t)row * m + r] : 0.0;
        }
    };
    load(0);
    for (int k0 = 0; k0 < m; k0 += KC) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = tid + 256 * q;
            As[e & (KC - 1)][e / KC] = ra[q];
        }
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const int e = tid + 256 * q;
            Gs[e / KC][e & (KC - 1)] = rg[q];
        }
        __syncthreads();
        if (k0 + KC < m) load(k0 + KC);
#pragma unroll
        for (int ks = 0; ks < KC / 4; ++ks) {
            const double b = As[ks * 4 + lk][ct * 16 + li];
            const double a = Gs[rt * 16 + li][ks * 4 + lk];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    const int j = c0 + ct * 16 + li;
    if (j >= n) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int t = rt * 16 + lk + 4 * r;
        if (t < nk) d.pnl[(size_t)t * d.ldp + j] = acc[r];
    }
}

// after a committed pivot (pend set by k_dual_commit, no stop) the rows of
// the panel follow the rows of inv(B) (k_dual_commit's rank-1 update):
// row pcur of the panel (G[p] := -G[p] / alpha), after the commit launch
// whose extra blocks updated the other rows from it (k_dual_commit): one
// read-modify-write per thread on the rows at once — a thread walking the
// 32 rows of its column took 22.7 us per pivot, one dependent memory round
// trip per row
__global__ void __launch_bounds__(256) k_panel_update_cur(SpxDev d)
{
    const DState *st = d.st;
    if (st->stop || !st->pend) return;
    const int cur = st->pcur;
    const double tp = st->pivot;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j == 0) d.st->page = st->page + 1;
    if (st->pk <= 0 || j >= d.n) return;
    double *g = d.pnl + (size_t)cur * d.ldp + j;
    *g = -*g / tp;
}

// the plan's panel size: the column-pass path on dense A outside rigorous
// mode, m >= GK_PANEL_MIN_M (default 1024: below it a pass over A costs
// little more than the panel's own kernels), GK_PANEL rows (default 32,
// 0 turns the panel off; read at every plan so that a caller can switch it)
int panel_wanted(const SpxDev &d, const DualPlan &pl)
{
    if (pl.rowpath || pl.colpath || pl.fupd || pl.rigorous || !d.A.dense || !d.pnl) return 0;
    const char *e = std::getenv("GK_PANEL");
    int k = e ? std::atoi(e) : 32;
    k = std::max(0, std::min(k, PANEL_MAX));
    const char *em = std::getenv("GK_PANEL_MIN_M");
    const int min_m = em ? std::atoi(em) : 1024;
    if (d.m < min_m || k < 2) return 0;
    // (panel_pick_dev gathers the 4 cdiv(m, 256) chuzr candidates in an LDS
    // array of 1024: m <= 65536, the explicit inverse's range)
    if (4 * cdiv(d.m, 256) > 1024) return 0;
    return k;
}

// updates a panel row may go through before the panel is refilled
// (GK_PANEL_AGE, default 100; read at every plan, as GK_PANEL)
int panel_age_max()
{
    const char *e = std::getenv("GK_PANEL_AGE");
    return e ? std::max(1, std::atoi(e)) : 100;
}

void panel_trow(hipStream_t s, const SpxDev &d, const DualPlan &pl, bool picked)
{
    const int m = d.m, n = d.n;
    // (picked: k_dual_top_grid's block 0 made the pick with the chuzr choice)
    if (!picked)
        hipLaunchKernelGGL(k_panel_pick, dim3(1), dim3(256), 0, s, d, 4 * cdiv(m, 256), pl.panel, pl.panel_age);
    hipLaunchKernelGGL(k_panel_gather, dim3(cdiv(m, 256), pl.panel), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_panel_mfma, dim3(cdiv(n, 32)), dim3(256), 0, s, d);
    // (trow itself: k_trow_finish reads the panel row of p, panel = 1)
    (void)n;
}

void panel_update(hipStream_t s, const SpxDev &d, const DualPlan &pl)
{
    (void)pl;
    // (the rows t != pcur: extra blocks of the k_dual_commit launch before
    // this, the same work as k_panel_update)
    hipLaunchKernelGGL(k_panel_update_cur, dim3(cdiv(d.n, 256)), dim3(256), 0, s, d);
}

}  // namespace gk
