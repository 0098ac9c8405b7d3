// Branch and bound on the MI355X: batched node LPs.
//
// Replaces ios_driver (glpios03.js:1) for cb_func == null.  The reference
// solves one node LP at a time with glp_simplex (ios_solve_node,
// glpios01.js:866) and walks the tree depth-first/best-local-bound.  Node LPs
// of B&B are tiny (gap 20x75, mas76 12x151) and one at a time they cannot
// occupy a GPU; here the open nodes are solved in BATCHES, one workgroup per
// node LP, with the whole simplex tableau of the node in LDS:
//
//   T = inv(B) [I | -A]   (m x (m+n), fp64, LDS),  x_B = -T_N x_N,
//   d = c - c_B' T        (reduced costs, internal minimisation form)
//
// Each workgroup builds inv(B) for its node's basis by Gauss-Jordan on
// [B | I | -A] (the parent's optimal basis: a warm start, dual feasible after
// the branching bound change), runs the bounded dual simplex to optimality,
// infeasibility or the incumbent cutoff, and returns the solution, its basis
// and the branching choice of the Driebeck-Tomlin heuristic (branch_drtom,
// glpios09.js:84) evaluated on its own tableau rows (the reference does this
// through glp_eval_tab_row / glp_dual_rtest, glpapi12.js:401/:687).
//
// The host driver (gk_ios_driver below) keeps the open nodes in a best-bound
// priority queue, prunes with the incumbent (ios_is_hopeful, glpios01.js:789)
// and the rounded bound (ios_round_bound, :730), and launches batches of up
// to 1024 nodes.  Objective and incumbent match the reference (objective
// parity); the order in which nodes are evaluated — and hence node counts —
// differs from the reference's sequential walk (SURVEY.md §8(a) design note).
#include "gk_device.h"
#include "gk_hostprof.h"
#include "../../include/glpk_mi355x.h"
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <x86intrin.h>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <queue>
#include <thread>
#include <string>
#include <vector>

namespace gk {

void set_err(const char *fmt, ...);

// node LP outcomes (status[]): OPT / INFEAS (dual unbounded) / CUTOFF (dual
// objective reached the incumbent) are final; FAIL (singular basis or a
// status the kernel cannot warm-start from) and ITLIM (iteration limit; the
// dual objective is still a valid bound) send a node to the engine fallback;
// PPINF: ios_preprocess_node proved the node infeasible (no LP solved)
enum : int { NODE_OPT = 0, NODE_INFEAS = 1, NODE_CUTOFF = 2, NODE_FAIL = 3, NODE_ITLIM = 4, NODE_PPINF = 5 };

struct NodeProb {
    int m, n, ld;                 // ld = m + n (row length of T)
    const double *A;              // dense col-major m x n (unscaled)
    const double *c;              // internal minimisation costs, [m+n] (0 for rows)
    const signed char *isint;     // [n]
    const double *rlb, *rub;      // [m] row bounds (the same at every node)
    // a sparse A (nnz <= m n / 2; nnz = 0: dense) also by rows and by
    // columns for the preprocessing: rptr[m+1] / rind / rval (column indices,
    // ascending) and cptr[n+1] / cind / cval (row indices, ascending)
    int nnz;
    const int *rptr, *rind, *cptr, *cind;
    const double *rval, *cval;
    double tol_int;
    int dth;                      // 1: choose the branching column by branch_drtom
};

struct NodeIO {
    const double *lb, *ub;        // [nb][m+n]
    const signed char *stat_in;   // [nb][m+n]  GLP_BS / NL / NU / NF / NS
    const double *cutoff;         // [nb]  stop once the dual objective reaches it
    const int *it_lim;            // [nb]  dual simplex iteration limit of the node
    const int *pp_pass;           // [nb]  ios_preprocess_node passes (0: none)
    double obj_bound;             // preprocessing: objective row bound (minimisation form, DBL_MAX: none)
    int *status, *pivots, *jj, *next;
    double *obj, *x, *dzb, *bnd;  // obj[nb], x[nb][m+n], dzb[nb][2n] (dn, up degradation
                                  // bounds of every fractional column), bnd[nb][2n] (final column bounds)
    signed char *stat_out;        // [nb][m+n]
    double *scratch;              // GLOBAL kernel: per-node work area (node_lp_lds(m, n) bytes each)
    size_t scratch_stride;        // in doubles
    // node records in HBM (the B&B bookkeeping on the device): an optimal
    // node stores its final tableau, column bounds and statuses; a child
    // starts from its parent's record — the tableau instead of inverting its
    // basis again (warm start), and, when br_j[b] >= 0, the bounds and
    // statuses with the branching change applied here (the host keeps no
    // arrays for such a child).  tab_in[b]: the parent's record or null;
    // tab_out[b]: where this node's goes (or null).  Record layout:
    // [0] pivots since the last inversion, [1..m] head, T (m x (m+n),
    // row-major), lb[n], ub[n] of the columns, stat[m+n] (bytes)
    const double *const *tab_in;
    double *const *tab_out;
    int tab_age_max;              // an older tableau is inverted again
    const int *br_j, *br_dir;     // [nb] branching column (-1: bounds from lb / ub / stat_in), 0 down / 1 up
    const double *br_val;         // [nb] the column's value in the parent's solution
    // check_integrality (glpios03.js:55) on the node's final bounds, and the
    // branching rules' candidates: fractional count, sum of integer
    // infeasibilities, first / last / most fractional column (0-based, -1:
    // none) and branch_mostf's direction
    int *nfrac, *jfirst, *jlast, *jmost, *nmost;
    double *iisum;
    unsigned long long *stamps;   // GK_BNB_LOG=2: [nb][8] device clock at the kernel's phases (null: off)
};

__host__ __device__ inline size_t node_rec_bounds(int m, int n) { return 1 + (size_t)m + (size_t)m * (m + n); }
__host__ __device__ inline size_t node_rec_doubles(int m, int n)
{
    return node_rec_bounds(m, n) + 2 * (size_t)n + ((size_t)m + n + 7) / 8;
}

// ---- small block helpers (blockDim.x = 256) --------------------------------
// argmax of key (ties: lowest idx); idx < 0 = none
__device__ int block_argmax(double key, int idx, double *shk, int *shi)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double k2 = __shfl_xor(key, o);
        const int i2 = __shfl_xor(idx, o);
        if (i2 >= 0 && (idx < 0 || k2 > key || (k2 == key && i2 < idx))) { key = k2; idx = i2; }
    }
    __syncthreads();
    if (lane == 0) { shk[w] = key; shi[w] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < (int)(blockDim.x >> 6); ++v)
            if (shi[v] >= 0 && (shi[0] < 0 || shk[v] > shk[0] || (shk[v] == shk[0] && shi[v] < shi[0]))) {
                shk[0] = shk[v];
                shi[0] = shi[v];
            }
    }
    __syncthreads();
    const int r = shi[0];
    __syncthreads();
    return r;
}

// dual ratio test choice: min ratio, then max |alfa|, then lowest idx
__device__ int block_ratio(double t, double a, int idx, double *shk, double *sha, int *shi)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double t2 = __shfl_xor(t, o), a2 = __shfl_xor(a, o);
        const int i2 = __shfl_xor(idx, o);
        if (i2 >= 0 && (idx < 0 || t2 < t || (t2 == t && (a2 > a || (a2 == a && i2 < idx))))) {
            t = t2; a = a2; idx = i2;
        }
    }
    __syncthreads();
    if (lane == 0) { shk[w] = t; sha[w] = a; shi[w] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < (int)(blockDim.x >> 6); ++v) {
            if (shi[v] < 0) continue;
            if (shi[0] < 0 || shk[v] < shk[0] || (shk[v] == shk[0] && (sha[v] > sha[0] || (sha[v] == sha[0] && shi[v] < shi[0])))) {
                shk[0] = shk[v]; sha[0] = sha[v]; shi[0] = shi[v];
            }
        }
    }
    __syncthreads();
    const int r = shi[0];
    __syncthreads();
    return r;
}

// block_argmax's order within one wave (every lane returns the choice): the
// largest key, then the lowest index — three DPP reductions instead of a
// six-round permute butterfly
__device__ int wave_argmax(double key, int idx)
{
    const double km = wmax(idx >= 0 ? key : -DBL_MAX);
    const unsigned c = (idx >= 0 && key == km) ? (unsigned)idx : 0x7fffffffu;
    const unsigned r = __ockl_wfred_min_u32(c);
    return r == 0x7fffffffu ? -1 : (int)r;
}

// block_ratio's order within one wave (every lane returns the choice): the
// smallest ratio, then the largest |alfa|, then the lowest index
__device__ int wave_ratio(double t, double a, int idx)
{
    const double tm = -wmax(idx >= 0 ? -t : -DBL_MAX);
    const bool at = idx >= 0 && t == tm;
    const double am = wmax(at ? a : -1.0);
    const unsigned c = (at && a == am) ? (unsigned)idx : 0x7fffffffu;
    const unsigned r = __ockl_wfred_min_u32(c);
    return r == 0x7fffffffu ? -1 : (int)r;
}

// the value v of the lane whose candidate is the wave's choice q (v >= 0;
// each index belongs to one lane)
__device__ __forceinline__ double wave_pick(double v, int mine, int q)
{
    return wmax(mine == q ? v : -DBL_MAX);
}

__device__ double block_sum256(double v, double *sh)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wsum(v);
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) r += sh[k];
    __syncthreads();
    return r;
}

__device__ __forceinline__ double nb_value(int st, double lb, double ub)
{
    switch (st) {
    case NL: return lb;
    case NU: return ub;
    case NF: return 0.0;
    default: return lb;   // NS
    }
}

// ---------------------------------------------------------------------------
// ios_preprocess_node (glpios02.js:1, called per node at glpios03.js:643-656):
// bound propagation over the rows of the node and the objective row under
// the incumbent.  The reference walks a LIFO list of rows, each row seeing
// the bounds tightened by the previous one; here a pass is two parallel
// phases over the whole node — one wave per row forms the row's activity
// bounds (prepare_row_info :2, check_row_bounds :137: infeasibility and
// redundant row bounds), then one thread per column intersects the implied
// bounds of all its rows (col_implied_bounds :74, check_col_bounds :177 with
// integer rounding) — repeated while some column changed efficiently
// (check_efficiency :245), at most max_pass times.  Every tightening is one
// the reference's rules derive, so the node's feasible set is unchanged.
// ri[6 i + {0..5}] = f_min, f_max, j_min, j_max, L, U of row i (row 0: the
// objective, sum c_j x_j <= incumbent in minimisation form).
// Returns 1 when the node is infeasible.  Called by the whole block.
// ---------------------------------------------------------------------------
struct NodeSp {                   // the sparse copies of A the kernel staged (null: dense A)
    const int *rptr, *rind, *cptr, *cind;
    const double *rval, *cval;
};

template <int ALDS>
__device__ int node_preprocess(const NodeProb &P, const double *cl, const signed char *isl, const double *Ar,
                               const NodeSp &sp, double objU, double *lb, double *ub, signed char *stat,
                               signed char *chg, double *ri, int max_pass)
{
    const int m = P.m, n = P.n;
    // a_ij: the row-major LDS copy (ALDS) or the column-major matrix in HBM
    auto aij = [&](int i, int j) { return ALDS ? Ar[(size_t)i * n + j] : P.A[(size_t)j * m + i]; };
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int i = threadIdx.x; i <= m; i += blockDim.x) {
        ri[6 * i + 4] = (i == 0) ? -DBL_MAX : lb[i - 1];
        ri[6 * i + 5] = (i == 0) ? objU : ub[i - 1];
    }
    __syncthreads();
    // "some column changed efficiently" of each pass, in three rotating
    // flags: the pass's last barrier publishes it together with the
    // infeasibility test; thread 0 clears the flag of the next pass, which no
    // thread still reads (a slow thread may still read the previous pass's)
    __shared__ int sh_eff[3];
    if (threadIdx.x == 0) sh_eff[0] = 0;
    for (int pass = 0; pass < max_pass; ++pass) {
        // ---- rows: activity bounds, infeasibility, redundant row bounds
        int bad = 0;
        if (threadIdx.x == 0) sh_eff[(pass + 1) % 3] = 0;
        for (int i = w; i <= m; i += nw) {
            double L = ri[6 * i + 4], U = ri[6 * i + 5];
            if (L == -DBL_MAX && U == DBL_MAX) continue;           // free row (wave-uniform)
            double smin = 0.0, smax = 0.0, cmin = 0.0, cmax = 0.0, jmin = 0.0, jmax = 0.0;
            auto term = [&](int j, double a) {
                if (a == 0.0) return;
                const double l = lb[m + j], u = ub[m + j];
                const double lo = a > 0.0 ? l : u, hi = a > 0.0 ? u : l;
                if ((a > 0.0 && l == -DBL_MAX) || (a < 0.0 && u == DBL_MAX)) { cmin += 1.0; jmin = fmax(jmin, j + 1); }
                else smin += a * lo;
                if ((a > 0.0 && u == DBL_MAX) || (a < 0.0 && l == -DBL_MAX)) { cmax += 1.0; jmax = fmax(jmax, j + 1); }
                else smax += a * hi;
            };
            if (i > 0 && sp.rptr)
                for (int t = sp.rptr[i - 1] + lane; t < sp.rptr[i]; t += 64) term(sp.rind[t], sp.rval[t]);
            else
                for (int j = lane; j < n; j += 64) term(j, (i == 0) ? cl[m + j] : aij(i - 1, j));
            smin = wsum(smin); smax = wsum(smax);
            cmin = wsum(cmin); cmax = wsum(cmax);
            jmin = wmax(jmin); jmax = wmax(jmax);
            // prepare_row_info: one unbounded term -> the sum of the others and
            // its column; two or more -> infinite
            const double fmin = cmin >= 2.0 ? -DBL_MAX : smin, fmax = cmax >= 2.0 ? DBL_MAX : smax;
            const int jn = cmin == 1.0 ? (int)jmin : 0, jx = cmax == 1.0 ? (int)jmax : 0;
            const double LL = jn == 0 ? fmin : -DBL_MAX, UU = jx == 0 ? fmax : DBL_MAX;
            if (L != -DBL_MAX && UU < L - 1e-3 * (1.0 + fabs(L))) bad = 1;
            if (U != DBL_MAX && LL > U + 1e-3 * (1.0 + fabs(U))) bad = 1;
            if (L != -DBL_MAX && LL > L - 1e-12 * (1.0 + fabs(L))) L = -DBL_MAX;
            if (U != DBL_MAX && UU < U + 1e-12 * (1.0 + fabs(U))) U = DBL_MAX;
            if (lane == 0) {
                ri[6 * i + 0] = fmin; ri[6 * i + 1] = fmax;
                ri[6 * i + 2] = jn; ri[6 * i + 3] = jx;
                ri[6 * i + 4] = L; ri[6 * i + 5] = U;
            }
        }
        if (__syncthreads_or(bad)) return 1;
        // ---- columns: implied bounds of every row the column is in
        int eff = 0;
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            const double l0 = lb[m + j], u0 = ub[m + j];
            const bool flag = isl[j] != 0;
            double lj = l0, uj = u0;
            // rows in order: the objective, then the rows of column j
            const int t0 = sp.cptr ? sp.cptr[j] : 0, t1 = sp.cptr ? sp.cptr[j + 1] : m;
            for (int t = t0 - 1; t < t1 && !bad; ++t) {
                const int i = (t < t0) ? 0 : (sp.cptr ? sp.cind[t] + 1 : t + 1);
                const double L = ri[6 * i + 4], U = ri[6 * i + 5];
                if (L == -DBL_MAX && U == DBL_MAX) continue;
                const double a = (t < t0) ? cl[m + j] : (sp.cptr ? sp.cval[t] : aij(i - 1, j));
                if (a == 0.0) continue;
                const double fmin = ri[6 * i + 0], fmax = ri[6 * i + 1];
                const int jn = (int)ri[6 * i + 2], jx = (int)ri[6 * i + 3];
                double ilb, iub, ll, uu;
                if (L == -DBL_MAX || fmax == DBL_MAX) ilb = -DBL_MAX;
                else if (jx == 0) ilb = L - (fmax - a * (a > 0.0 ? u0 : l0));
                else if (jx == j + 1) ilb = L - fmax;
                else ilb = -DBL_MAX;
                if (U == DBL_MAX || fmin == -DBL_MAX) iub = DBL_MAX;
                else if (jn == 0) iub = U - (fmin - a * (a > 0.0 ? l0 : u0));
                else if (jn == j + 1) iub = U - fmin;
                else iub = DBL_MAX;
                if (fabs(a) < 1e-6) { ll = -DBL_MAX; uu = DBL_MAX; }
                else if (a > 0.0) {
                    ll = ilb == -DBL_MAX ? -DBL_MAX : ilb / a;
                    uu = iub == DBL_MAX ? DBL_MAX : iub / a;
                } else {
                    ll = iub == DBL_MAX ? -DBL_MAX : iub / a;
                    uu = ilb == -DBL_MAX ? DBL_MAX : ilb / a;
                }
                if (flag) {
                    if (ll != -DBL_MAX) ll = (ll - floor(ll) < 1e-3 ? floor(ll) : ceil(ll));
                    if (uu != DBL_MAX) uu = (ceil(uu) - uu < 1e-3 ? ceil(uu) : floor(uu));
                }
                const double lp = lj, up = uj;
                if (lj != -DBL_MAX && uu < lj - 1e-3 * (1.0 + fabs(lj))) { bad = 1; break; }
                if (uj != DBL_MAX && ll > uj + 1e-3 * (1.0 + fabs(uj))) { bad = 1; break; }
                if (ll != -DBL_MAX && lj < ll - 1e-3 * (1.0 + fabs(ll))) lj = ll;
                if (uu != DBL_MAX && uj > uu + 1e-3 * (1.0 + fabs(uu))) uj = uu;
                if (!(lj == -DBL_MAX || uj == DBL_MAX)) {
                    const double t1 = fabs(lj), t2 = fabs(uj);
                    if (lj > uj - 1e-10 * (1.0 + (t1 <= t2 ? t1 : t2))) {
                        if (lj == lp) uj = lj;
                        else if (uj == up) lj = uj;
                        else if (t1 <= t2) uj = lj;
                        else lj = uj;
                    }
                }
            }
            // check_efficiency (:245)
            if (l0 < lj) {
                if (flag || l0 == -DBL_MAX) eff = 1;
                else {
                    const double r = (u0 == DBL_MAX) ? 1.0 + fabs(l0) : 1.0 + (u0 - l0);
                    if (lj - l0 >= 0.25 * r) eff = 1;
                }
            }
            if (u0 > uj) {
                if (flag || u0 == DBL_MAX) eff = 1;
                else {
                    const double r = (l0 == -DBL_MAX) ? 1.0 + fabs(u0) : 1.0 + (u0 - l0);
                    if (u0 - uj >= 0.25 * r) eff = 1;
                }
            }
            lb[m + j] = lj;
            ub[m + j] = uj;
        }
        if (eff) sh_eff[pass % 3] = 1;
        if (__syncthreads_or(bad)) return 1;
        if (!sh_eff[pass % 3]) break;
    }
    // relaxed bounds of the basic rows (non-active: dual feasibility kept);
    // statuses of non-basic columns whose type changed (glp_set_col_bnds):
    // fixed -> NS, a free column that gained a bound is re-chosen once the
    // reduced costs are known (chg)
    for (int i = threadIdx.x; i < m; i += blockDim.x)
        if (stat[i] == BS) {
            lb[i] = ri[6 * (i + 1) + 4];
            ub[i] = ri[6 * (i + 1) + 5];
        }
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const int k = m + j;
        if (stat[k] == BS) continue;
        if (lb[k] == ub[k]) stat[k] = NS;
        else if (stat[k] == NF && (lb[k] != -DBL_MAX || ub[k] != DBL_MAX)) chg[j] = 1;
    }
    __syncthreads();
    return 0;
}

// ---------------------------------------------------------------------------
// one workgroup = one node LP
// LDS: M[m][2m+n] during the inversion, then T[m][m+n]; lb, ub, x, d [m+n];
// fcol[m]; preprocessing row info [6 (m+1)]; head[m], stat[m+n], chg[n].
// GLOBAL = 1: the same work area in a per-node slice of HBM (node LPs beyond
// 64 KiB of LDS; L2 serves the workgroup's sweeps).
// ---------------------------------------------------------------------------
template <int GLOBAL, int ALDS>
__global__ void __launch_bounds__(256) k_node_lp(NodeProb P, NodeIO io)
{
    extern __shared__ double lds_[];
    double *lds = GLOBAL ? io.scratch + (size_t)blockIdx.x * io.scratch_stride : lds_;
    __shared__ double shk[4];
    __shared__ int shi[4];
    __shared__ int sh_flag;
    const int m = P.m, n = P.n, N = m + n, b = blockIdx.x;
    const int W = 2 * m + n;                 // width of [B | I | -A]
    // phases: 0 entry, 5 bounds loaded, 1 preprocessed, 2 tableau (warm or
    // inverted), 3 x / d formed, 4 simplex done, 7 exit
#define NODE_STAMP(ph) \
    do { if (io.stamps && threadIdx.x == 0) io.stamps[(size_t)b * 8 + (ph)] = wall_clock64(); } while (0)
    NODE_STAMP(0);
    double *M = lds;                          // m * W
    double *lb = M + (size_t)m * W, *ub = lb + N, *x = ub + N, *d = x + N;
    double *fcol = d + N;                     // m
    double *rinfo = fcol + m;                 // 6 (m + 1)
    double *cl = rinfo + 6 * (m + 1);         // N: the costs
    double *dzt = cl + N;                     // 4 m: branching degradations of the candidates
    double *gam = dzt + 4 * m;                // m: projected steepest-edge weights of the rows
    double *Ar = gam + m;                     // ALDS: A row-major (m x n)
    const int nzl = ALDS ? P.nnz : 0;         // sparse copies staged in LDS
    double *rv = Ar + (ALDS ? (size_t)m * n : 0), *cv = rv + nzl;
    int *head = (int *)(cv + nzl);
    int *rowof = head + m;                    // N: row of a basic variable
    int *cand = rowof + N;                    // m: fractional basic integer columns
    int *rp = cand + m, *ri_ = rp + (nzl ? m + 1 : 0), *cp = ri_ + nzl, *ci = cp + (nzl ? n + 1 : 0);
    signed char *stat = (signed char *)(ci + nzl);
    signed char *chg = stat + N;              // n
    signed char *isl = chg + n;               // n: integer flags
    signed char *refsp = isl + n;             // N: the pricing's reference space
    // the problem's costs, integer flags and (ALDS) matrix staged in LDS:
    // every loop below reads them many times, some from one thread
    for (int k = threadIdx.x; k < N; k += blockDim.x) cl[k] = P.c[k];
    for (int j = threadIdx.x; j < n; j += blockDim.x) isl[j] = P.isint[j];
    if (ALDS)
        for (int e = threadIdx.x; e < m * n; e += blockDim.x) {
            const int j = e / m, i = e - j * m;
            Ar[(size_t)i * n + j] = P.A[e];
        }
    NodeSp sp{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (P.nnz > 0) {
        if (nzl) {
            for (int t = threadIdx.x; t < nzl; t += blockDim.x) {
                rv[t] = P.rval[t]; cv[t] = P.cval[t];
                ri_[t] = P.rind[t]; ci[t] = P.cind[t];
            }
            for (int i = threadIdx.x; i <= m; i += blockDim.x) rp[i] = P.rptr[i];
            for (int j = threadIdx.x; j <= n; j += blockDim.x) cp[j] = P.cptr[j];
            sp = NodeSp{rp, ri_, cp, ci, rv, cv};
        } else sp = NodeSp{P.rptr, P.rind, P.cptr, P.cind, P.rval, P.cval};
    }
    double *gbnd = io.bnd + (size_t)b * 2 * n, *gdz = io.dzb + (size_t)b * 2 * n;
    const double *tin = io.tab_in ? io.tab_in[b] : nullptr;
    const int brj = io.br_j ? io.br_j[b] : -1;
    if (brj >= 0) {
        // a child built here from its parent's stored record (fill_child of
        // the host driver, on the device): the parent's final column bounds
        // and statuses, the branching bound (glpios03.js:141-186), statuses
        // that follow the column types (glp_set_col_bnds)
        const double *rb = tin + node_rec_bounds(m, n);
        const signed char *rs = (const signed char *)(rb + 2 * (size_t)n);
        for (int k = threadIdx.x; k < N; k += blockDim.x) {
            double l, u;
            if (k < m) { l = P.rlb[k]; u = P.rub[k]; }
            else { l = rb[k - m]; u = rb[n + k - m]; }
            signed char s = rs[k];
            if (k - m == brj) {
                const double beta = io.br_val[b];
                if (io.br_dir[b] == 0) u = floor(beta);
                else l = ceil(beta);
            }
            if (k >= m && s != BS) {
                if (l == u) s = NS;
                else if (s == NS) s = (l != -DBL_MAX) ? NL : (u != DBL_MAX ? NU : NF);
            }
            lb[k] = l;
            ub[k] = u;
            stat[k] = s;
        }
    } else {
        const double *glb = io.lb + (size_t)b * N, *gub = io.ub + (size_t)b * N;
        const signed char *gst = io.stat_in + (size_t)b * N;
        for (int k = threadIdx.x; k < N; k += blockDim.x) {
            lb[k] = glb[k];
            ub[k] = gub[k];
            stat[k] = gst[k];
        }
    }
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        chg[j] = 0;
        gdz[2 * j] = 0.0;
        gdz[2 * j + 1] = 0.0;
    }
    __syncthreads();
    auto put_bounds = [&]() {
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            gbnd[2 * j] = lb[m + j];
            gbnd[2 * j + 1] = ub[m + j];
        }
    };
    NODE_STAMP(5);
    const int max_pass = io.pp_pass[b];
    if (max_pass > 0 && node_preprocess<ALDS>(P, cl, isl, Ar, sp, io.obj_bound, lb, ub, stat, chg, rinfo, max_pass)) {
        put_bounds();
        if (threadIdx.x == 0) { io.status[b] = NODE_PPINF; io.pivots[b] = 0; io.jj[b] = 0; io.obj[b] = 0.0; }
        NODE_STAMP(7);
        return;
    }
    put_bounds();
    NODE_STAMP(1);
    // warm start: the parent's tableau, when its basis is still this node's
    // (the node's statuses come from the parent's final ones; preprocessing
    // only moves non-basic columns) and it is young enough
    int age = 0;
    if (tin) {
        // the parent's header staged in LDS (cand: m ints, free until the
        // branching), then checked by every thread at once
        int *hin = cand;
        age = (int)tin[0];
        for (int i = threadIdx.x; i < m; i += blockDim.x) hin[i] = (int)tin[1 + i];
        __syncthreads();
        int bad = age >= io.tab_age_max;
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            const int k = hin[i];
            if (k < 0 || k >= N || stat[k] != BS) bad = 1;
        }
        int nbs = 0;
        for (int k0 = 0; k0 < N; k0 += blockDim.x) {
            const int k = k0 + threadIdx.x;
            nbs += __syncthreads_count(k < N && stat[k] == BS);
        }
        if (__syncthreads_or(bad || nbs != m)) { tin = nullptr; age = 0; }
    }
#define T_(i, j) M[(size_t)(i) * W + m + (j)]
    if (tin) {
        // the rows in variable order, as the inversion below leaves them
        // (the dual ratio tests break ties by row: a warm-started node then
        // takes the pivots a cold-started one would)
        int *rk = (int *)fcol;
        const int *hin = cand;
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            const int k = hin[i];
            int r = 0;
            for (int i2 = 0; i2 < m; ++i2) r += hin[i2] < k;
            rk[i] = r;
            head[r] = k;
        }
        __syncthreads();
        const double *tt = tin + 1 + m;
        for (int e = threadIdx.x; e < m * N; e += blockDim.x) {
            const int i = e / N, k = e - i * N;
            T_(rk[i], k) = tt[e];
        }
        __syncthreads();
    } else {
    // basis header in variable order (glp_factorize's head, glpapi12.js:44-67)
    if (threadIdx.x == 0) {
        int j = 0;
        for (int k = 0; k < N && j <= m; ++k)
            if (stat[k] == BS) {
                if (j < m) head[j] = k;
                j++;
            }
        sh_flag = (j == m) ? 0 : 1;
    }
    __syncthreads();
    if (sh_flag) {
        if (threadIdx.x == 0) { io.status[b] = NODE_FAIL; io.pivots[b] = 0; io.jj[b] = 0; }
        return;
    }
    // M = [B | I | -A]: column k of (I | -A) is e_k (k < m) or -A[:, k-m]
    for (int e = threadIdx.x; e < m * W; e += blockDim.x) {
        const int i = e / W, c = e % W;
        double v;
        if (c < m) {
            const int k = head[c];
            v = (k < m) ? (i == k ? 1.0 : 0.0) : -(ALDS ? Ar[(size_t)i * n + (k - m)] : P.A[(size_t)(k - m) * m + i]);
        } else if (c < 2 * m) {
            v = (i == c - m) ? 1.0 : 0.0;
        } else {
            v = -(ALDS ? Ar[(size_t)i * n + (c - 2 * m)] : P.A[(size_t)(c - 2 * m) * m + i]);
        }
        M[(size_t)i * W + c] = v;
    }
    __syncthreads();
    // Gauss-Jordan with partial pivoting on the left m x m block
    for (int k = 0; k < m; ++k) {
        double key = -1.0;
        int idx = -1;
        for (int i = k + threadIdx.x; i < m; i += blockDim.x) {
            const double v = fabs(M[(size_t)i * W + k]);
            if (idx < 0 || v > key) { key = v; idx = i; }
        }
        const int piv = block_argmax(key, idx, shk, shi);
        const bool singular = piv < 0 || fabs(M[(size_t)piv * W + k]) < 1e-12;
        __syncthreads();                      // every wave has read M[piv][k] before the swap moves it
        if (singular) {
            if (threadIdx.x == 0) { io.status[b] = NODE_FAIL; io.pivots[b] = 0; io.jj[b] = 0; }
            return;
        }
        if (piv != k)
            for (int c = threadIdx.x; c < W; c += blockDim.x) {
                const double t = M[(size_t)k * W + c];
                M[(size_t)k * W + c] = M[(size_t)piv * W + c];
                M[(size_t)piv * W + c] = t;
            }
        __syncthreads();
        const double inv = 1.0 / M[(size_t)k * W + k];
        __syncthreads();                      // every thread has read the pivot before row k is scaled
        for (int c = threadIdx.x; c < W; c += blockDim.x) M[(size_t)k * W + c] *= inv;
        // multipliers of column k, saved before the elimination overwrites it
        for (int i = threadIdx.x; i < m; i += blockDim.x) fcol[i] = (i == k) ? 0.0 : M[(size_t)i * W + k];
        __syncthreads();
        for (int e = threadIdx.x; e < m * W; e += blockDim.x) {
            const int i = e / W, c = e % W;
            const double f = fcol[i];
            if (f != 0.0) M[(size_t)i * W + c] -= f * M[(size_t)k * W + c];
        }
        __syncthreads();
    }
    // T[i][j] = M[i][m + j]  (row length W kept; T(i, j) = M[i*W + m + j])
    }
    NODE_STAMP(2);
    // d = c - c_B' T  (c_B staged in fcol)
    for (int i = threadIdx.x; i < m; i += blockDim.x) fcol[i] = cl[head[i]];
    __syncthreads();
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        if (stat[k] == BS) { d[k] = 0.0; continue; }
        double s = cl[k];
        for (int i = 0; i < m; ++i) {
            const double cb = fcol[i];
            if (cb != 0.0) s -= cb * T_(i, k);
        }
        d[k] = s;
    }
    __syncthreads();
    // a free column that gained a bound in preprocessing: the bound its
    // reduced cost allows (a warm start must stay dual feasible)
    {
        int bad = 0;
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            if (!chg[j]) continue;
            const int k = m + j;
            const bool hl = lb[k] != -DBL_MAX, hu = ub[k] != DBL_MAX;
            if (hl && hu) stat[k] = d[k] >= 0.0 ? NL : NU;
            else if (hl) { stat[k] = NL; if (d[k] < -1e-9) bad = 1; }
            else { stat[k] = NU; if (d[k] > 1e-9) bad = 1; }
        }
        if (__syncthreads_or(bad)) {
            if (threadIdx.x == 0) { io.status[b] = NODE_FAIL; io.pivots[b] = 0; io.jj[b] = 0; }
            return;
        }
    }
    // x_N and x_B = -T_N x_N
    for (int k = threadIdx.x; k < N; k += blockDim.x) x[k] = (stat[k] == BS) ? 0.0 : nb_value(stat[k], lb[k], ub[k]);
    __syncthreads();
    {
        // one wave per row, lanes over the columns
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
        for (int i = wv; i < m; i += nwv) {
            double sx = 0.0;
            for (int k = lane; k < N; k += 64)
                if (stat[k] != BS && x[k] != 0.0) sx += T_(i, k) * x[k];
            sx = wsum(sx);
            if (lane == 0) x[head[i]] = -sx;
        }
    }
    __syncthreads();
    NODE_STAMP(3);
    // ---- bounded dual simplex ------------------------------------------
    // the reference's node LP is glp_simplex with meth GLP_DUALP and the
    // default SMCP (glpios01.js:866-910): projected steepest-edge chuzr
    // (glpspx02.js:572) and the Harris two-pass chuzc with rtol = 0.30 tol_dj
    // (glpspx02.js:793, called at :1859) on the row sorted with tol_bnd
    // (sort_trow :754, called at :1851)
    const double tol_bnd = 1e-7, tol_dj = 1e-7, kappa = 0.10, rtol = 0.30 * tol_dj;
    const double cutoff = io.cutoff[b];
    const int it_lim = io.it_lim[b];
    int it = 0, status = NODE_OPT;
    // a pivot is three barriers: wave 0 takes the whole decision (objective
    // and cutoff, chuzr, the ratio test on row p: wave reductions only) while
    // the other waves wait; then one update phase that reads row p and
    // column q as they were (x, d and every other entry of T) and one that
    // rewrites row p, column q and the header
    __shared__ int sh_st, sh_p, sh_q;
    __shared__ double sh_tq, sh_dq, sh_apq;
    for (;;) {
        if (it % 1000 == 0) {
            // reset_refsp (glpspx02.js:497): the reference space is the
            // current basic set, every weight 1 — at the start of the node's
            // solve (refct = 0) and after every 1000 weight updates
            for (int k = threadIdx.x; k < N; k += blockDim.x) refsp[k] = stat[k] == BS;
            for (int i = threadIdx.x; i < m; i += blockDim.x) gam[i] = 1.0;
            __syncthreads();
        }
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            int dec = -1, p = -1, q = -1;
            // objective (dual objective of the current dual feasible basis)
            double zs = 0.0;
            for (int k = lane; k < N; k += 64) zs += cl[k] * x[k];
            const double z = wsum(zs);
            if (z >= cutoff) dec = NODE_CUTOFF;
            else {
                // chuzr: the largest squared bound violation over the row's
                // weight; the first row among equals
                double key = 0.0;
                int idx = -1;
                for (int i = lane; i < m; i += 64) {
                    const int k = head[i];
                    const double v = x[k];
                    double r = 0.0;
                    if (lb[k] != -DBL_MAX && v < lb[k] - tol_bnd * (1.0 + kappa * fabs(lb[k]))) r = lb[k] - v;
                    if (ub[k] != DBL_MAX && v > ub[k] + tol_bnd * (1.0 + kappa * fabs(ub[k]))) r = ub[k] - v;
                    if (r == 0.0) continue;
                    const double g = fmax(gam[i], DBL_EPSILON), s = r * r / g;
                    if (s > key) { key = s; idx = i; }
                }
                p = wave_argmax(key, idx);
                if (p < 0) dec = NODE_OPT;                 // primal feasible: optimal
                else if (it >= it_lim) dec = NODE_ITLIM;
            }
            if (dec < 0) {
                const int kp = head[p];
                const bool to_lb = x[kp] < lb[kp];
                // x_p = -sum T[p,k] x_k: the reference's row trow_k = -T[p,k];
                // alfa = s trow_k with s = sign(delta) (+1: x_p rises to lb)
                const double s = to_lb ? 1.0 : -1.0;
                double rmax = 0.0;
                for (int k = lane; k < N; k += 64)
                    if (stat[k] != BS && stat[k] != NS) rmax = fmax(rmax, fabs(T_(p, k)));
                rmax = wmax(rmax);
                const double eps = tol_bnd * (1.0 + 0.01 * rmax);
                // first pass: the bounds relaxed by rtol, smallest step
                // (the larger |alfa| among equal steps)
                double bt = 0.0, ba = 0.0;
                int bq = -1;
                for (int k = lane; k < N; k += 64) {
                    const int st = stat[k];
                    if (st == BS || st == NS) continue;
                    const double a = T_(p, k);
                    if (fabs(a) < eps) continue;
                    const double alfa = -s * a;
                    double t;
                    if (alfa > 0.0) {
                        if (st != NL && st != NF) continue;
                        t = (d[k] + rtol) / alfa;
                    } else {
                        if (st != NU && st != NF) continue;
                        t = (d[k] - rtol) / alfa;
                    }
                    if (t < 0.0) t = 0.0;
                    if (bq < 0 || t < bt || (t == bt && fabs(alfa) > ba)) { bt = t; ba = fabs(alfa); bq = k; }
                }
                q = wave_ratio(bt, ba, bq);
                double teta = 0.0;
                if (q >= 0) {
                    const double tmax = wave_pick(bt, bq, q);
                    teta = tmax;
                    if (tmax > 0.0) {
                        // second pass: within the relaxed step, the largest |alfa|
                        double ka = -1.0, kt = 0.0;
                        int kq = -1;
                        for (int k = lane; k < N; k += 64) {
                            const int st = stat[k];
                            if (st == BS || st == NS) continue;
                            const double a = T_(p, k);
                            if (fabs(a) < eps) continue;
                            const double alfa = -s * a;
                            if (alfa > 0.0 ? (st != NL && st != NF) : (st != NU && st != NF)) continue;
                            double t = d[k] / alfa;
                            if (t < 0.0) t = 0.0;
                            if (t <= tmax && fabs(alfa) > ka) { ka = fabs(alfa); kq = k; kt = t; }
                        }
                        q = wave_argmax(ka, kq);
                        teta = wave_pick(kt, kq, q);
                    }
                }
                if (q < 0) dec = NODE_INFEAS;              // dual unbounded
                else if (lane == 0) {
                    const double apq = T_(p, q);
                    const double bound = to_lb ? lb[kp] : ub[kp];
                    sh_apq = apq;
                    sh_tq = (x[kp] - bound) / apq;         // step of x_q
                    sh_dq = -s * teta;                     // -new_dq: d_k -= dq T[p,k], d_kp = -dq
                }
            }
            if (lane == 0) { sh_st = dec; sh_p = p; sh_q = q; }
        }
        __syncthreads();
        if (sh_st >= 0) { status = sh_st; break; }
        // pivot (p, q)
        const int p = sh_p, q = sh_q, kp = head[p];
        const double apq = sh_apq, tq = sh_tq, dq = sh_dq;
        // x update (basic variables of rows i != p)
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            if (i == p) continue;
            const double a = T_(i, q);
            if (a != 0.0) x[head[i]] -= a * tq;
        }
        // reduced costs: d_k -= dq * T[p,k]
        for (int k = threadIdx.x; k < N; k += blockDim.x) {
            if (k == q) continue;
            const double a = T_(p, k);
            if (a != 0.0) d[k] -= dq * a;
        }
        // T update outside row p and column q: row i -= T[i,q] (row p / apq),
        // a wave per row, lanes along it.  The rows' projected steepest-edge
        // weights of the adjacent basis come from the rows themselves:
        // gamma_i = [x_B(i) in the reference space] + sum of T[i,k]^2 over
        // the non-basic non-fixed k of the reference space — the quantity
        // update_gamma (glpspx02.js:1075) carries by recurrence, exact here
        // because the tableau is explicit.  A row with T[i,q] = 0 keeps its
        // weight (its entries in columns q and kp are zero before and after).
        {
            const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
            const bool kp_in = refsp[kp] && lb[kp] != ub[kp];     // x_kp leaves non-fixed
            for (int i = wv; i < m; i += nwv) {
                const double f = (i == p) ? 0.0 : T_(i, q);
                if (i != p && f == 0.0) continue;
                double g = 0.0;
                for (int k = lane; k < N; k += 64) {
                    if (k == q) continue;
                    const double r = T_(p, k) / apq;
                    double v;
                    if (i == p) v = r;
                    else {
                        v = T_(i, k) - f * r;
                        T_(i, k) = v;
                    }
                    const bool in = (k == kp) ? kp_in : (refsp[k] && stat[k] != BS && stat[k] != NS);
                    if (in) g += v * v;
                }
                g = wsum(g);
                if (lane == 0) gam[i] = (refsp[i == p ? q : head[i]] ? 1.0 : 0.0) + g;
            }
        }
        __syncthreads();
        for (int k = threadIdx.x; k < N; k += blockDim.x) T_(p, k) /= apq;
        for (int i = threadIdx.x; i < m; i += blockDim.x)
            if (i != p) T_(i, q) = 0.0;
        if (threadIdx.x == 0) {
            const bool to_lb = x[kp] < lb[kp];
            const double bound = to_lb ? lb[kp] : ub[kp];
            x[q] += tq;
            x[kp] = bound;
            d[q] = 0.0;
            d[kp] = -dq;
            stat[kp] = to_lb ? (lb[kp] == ub[kp] ? NS : NL) : (lb[kp] == ub[kp] ? NS : NU);
            stat[q] = BS;
            head[p] = q;
        }
        __syncthreads();
        it++;
    }
    __syncthreads();
    NODE_STAMP(4);
    // the children's warm start
    double *tout = io.tab_out ? io.tab_out[b] : nullptr;
    if (tout && status == NODE_OPT) {
        if (threadIdx.x == 0) tout[0] = (double)(age + it);
        for (int i = threadIdx.x; i < m; i += blockDim.x) tout[1 + i] = (double)head[i];
        double *tt = tout + 1 + m;
        for (int e = threadIdx.x; e < m * N; e += blockDim.x) {
            const int i = e / N, k = e - i * N;
            tt[e] = T_(i, k);
        }
    }
    double zs = 0.0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) zs += cl[k] * x[k];
    const double z = block_sum256(zs, shk);
    // outputs
    double *gx = io.x + (size_t)b * N;
    signed char *gso = io.stat_out + (size_t)b * N;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        gx[k] = x[k];
        gso[k] = stat[k];
    }
    if (status != NODE_OPT) {
        if (threadIdx.x == 0) {
            io.status[b] = status;
            io.obj[b] = z;
            io.pivots[b] = it;
            io.jj[b] = 0;
        }
        NODE_STAMP(7);
        return;
    }
    // ---- fix_by_red_cost (glpios03.js:307, called at :801 once an incumbent
    // exists): a non-basic integer column whose reduced cost alone lifts the
    // node's objective to the incumbent is fixed on its current bound (the
    // LP solution does not change; the children inherit the fixing through
    // the node's final bounds, and the branching below skips it as NS)
    if (io.obj_bound < DBL_MAX) {
        const double best = io.obj_bound;
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            const int k = m + j;
            if (!isl[j]) continue;
            double dj = d[k];
            if (stat[k] == NL) {
                if (dj < 0.0) dj = 0.0;
                if (z + dj >= best) { ub[k] = lb[k]; stat[k] = NS; }
            } else if (stat[k] == NU) {
                if (dj > 0.0) dj = 0.0;
                if (z - dj >= best) { lb[k] = ub[k]; stat[k] = NS; }
            }
        }
        __syncthreads();
        put_bounds();
    }
    // ---- ios_eval_degrad (glpios03.js:188) for every fractional column and
    // branch_drtom (glpios09.js:84) on the node's own tableau rows ---------
    // columns in order; x_j basic and fractional; the dual ratio test of
    // glp_dual_rtest (glpapi12.js:687) on the row x_j = sum alfa_k x_k,
    // alfa_k = -T[i,k]; delta z = d_k * delta x_k.  dzb (the one-pivot dual
    // bound of each branch, DBL_MAX: the branch has no feasible point) goes
    // to the host for whichever column the branching rule picks; with DTH
    // the choice uses Tomlin's rounding of delta x_k on integer columns
    // The candidates are evaluated in parallel, one wave per column (a
    // wave-wide ratio test per branch, no block barrier), and the choice
    // then walks them in column order as the reference does, stopping at
    // the first column with a branch that has no feasible point
    __shared__ int sh_jj, sh_next;
    __shared__ double sh_degrad;
    __shared__ int sh_wc[4];
    for (int i = threadIdx.x; i < m; i += blockDim.x) rowof[head[i]] = i;
    if (threadIdx.x == 0) { sh_jj = 0; sh_next = 0; sh_degrad = -1.0; }
    // the fractional basic integer columns in column order (ballot compaction)
    int ncand = 0;
    for (int j0 = 0; j0 < n; j0 += blockDim.x) {
        const int j = j0 + threadIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        bool f = false;
        if (j < n && stat[m + j] == BS && isl[j]) {
            const double xv = x[m + j];
            f = fabs(xv - floor(xv + 0.5)) > P.tol_int;
        }
        const unsigned long long msk = __ballot(f);
        if (lane == 0) sh_wc[wv] = __popcll(msk);
        __syncthreads();
        int base = ncand, tot = 0;
        for (int v = 0; v < (int)(blockDim.x >> 6); ++v) {
            if (v < wv) base += sh_wc[v];
            tot += sh_wc[v];
        }
        if (f) cand[base + __popcll(msk & ((1ull << lane) - 1ull))] = j;
        ncand += tot;
        __syncthreads();
    }
    const int any_frac = ncand > 0;
    {
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
        for (int c = wv; c < ncand; c += nwv) {
            const int j = cand[c], k = m + j, row = rowof[k];
            const double xv = x[k];
            // both branches in one sweep: dir -1 (down), +1 (up)
            double bt0 = 0.0, ba0 = 0.0, bt1 = 0.0, ba1 = 0.0;
            int bq0 = -1, bq1 = -1;
            for (int kk = lane; kk < N; kk += 64) {
                const int st = stat[kk];
                if (st == BS || st == NS) continue;
                const double tr = T_(row, kk), dk = d[kk];
#pragma unroll
                for (int kase = 0; kase < 2; ++kase) {
                    const double alfa = kase == 0 ? tr : -tr;      // dir * (-T[row, kk])
                    double t;
                    if (st == NL) {
                        if (alfa < +1e-9) continue;
                        t = dk / alfa;
                    } else if (st == NU) {
                        if (alfa > -1e-9) continue;
                        t = dk / alfa;
                    } else {
                        if (-1e-9 < alfa && alfa < +1e-9) continue;
                        t = 0.0;
                    }
                    if (t < 0.0) t = 0.0;
                    double &bt = kase == 0 ? bt0 : bt1, &ba = kase == 0 ? ba0 : ba1;
                    int &bq = kase == 0 ? bq0 : bq1;
                    if (bq < 0 || t < bt || (t == bt && fabs(alfa) > ba)) { bt = t; ba = fabs(alfa); bq = kk; }
                }
            }
            double dz[2], dzb[2];
#pragma unroll
            for (int kase = 0; kase < 2; ++kase) {
                const int kq = wave_ratio(kase == 0 ? bt0 : bt1, kase == 0 ? ba0 : ba1, kase == 0 ? bq0 : bq1);
                if (kq < 0) dz[kase] = dzb[kase] = DBL_MAX;
                else {
                    const double alfa = -T_(row, kq);
                    const double delta_j = (kase == 0 ? floor(xv) : ceil(xv)) - xv;
                    double delta_k = delta_j / alfa;
                    double dk = d[kq];
                    const int st = stat[kq];
                    if ((st == NL && dk < 0.0) || (st == NU && dk > 0.0) || st == NF) dk = 0.0;
                    // the objective after this one dual pivot bounds the branch
                    dzb[kase] = fabs(dk * delta_k);
                    if (kq >= m && isl[kq - m] && fabs(delta_k - floor(delta_k + 0.5)) > 1e-3)
                        delta_k = delta_k > 0.0 ? ceil(delta_k) : floor(delta_k);
                    dz[kase] = fabs(dk * delta_k);   // Tomlin's estimate: choice only
                }
            }
            if (lane == 0) {
                dzt[4 * c] = dz[0]; dzt[4 * c + 1] = dz[1];
                dzt[4 * c + 2] = dzb[0]; dzt[4 * c + 3] = dzb[1];
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int c = 0; c < ncand; ++c) {
            const int j = cand[c];
            const double dz0 = dzt[4 * c], dz1 = dzt[4 * c + 1];
            gdz[2 * j] = dzt[4 * c + 2];
            gdz[2 * j + 1] = dzt[4 * c + 3];
            if (P.dth && (sh_degrad < dz0 || sh_degrad < dz1)) {
                sh_jj = j + 1;
                if (dz0 < dz1) { sh_next = -1; sh_degrad = dz1; }
                else { sh_next = +1; sh_degrad = dz0; }
                if (sh_degrad == DBL_MAX) break;
            }
        }
    }
    if (threadIdx.x == 0) {
        int jj = sh_jj, next = sh_next;
        if (!P.dth) {
            // the host applies the branching rule; report the first candidate
            jj = ncand ? cand[0] + 1 : 0;
        } else if (any_frac && sh_degrad < 1e-6 * (1.0 + 0.001 * fabs(z))) {
            // branch_mostf (glpios09.js:62): value closest to floor + 1/2
            double most = DBL_MAX;
            jj = 0;
            for (int c = 0; c < ncand; ++c) {
                const int j = cand[c];
                const double beta = x[m + j];
                const double temp = floor(beta) + 0.5;
                if (most > fabs(beta - temp)) {
                    jj = j + 1;
                    most = fabs(beta - temp);
                    next = beta < temp ? -1 : +1;
                }
            }
        }
        // check_integrality (glpios03.js:55) as the host driver states it
        // (MipSolver::integrality), in column order: the count, the sum of
        // integer infeasibilities, and the candidates of branch_first /
        // branch_last / branch_mostf (glpios09.js:28-82)
        // (a subset of the candidates above: integer columns have integral
        // bounds, glp_intopt's precondition kept by the preprocessing)
        int nf = 0, jf = -1, jl = -1, jm = -1, nm = 0;
        double ii = 0.0, most = DBL_MAX;
        bool jj_cand = false;
        const double tol = P.tol_int;
        for (int c = 0; c < ncand; ++c) {
            const int j = cand[c], k = m + j;
            const double v = x[k], l = lb[k], u = ub[k];
            if (l != -DBL_MAX) {
                if (l - tol <= v && v <= l + tol) continue;
                if (v < l) continue;
            }
            if (u != DBL_MAX) {
                if (u - tol <= v && v <= u + tol) continue;
                if (v > u) continue;
            }
            const double r = floor(v + 0.5);
            if (r - tol <= v && v <= r + tol) continue;
            nf++;
            if (jf < 0) jf = j;
            jl = j;
            if (jj == j + 1) jj_cand = true;
            const double t1 = v - floor(v), t2 = ceil(v) - v;
            ii += (t1 <= t2 ? t1 : t2);
            const double temp = floor(v) + 0.5;
            if (most > fabs(v - temp)) {
                jm = j;
                most = fabs(v - temp);
                nm = v < temp ? -1 : +1;
            }
        }
        io.nfrac[b] = nf;
        io.iisum[b] = ii;
        io.jfirst[b] = jf;
        io.jlast[b] = jl;
        io.jmost[b] = jm;
        io.nmost[b] = nm;
        io.status[b] = NODE_OPT;
        io.obj[b] = z;
        io.pivots[b] = it;
        // the tableau's choice only if it is a candidate of the host's test
        io.jj[b] = (any_frac && jj_cand) ? jj : 0;
        io.next[b] = next;
    }
    // the children's record: final column bounds and statuses
    if (tout) {
        double *rb = tout + node_rec_bounds(m, n);
        signed char *rs = (signed char *)(rb + 2 * (size_t)n);
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            rb[j] = lb[m + j];
            rb[n + j] = ub[m + j];
        }
        for (int k = threadIdx.x; k < N; k += blockDim.x) rs[k] = stat[k];
    }
    NODE_STAMP(7);
#undef T_
#undef NODE_STAMP
}

// the node kernel's work area (alds: with the row-major copy of A and, for
// a sparse A, its copies by rows and columns)
size_t node_lp_lds(int m, int n, int alds = 0, int nnz = 0)
{
    const size_t N = (size_t)m + n, z = alds ? (size_t)nnz : 0;
    return sizeof(double) * ((size_t)m * (2 * m + n) + 5 * N + 6 * (size_t)m + 6 * ((size_t)m + 1) +
                             (alds ? (size_t)m * n : 0) + 2 * z) +
           sizeof(int) * (2 * (size_t)m + N + (z ? (size_t)m + n + 2 + 2 * z : 0)) + 2 * N + 2 * (size_t)n + 16;
}

constexpr size_t NODE_LDS_MAX = 64 * 1024;
// the node kernel's work area per node beyond which the node LPs go to the
// engine (GK_BNB_ENGINE_BYTES, default 1 MiB: m (2m + n) doubles streamed by
// one CU per pivot against the revised simplex on a factor; sparsebig1, 1.8
// MB per node: 0.58 s and 4,818 node LPs in the node kernel, 0.53 s and 410
// in engine mode — reference 297); engine mode solves engine_batch() nodes per
// search step
static size_t engine_node_bytes()
{
    const char *e = std::getenv("GK_BNB_ENGINE_BYTES");        // (read per search: tests switch it)
    return e ? (size_t)std::max(0LL, std::atoll(e)) : ((size_t)1 << 20);
}
static int engine_batch()                             // GK_BNB_ENGINE_BATCH (experiments), default 8
{
    static const int b = [] {
        const char *e = std::getenv("GK_BNB_ENGINE_BATCH");
        return e ? std::max(1, std::min(std::atoi(e), 64)) : 8;
    }();
    return b;
}

void launch_node_lp(hipStream_t s, const NodeProb &P, const NodeIO &io, int nb)
{
    if (node_lp_lds(P.m, P.n, 1, P.nnz) <= NODE_LDS_MAX)
        hipLaunchKernelGGL((k_node_lp<0, 1>), dim3(nb), dim3(256), node_lp_lds(P.m, P.n, 1, P.nnz), s, P, io);
    else if (node_lp_lds(P.m, P.n) <= NODE_LDS_MAX)
        hipLaunchKernelGGL((k_node_lp<0, 0>), dim3(nb), dim3(256), node_lp_lds(P.m, P.n), s, P, io);
    else hipLaunchKernelGGL((k_node_lp<1, 0>), dim3(nb), dim3(256), 0, s, P, io);
}

// ---------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------
namespace {

template <typename T>
struct DevArr {
    T *p = nullptr;
    size_t n = 0;
    void ensure(size_t cnt)
    {
        if (cnt <= n && p) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        if (hipMalloc((void **)&p, std::max<size_t>(cnt, 1) * sizeof(T)) != hipSuccess) p = nullptr;
        n = p ? std::max<size_t>(cnt, 1) : 0;
    }
    ~DevArr()
    {
        if (p) (void)hipFree(p);
    }
};

template <typename T>
struct HostArr {
    T *p = nullptr;
    size_t n = 0;
    void ensure(size_t cnt)
    {
        if (cnt <= n && p) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        if (hipHostMalloc((void **)&p, std::max<size_t>(cnt, 1) * sizeof(T), hipHostMallocDefault) != hipSuccess)
            p = nullptr;
        n = p ? std::max<size_t>(cnt, 1) : 0;
    }
    ~HostArr()
    {
        if (p) (void)hipHostFree(p);
    }
};

// the node records kept in HBM (NodeIO tab_in / tab_out): slots of
// node_rec_doubles(m, n) in chunks that never move (a slot's address goes
// into the kernel's tab_in / tab_out), reference counted — one reference for
// the batch that writes the record, one per child or parked node reading it.
// At most cap_bytes of them (GK_BNB_TAB_MB, default 8 GiB of the 288 GiB);
// beyond that a node stores none: the host fills its children's arrays and
// they invert their basis
struct TabStore {
    static constexpr int CHUNK = 1024;
    std::vector<double *> chunks;
    std::vector<int> ref, freel;
    size_t slot = 0, cap_bytes = 0;
    ~TabStore() { clear(); }
    void clear()
    {
        for (double *p : chunks) (void)hipFree(p);
        chunks.clear();
        ref.clear();
        freel.clear();
    }
    // a new search: keep the chunks when the slot size is the same
    void reset(size_t doubles, size_t cap)
    {
        if (doubles != slot) clear();
        slot = doubles;
        cap_bytes = cap;
        freel.clear();
        for (int i = (int)ref.size() - 1; i >= 0; i--) freel.push_back(i);
        std::fill(ref.begin(), ref.end(), 0);
    }
    int alloc()
    {
        if (freel.empty()) {
            const size_t bytes = slot * sizeof(double) * CHUNK;
            if ((chunks.size() + 1) * bytes > cap_bytes) return -1;
            double *p = nullptr;
            if (hipMalloc((void **)&p, bytes) != hipSuccess) return -1;
            chunks.push_back(p);
            const int base = (int)ref.size();
            ref.resize(ref.size() + CHUNK, 0);
            for (int i = CHUNK - 1; i >= 0; i--) freel.push_back(base + i);
        }
        const int t = freel.back();
        freel.pop_back();
        ref[t] = 1;
        return t;
    }
    void inc(int t)
    {
        if (t >= 0) ref[t]++;
    }
    void dec(int t)
    {
        if (t >= 0 && --ref[t] == 0) freel.push_back(t);
    }
    double *ptr(int t) const { return t < 0 ? nullptr : chunks[t / CHUNK] + (size_t)(t % CHUNK) * slot; }
};

// what a node knows about its parent (the reference keeps it in node.up and
// in the branching fields of the parent: glpios01.js, glpios03.js:141)
struct NodeMeta {
    int tab = -1;                 // the parent's record (TabStore slot), -1: none
    bool inl = true;              // the pool slot holds the node's bounds and statuses;
                                  // false: the kernel builds them from the record tab
    int br_dir = 0;               // 0: the down branch (ub = floor), 1: up (lb = ceil)
    int arr = -1;                 // inline nodes: the slot of their arrays in NodePool::bnd / st
    int level = 0;
    int br_var = -1;              // column the parent branched on (0-based); -1: root
    double br_val = 0.0;          // its value in the parent's LP solution (ios_pcost_update)
    double up_lpobj = 0.0;        // the parent's LP objective (minimisation form)
    double up_bound = 0.0;        // the parent's local bound (best projection)
    double up_ii = 0.0;           // the parent's sum of integer infeasibilities
    double lpz = 0.0;             // its own LP objective estimate (minimisation form): the parent's
                                  // objective plus the branch's degradation (branch_on's node.lp_obj)
};

// an open node: its local bound, the selection keys of the backtracking
// technique (smaller first), creation order and its slot in the node pool
struct NodeRec {
    double bound;
    double key, key2;
    long long seq;
    int slot;
};

struct NodeWorse {                // heap order: a is selected after b
    bool operator()(const NodeRec &a, const NodeRec &b) const
    {
        if (a.key != b.key) return a.key > b.key;
        if (a.key2 != b.key2) return a.key2 > b.key2;
        return a.seq > b.seq;
    }
};

// node slots (the parent information), recycled through a free list, and —
// only for the nodes that need them on the host (inline: the root, nodes
// received from another rank, children whose parent has no record) — array
// slots of 2 n doubles (lb | ub of the structurals) and m + n statuses.  The
// storage is kept by the context from one search to the next (take / give)
struct NodePool {
    int n = 0, N = 0;
    TabStore *tabs = nullptr;
    std::vector<double> bnd;
    std::vector<signed char> st;
    std::vector<NodeMeta> meta;
    std::vector<int> freel, afree;
    int narr = 0;
    int alloc()
    {
        int sl;
        if (!freel.empty()) {
            sl = freel.back();
            freel.pop_back();
            meta[sl] = NodeMeta{};
        } else {
            sl = (int)meta.size();
            meta.emplace_back();
        }
        return sl;
    }
    // the node's bound and status arrays (inline nodes); called on the
    // search's own thread (the storage may grow), before any worker fills them
    void need_arrays(int sl)
    {
        NodeMeta &mt = meta[sl];
        if (mt.arr >= 0) return;
        if (!afree.empty()) {
            mt.arr = afree.back();
            afree.pop_back();
            return;
        }
        mt.arr = narr++;
        if ((size_t)narr * 2 * n > bnd.size()) {
            bnd.resize(std::max<size_t>((size_t)narr * 2 * n, 2 * bnd.size()));
            st.resize(std::max<size_t>((size_t)narr * N, 2 * st.size()));
        }
    }
    void release(int sl)
    {
        if (tabs) tabs->dec(meta[sl].tab);
        meta[sl].tab = -1;
        meta[sl].inl = true;
        if (meta[sl].arr >= 0) afree.push_back(meta[sl].arr);
        meta[sl].arr = -1;
        freel.push_back(sl);
    }
    double *lb(int sl) { return bnd.data() + (size_t)meta[sl].arr * 2 * n; }
    double *ub(int sl) { return bnd.data() + (size_t)meta[sl].arr * 2 * n + n; }
    signed char *stat(int sl) { return st.data() + (size_t)meta[sl].arr * N; }
    // a new search: every slot free, the storage's capacity kept
    void reset(int n_, int N_)
    {
        if (n_ != n || N_ != N) { bnd.clear(); st.clear(); }
        n = n_;
        N = N_;
        meta.clear();
        freel.clear();
        afree.clear();
        narr = 0;
    }
};

// check_integrality's results from the node kernel (NodeIO nfrac ...)
struct KInt {
    int nfrac, jf, jl, jm, nm;
    double ii;
};

// one batch entry: a node LP, or a pseudocost probe (a node with one
// column fixed, 30 dual pivots: eval_degrad, glpios09.js:337)
struct Entry {
    int kind;                     // 0 node, 1 probe
    NodeRec nd;
    int pid, j, dir;              // probe: parked node, column, 0 down / 1 up
    int tab_out = -1;             // node: the TabStore slot its tableau goes to
};

// packed batch buffers (one copy each way): byte offsets for nb entries
struct Layout {
    size_t lb, ub, cut, brv, tin, tout, itl, pp, brj, brd, st, in_end;
    size_t obj, ii, dz, x, bnd, stat, piv, jj, next, nf, jf, jl, jm, nm, sto, out_end;
    Layout(size_t N, size_t n, size_t nb)
    {
        lb = 0; ub = lb + 8 * nb * N; cut = ub + 8 * nb * N; brv = cut + 8 * nb; tin = brv + 8 * nb;
        tout = tin + 8 * nb; itl = tout + 8 * nb; pp = itl + 4 * nb; brj = pp + 4 * nb; brd = brj + 4 * nb;
        st = brd + 4 * nb; in_end = st + nb * N;
        obj = 0; ii = obj + 8 * nb; dz = ii + 8 * nb; x = dz + 16 * nb * n; bnd = x + 8 * nb * N;
        stat = bnd + 16 * nb * n; piv = stat + 4 * nb; jj = piv + 4 * nb; next = jj + 4 * nb; nf = next + 4 * nb;
        jf = nf + 4 * nb; jl = jf + 4 * nb; jm = jl + 4 * nb; nm = jm + 4 * nb; sto = nm + 4 * nb;
        out_end = sto + nb * N;
    }
};

struct BatchBuf {
    DevArr<char> din, dout;
    DevArr<unsigned long long> dstamp;      // GK_BNB_LOG=2: the node kernel's phase stamps
    HostArr<char> hin, hout;
    hipEvent_t done = nullptr;
    std::vector<Entry> ents;
    int nb = 0;
    ~BatchBuf()
    {
        if (done) (void)hipEventDestroy(done);
    }
};

// a node whose branching column waits for pseudocost probes (PCH)
struct Parked {
    NodeRec nd;
    NodeMeta meta;
    double z = 0.0, bound = 0.0, ii = 0.0;
    std::vector<double> x, bnd;
    std::vector<double> dzb;             // the kernel's one-pivot branch bounds (ios_eval_degrad)
    std::vector<double> probe;           // probe[2 j + dir]: degradation from the probe LP
    std::vector<signed char> so;
    std::vector<int> cand;
    int pending = 0;
    int tab = -1;                        // its tableau (the probes' and the children's warm start)
};

// the device and pinned host buffers of the driver, kept by the context
// from one glp_intopt to the next (allocating them — hipHostMalloc of the
// packed batch buffers above all — cost a search of gap several
// milliseconds when it was done per call); the arrays only grow
// host workers for the per-node parts of a batch's processing (integrality
// scans and the children's bound / status arrays), persistent across
// searches: for(n, fn) runs fn(i) for i < n on the workers and the caller,
// chunks claimed from an atomic counter, and returns when all are done
struct HostWorkers {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done;
    std::function<void(int)> fn;
    std::atomic<int> next{0};
    int n = 0, chunk = 1, busy = 0;
    unsigned long long gen = 0;
    bool stop = false;
    explicit HostWorkers(int k)
    {
        for (int t = 0; t < k; t++) th.emplace_back([this] { loop(); });
    }
    ~HostWorkers()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
    void work()
    {
        for (;;) {
            const int i0 = next.fetch_add(chunk);
            if (i0 >= n) return;
            const int i1 = std::min(n, i0 + chunk);
            for (int i = i0; i < i1; i++) fn(i);
        }
    }
    void loop()
    {
        unsigned long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
            }
            work();
            {
                std::lock_guard<std::mutex> lk(mu);
                if (--busy == 0) done.notify_one();
            }
        }
    }
    void run(int cnt, int ch, std::function<void(int)> f)
    {
        if (cnt <= 0) return;
        if (th.empty() || cnt < 2 * ch) {
            for (int i = 0; i < cnt; i++) f(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            fn = std::move(f);
            n = cnt;
            chunk = ch;
            next.store(0);
            busy = (int)th.size();
            gen++;
        }
        cv.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return busy == 0; });
    }
};

static int bnb_threads()
{
    static const int v = [] {
        const char *e = std::getenv("GK_BNB_THREADS");
        if (e) return std::max(0, std::min(std::atoi(e), 16));
        const unsigned hc = std::thread::hardware_concurrency();
        return (int)std::min(3u, hc > 1 ? hc - 1 : 0u);
    }();
    return v;
}

struct MipCache {
    BatchBuf bufs[2];
    DevArr<double> dA, dc, dscratch, drb, dspv;
    DevArr<int> dspi;
    std::vector<int> hspi;                   // host staging of the sparse copies (alive until the copies ran)
    std::vector<double> hspv;
    DevArr<signed char> dint;
    TabStore tabs;
    NodePool pool;                           // the node storage, kept between searches
    HostWorkers *workers = nullptr;          // made with the first search that has work for them
    ~MipCache() { delete workers; }
};

}  // namespace

}  // namespace gk
void **gk_ctx_mip_cache(gk_ctx *c, void (**freer)(void *));
void mip_cache_free_hook(void *p) { delete (gk::MipCache *)p; }
namespace gk {

// ---------------------------------------------------------------------------
// one glp_intopt search (ios_driver, glpios03.js:1) on one GPU
// ---------------------------------------------------------------------------
struct MipSolver {
    bool engine = false;                      // engine mode: every node LP by the engine (gk_ios_driver)
    gk_ctx *ctx = nullptr;
    hipStream_t s = nullptr;
    gk_mip *mip = nullptr;
    const gk_iocp *parm = nullptr;
    int m = 0, n = 0, N = 0;
    double sign = 1.0, c0 = 0.0;
    std::vector<double> A, c, rlb, rub, clb, cub;
    std::vector<signed char> isint;
    MipCache *cache = nullptr;
    BatchBuf *bufs = nullptr;
    NodePool pool;
    NodeProb P{};
    int BMAX = 0;
    size_t stride = 0;
    int node_it_lim = 10000;
    // search state
    std::vector<NodeRec> open;                // heap (NodeWorse)
    std::vector<NodeRec> dive, next_dive;     // preferred children (T.child): evaluated in the next batch
    long long seq = 0;
    bool have = false;                        // incumbent of this rank (with x)
    double best = DBL_MAX, gbest = DBL_MAX;   // minimisation form; gbest: best over all ranks
    std::vector<double> xbest;
    long long lp_solves = 0, pivots = 0, created = 1, fallbacks = 0, probes = 0, pp_fathomed = 0;
    int err = 0;                              // GLP_EFAIL: a node LP could not be solved at all
    bool root_seen = false;
    double root_bound = 0.0, root_ii = 0.0;   // best projection (glpios12.js:19)
    // pseudocosts (ios_pcost_init, glpios09.js:272)
    bool pcost_on = false;
    std::vector<int> dn_cnt, up_cnt;
    std::vector<double> dn_sum, up_sum;
    std::vector<Parked> parked;
    std::vector<int> parked_free;
    std::vector<Entry> probeq;
    // engine fallback (ios_solve_node with glp_simplex, glpios01.js:866)
    gk_bfd *fb = nullptr;
    unsigned long long fb_version = 0;
    // engine mode: one context (stream) and factor per concurrent node LP
    struct EngW {
        gk_ctx *ctx = nullptr;
        gk_bfd *fb = nullptr;
        unsigned long long ver = 0;
    };
    std::vector<EngW> engw;
    // ios_round_bound (glpios01.js:730): objective integrality
    bool round_ok = false;
    double round_s = 0.0, round_d = 1.0;

    ~MipSolver()
    {
        if (fb) gk_bfd_destroy(fb);
        for (EngW &w : engw) {
            if (w.fb) gk_bfd_destroy(w.fb);
            if (w.ctx) gk_ctx_destroy(w.ctx);
        }
    }

    size_t in_bytes(int nb) const { return Layout(N, n, nb).in_end; }
    size_t out_bytes(int nb) const { return Layout(N, n, nb).out_end; }
    bool alloc_batch(int B)
    {
        BMAX = B;
        for (int q = 0; q < 2; q++) {
            BatchBuf &bf = bufs[q];
            bf.din.ensure(in_bytes(B) + 64); bf.dout.ensure(out_bytes(B) + 64);
            bf.hin.ensure(in_bytes(B) + 64); bf.hout.ensure(out_bytes(B) + 64);
            if (!bf.done && hipEventCreateWithFlags(&bf.done, hipEventDisableTiming) != hipSuccess) return false;
            if (!bf.din.p || !bf.dout.p || !bf.hin.p || !bf.hout.p) return false;
        }
        return true;
    }

    // min-form bound -> rounded min-form bound
    double round_bound(double z) const
    {
        if (!round_ok || z == DBL_MAX || z == -DBL_MAX) return z;
        // the reference rounds in the original direction; in minimisation
        // form both cases are "round up" of (bound - s) / d
        const double s0 = sign * (round_s - c0), d = round_d;
        const double h = (z - s0) / d;
        if (h >= std::floor(h) + 0.001) return d * std::ceil(h) + s0;
        return z;
    }
    double bestall() const { return std::min(best, gbest); }
    // ios_is_hopeful (glpios01.js:789)
    bool hopeful(double bound) const
    {
        const double b = bestall();
        if (b == DBL_MAX) return true;
        const double eps = parm->tol_obj * (1.0 + std::fabs(c0 + sign * b));
        return bound < b - eps;
    }

    // ---- node selection (ios_choose_node, glpios12.js:2) -----------------
    void set_keys(NodeRec &r) const
    {
        const NodeMeta &mt = pool.meta[r.slot];
        r.key2 = 0.0;
        switch (parm->bt_tech) {
        case 1: r.key = -(double)r.seq; break;                      // DFS: the newest node (T.tail)
        case 2: r.key = (double)r.seq; break;                       // BFS: the oldest node (T.head)
        case 4:                                                     // BPH
            if (bestall() == DBL_MAX || !root_seen || root_ii <= 0.0) r.key = mt.up_ii;   // most_feas
            else r.key = mt.up_bound + (bestall() - root_bound) / root_ii * mt.up_ii;  // best_proj
            break;
        default:                                                    // BLB: best local bound, then
            r.key = r.bound;                                        // (best_node, glpios12.js:49) the
            r.key2 = sign > 0 ? mt.up_ii : mt.lpz;                  // parent's ii_sum (MIN) or the best
            break;                                                  // lp_obj (MAX)
        }
    }
    // best_node's window (glpios12.js:49-87): the subproblems whose local
    // bound is within 0.001 (1 + |bound|) of the best are equally good, and
    // among them the one with the least parent ii_sum (minimisation) or the
    // best lp_obj (maximisation) is chosen, the earliest created on ties.
    // Opt-in (GK_BNB_BLB_WINDOW: the open-list size up to which the window is
    // scanned; default 0, off): with the batched search it changed no node
    // count on gap or the C5s fixtures (profiles/r06_bnb_selection.txt) and
    // its scans cost C5s 12x30 21 -> 128 ms
    static int blb_window_max()
    {
        static const int v = [] {
            const char *e = std::getenv("GK_BNB_BLB_WINDOW");
            return e ? std::max(0, std::atoi(e)) : 0;
        }();
        return v;
    }
    double window_eps(double key) const { return 0.001 * (1.0 + std::fabs(c0 + sign * key)); }
    std::vector<NodeRec> win_buf;
    void push_open(NodeRec r)
    {
        const unsigned long long t0 = tsc_on ? tsc() : 0ull;
        set_keys(r);
        open.push_back(r);
        std::push_heap(open.begin(), open.end(), NodeWorse());
        if (tsc_on) tsc_heap += tsc() - t0;
    }
    NodeRec pop_heap1()
    {
        std::pop_heap(open.begin(), open.end(), NodeWorse());
        NodeRec r = open.back();
        open.pop_back();
        return r;
    }
    NodeRec pop_open()
    {
        const int wmax = blb_window_max();
        if (parm->bt_tech != 3 || wmax == 0 || (int)open.size() > wmax || open.size() < 2) return pop_heap1();
        NodeRec best = pop_heap1();
        const double lim = best.key + window_eps(best.key);
        win_buf.clear();
        while (!open.empty() && open.front().key <= lim) win_buf.push_back(pop_heap1());
        for (NodeRec &r : win_buf)
            if (r.key2 < best.key2 || (r.key2 == best.key2 && r.seq < best.seq)) std::swap(best, r);
        for (const NodeRec &r : win_buf) {
            open.push_back(r);
            std::push_heap(open.begin(), open.end(), NodeWorse());
        }
        return best;
    }
    // the best projection keys depend on the incumbent
    void rekey()
    {
        if (parm->bt_tech != 4) return;
        for (NodeRec &r : open) set_keys(r);
        std::make_heap(open.begin(), open.end(), NodeWorse());
    }
    int cur_tab = -1;                         // the tableau of the node being analysed (its children's warm start)
    int bingos = 0;                           // new incumbents not yet reported
    std::vector<int> cand_buf;                // node_done's fractional columns
    // GK_BNB_LOG: time stamp counter ticks of node_done's parts (host profile)
    bool tsc_on = false;
    unsigned long long tsc_int = 0, tsc_choose = 0, tsc_child = 0, tsc_heap = 0;
    static unsigned long long tsc() { return __rdtsc(); }
    void new_incumbent(double z, const double *x)
    {
        const double before = bestall();
        have = true;
        bingos++;
        best = z;
        std::memcpy(xbest.data(), x, N * sizeof(double));
        if (bestall() != before) rekey();
    }
    void set_gbest(double b)
    {
        if (b < gbest) {
            gbest = b;
            rekey();
        }
    }

    // check_integrality (glpios03.js:55): fractional integer columns and the
    // sum of integer infeasibilities, on the node's own (possibly tightened)
    // column bounds
    int integrality(const double *x, const signed char *so, const double *bl, const double *bu,
                    std::vector<int> &cand, double &ii_sum) const
    {
        cand.clear();
        ii_sum = 0.0;
        const double tol = parm->tol_int;
        for (int j = 0; j < n; j++) {
            if (!isint[j] || so[m + j] != BS) continue;
            const double v = x[m + j], l = bl[j], u = bu[j];
            if (l != -DBL_MAX) {
                if (l - tol <= v && v <= l + tol) continue;
                if (v < l) continue;
            }
            if (u != DBL_MAX) {
                if (u - tol <= v && v <= u + tol) continue;
                if (v > u) continue;
            }
            const double r = std::floor(v + 0.5);
            if (r - tol <= v && v <= r + tol) continue;
            cand.push_back(j);
            const double t1 = v - std::floor(v), t2 = std::ceil(v) - v;
            ii_sum += (t1 <= t2 ? t1 : t2);
        }
        return (int)cand.size();
    }

    // branch_first / branch_last / branch_mostf (glpios09.js:28-82); next:
    // -1 down, +1 up
    static int next_of(double beta) { return (beta - std::floor(beta) < std::ceil(beta) - beta) ? -1 : +1; }
    int choose_simple(int tech, const std::vector<int> &cand, const double *x, int &next) const
    {
        if (tech == 1 || tech == 2) {
            const int j = tech == 1 ? cand.front() : cand.back();
            next = next_of(x[m + j]);
            return j;
        }
        int jj = -1;
        double most = DBL_MAX;
        for (int j : cand) {
            const double beta = x[m + j], temp = std::floor(beta) + 0.5;
            if (most > std::fabs(beta - temp)) {
                jj = j;
                most = std::fabs(beta - temp);
                next = beta < temp ? -1 : +1;
            }
        }
        return jj;
    }

    // ios_pcost_branch (glpios09.js:336) over pseudocosts that are all
    // initialised (probe[] holds the probes of this node, DBL_MAX: that
    // branch has no feasible point); returns the column, next through *next
    int choose_pcost(const std::vector<int> &cand, const double *x, const double *probe, int &next)
    {
        int jjj = -1;
        double dmax = -1.0;
        for (int j : cand) {
            const double beta = x[m + j];
            double psi;
            if (dn_cnt[j] == 0) {
                const double dg = probe[2 * j];
                if (dg == DBL_MAX) { next = -1; return j; }
                dn_cnt[j] = 1;
                dn_sum[j] = dg / (beta - std::floor(beta));
            }
            psi = dn_sum[j] / dn_cnt[j];
            const double d1 = psi * (beta - std::floor(beta));
            if (up_cnt[j] == 0) {
                const double dg = probe[2 * j + 1];
                if (dg == DBL_MAX) { next = +1; return j; }
                up_cnt[j] = 1;
                up_sum[j] = dg / (std::ceil(beta) - beta);
            }
            psi = up_sum[j] / up_cnt[j];
            const double d2 = psi * (std::ceil(beta) - beta);
            const double d = d1 > d2 ? d1 : d2;
            if (dmax < d) {
                dmax = d;
                jjj = j;
                next = d1 <= d2 ? -1 : +1;
            }
        }
        if (dmax == 0.0) return choose_simple(3, cand, x, next);
        return jjj;
    }

    // a child whose bound and status arrays are filled after the batch's
    // sequential pass (process(): many children filled by the workers)
    struct FillJob {
        int slot, j, kase;
        double beta;
        const double *bl, *bu;
        const signed char *so;
    };
    std::vector<FillJob> *defer = nullptr;
    // per-entry scratch of a batch's processing: column bounds (bl | bu),
    // fractional columns, their count and the sum of integer infeasibilities
    std::vector<double> eb;
    std::vector<FillJob> jobs;
    void fill_child(const FillJob &f)
    {
        double *l = pool.lb(f.slot), *u = pool.ub(f.slot);
        std::memcpy(l, f.bl, n * sizeof(double));
        std::memcpy(u, f.bu, n * sizeof(double));
        if (f.kase == 0) u[f.j] = std::floor(f.beta);
        else l[f.j] = std::ceil(f.beta);
        signed char *cs = pool.stat(f.slot);
        std::memcpy(cs, f.so, N);
        for (int q = 0; q < n; q++) {                 // statuses follow the column types (glp_set_col_bnds)
            if (cs[m + q] == BS) continue;
            if (l[q] == u[q]) cs[m + q] = NS;
            else if (cs[m + q] == NS) cs[m + q] = (l[q] != -DBL_MAX) ? NL : (u[q] != DBL_MAX ? NU : NF);
        }
    }

    // branch_on (glpios03.js:141): the two children, the preferred one
    // (T.child) first into the next batch
    void branch(const NodeRec &nd, const NodeMeta &mt, double z, double bound, double ii, const double *x,
                const signed char *so, const double *bl, const double *bu, int j, int next, double dn, double up)
    {
        const double beta = x[m + j];
        const double dz[2] = {dn, up};
        const int first = next < 0 ? 0 : 1;
        bool dived = false;
        for (int r = 0; r < 2; r++) {
            const int kase = (r == 0) ? first : 1 - first;
            if (dz[kase] == DBL_MAX) continue;        // that branch has no feasible point
            const double cb = std::max(bound, round_bound(z + dz[kase]));
            if (!hopeful(cb)) continue;
            const int sl = pool.alloc();
            NodeMeta &cm = pool.meta[sl];
            cm.tab = cur_tab;
            cm.br_dir = kase;
            if (cur_tab >= 0) {
                // the parent's record holds the arrays: the kernel builds the child
                pool.tabs->inc(cur_tab);
                cm.inl = false;
            } else {
                cm.inl = true;
                pool.need_arrays(sl);
                const FillJob fj{sl, j, kase, beta, bl, bu, so};
                if (defer) defer->push_back(fj);
                else fill_child(fj);
            }
            cm.level = mt.level + 1;
            cm.br_var = j;
            cm.br_val = beta;
            cm.up_lpobj = z;
            cm.up_bound = bound;
            cm.up_ii = ii;
            cm.lpz = z + dz[kase];
            NodeRec c{cb, 0.0, 0.0, seq++, sl};
            set_keys(c);
            if (!dived) {
                next_dive.push_back(c);
                dived = true;
            } else
                push_open(c);
            created++;
        }
    }

    // node_done split for the batch's workers: everything that does not
    // depend on the search state (the rounded local bound, the branching
    // column and direction from the kernel's candidates, the children's
    // rounded bounds) is planned in parallel; node_done_planned then takes
    // the decisions in entry order exactly as node_done does (the same
    // hopeful tests against the same incumbent, the same allocations and
    // queue pushes).  For a kernel-solved node whose children get records,
    // with any branching rule but pseudocosts
    struct Plan {
        double bound, beta, ii, dz[2], cb[2];
        int j, next, nfrac;
    };
    std::vector<Plan> plans;                  // per batch entry
    std::vector<char> planned;
    void plan_node(Plan &pl, const NodeRec &nd, double z, const double *x, const double *dzb, int kjj, int knext,
                   const KInt &ki) const
    {
        pl.bound = std::max(nd.bound, round_bound(z));
        pl.nfrac = ki.nfrac;
        pl.ii = ki.ii;
        if (pl.nfrac == 0) return;
        int j, next;
        switch (parm->br_tech) {
        case 1: j = ki.jf; next = next_of(x[m + j]); break;
        case 2: j = ki.jl; next = next_of(x[m + j]); break;
        case 3: j = ki.jm; next = ki.nm; break;
        default:
            if (kjj > 0) { j = kjj - 1; next = knext; }
            else { j = ki.jm; next = ki.nm; }
            break;
        }
        pl.j = j;
        pl.next = next;
        pl.beta = x[m + j];
        for (int kase = 0; kase < 2; kase++) {
            pl.dz[kase] = dzb[2 * j + kase];
            pl.cb[kase] = pl.dz[kase] == DBL_MAX ? DBL_MAX : std::max(pl.bound, round_bound(z + pl.dz[kase]));
        }
    }
    void node_done_planned(const NodeRec &nd, double z, const double *x, const Plan &pl)
    {
        const NodeMeta &mt0 = pool.meta[nd.slot];
        if (!hopeful(pl.bound)) return;
        if (pl.nfrac == 0) {
            if (!have || z < best) new_incumbent(z, x);
            return;
        }
        const int level = mt0.level;
        if (level == 0 && !root_seen) {
            root_seen = true;
            root_bound = pl.bound;
            root_ii = pl.ii;
        }
        const int first = pl.next < 0 ? 0 : 1;
        bool dived = false;
        for (int r = 0; r < 2; r++) {
            const int kase = (r == 0) ? first : 1 - first;
            if (pl.dz[kase] == DBL_MAX) continue;     // that branch has no feasible point
            if (!hopeful(pl.cb[kase])) continue;
            const int sl = pool.alloc();               // (may move pool.meta: mt0 is not used below)
            NodeMeta &cm = pool.meta[sl];
            cm.tab = cur_tab;
            cm.br_dir = kase;
            pool.tabs->inc(cur_tab);
            cm.inl = false;
            cm.level = level + 1;
            cm.br_var = pl.j;
            cm.br_val = pl.beta;
            cm.up_lpobj = z;
            cm.up_bound = pl.bound;
            cm.up_ii = pl.ii;
            cm.lpz = z + pl.dz[kase];
            NodeRec c{pl.cb[kase], 0.0, 0.0, seq++, sl};
            if (!dived) {
                set_keys(c);
                next_dive.push_back(c);
                dived = true;
            } else
                push_open(c);
            created++;
        }
    }

    // the result of one node LP (kernel or fallback): incumbent, pruning,
    // branching (ios_driver's "analyze" part, glpios03.js:670-905)
    // returns true when the node is parked (its pool slot stays in use)
    bool node_done(const NodeRec &nd, double z, const double *x, const signed char *so, const double *bl,
                   const double *bu, const double *dzb, int kjj, int knext, bool tableau, const int *pcand = nullptr,
                   int npcand = -1, double pii = 0.0, const KInt *ki = nullptr)
    {
        const NodeMeta mt = pool.meta[nd.slot];
        // ios_pcost_update (glpios09.js:288)
        if (pcost_on && mt.br_var >= 0) {
            const double dx = x[m + mt.br_var] - mt.br_val;
            if (dx != 0.0) {
                const double psi = std::fabs((z - mt.up_lpobj) / dx);
                if (dx < 0.0) { dn_cnt[mt.br_var]++; dn_sum[mt.br_var] += psi; }
                else { up_cnt[mt.br_var]++; up_sum[mt.br_var] += psi; }
            }
        }
        const double bound = std::max(nd.bound, round_bound(z));
        if (!hopeful(bound)) return false;
        std::vector<int> &cand = cand_buf;           // reused: no allocation per node
        double ii = 0.0;
        const unsigned long long ti0 = tsc_on ? tsc() : 0ull;
        int nfrac;
        if (ki) {                                    // scanned by the node kernel
            nfrac = ki->nfrac;
            ii = ki->ii;
        } else if (npcand >= 0) {                    // scanned by the batch's workers
            cand.assign(pcand, pcand + npcand);
            ii = pii;
            nfrac = npcand;
        } else
            nfrac = integrality(x, so, bl, bu, cand, ii);
        const unsigned long long ti1 = tsc_on ? tsc() : 0ull;
        if (tsc_on) tsc_int += ti1 - ti0;
        if (nfrac == 0) {
            if (!have || z < best) new_incumbent(z, x);
            return false;
        }
        if (mt.level == 0 && !root_seen) {
            root_seen = true;
            root_bound = bound;
            root_ii = ii;
        }
        int j = -1, next = 0;
        if (ki && parm->br_tech != 5) {
            // the kernel's candidates (the same rules as choose_simple)
            switch (parm->br_tech) {
            case 1: j = ki->jf; next = next_of(x[m + j]); break;
            case 2: j = ki->jl; next = next_of(x[m + j]); break;
            case 3: j = ki->jm; next = ki->nm; break;
            default:
                if (kjj > 0) { j = kjj - 1; next = knext; }
                else { j = ki->jm; next = ki->nm; }
                break;
            }
        } else switch (parm->br_tech) {
        case 1: case 2: case 3:
            j = choose_simple(parm->br_tech, cand, x, next);
            break;
        case 5:
            if (!tableau) { j = choose_simple(3, cand, x, next); break; }
            if (!pcost_on) {
                pcost_on = true;
                dn_cnt.assign(n, 0); up_cnt.assign(n, 0); dn_sum.assign(n, 0.0); up_sum.assign(n, 0.0);
            }
            {
                // probes for the pseudocosts still missing (eval_psi :397),
                // solved in the next batches; the node waits parked
                std::vector<std::pair<int, int>> need;
                for (int q : cand) {
                    if (dn_cnt[q] == 0) need.emplace_back(q, 0);
                    if (up_cnt[q] == 0) need.emplace_back(q, 1);
                }
                if (!need.empty()) {
                    int pid;
                    if (!parked_free.empty()) { pid = parked_free.back(); parked_free.pop_back(); }
                    else { pid = (int)parked.size(); parked.emplace_back(); }
                    Parked &pk = parked[pid];
                    pk.nd = nd; pk.meta = mt; pk.z = z; pk.bound = bound; pk.ii = ii;
                    pk.x.assign(x, x + N);
                    pk.so.assign(so, so + N);
                    pk.bnd.resize(2 * (size_t)n);
                    std::memcpy(pk.bnd.data(), bl, n * sizeof(double));
                    std::memcpy(pk.bnd.data() + n, bu, n * sizeof(double));
                    pk.dzb.assign(dzb, dzb + 2 * (size_t)n);
                    pk.probe.assign(2 * (size_t)n, 0.0);
                    pk.cand = cand;
                    pk.pending = (int)need.size();
                    pk.tab = cur_tab;
                    if (pool.tabs) pool.tabs->inc(cur_tab);
                    for (auto &pr : need) {
                        Entry e{};
                        e.kind = 1; e.nd = nd; e.pid = pid; e.j = pr.first; e.dir = pr.second;
                        probeq.push_back(e);
                    }
                    return true;                      // the slot stays alive while parked
                }
                j = choose_pcost(cand, x, nullptr, next);
            }
            break;
        default:                                      // DTH: the kernel's choice on the tableau
            if (kjj > 0 && std::find(cand.begin(), cand.end(), kjj - 1) != cand.end()) { j = kjj - 1; next = knext; }
            else j = choose_simple(3, cand, x, next);
            break;
        }
        const double dn = tableau ? dzb[2 * j] : 0.0, up = tableau ? dzb[2 * j + 1] : 0.0;
        const unsigned long long tb0 = tsc_on ? tsc() : 0ull;
        if (tsc_on) tsc_choose += tb0 - ti1;
        branch(nd, mt, z, bound, ii, x, so, bl, bu, j, next, dn, up);
        if (tsc_on) tsc_child += tsc() - tb0;
        return false;
    }

    // a record child's bounds and statuses into its pool slot (the
    // sharded exchange and the engine fallback read them on the host); its
    // record stays referenced for the warm start
    void materialize(int sl)
    {
        NodeMeta &mt = pool.meta[sl];
        if (mt.inl) return;
        const size_t bytes = 2 * (size_t)n * sizeof(double) + (size_t)N;
        std::vector<double> rec((bytes + 7) / 8);
        (void)hipMemcpy(rec.data(), pool.tabs->ptr(mt.tab) + node_rec_bounds(m, n), bytes, hipMemcpyDeviceToHost);
        std::vector<signed char> so(N);
        std::memcpy(so.data(), rec.data() + 2 * n, N);
        pool.need_arrays(sl);
        fill_child(FillJob{sl, mt.br_var, mt.br_dir, mt.br_val, rec.data(), rec.data() + n, so.data()});
        pool.meta[sl].inl = true;
    }

    void parked_done(int pid)
    {
        Parked &pk = parked[pid];
        int next = 0;
        const int j = choose_pcost(pk.cand, pk.x.data(), pk.probe.data(), next);
        const double *bl = pk.bnd.data(), *bu = pk.bnd.data() + n;
        const double dn = pk.dzb[2 * j], up = pk.dzb[2 * j + 1];
        cur_tab = pk.tab;
        branch(pk.nd, pk.meta, pk.z, pk.bound, pk.ii, pk.x.data(), pk.so.data(), bl, bu, j, next, dn, up);
        cur_tab = -1;
        if (pool.tabs) pool.tabs->dec(pk.tab);
        pk.tab = -1;
        parked_free.push_back(pid);
    }

    // ios_solve_node with the full engine (glp_simplex, meth = GLP_DUALP,
    // the incumbent as objective limit): a node LP the batched kernel could
    // not finish.  Returns 0 solved (OPT: *opt = true), 0 fathomed, or
    // GLP_EFAIL.
    int fallback(const NodeRec &nd, const double *bl, const double *bu, std::vector<double> &x,
                 std::vector<signed char> &so, double &z, bool &opt);
    // its solve on a given context / factor (no search state written: the
    // engine-mode workers run it concurrently, one node LP each); the
    // degradations into *D when given
    struct Degrad;
    int solve_node(gk_ctx *c, gk_bfd *f, unsigned long long ver, const NodeRec &nd, const double *bl,
                   const double *bu, std::vector<double> &x, std::vector<signed char> &so, double &z, bool &opt,
                   long long &piv, Degrad *D);
    // engine mode: what the node kernel returns besides the solution, from
    // the engine's factor of the node's optimal basis — the fractional
    // columns, ios_eval_degrad's degradations of every one of them
    // (glpios01.js:615, minimisation form, DBL_MAX: that branch is
    // infeasible) and branch_drtom's choice (glpios09.js:84; 0 when its
    // degradation is negligible: the host takes the most fractional)
    struct Degrad {
        std::vector<int> cand;
        double ii = 0.0;
        std::vector<double> dz;               // 2 n: down | up per column
        int kjj = 0, knext = 0;
        bool ok = false;
    } dg;
    void engine_degrad(gk_bfd *f, Degrad &D, gk_lp &L, const std::vector<double> &x,
                       const std::vector<signed char> &so, const double *bl, const double *bu) const;
};

int gk_spx_node(gk_ctx *ctx, gk_lp *lp, gk_bfd *bfd, const gk_smcp *parm);

static unsigned long long engine_a_version()
{
    static std::atomic<unsigned long long> ver{0};
    return (1ull << 62) | ++ver;                    // A uploaded once per factor and search
}

int MipSolver::fallback(const NodeRec &nd, const double *bl, const double *bu, std::vector<double> &x,
                        std::vector<signed char> &so, double &z, bool &opt)
{
    opt = false;
    fallbacks++;
    // GK_BNB_FRESH_FB=1 (diagnostics): a new factor handle for every node LP
    static const bool fresh = [] {
        const char *e = std::getenv("GK_BNB_FRESH_FB");
        return e && std::atoi(e) != 0;
    }();
    if (fresh && fb) {
        gk_bfd_destroy(fb);
        fb = nullptr;
    }
    if (!fb) {
        fb = gk_bfd_create(ctx);
        if (!fb) return 5;
        fb_version = engine_a_version();
    }
    materialize(nd.slot);
    long long piv = 0;
    const int ret = solve_node(ctx, fb, fb_version, nd, bl, bu, x, so, z, opt, piv, engine ? &dg : nullptr);
    pivots += piv;
    return ret;
}

int MipSolver::solve_node(gk_ctx *c, gk_bfd *f, unsigned long long ver, const NodeRec &nd, const double *bl,
                          const double *bu, std::vector<double> &x, std::vector<signed char> &so, double &z,
                          bool &opt, long long &piv, Degrad *D)
{
    const gk_lp &R = mip->lp;
    opt = false;
    piv = 0;
    std::vector<signed char> ctype(n + 1), rstat(m + 1), cstat(n + 1);
    std::vector<double> clo(n + 1, 0.0), cup(n + 1, 0.0);
    std::vector<int> head(m + 1), rbind(m + 1), cbind(n + 1);
    std::vector<double> rprim(m + 1), rdual(m + 1), cprim(n + 1), cdual(n + 1);
    for (int j = 0; j < n; j++) {
        const double l = bl[j], u = bu[j];
        ctype[j + 1] = (l == -DBL_MAX && u == DBL_MAX) ? 1 : (u == DBL_MAX ? 2 : (l == -DBL_MAX ? 3 : (l != u ? 4 : 5)));
        clo[j + 1] = l == -DBL_MAX ? 0.0 : l;
        cup[j + 1] = u == DBL_MAX ? 0.0 : u;
    }
    gk_smcp sp{};
    sp.msg_lev = 1; sp.meth = 2; sp.pricing = 0x22; sp.r_test = 0x22;     // GLP_MSG_ERR, GLP_DUALP, PSE, Harris
    sp.tol_bnd = 1e-7; sp.tol_dj = 1e-7; sp.tol_piv = 1e-10;
    sp.obj_ll = -DBL_MAX; sp.obj_ul = DBL_MAX;
    if (bestall() != DBL_MAX) {
        const double mo = c0 + sign * bestall();
        if (sign > 0) sp.obj_ul = mo; else sp.obj_ll = mo;
    }
    sp.it_lim = 0x7fffffff; sp.tm_lim = 0x7fffffff; sp.out_frq = 500; sp.out_dly = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        const signed char *st0 = pool.stat(nd.slot);
        for (int i = 0; i < m; i++) rstat[i + 1] = attempt == 0 ? st0[i] : (signed char)BS;
        for (int j = 0; j < n; j++) {
            signed char v = attempt == 0 ? st0[m + j] : (signed char)NL;
            if (v != BS) {                            // statuses consistent with the node's column types
                const int t = ctype[j + 1];
                if (t == 5) v = NS;
                else if (t == 1) v = NF;
                else if (t == 2) v = NL;
                else if (t == 3) v = NU;
                else if (v != NL && v != NU) v = NL;
            }
            cstat[j + 1] = v;
        }
        int k = 0;
        for (int i = 1; i <= m; i++) if (rstat[i] == BS && k < m) head[++k] = i;
        for (int j = 1; j <= n; j++) if (cstat[j] == BS && k < m) head[++k] = m + j;
        if (k != m) continue;
        gk_lp L{};
        L.m = m; L.n = n; L.nnz = R.nnz; L.dir = R.dir; L.c0 = R.c0;
        L.row_type = R.row_type; L.row_lb = R.row_lb; L.row_ub = R.row_ub; L.rii = R.rii;
        L.col_type = ctype.data(); L.col_lb = clo.data(); L.col_ub = cup.data(); L.col_coef = R.col_coef; L.sjj = R.sjj;
        L.A_ptr = R.A_ptr; L.A_ind = R.A_ind; L.A_val = R.A_val; L.a_version = ver;
        L.head = head.data(); L.row_stat = rstat.data(); L.col_stat = cstat.data();
        L.row_bind = rbind.data(); L.col_bind = cbind.data();
        L.row_prim = rprim.data(); L.row_dual = rdual.data(); L.col_prim = cprim.data(); L.col_dual = cdual.data();
        const int ret = gk_spx_node(c, &L, f, &sp);
        if (ret == 6 || ret == 7) return 0;           // GLP_EOBJLL / EOBJUL: no better than the incumbent
        if (ret != 0) continue;
        if (L.dbs_stat != 2) break;                   // no dual feasible solution: the reference fails here
        if (L.pbs_stat != 2) return 0;                // infeasible, or no better than the incumbent
        x.assign(N, 0.0);
        so.assign(N, 0);
        for (int i = 0; i < m; i++) { x[i] = rprim[i + 1]; so[i] = rstat[i + 1]; }
        for (int j = 0; j < n; j++) { x[m + j] = cprim[j + 1]; so[m + j] = cstat[j + 1]; }
        z = sign * (L.obj_val - c0);
        piv = L.it_cnt;
        opt = true;
        if (D) engine_degrad(f, *D, L, x, so, bl, bu);
        return 0;
    }
    return 5;                                         // GLP_EFAIL (ios_driver, glpios03.js:669-673)
}

void MipSolver::engine_degrad(gk_bfd *f, Degrad &D, gk_lp &L, const std::vector<double> &x,
                              const std::vector<signed char> &so, const double *bl, const double *bu) const
{
    D.ok = false;
    D.kjj = 0;
    D.knext = 0;
    (void)integrality(x.data(), so.data(), bl, bu, D.cand, D.ii);
    D.dz.assign(2 * (size_t)n, 0.0);
    const int nk = (int)D.cand.size();
    if (nk == 0) { D.ok = true; return; }
    // the tableau rows of the fractional basic columns (glp_eval_tab_row),
    // one pass on the engine's factor of this node's final basis
    std::vector<int> kk(nk);
    for (int t = 0; t < nk; t++) kk[t] = m + D.cand[t] + 1;
    const int N1 = m + n;
    std::vector<double> alfa((size_t)nk * N1);
    if (gk_bfd_eval_tab_rows(f, &L, nk, kk.data(), alfa.data(), 0) != 0) return;
    const double obj = (L.dir == 1) ? +1.0 : -1.0;   // GLP_MIN = 1
    auto stat_of = [&](int k) { return k <= m ? L.row_stat[k] : L.col_stat[k - m]; };
    auto dual_of = [&](int k) { return k <= m ? L.row_dual[k] : L.col_dual[k - m]; };
    // glp_dual_rtest (glpapi12.js:687) over the row's non-zeros in variable order
    auto rtest = [&](const double *row, int dir, double &alfa_k) {
        int piv = 0;
        double teta = DBL_MAX, big = 0.0;
        for (int k = 1; k <= N1; k++) {
            const double v = row[k - 1];
            if (v == 0.0) continue;
            const int st = stat_of(k);
            if (st == BS) continue;
            const double a = dir > 0 ? v : -v, cost = dual_of(k);
            double temp;
            if (st == NL) { if (a < 1e-9) continue; temp = (obj * cost) / a; }
            else if (st == NU) { if (a > -1e-9) continue; temp = (obj * cost) / a; }
            else if (st == NF) { if (-1e-9 < a && a < 1e-9) continue; temp = 0.0; }
            else continue;                                    // NS
            if (temp < 0.0) temp = 0.0;
            if (teta > temp || (teta == temp && big < std::fabs(a))) {
                piv = k;
                teta = temp;
                big = std::fabs(a);
                alfa_k = v;
            }
        }
        return piv;
    };
    // the reduced cost of x[k] with the sign correction of a degenerate basis
    auto dk_of = [&](int k) {
        const int st = stat_of(k);
        double d = dual_of(k);
        if (obj > 0) { if ((st == NL && d < 0.0) || (st == NU && d > 0.0) || st == NF) d = 0.0; }
        else if ((st == NL && d > 0.0) || (st == NU && d < 0.0) || st == NF) d = 0.0;
        return d;
    };
    int jj = -1, next = 0;
    double degrad = -1.0;
    const double objv = L.obj_val;
    for (int t = 0; t < nk; t++) {
        const int j = D.cand[t];
        const double *row = alfa.data() + (size_t)t * N1;
        const double beta = x[m + j];
        double dz_e[2], dz_t[2];                               // eval_degrad / branch_drtom (Tomlin)
        for (int c = 0; c < 2; c++) {
            const int kase = c == 0 ? -1 : +1;
            double a = 0.0;
            const int k = rtest(row, kase, a);
            if (k == 0) {
                dz_e[c] = dz_t[c] = obj * DBL_MAX;
                continue;
            }
            const double dj = (kase < 0 ? std::floor(beta) : std::ceil(beta)) - beta;
            const double g = dk_of(k);
            dz_e[c] = g * (dj / a);
            double dkk = dj / a;
            if (k > m && mip->col_kind[k - m] != 1) {       // Tomlin: an integer x[k] moves by at least one
                if (std::fabs(dkk - std::floor(dkk + 0.5)) > 1e-3) dkk = dkk > 0.0 ? std::ceil(dkk) : std::floor(dkk);
            }
            dz_t[c] = g * dkk;
        }
        // minimisation-form degradations of the two branches (the bounds)
        for (int c = 0; c < 2; c++)
            D.dz[2 * (size_t)j + c] = (std::fabs(dz_e[c]) == DBL_MAX) ? DBL_MAX : std::max(0.0, obj * dz_e[c]);
        if (degrad < std::fabs(dz_t[0]) || degrad < std::fabs(dz_t[1])) {
            jj = j;
            if (std::fabs(dz_t[0]) < std::fabs(dz_t[1])) { next = -1; degrad = std::fabs(dz_t[1]); }
            else { next = +1; degrad = std::fabs(dz_t[0]); }
            if (degrad == DBL_MAX) break;
        }
    }
    if (jj >= 0 && !(degrad < 1e-6 * (1.0 + 0.001 * std::fabs(objv)))) {
        D.kjj = jj + 1;
        D.knext = next;
    }
    D.ok = true;
}

static void setup_rounding(MipSolver &S, const gk_mip *mip)
{
    // ios_round_bound: all objective coefficients of non-fixed columns
    // integral and on integer columns; s = c0 + sum over fixed columns
    const gk_lp &L = mip->lp;
    double s = L.c0;
    std::vector<long long> cs;
    for (int j = 1; j <= S.n; j++) {
        const double cj = L.col_coef[j];
        if (cj == 0.0) continue;
        if (L.col_type[j] == 5) {                       // GLP_FX
            s += cj * L.col_lb[j];
            continue;
        }
        if (mip->col_kind[j] != 2 || cj != std::floor(cj) || std::fabs(cj) > 2147483647.0) return;
        cs.push_back((long long)std::fabs(cj));
    }
    if (cs.empty()) return;
    long long g = 0;
    for (long long v : cs) {
        long long a = g, b = v;
        while (b) { long long t = a % b; a = b; b = t; }
        g = a;
    }
    if (g <= 0) return;
    S.round_ok = true;
    S.round_s = s;
    S.round_d = (double)g;
}

// ---------------------------------------------------------------------------
// open-node exchange between ranks: at every sync epoch
// the ranks all-gather {incumbent, best open bound, open nodes, active};
// every rank derives the same plan from it — idle ranks paired with the
// ranks holding the most open nodes, each donor handing over up to half of
// its queue (at most XFER_MAX nodes, best first) — and the node descriptors
// (bounds, warm-start basis, parent information) travel in one more
// all-gather of fixed-size blocks.
// ---------------------------------------------------------------------------
struct ShardMsg {
    double best, bound;
    long long open;
    int active, err;          // err: this rank's search failed (every rank then stops at this epoch)
};
constexpr int XFER_MAX = 32;

static size_t desc_bytes(int n, int N)
{
    return (((size_t)6 * 8 + 2 * 4 + 16 * (size_t)n + (size_t)N) + 7) & ~(size_t)7;
}

static void put_desc(MipSolver &S, const NodeRec &r, char *p)
{
    S.materialize(r.slot);
    const NodeMeta &mt = S.pool.meta[r.slot];
    double *d = (double *)p;
    d[0] = r.bound; d[1] = mt.br_val; d[2] = mt.up_lpobj; d[3] = mt.up_bound; d[4] = mt.up_ii; d[5] = 0.0;
    int *iv = (int *)(d + 6);
    iv[0] = mt.level; iv[1] = mt.br_var;
    double *bl = (double *)(iv + 2);
    std::memcpy(bl, S.pool.lb(r.slot), S.n * sizeof(double));
    std::memcpy(bl + S.n, S.pool.ub(r.slot), S.n * sizeof(double));
    std::memcpy((char *)(bl + 2 * S.n), S.pool.stat(r.slot), S.N);
}

static void get_desc(MipSolver &S, const char *p)
{
    const double *d = (const double *)p;
    const int sl = S.pool.alloc();
    S.pool.need_arrays(sl);
    NodeMeta &mt = S.pool.meta[sl];
    mt.tab = -1;                          // the sender's tableau stays on its GPU
    mt.br_val = d[1]; mt.up_lpobj = d[2]; mt.up_bound = d[3]; mt.up_ii = d[4];
    const int *iv = (const int *)(d + 6);
    mt.level = iv[0]; mt.br_var = iv[1];
    const double *bl = (const double *)(iv + 2);
    std::memcpy(S.pool.lb(sl), bl, S.n * sizeof(double));
    std::memcpy(S.pool.ub(sl), bl + S.n, S.n * sizeof(double));
    std::memcpy(S.pool.stat(sl), (const char *)(bl + 2 * S.n), S.N);
    S.push_open(NodeRec{d[0], 0.0, 0.0, S.seq++, sl});
}

// one sync epoch; returns the number of ranks with work (0 ends the run) or
// -1 when a collective failed.  Every stop decision is taken from the
// gathered blocks, which are the same on every rank, so all ranks leave the
// loop at the same epoch and meet again in gk_ios_driver_comm's final
// all-gather: a rank whose search failed (local_err) ends the epoch for all
// (peer_err on the others), and the relative mip gap (glpios03.js:613-620)
// is tested on the global incumbent against the global best open bound —
// only while some rank still holds open nodes (the reference tests it for a
// selected subproblem, never on an empty tree, glpios03.js:522-528)
static int shard_epoch(MipSolver &S, const gk_ios_shard *sh, bool have_work, long long &moved, bool local_err,
                       double mip_gap, bool &gap_stop, bool &peer_err)
{
    const int size = sh->size, rank = sh->rank;
    ShardMsg me{};
    me.best = S.best;
    me.bound = DBL_MAX;
    for (const NodeRec &r : S.open) me.bound = std::min(me.bound, r.bound);
    for (const NodeRec &r : S.dive) me.bound = std::min(me.bound, r.bound);
    me.open = (long long)(S.open.size() + S.dive.size());
    me.active = (have_work && !local_err) ? 1 : 0;
    me.err = local_err ? 1 : 0;
    std::vector<ShardMsg> all(size);
    if (sh->allgather(sh->info, &me, sizeof me, all.data()) != 0) return -1;
    int nact = 0, nerr = 0;
    long long nopen = 0;
    double gb = DBL_MAX, gbound = DBL_MAX;
    for (const ShardMsg &x : all) {
        nact += x.active;
        nerr += x.err;
        nopen += x.open;
        gb = std::min(gb, x.best);
        if (x.open > 0) gbound = std::min(gbound, x.bound);
    }
    S.set_gbest(gb);
    if (nerr > 0) {
        peer_err = !local_err;
        return 0;
    }
    if (mip_gap > 0.0 && gb < DBL_MAX && nopen > 0) {
        const double bm = S.c0 + S.sign * gb, bb = S.c0 + S.sign * gbound;
        if (std::fabs(bm - bb) / (std::fabs(bm) + DBL_EPSILON) <= mip_gap) {
            gap_stop = true;
            return 0;
        }
    }
    if (nact == 0) return 0;
    // the plan (identical on every rank)
    std::vector<int> idle, donors;
    for (int r = 0; r < size; r++) {
        if (!all[r].active && all[r].open == 0) idle.push_back(r);
        else if (all[r].open >= 2) donors.push_back(r);
    }
    std::stable_sort(donors.begin(), donors.end(), [&](int a, int b) { return all[a].open > all[b].open; });
    const int pairs = (int)std::min(idle.size(), donors.size());
    if (pairs == 0) return nact;
    const size_t db = desc_bytes(S.n, S.N), blk = 16 + XFER_MAX * db;
    std::vector<char> send(blk, 0), recv(blk * size);
    int *hdr = (int *)send.data();
    hdr[0] = 0; hdr[1] = -1;
    for (int k = 0; k < pairs; k++) {
        if (donors[k] != rank) continue;
        const int give = (int)std::min<long long>(XFER_MAX, all[rank].open / 2);
        hdr[1] = idle[k];
        for (int g = 0; g < give && !S.open.empty(); g++) {
            const NodeRec r = S.pop_open();
            put_desc(S, r, send.data() + 16 + g * db);
            S.pool.release(r.slot);
            hdr[0]++;
        }
    }
    if (sh->allgather(sh->info, send.data(), blk, recv.data()) != 0) return -1;
    for (int r = 0; r < size; r++) {
        const int *h = (const int *)(recv.data() + r * blk);
        if (h[1] != rank) continue;
        for (int g = 0; g < h[0]; g++) get_desc(S, recv.data() + r * blk + 16 + g * db);
        moved += h[0];
    }
    return nact + pairs;                  // receivers have work now
}

}  // namespace gk

using namespace gk;

int gk_ctx_device(gk_ctx *);
hipStream_t gk_ctx_stream(gk_ctx *);
void gk_ctx_ios_report(gk_ctx *c, gk_report_fn *fn, void **ud);

extern "C" int gk_ios_driver(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm)
{
    return gk_ios_driver_sharded(ctx, mip, parm, nullptr);
}

extern "C" int gk_ios_driver_sharded_inc(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, const gk_ios_shard *shard,
                                         double (*inc)(void *info, double mine), void *inc_info);

extern "C" int gk_ios_driver_sharded(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, const gk_ios_shard *shard)
{
    return gk_ios_driver_sharded_inc(ctx, mip, parm, shard, nullptr, nullptr);
}

// inc (optional): publishes this rank's incumbent (internal minimisation
// form, DBL_MAX: none) and returns the best over the ranks; called before
// every batch of the split search (gk_comm's shared word)
extern "C" int gk_ios_driver_sharded_inc(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, const gk_ios_shard *shard,
                                         double (*inc)(void *info, double mine), void *inc_info)
{
    if (!ctx || !mip || !parm) { set_err("gk_ios_driver: null argument"); return GK_EABI; }
    const int rank = shard ? shard->rank : 0, size = shard ? shard->size : 1;
    if (size < 1 || rank < 0 || rank >= size || (size > 1 && !shard->exchange && !shard->allgather)) {
        set_err("gk_ios_driver: invalid shard %d of %d", rank, size);
        return GK_EABI;
    }
    // glp_intopt's parameter checks (glpapi09.js:240-262)
    if (parm->br_tech < 1 || parm->br_tech > 5) { set_err("glp_intopt: br_tech = %d; invalid parameter", parm->br_tech); return GK_EABI; }
    if (parm->bt_tech < 1 || parm->bt_tech > 4) { set_err("glp_intopt: bt_tech = %d; invalid parameter", parm->bt_tech); return GK_EABI; }
    if (parm->pp_tech < 0 || parm->pp_tech > 2) { set_err("glp_intopt: pp_tech = %d; invalid parameter", parm->pp_tech); return GK_EABI; }
    // ramp_nodes < 0: split the root alone (rank 0 starts with all the work;
    // exercises the open-node exchange)
    const int ramp = (shard && shard->ramp_nodes < 0) ? 0 : ((shard && shard->ramp_nodes > 0) ? shard->ramp_nodes : 8);
    const int sync_every = (shard && shard->sync_every > 0) ? shard->sync_every : 4;
    const gk_lp &L = mip->lp;
    const int m = L.m, n = L.n;
    if (m < 1 || n < 1) { set_err("gk_ios_driver: m = %d, n = %d; invalid dimensions", m, n); return GK_EABI; }
    if (L.pbs_stat != 2 || L.dbs_stat != 2) {
        set_err("gk_ios_driver: optimal basis to initial LP relaxation not provided");
        return GK_EABI;
    }
    // node LPs up to 64 KiB keep their tableau in LDS; larger ones work in a
    // per-node slice of HBM, batches sized to at most 8 GiB of work area.
    // Past engine_node_bytes() of work area per node (the dense tableau
    // T = inv(B)[I | -A] streamed by one workgroup per pivot no longer pays)
    // every node LP is solved by the engine instead — ios_solve_node's
    // glp_simplex (glpios01.js:866) on the revised simplex with its factor
    // (the explicit inverse or the sparse LU), warm-started from the parent's
    // final basis (MipSolver::fallback); the node kernel is not launched
    const size_t lds = node_lp_lds(m, n);
    const size_t SCRATCH_MAX = (size_t)8 << 30;
    const bool eng = lds > engine_node_bytes();
    if (hipSetDevice(gk_ctx_device(ctx)) != hipSuccess) { set_err("gk_ios_driver: hipSetDevice failed"); return GK_EABI; }
    hipStream_t s = gk_ctx_stream(ctx);
    const auto t0 = std::chrono::steady_clock::now();
    HostProf host_prof_;                                  // GK_HOST_PROF (diagnostics)
    MipSolver S;
    S.ctx = ctx; S.s = s; S.mip = mip; S.parm = parm;
    S.m = m; S.n = n; S.N = m + n;
    S.sign = (L.dir == 1) ? 1.0 : -1.0;                   // GLP_MIN = 1
    S.c0 = L.c0;
    S.xbest.assign(S.N, 0.0);
    if (const char *e = std::getenv("GK_TEST_NODE_IT_LIM")) {   // test knob: force node LPs onto the fallback
        const int v = std::atoi(e);
        if (v >= 0) S.node_it_lim = v;
    }
    const double INF = DBL_MAX;
    S.rlb.resize(m); S.rub.resize(m); S.clb.resize(n); S.cub.resize(n);
    auto bnds = [&](int type, double lb, double ub, double &l, double &u) {
        switch (type) {
        case 1: l = -INF; u = +INF; break;               // FR
        case 2: l = lb; u = +INF; break;                 // LO
        case 3: l = -INF; u = ub; break;                 // UP
        case 4: l = lb; u = ub; break;                   // DB
        default: l = lb; u = lb; break;                  // FX
        }
    };
    for (int i = 0; i < m; i++) bnds(L.row_type[i + 1], L.row_lb[i + 1], L.row_ub[i + 1], S.rlb[i], S.rub[i]);
    for (int j = 0; j < n; j++) bnds(L.col_type[j + 1], L.col_lb[j + 1], L.col_ub[j + 1], S.clb[j], S.cub[j]);
    S.engine = eng;
    // (engine mode: no dense copy of A — the engine reads the CSC arrays)
    S.A.assign(eng ? 0 : (size_t)m * n, 0.0);
    for (int j = 1; j <= n; j++)
        for (int t = L.A_ptr[j]; t < L.A_ptr[j + 1]; t++) {
            const int i = L.A_ind[t];
            if (i < 1 || i > m) { set_err("gk_ios_driver: A_ind[%d] = %d; out of range", t, i); return GK_EABI; }
            if (!eng) S.A[(size_t)(j - 1) * m + (i - 1)] += L.A_val[t];
        }
    S.c.assign(S.N, 0.0);
    S.isint.assign(n, 0);
    for (int j = 0; j < n; j++) {
        S.c[m + j] = S.sign * L.col_coef[j + 1];
        S.isint[j] = (mip->col_kind[j + 1] == 2) ? 1 : 0;
    }
    setup_rounding(S, mip);
    // device problem
    {
        void (*freer)(void *) = nullptr;
        void **slot = gk_ctx_mip_cache(ctx, &freer);
        if (!*slot) *slot = new MipCache;
        (void)freer;
        S.cache = (MipCache *)*slot;
        S.bufs = S.cache->bufs;
        if (!S.cache->workers && bnb_threads() > 0) S.cache->workers = new HostWorkers(bnb_threads());
        // the previous search may have left events in use: nothing of it is in flight
    }
    MipCache &Cc = *S.cache;
    Cc.dA.ensure(S.A.size()); Cc.dc.ensure(S.N); Cc.dint.ensure(n); Cc.drb.ensure(2 * (size_t)m);
    // (engine mode: the batch is the order the node LPs are solved in, one
    // after another; engine_batch() of them keeps the search order of the
    // batched search's narrow batches)
    const int BMAX = eng ? engine_batch()
                         : (lds <= NODE_LDS_MAX ? 1024
                                                : (int)std::max<size_t>(1, std::min<size_t>(1024, SCRATCH_MAX / lds)));
    S.stride = (lds + 255) / 256 * 32;                    // doubles, 256-byte aligned slices
    if (lds > NODE_LDS_MAX && !eng) {
        Cc.dscratch.ensure(S.stride * BMAX);
        if (!Cc.dscratch.p) { set_err("gk_ios_driver: out of memory (node work area)"); return GK_EABI; }
    }
    if (!S.alloc_batch(BMAX) || !Cc.dA.p || !Cc.dc.p || !Cc.dint.p || !Cc.drb.p) {
        set_err("gk_ios_driver: out of memory");
        return GK_EABI;
    }
    (void)hipMemcpyAsync(Cc.dA.p, S.A.data(), S.A.size() * sizeof(double), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(Cc.dc.p, S.c.data(), S.N * sizeof(double), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(Cc.dint.p, S.isint.data(), n, hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(Cc.drb.p, S.rlb.data(), m * sizeof(double), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(Cc.drb.p + m, S.rub.data(), m * sizeof(double), hipMemcpyHostToDevice, s);
    NodeProb &P = S.P;
    P.m = m; P.n = n; P.ld = S.N; P.A = Cc.dA.p; P.c = Cc.dc.p; P.isint = Cc.dint.p; P.tol_int = parm->tol_int;
    P.rlb = Cc.drb.p; P.rub = Cc.drb.p + m;
    // a sparse A by rows and by columns for the node preprocessing
    P.nnz = 0;
    P.rptr = P.rind = P.cptr = P.cind = nullptr;
    P.rval = P.cval = nullptr;
    if (!eng) {
        size_t nz = 0;
        for (double v : S.A) nz += v != 0.0;
        if (nz > 0 && 2 * nz <= (size_t)m * n) {
            std::vector<int> rptr(m + 1, 0), cptr(n + 1, 0), rind(nz), cind(nz);
            std::vector<double> rval(nz), cval(nz);
            for (int j = 0; j < n; j++)
                for (int i = 0; i < m; i++)
                    if (S.A[(size_t)j * m + i] != 0.0) { rptr[i + 1]++; cptr[j + 1]++; }
            for (int i = 0; i < m; i++) rptr[i + 1] += rptr[i];
            for (int j = 0; j < n; j++) cptr[j + 1] += cptr[j];
            std::vector<int> rfill(rptr.begin(), rptr.end() - 1);
            size_t t = 0;
            for (int j = 0; j < n; j++)
                for (int i = 0; i < m; i++) {
                    const double v = S.A[(size_t)j * m + i];
                    if (v == 0.0) continue;
                    cind[t] = i; cval[t] = v; t++;
                    rind[rfill[i]] = j; rval[rfill[i]] = v; rfill[i]++;
                }
            Cc.dspi.ensure((size_t)m + n + 2 + 2 * nz);
            Cc.dspv.ensure(2 * nz);
            if (Cc.dspi.p && Cc.dspv.p) {
                int *pi = Cc.dspi.p;
                double *pv = Cc.dspv.p;
                // one copy each way, ordered on the search's stream before its first batch
                Cc.hspi.assign(rptr.begin(), rptr.end());
                Cc.hspi.insert(Cc.hspi.end(), cptr.begin(), cptr.end());
                Cc.hspi.insert(Cc.hspi.end(), rind.begin(), rind.end());
                Cc.hspi.insert(Cc.hspi.end(), cind.begin(), cind.end());
                Cc.hspv.assign(rval.begin(), rval.end());
                Cc.hspv.insert(Cc.hspv.end(), cval.begin(), cval.end());
                (void)hipMemcpyAsync(pi, Cc.hspi.data(), Cc.hspi.size() * sizeof(int), hipMemcpyHostToDevice, s);
                (void)hipMemcpyAsync(pv, Cc.hspv.data(), Cc.hspv.size() * sizeof(double), hipMemcpyHostToDevice, s);
                P.nnz = (int)nz;
                P.rptr = pi; P.cptr = pi + m + 1; P.rind = pi + m + n + 2; P.cind = pi + m + n + 2 + nz;
                P.rval = pv; P.cval = pv + nz;
            }
        }
    }
    P.dth = (parm->br_tech == 4) ? 1 : 0;
    NodePool &pool = S.pool;
    // the node storage of the previous search on this context (capacity kept)
    std::swap(S.pool, Cc.pool);
    struct PoolBack {
        NodePool &a, &b;
        ~PoolBack() { std::swap(a, b); }
    } pool_back{S.pool, Cc.pool};
    pool.reset(n, S.N);
    // warm start store (GK_BNB_WARM=0: every node inverts its basis;
    // GK_BNB_TAB_MB: its size limit)
    const size_t tab_cap = eng ? (size_t)0 : [] {
        const char *w = std::getenv("GK_BNB_WARM");
        if (w && std::atoi(w) == 0) return (size_t)0;
        const char *e = std::getenv("GK_BNB_TAB_MB");
        return (size_t)(e ? std::max(0, std::atoi(e)) : 8192) << 20;
    }();
    Cc.tabs.reset(node_rec_doubles(m, n), tab_cap);
    pool.tabs = &Cc.tabs;
    // root node: the optimal basis of the initial LP relaxation
    {
        const int sl = pool.alloc();
        pool.need_arrays(sl);
        std::memcpy(pool.lb(sl), S.clb.data(), n * sizeof(double));
        std::memcpy(pool.ub(sl), S.cub.data(), n * sizeof(double));
        signed char *st = pool.stat(sl);
        for (int i = 0; i < m; i++) st[i] = L.row_stat[i + 1];
        for (int j = 0; j < n; j++) st[m + j] = L.col_stat[j + 1];
        S.push_open(NodeRec{-INF, 0.0, 0.0, S.seq++, sl});
    }
    // ios_preprocess_node passes of a node (glpios03.js:643-656)
    auto pp_passes = [&](int level) {
        if (parm->pp_tech == 2) return level == 0 ? 100 : 10;
        if (parm->pp_tech == 1) return level == 0 ? 100 : 0;
        return 0;
    };
    // single GPU: two batches in flight — the host assembles and launches
    // batch k + 1 before it processes the results of batch k (more
    // speculative nodes, the GPU never waits for the host)
    static const int depth_env = [] {
        const char *e = std::getenv("GK_BNB_DEPTH");           // (experiments) batches in flight, 1 or 2
        return e ? std::atoi(e) : 2;
    }();
    const int depth = (size == 1 && !eng) ? (depth_env == 1 ? 1 : 2) : 1;
    int inflight[2] = {0, 0}, cur = 0;
    bool fail_sync = false;
    long long moved = 0;
    // GK_BNB_LOG=1: where the search's wall time goes (stderr)
    static const int bnb_lvl = [] {
        const char *e = std::getenv("GK_BNB_LOG");
        return e ? std::max(1, std::atoi(e)) : 0;
    }();
    static const bool bnb_log = bnb_lvl > 0;
    // GK_BNB_LOG=2: device time of the node kernel's phases (sums over the
    // entries that reach the end, in device clock ticks) and batch spans
    double ph_sum[7] = {0, 0, 0, 0, 0, 0, 0}, span_sum = 0.0;
    long long ph_cnt = 0, pp_cnt = 0;
    std::vector<unsigned long long> hst;
    S.tsc_on = bnb_log;
    const unsigned long long tsc_beg = bnb_log ? MipSolver::tsc() : 0ull;
    double t_launch = 0.0, t_wait = 0.0, t_proc = 0.0, t_nd = 0.0;
    long long n_batches = 0, n_ents = 0;
    auto secs = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    };
    auto launch = [&](BatchBuf &bf) {
        const auto tl0 = std::chrono::steady_clock::now();
        n_batches++;
        n_ents += (long long)bf.ents.size();
        const int nb = (int)bf.ents.size();
        bf.nb = nb;
        if (eng) return;                                  // (engine mode: solved in process)
        const double ball = S.bestall();
        const double cut = ball < INF ? ball - parm->tol_obj * (1.0 + std::fabs(S.c0 + S.sign * ball)) : INF;
        const Layout Y(S.N, n, nb);
        char *h = bf.hin.p;
        double *hl = (double *)(h + Y.lb), *hu = (double *)(h + Y.ub), *hc = (double *)(h + Y.cut);
        int *hit = (int *)(h + Y.itl), *hpp = (int *)(h + Y.pp);
        signed char *hs = (signed char *)(h + Y.st);
        const double **htin = (const double **)(h + Y.tin);
        double **htout = (double **)(h + Y.tout);
        int *hbj = (int *)(h + Y.brj), *hbd = (int *)(h + Y.brd);
        double *hbv = (double *)(h + Y.brv);
        for (int b = 0; b < nb; b++) {
            Entry &e = bf.ents[b];
            double *l = hl + (size_t)b * S.N, *u = hu + (size_t)b * S.N;
            hbj[b] = -1;
            hbd[b] = 0;
            hbv[b] = 0.0;
            if (e.kind == 0) {
                const int sl = e.nd.slot;
                const NodeMeta &mt = pool.meta[sl];
                htin[b] = Cc.tabs.ptr(mt.tab);
                e.tab_out = tab_cap ? Cc.tabs.alloc() : -1;
                htout[b] = Cc.tabs.ptr(e.tab_out);
                if (!mt.inl) {
                    // the kernel builds the node from its parent's record
                    hbj[b] = mt.br_var;
                    hbd[b] = mt.br_dir;
                    hbv[b] = mt.br_val;
                } else {
                    std::memcpy(l, S.rlb.data(), m * sizeof(double));
                    std::memcpy(u, S.rub.data(), m * sizeof(double));
                    std::memcpy(l + m, pool.lb(sl), n * sizeof(double));
                    std::memcpy(u + m, pool.ub(sl), n * sizeof(double));
                    std::memcpy(hs + (size_t)b * S.N, pool.stat(sl), S.N);
                }
                hc[b] = cut;
                hit[b] = S.node_it_lim;
                hpp[b] = pp_passes(mt.level);
            } else {
                // eval_degrad (glpios09.js:337): x_j fixed at floor / ceil,
                // 30 dual pivots from the node's optimal basis
                const Parked &pk = S.parked[e.pid];
                std::memcpy(l, S.rlb.data(), m * sizeof(double));
                std::memcpy(u, S.rub.data(), m * sizeof(double));
                std::memcpy(l + m, pk.bnd.data(), n * sizeof(double));
                std::memcpy(u + m, pk.bnd.data() + n, n * sizeof(double));
                const double beta = pk.x[m + e.j], v = e.dir == 0 ? std::floor(beta) : std::ceil(beta);
                l[m + e.j] = u[m + e.j] = v;
                std::memcpy(hs + (size_t)b * S.N, pk.so.data(), S.N);
                htin[b] = Cc.tabs.ptr(pk.tab);
                htout[b] = nullptr;
                hc[b] = INF;
                hit[b] = 30;
                hpp[b] = 0;
            }
        }
        (void)hipMemcpyAsync(bf.din.p, bf.hin.p, Y.in_end, hipMemcpyHostToDevice, s);
        char *din = bf.din.p, *dout = bf.dout.p;
        NodeIO io;
        io.lb = (const double *)(din + Y.lb); io.ub = (const double *)(din + Y.ub);
        io.cutoff = (const double *)(din + Y.cut); io.it_lim = (const int *)(din + Y.itl);
        io.pp_pass = (const int *)(din + Y.pp); io.stat_in = (const signed char *)(din + Y.st);
        io.obj_bound = ball;
        io.obj = (double *)(dout + Y.obj); io.dzb = (double *)(dout + Y.dz); io.x = (double *)(dout + Y.x);
        io.bnd = (double *)(dout + Y.bnd); io.status = (int *)(dout + Y.stat); io.pivots = (int *)(dout + Y.piv);
        io.jj = (int *)(dout + Y.jj); io.next = (int *)(dout + Y.next); io.stat_out = (signed char *)(dout + Y.sto);
        io.scratch = Cc.dscratch.p;
        io.scratch_stride = S.stride;
        io.tab_in = (const double *const *)(din + Y.tin);
        io.tab_out = (double *const *)(din + Y.tout);
        io.tab_age_max = 100;
        io.br_j = (const int *)(din + Y.brj); io.br_dir = (const int *)(din + Y.brd);
        io.br_val = (const double *)(din + Y.brv);
        io.stamps = nullptr;
        if (bnb_lvl >= 2) {
            bf.dstamp.ensure((size_t)S.BMAX * 8);
            (void)hipMemsetAsync(bf.dstamp.p, 0, (size_t)nb * 8 * sizeof(unsigned long long), s);
            io.stamps = bf.dstamp.p;
        }
        io.nfrac = (int *)(dout + Y.nf); io.jfirst = (int *)(dout + Y.jf); io.jlast = (int *)(dout + Y.jl);
        io.jmost = (int *)(dout + Y.jm); io.nmost = (int *)(dout + Y.nm); io.iisum = (double *)(dout + Y.ii);
        launch_node_lp(s, P, io, nb);
        (void)hipMemcpyAsync(bf.hout.p, bf.dout.p, Y.out_end, hipMemcpyDeviceToHost, s);
        (void)hipEventRecord(bf.done, s);
        t_launch += secs(tl0);
    };
    auto process = [&](BatchBuf &bf) {
        if (eng) {
            // engine mode: every node LP by the engine from its parent's
            // basis, in entry order (the search's decisions as node_done
            // takes them for a fallback node: host integrality scan and
            // branching, no tableau, no probes)
            const auto tp0 = std::chrono::steady_clock::now();
            const std::vector<double> zeros(2 * (size_t)n, 0.0);
            // the batch's node LPs solved concurrently, one context and
            // factor per worker (each LP's path is its own: the same solution
            // as one at a time), then the search's decisions in entry order.
            // Each LP's objective limit is the incumbent at the batch's
            // start: an LP a newer incumbent would have cut off is solved to
            // its optimum and pruned by node_done's hopeful test instead,
            // the same decision; a failed one is re-solved in order with the
            // current incumbent, as one at a time would have solved it
            struct Res {
                std::vector<double> bnd, x;
                std::vector<signed char> so;
                double z = 0.0;
                bool opt = false;
                int ret = 0;
                long long piv = 0;
                MipSolver::Degrad dg;
            };
            const int ne = (int)bf.ents.size();
            std::vector<Res> res(ne);
            for (int i = 0; i < ne; i++) {
                // (the node's bounds copied out: branching allocates pool
                // slots, which may move the pool's arrays)
                const int sl = bf.ents[i].nd.slot;
                S.materialize(sl);
                res[i].bnd.resize(2 * (size_t)n);
                std::memcpy(res[i].bnd.data(), pool.lb(sl), n * sizeof(double));
                std::memcpy(res[i].bnd.data() + n, pool.ub(sl), n * sizeof(double));
            }
            // (opt-in, GK_BNB_ENGINE_CONCURRENT=1: measured 2.2x faster on
            // the sparse MIPs, but its node counts varied from run to run
            // — 377 / 410 / 448 node LPs on sparsebig1 — where one at a
            // time gives the pinned 410 every run; the cause is not found,
            // so the default solves the batch in order on one factor)
            static const bool conc = [] {
                const char *e = std::getenv("GK_BNB_ENGINE_CONCURRENT");
                return e && std::atoi(e) != 0;
            }();
            static const int wmax = [] {                  // GK_BNB_ENGINE_WORKERS (diagnostics): at most this many
                const char *e = std::getenv("GK_BNB_ENGINE_WORKERS");
                return e ? std::max(1, std::atoi(e)) : 64;
            }();
            const int W = (S.err || !conc) ? 0 : std::min(std::min(ne, engine_batch()), wmax);
            int dev = 0;
            (void)hipGetDevice(&dev);                     // (the search's device: its contexts' and the workers')
            while ((int)S.engw.size() < W) {
                MipSolver::EngW w;
                w.ctx = gk_ctx_create(dev);
                w.fb = w.ctx ? gk_bfd_create(w.ctx) : nullptr;
                w.ver = engine_a_version();
                S.engw.push_back(w);
            }
            bool wok = true;
            for (int w = 0; w < W; w++) wok = wok && S.engw[w].fb;
            auto work = [&](int w) {
                (void)hipSetDevice(dev);
                const MipSolver::EngW &ew = S.engw[w];
                for (int i = w; i < ne; i += W) {
                    Res &r = res[i];
                    try {
                        r.ret = S.solve_node(ew.ctx, ew.fb, ew.ver, bf.ents[i].nd, r.bnd.data(), r.bnd.data() + n,
                                             r.x, r.so, r.z, r.opt, r.piv, &r.dg);
                    } catch (...) {
                        r.ret = 5;                        // (re-solved in order below)
                    }
                }
            };
            if (W > 0 && wok) {
                std::vector<std::thread> th;
                for (int w = 1; w < W; w++) th.emplace_back(work, w);
                work(0);
                for (auto &t : th) t.join();
            }
            for (int i = 0; i < ne; i++) {
                const NodeRec &nd = bf.ents[i].nd;
                Res &r = res[i];
                if (!S.err) {
                    S.lp_solves++;
                    if (!(W > 0 && wok) || r.ret) {
                        // (no workers, or a failure: solved here, in order)
                        r.ret = S.fallback(nd, r.bnd.data(), r.bnd.data() + n, r.x, r.so, r.z, r.opt);
                        r.dg = S.dg;
                    } else {
                        S.fallbacks++;
                        S.pivots += r.piv;
                    }
                    if (r.ret) S.err = r.ret;
                    else if (r.opt) {
                        // the tableau's degradations and branch_drtom's choice
                        // (engine_degrad) as the node kernel returns them;
                        // pseudocost branching without probes
                        const MipSolver::Degrad &D = r.dg;
                        const bool tab = D.ok && parm->br_tech != 5;
                        S.node_done(nd, r.z, r.x.data(), r.so.data(), r.bnd.data(), r.bnd.data() + n,
                                    tab ? D.dz.data() : zeros.data(), tab ? D.kjj : 0, tab ? D.knext : 0, tab,
                                    D.ok ? D.cand.data() : nullptr, D.ok ? (int)D.cand.size() : -1, D.ii);
                    }
                }
                pool.release(nd.slot);
            }
            bf.ents.clear();
            for (const NodeRec &c : S.next_dive) S.dive.push_back(c);
            S.next_dive.clear();
            t_proc += secs(tp0);
            return;
        }
        const auto tw0 = std::chrono::steady_clock::now();
        if (hipEventSynchronize(bf.done) != hipSuccess) { fail_sync = true; return; }
        t_wait += secs(tw0);
        if (bnb_lvl >= 2 && bf.nb > 0) {
            hst.resize((size_t)bf.nb * 8);
            (void)hipMemcpy(hst.data(), bf.dstamp.p, hst.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0;
            for (int b = 0; b < bf.nb; b++) {
                const unsigned long long *t = hst.data() + (size_t)b * 8;
                if (t[0]) lo = std::min(lo, t[0]);
                if (t[7]) hi = std::max(hi, t[7]);
                if (t[0] && t[7] && !t[1]) { pp_cnt++; ph_sum[5] += (double)(t[7] - t[0]); }
                if (!(t[0] && t[5] && t[1] && t[2] && t[3] && t[4] && t[7])) continue;
                ph_cnt++;
                ph_sum[6] += (double)(t[5] - t[0]);
                ph_sum[0] += (double)(t[1] - t[5]);
                ph_sum[1] += (double)(t[2] - t[1]);
                ph_sum[2] += (double)(t[3] - t[2]);
                ph_sum[3] += (double)(t[4] - t[3]);
                ph_sum[4] += (double)(t[7] - t[4]);
            }
            if (hi > lo) span_sum += (double)(hi - lo);
        }
        const auto tp0 = std::chrono::steady_clock::now();
        struct Acc { double &t; std::chrono::steady_clock::time_point a; ~Acc() {
            t += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count(); } } acc_{t_proc, tp0};
        const int nb = bf.nb;
        const Layout Y(S.N, n, nb);
        const char *h = bf.hout.p;
        const double *hobj = (const double *)(h + Y.obj), *hdz = (const double *)(h + Y.dz);
        const double *hx = (const double *)(h + Y.x), *hb = (const double *)(h + Y.bnd);
        const int *hstat = (const int *)(h + Y.stat), *hpiv = (const int *)(h + Y.piv);
        const int *hjj = (const int *)(h + Y.jj), *hnext = (const int *)(h + Y.next);
        const signed char *hso = (const signed char *)(h + Y.sto);
        const int *hnf = (const int *)(h + Y.nf), *hjf = (const int *)(h + Y.jf), *hjl = (const int *)(h + Y.jl);
        const int *hjm = (const int *)(h + Y.jm), *hnm = (const int *)(h + Y.nm);
        const double *hii = (const double *)(h + Y.ii);
        std::vector<double> fx;
        std::vector<signed char> fso;
        const std::vector<double> zeros(2 * (size_t)n, 0.0);
        // (1) per entry, on the workers: the column bounds the node kernel
        // returned (interleaved lb / ub) into bl | bu — only where the host
        // reads them: the engine fallback, pseudocost branching (its
        // integrality scan and parked nodes), and children that get no
        // record (the record store is full).  The integrality scan itself
        // comes from the kernel (NodeIO nfrac ...) except for PCH
        HostWorkers *W = S.cache->workers;
        const bool pch = parm->br_tech == 5;
        const bool par = W && !pch;
        S.eb.resize((size_t)nb * 2 * n);
        auto prep = [&](int b) {
            const Entry &e = bf.ents[b];
            if (e.kind != 0) return;
            if (hstat[b] == NODE_OPT && e.tab_out >= 0 && !pch) return;
            const double *bb = hb + (size_t)b * 2 * n;
            double *bl = S.eb.data() + (size_t)b * 2 * n, *bu = bl + n;
            for (int j = 0; j < n; j++) { bl[j] = bb[2 * j]; bu[j] = bb[2 * j + 1]; }
        };
        // the search-state-free part of node_done, planned on the workers
        S.plans.resize(nb);
        S.planned.assign(nb, 0);
        auto plan = [&](int b) {
            const Entry &e = bf.ents[b];
            if (e.kind != 0) return;
            prep(b);
            if (hstat[b] != NODE_OPT || e.tab_out < 0 || pch) return;
            const KInt ki{hnf[b], hjf[b], hjl[b], hjm[b], hnm[b], hii[b]};
            S.plan_node(S.plans[b], e.nd, hobj[b], hx + (size_t)b * S.N, hdz + (size_t)b * 2 * n, hjj[b], hnext[b], ki);
            S.planned[b] = 1;
        };
        if (par) W->run(nb, 16, plan);
        else
            for (int b = 0; b < nb; b++) plan(b);
        // (2) in entry order (the search's decisions): incumbent, pruning,
        // branching; a child's bound and status arrays are only recorded
        S.jobs.clear();
        S.defer = par ? &S.jobs : nullptr;
        for (int b = 0; b < nb; b++) {
            const Entry &e = bf.ents[b];
            const int st = hstat[b];
            const double *x = hx + (size_t)b * S.N;
            const double *fbl = S.eb.data() + (size_t)b * 2 * n, *fbu = fbl + n;
            S.pivots += hpiv[b];
            if (e.kind == 1) {
                // the probe's degradation (eval_degrad :337-392)
                S.probes++;
                Parked &pk = S.parked[e.pid];
                double dg;
                if (st == NODE_INFEAS) dg = DBL_MAX;
                else if (st == NODE_OPT || st == NODE_ITLIM) {
                    dg = hobj[b] - pk.z;
                    if (dg < 1e-6 * (1.0 + 0.001 * std::fabs(S.c0 + S.sign * pk.z))) dg = 0.0;
                } else dg = 0.0;                   // the simplex failed
                pk.probe[2 * e.j + e.dir] = dg;
                if (--pk.pending == 0) S.parked_done(e.pid);
                continue;
            }
            const NodeRec &nd = e.nd;
            if (st == NODE_PPINF) S.pp_fathomed++;
            else S.lp_solves++;
            if (st == NODE_OPT) {
                const auto tn0 = bnb_log ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
                S.cur_tab = e.tab_out;
                if (S.planned[b])
                    S.node_done_planned(nd, hobj[b], x, S.plans[b]);
                else {
                    const KInt ki{hnf[b], hjf[b], hjl[b], hjm[b], hnm[b], hii[b]};
                    S.node_done(nd, hobj[b], x, hso + (size_t)b * S.N, fbl, fbu, hdz + (size_t)b * 2 * n, hjj[b],
                                hnext[b], true, nullptr, -1, 0.0, pch ? nullptr : &ki);
                }
                S.cur_tab = -1;
                if (bnb_log) t_nd += secs(tn0);
            } else if ((st == NODE_FAIL || st == NODE_ITLIM) && !S.err) {
                double z = 0.0;
                bool opt = false;
                const int ret = S.fallback(nd, fbl, fbu, fx, fso, z, opt);
                if (ret) S.err = ret;
                else if (opt) {
                    // fx / fso are reused by the next fallback: its children are filled now
                    std::vector<MipSolver::FillJob> *dj = S.defer;
                    S.defer = nullptr;
                    S.node_done(nd, z, fx.data(), fso.data(), fbl, fbu, zeros.data(), 0, 0, false);
                    S.defer = dj;
                }
            }
            Cc.tabs.dec(e.tab_out);
            pool.release(nd.slot);
        }
        S.defer = nullptr;
        // (3) the children's arrays, on the workers (slots are final: the
        // pool does not grow any more in this batch)
        if (!S.jobs.empty()) {
            const auto tf0 = bnb_log ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
            W->run((int)S.jobs.size(), 16, [&](int i) { S.fill_child(S.jobs[i]); });
            if (bnb_log) t_nd += secs(tf0);
        }
        bf.ents.clear();
        for (const NodeRec &c : S.next_dive) S.dive.push_back(c);
        S.next_dive.clear();
    };
    auto drain = [&]() {
        for (int k = 0; k < 2; k++) {
            const int sb = (cur + k) & 1;
            if (inflight[sb]) { process(S.bufs[sb]); inflight[sb] = 0; }
        }
    };
    auto release_all = [&]() {
        for (const NodeRec &r : S.open) pool.release(r.slot);
        S.open.clear();
        for (const NodeRec &d : S.dive) pool.release(d.slot);
        S.dive.clear();
        S.probeq.clear();
    };
    // sharded runs: every rank evaluates the same first
    // batches (deterministic, identical on every GPU) until the frontier holds
    // ramp * size nodes, then keeps the nodes i = rank (mod size) of the
    // frontier in (bound, creation) order; at every sync_every batches the
    // ranks exchange the incumbent and, with an all-gather, hand open nodes
    // to idle ranks (the collective is called by idle ranks too, until no
    // rank has work left)
    bool split_done = (size == 1), timed_out = false, gap_hit = false;
    // batch width before the first incumbent (GK_BNB_PRECAP; 0: no limit).
    // 8 measured best on gap (profiles/r03_bnb_precap_sweep.txt): 495 node
    // LPs against 3959 uncapped (the reference: 196) at the same wall time
    static const int pre_cap_env = [] {
        const char *e = std::getenv("GK_BNB_PRECAP");
        return e ? std::atoi(e) : 8;
    }();
    const int pre_cap = pre_cap_env > 0 ? pre_cap_env : 1 << 30;
    static const int post_cap_env = [] {
        const char *e = std::getenv("GK_BNB_CAP");              // (experiments) batch width with an incumbent
        return e ? std::atoi(e) : 0;
    }();
    const int post_cap = post_cap_env > 0 ? post_cap_env : 1 << 30;
    static const int winbatch_min = [] {
        const char *e = std::getenv("GK_BNB_WINBATCH");        // 0: batches as wide as BMAX
        return e ? std::max(0, std::atoi(e)) : 0;
    }();
    int since_sync = 0;
    // show_progress (glpios03.js:2-48) through the context's report hook, and
    // the relative gap of ios_relative_gap (glpios01.js:842): both need the
    // best local bound over the active subproblems (open, preferred children,
    // in flight, parked for pseudocost probes)
    gk_report_fn rfn = nullptr;
    void *rud = nullptr;
    gk_ctx_ios_report(ctx, &rfn, &rud);
    const bool rpt_on = rfn && parm->msg_lev >= 2;                          // GLP_MSG_ON
    auto active = [&](double &bnd) {
        long long a = 0;
        bnd = INF;
        auto take = [&](const NodeRec &r) { a++; bnd = std::min(bnd, r.bound); };
        for (const NodeRec &r : S.open) take(r);
        for (const NodeRec &r : S.dive) take(r);
        for (const NodeRec &r : S.next_dive) take(r);
        for (int k = 0; k < 2; k++)
            if (inflight[k])
                for (const Entry &e : S.bufs[k].ents)
                    if (e.kind == 0) take(e.nd);
        for (size_t p = 0; p < S.parked.size(); p++)
            if (std::find(S.parked_free.begin(), S.parked_free.end(), (int)p) == S.parked_free.end())
                take(S.parked[p].nd);
        return a;
    };
    auto tm_lag = std::chrono::steady_clock::time_point{};
    bool lag_set = false;
    auto report = [&](int bingo) {
        double bnd;
        const long long a = active(bnd);
        const int code = (bingo ? 1 : 0) | (S.have ? 2 : 0) | (a == 0 ? 4 : 0);
        const double obj = S.have ? S.c0 + S.sign * S.best : 0.0;
        // -DBL_MAX (the root's bound) prints as -inf / +inf by direction
        const double ob = (bnd == -INF) ? -S.sign * DBL_MAX : (bnd == INF ? S.sign * DBL_MAX : S.c0 + S.sign * bnd);
        rfn(rud, GK_RPT_MIP, code, (int)(L.it_cnt + S.pivots), (int)std::min<long long>(a, 0x7fffffff), obj, ob,
            (int)std::min<long long>(S.created - a, 0x7fffffff));
        tm_lag = std::chrono::steady_clock::now();
        lag_set = true;
    };
    // DBL_MAX (no stop) without an incumbent or once the tree is empty: the
    // reference ends an exhausted search with GLP_OPT before any gap test
    // (glpios03.js:522-528) and tests the gap only for a selected subproblem
    auto rel_gap = [&]() {
        if (!S.have) return DBL_MAX;
        double bnd;
        if (active(bnd) == 0) return DBL_MAX;
        const double bm = S.c0 + S.sign * S.best, bb = S.c0 + S.sign * bnd;
        return std::fabs(bm - bb) / (std::fabs(bm) + DBL_EPSILON);
    };
    bool peer_err = false;
    const bool sharded = size > 1 && shard && shard->allgather;
    for (;;) {
        // a failed rank of a sharded search leaves at the next epoch, with
        // the others (shard_epoch), not on its own
        if ((fail_sync || S.err) && !(sharded && split_done)) break;
        if (rpt_on) {
            if (S.bingos) { S.bingos = 0; report(1); }
            // every out_frq milliseconds (glpios03.js:603-607; the first line at the root)
            if (!lag_set || (double)(parm->out_frq - 1) <=
                                1000.0 * std::chrono::duration<double>(std::chrono::steady_clock::now() - tm_lag).count())
                report(0);
        }
        // the relative mip gap (glpios03.js:613-620); a sharded search
        // tests it on the global incumbent and bound inside shard_epoch
        if (size == 1 && parm->mip_gap > 0.0 && S.have && rel_gap() <= parm->mip_gap) {
            gap_hit = true;
            drain();
            if (rpt_on && S.bingos) { S.bingos = 0; report(1); }
            release_all();
            break;
        }
        const bool any_inflight = inflight[0] || inflight[1];
        bool have_work = !S.err && !fail_sync && (!S.open.empty() || !S.dive.empty() || !S.probeq.empty() || any_inflight);
        if (have_work && parm->tm_lim < 0x7fffffff &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1000.0 >= parm->tm_lim) {
            timed_out = true;
            drain();
            release_all();
            have_work = false;
        }
        if (!split_done) {
            if (!have_work) break;                        // the tree ended during the ramp-up: same on every rank
            if (S.probeq.empty() && !any_inflight &&
                (long long)S.open.size() + (long long)S.dive.size() >= (long long)ramp * size) {
                std::vector<NodeRec> front(S.dive.begin(), S.dive.end());
                for (const NodeRec &r : S.open) front.push_back(r);
                S.open.clear();
                S.dive.clear();
                std::sort(front.begin(), front.end(), [](const NodeRec &a, const NodeRec &b) {
                    return a.bound != b.bound ? a.bound < b.bound : a.seq < b.seq;
                });
                for (size_t i = 0; i < front.size(); i++) {
                    if ((int)(i % size) == rank) S.push_open(front[i]);
                    else pool.release(front[i].slot);
                }
                split_done = true;
                continue;
            }
        }
        if (split_done && size > 1 && (since_sync >= sync_every || !have_work)) {
            since_sync = 0;
            if (shard->allgather) {
                if (!have_work) drain();
                bool gstop = false;
                const int act = shard_epoch(S, shard, have_work, moved, S.err != 0 || fail_sync, parm->mip_gap, gstop,
                                            peer_err);
                if (act < 0) { set_err("gk_ios_driver: shard all-gather failed"); return GK_EABI; }
                if (gstop) {
                    gap_hit = true;
                    drain();
                    if (rpt_on && S.bingos) { S.bingos = 0; report(1); }
                    release_all();
                }
                if (act == 0) break;
                have_work = !S.open.empty() || !S.dive.empty() || !S.probeq.empty() || inflight[0] || inflight[1];
                if (!have_work) continue;
            } else {
                double bx = S.best;
                const int active = shard->exchange(shard->info, &bx, have_work ? 1 : 0);
                S.set_gbest(bx);
                if (active == 0) break;
                if (!have_work) continue;
            }
        }
        if (!have_work) break;
        since_sync++;
        if (inc && split_done) S.set_gbest(inc(inc_info, S.best));
        // assemble the next batch into the free buffer set: pseudocost
        // probes first (they unblock parked nodes), then the preferred
        // children, then the open nodes in the order of bt_tech
        BatchBuf &bf = S.bufs[cur];
        if (inflight[cur]) { process(bf); inflight[cur] = 0; }
        if (S.err) break;
        bf.ents.clear();
        // until the first incumbent prunes, a wide batch is mostly nodes a
        // sequential walk never solves (the reference dives for an incumbent
        // first): the batch widens to BMAX once one exists
        const int cap = S.have ? std::min(S.BMAX, post_cap) : std::min(S.BMAX, pre_cap);
        {
            size_t k = 0;
            for (; k < S.probeq.size() && (int)bf.ents.size() < cap; k++) bf.ents.push_back(S.probeq[k]);
            S.probeq.erase(S.probeq.begin(), S.probeq.begin() + k);
        }
        {
            std::vector<NodeRec> keep;
            for (const NodeRec &nd : S.dive) {
                if (!S.hopeful(nd.bound)) { pool.release(nd.slot); continue; }
                if ((int)bf.ents.size() < cap) bf.ents.push_back(Entry{0, nd, 0, 0, 0});
                else S.push_open(nd);
            }
            S.dive.clear();
        }
        // (with an incumbent, GK_BNB_WINBATCH: the open nodes of a batch are
        // those within best_node's window of its first one — the nodes a
        // sequential walk treats as equally good — and at least
        // winbatch_min of them)
        double wlim = DBL_MAX;
        while (!S.open.empty() && (int)bf.ents.size() < cap) {
            if (S.have && winbatch_min > 0 && (int)bf.ents.size() >= winbatch_min && S.open.front().key > wlim) break;
            const NodeRec nd = S.pop_open();
            if (!S.hopeful(nd.bound)) { pool.release(nd.slot); continue; }
            if (wlim == DBL_MAX && parm->bt_tech == 3) wlim = nd.key + S.window_eps(nd.key);
            bf.ents.push_back(Entry{0, nd, 0, 0, 0});
        }
        if (!bf.ents.empty()) {
            launch(bf);
            inflight[cur] = 1;
        }
        const int prev = cur ^ 1;
        if (depth == 1 || bf.ents.empty()) {
            // no pipelining (sharded runs), or nothing new to launch: finish
            // what is in flight, oldest first
            if (inflight[prev]) { process(S.bufs[prev]); inflight[prev] = 0; }
            if (depth == 1 && inflight[cur]) { process(bf); inflight[cur] = 0; }
        } else if (inflight[prev]) {
            process(S.bufs[prev]);
            inflight[prev] = 0;
        }
        cur ^= 1;
    }
    if (fail_sync) {
        set_err("gk_ios_driver: node batch failed: %s", hipGetErrorString(hipGetLastError()));
        return GK_EABI;
    }
    if (S.err || peer_err) {                              // the reference's "unable to solve current LP relaxation"
        drain();
        release_all();
    }
    if (rpt_on) {
        if (S.bingos) { S.bingos = 0; report(1); }
        report(0);                                        // glpios03.js:941-943
    }
    if (bnb_log)
        fprintf(stderr, "[gk bnb] %.3f ms: %lld batches, %lld entries (%.1f per batch); host launch %.3f ms, "
                        "wait %.3f ms, process %.3f ms (node_done %.3f); open %zu; lp %lld, pp-fathomed %lld, created %lld\n",
                1e3 * secs(t0), n_batches, n_ents, n_batches ? (double)n_ents / n_batches : 0.0, 1e3 * t_launch,
                1e3 * t_wait, 1e3 * t_proc, 1e3 * t_nd, S.open.size(), S.lp_solves, S.pp_fathomed, S.created);
    if (bnb_lvl >= 2) {
        const double us = 0.01;                           // device clock: 100 MHz
        const double c = ph_cnt ? 1.0 / (double)ph_cnt : 0.0;
        fprintf(stderr, "[gk bnb] node kernel, mean us per node LP (%lld): load %.2f, preprocess %.2f, tableau %.2f, "
                        "x/d %.2f, simplex %.2f, branching+records %.2f; preprocess-fathomed (%lld) %.2f; "
                        "batch spans %.3f ms in all\n", ph_cnt, ph_sum[6] * c * us, ph_sum[0] * c * us, ph_sum[1] * c * us,
                ph_sum[2] * c * us, ph_sum[3] * c * us, ph_sum[4] * c * us, pp_cnt,
                pp_cnt ? ph_sum[5] / (double)pp_cnt * us : 0.0, span_sum * us * 1e-3);
    }
    if (bnb_log) {
        const double tpms = (double)(MipSolver::tsc() - tsc_beg) / (1e3 * secs(t0));     // ticks per ms
        fprintf(stderr, "[gk bnb] node_done parts: integrality %.3f ms, choice %.3f ms, children (incl. heap) %.3f ms, "
                        "heap pushes %.3f ms\n", S.tsc_int / tpms, S.tsc_choose / tpms, S.tsc_child / tpms,
                S.tsc_heap / tpms);
    }
    mip->lp_solves = S.lp_solves;
    mip->nodes_created = S.created;
    mip->pivots = S.pivots;
    mip->node_fallbacks = S.fallbacks;
    mip->probe_lps = S.probes;
    mip->pp_fathomed = S.pp_fathomed;
    mip->nodes_moved = moved;
    if (S.have) {
        mip->mip_stat = (timed_out || S.err || gap_hit || peer_err) ? 2 : 5;     // GLP_FEAS / GLP_OPT
        mip->mip_obj = S.c0 + S.sign * S.best;
        for (int i = 0; i < m; i++) mip->row_mipx[i + 1] = S.xbest[i];
        for (int j = 0; j < n; j++)
            mip->col_mipx[j + 1] = S.isint[j] ? std::floor(S.xbest[m + j] + 0.5) : S.xbest[m + j];
    } else {
        mip->mip_stat = (timed_out || S.err || peer_err) ? 1 : 4;     // GLP_UNDEF / GLP_NOFEAS
        mip->mip_obj = 0.0;
    }
    if (S.err) return S.err;                              // GLP_EFAIL
    if (peer_err) return 0x05;                            // another rank's GLP_EFAIL ends this one's search too
    if (gap_hit) return 0x0E;                             // GLP_EMIPGAP
    return timed_out ? 0x09 : 0;                          // GLP_ETMLIM
}
