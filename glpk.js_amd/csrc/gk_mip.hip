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
#include "../../include/glpk_mi355x.h"
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <queue>
#include <string>
#include <vector>

namespace gk {

void set_err(const char *fmt, ...);

enum : int { NODE_OPT = 0, NODE_INFEAS = 1, NODE_CUTOFF = 2, NODE_FAIL = 3 };

struct NodeProb {
    int m, n, ld;                 // ld = m + n (row length of T)
    const double *A;              // dense col-major m x n (unscaled)
    const double *c;              // internal minimisation costs, [m+n] (0 for rows)
    const signed char *isint;     // [n]
    double tol_int;
};

struct NodeIO {
    const double *lb, *ub;        // [nb][m+n]
    const signed char *stat_in;   // [nb][m+n]  GLP_BS / NL / NU / NF / NS
    const double *cutoff;         // [nb]  stop once the dual objective reaches it
    int *status, *pivots, *jj, *next;
    double *obj, *x, *dz;         // obj[nb], x[nb][m+n], dz[nb][2]
    signed char *stat_out;        // [nb][m+n]
    int it_lim;
    double *scratch;              // GLOBAL kernel: per-node work area (node_lp_lds(m, n) bytes each)
    size_t scratch_stride;        // in doubles
};

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
// one workgroup = one node LP
// LDS: M[m][2m+n] during the inversion, then T[m][m+n]; lb, ub, x, d [m+n];
// head[m], stat[m+n].  GLOBAL = 1: the same work area in a per-node slice of
// HBM (node LPs beyond 64 KiB of LDS; L2 serves the workgroup's sweeps).
// ---------------------------------------------------------------------------
template <int GLOBAL>
__global__ void __launch_bounds__(256) k_node_lp(NodeProb P, NodeIO io)
{
    extern __shared__ double lds_[];
    double *lds = GLOBAL ? io.scratch + (size_t)blockIdx.x * io.scratch_stride : lds_;
    __shared__ double shk[4], sha[4];
    __shared__ int shi[4];
    __shared__ int sh_flag;
    const int m = P.m, n = P.n, N = m + n, b = blockIdx.x;
    const int W = 2 * m + n;                 // width of [B | I | -A]
    double *M = lds;                          // m * W
    double *lb = M + (size_t)m * W, *ub = lb + N, *x = ub + N, *d = x + N;
    double *fcol = d + N;                     // m
    int *head = (int *)(fcol + m);
    signed char *stat = (signed char *)(head + m);
    const double *glb = io.lb + (size_t)b * N, *gub = io.ub + (size_t)b * N;
    const signed char *gst = io.stat_in + (size_t)b * N;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        lb[k] = glb[k];
        ub[k] = gub[k];
        stat[k] = gst[k];
    }
    __syncthreads();
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
        if (threadIdx.x == 0) { io.status[b] = NODE_FAIL; io.pivots[b] = 0; }
        return;
    }
    // M = [B | I | -A]: column k of (I | -A) is e_k (k < m) or -A[:, k-m]
    for (int e = threadIdx.x; e < m * W; e += blockDim.x) {
        const int i = e / W, c = e % W;
        double v;
        if (c < m) {
            const int k = head[c];
            v = (k < m) ? (i == k ? 1.0 : 0.0) : -P.A[(size_t)(k - m) * m + i];
        } else if (c < 2 * m) {
            v = (i == c - m) ? 1.0 : 0.0;
        } else {
            v = -P.A[(size_t)(c - 2 * m) * m + i];
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
            if (threadIdx.x == 0) { io.status[b] = NODE_FAIL; io.pivots[b] = 0; }
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
#define T_(i, j) M[(size_t)(i) * W + m + (j)]
    // x_N and x_B = -T_N x_N
    for (int k = threadIdx.x; k < N; k += blockDim.x) x[k] = (stat[k] == BS) ? 0.0 : nb_value(stat[k], lb[k], ub[k]);
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        double s = 0.0;
        for (int k = 0; k < N; ++k)
            if (stat[k] != BS && x[k] != 0.0) s += T_(i, k) * x[k];
        x[head[i]] = -s;
    }
    // d = c - c_B' T
    __syncthreads();
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        if (stat[k] == BS) { d[k] = 0.0; continue; }
        double s = P.c[k];
        for (int i = 0; i < m; ++i) {
            const double cb = P.c[head[i]];
            if (cb != 0.0) s -= cb * T_(i, k);
        }
        d[k] = s;
    }
    __syncthreads();
    // ---- bounded dual simplex ------------------------------------------
    const double tol_p = 1e-7, tol_piv = 1e-7;
    const double cutoff = io.cutoff[b];
    int it = 0, status = NODE_OPT;
    for (;;) {
        // objective (dual objective of the current dual feasible basis)
        double zs = 0.0;
        for (int k = threadIdx.x; k < N; k += blockDim.x) zs += P.c[k] * x[k];
        const double z = block_sum256(zs, shk);
        if (z >= cutoff) { status = NODE_CUTOFF; break; }
        // chuzr: largest bound violation
        double key = 0.0;
        int idx = -1;
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            const int k = head[i];
            const double v = x[k];
            double r = 0.0;
            if (v < lb[k] - tol_p * (1.0 + fabs(lb[k]))) r = lb[k] - v;
            else if (v > ub[k] + tol_p * (1.0 + fabs(ub[k]))) r = v - ub[k];
            if (r > 0.0 && (idx < 0 || r > key)) { key = r; idx = i; }
        }
        const int p = block_argmax(key, idx, shk, shi);
        if (p < 0) break;                                  // primal feasible: optimal
        if (it >= io.it_lim) { status = NODE_FAIL; break; }
        const int kp = head[p];
        const bool to_lb = x[kp] < lb[kp];
        // ratio test on row p: x_p = -sum T[p,j] x_j
        double rmax = 0.0;
        for (int k = threadIdx.x; k < N; k += blockDim.x)
            if (stat[k] != BS) rmax = fmax(rmax, fabs(T_(p, k)));
        {
            __syncthreads();
            const double r = wmax(rmax);
            if ((threadIdx.x & 63) == 0) shk[threadIdx.x >> 6] = r;
            __syncthreads();
            rmax = fmax(fmax(shk[0], shk[1]), fmax(shk[2], shk[3]));
            __syncthreads();
        }
        const double eps = tol_piv * (1.0 + 0.01 * rmax);
        double bt = 0.0, ba = 0.0;
        int bq = -1;
        for (int k = threadIdx.x; k < N; k += blockDim.x) {
            const int st = stat[k];
            if (st == BS || st == NS) continue;
            const double a = T_(p, k);
            if (fabs(a) < eps) continue;
            // x_p changes by -a per unit increase of x_k
            bool ok;
            if (to_lb) ok = (st == NL && a < 0.0) || (st == NU && a > 0.0) || (st == NF);
            else ok = (st == NL && a > 0.0) || (st == NU && a < 0.0) || (st == NF);
            if (!ok) continue;
            // the step that keeps d dual feasible: d_k - (d_q / a_pq) a_k
            double t = (st == NF) ? fabs(d[k]) / fabs(a) : (to_lb ? -d[k] / a : d[k] / a);
            if (t < 0.0) t = 0.0;
            if (bq < 0 || t < bt || (t == bt && fabs(a) > ba)) { bt = t; ba = fabs(a); bq = k; }
        }
        const int q = block_ratio(bt, ba, bq, shk, sha, shi);
        if (q < 0) { status = NODE_INFEAS; break; }        // dual unbounded
        // pivot (p, q)
        const double apq = T_(p, q);
        const double bound = to_lb ? lb[kp] : ub[kp];
        const double tq = (x[kp] - bound) / apq;         // step of x_q
        const double dq = d[q] / apq;
        __syncthreads();
        // x update
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
        __syncthreads();
        if (threadIdx.x == 0) {
            x[q] += tq;
            x[kp] = bound;
            d[q] = 0.0;
            d[kp] = -dq;
            stat[kp] = to_lb ? (lb[kp] == ub[kp] ? NS : NL) : (lb[kp] == ub[kp] ? NS : NU);
            stat[q] = BS;
            head[p] = q;
        }
        // T update: row p /= apq; row i -= T[i,q] row p
        __syncthreads();
        for (int k = threadIdx.x; k < N; k += blockDim.x) T_(p, k) /= apq;
        __syncthreads();
        for (int e = threadIdx.x; e < m * N; e += blockDim.x) {
            const int i = e / N, k = e % N;
            if (i == p) continue;
            const double f = T_(i, q);
            if (f != 0.0 && k != q) T_(i, k) -= f * T_(p, k);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < m; i += blockDim.x)
            if (i != p) T_(i, q) = 0.0;
        __syncthreads();
        it++;
    }
    __syncthreads();
    double zs = 0.0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) zs += P.c[k] * x[k];
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
        return;
    }
    // ---- branch_drtom (glpios09.js:84) on the node's own tableau rows ----
    // columns in order; x_j basic and fractional; the dual ratio test of
    // glp_dual_rtest (glpapi12.js:687) on the row x_j = sum alfa_k x_k,
    // alfa_k = -T[i,k]; delta z = d_k * delta x_k with Tomlin's rounding
    __shared__ int sh_jj, sh_next, sh_brk;
    __shared__ double sh_degrad, sh_dn, sh_up;
    if (threadIdx.x == 0) { sh_jj = 0; sh_next = 0; sh_degrad = -1.0; sh_dn = 0.0; sh_up = 0.0; sh_brk = 0; }
    __syncthreads();
    int any_frac = 0;
    // visit the basic structural columns in increasing j
    for (int j = 0; j < n; ++j) {
        const int k = m + j;
        if (stat[k] != BS || !P.isint[j]) continue;
        const double xv = x[k];
        if (fabs(xv - floor(xv + 0.5)) <= P.tol_int) continue;
        any_frac = 1;
        int row = -1;
        for (int i = 0; i < m; ++i)
            if (head[i] == k) { row = i; break; }
        double dz[2], dzb[2];
        for (int kase = 0; kase < 2; ++kase) {
            const double dir = kase == 0 ? -1.0 : +1.0;
            double bt = 0.0, ba = 0.0;
            int bq = -1;
            for (int kk = threadIdx.x; kk < N; kk += blockDim.x) {
                const int st = stat[kk];
                if (st == BS || st == NS) continue;
                const double alfa = dir * (-T_(row, kk));
                double t;
                if (st == NL) {
                    if (alfa < +1e-9) continue;
                    t = d[kk] / alfa;
                } else if (st == NU) {
                    if (alfa > -1e-9) continue;
                    t = d[kk] / alfa;
                } else {
                    if (-1e-9 < alfa && alfa < +1e-9) continue;
                    t = 0.0;
                }
                if (t < 0.0) t = 0.0;
                if (bq < 0 || t < bt || (t == bt && fabs(alfa) > ba)) { bt = t; ba = fabs(alfa); bq = kk; }
            }
            const int kq = block_ratio(bt, ba, bq, shk, sha, shi);
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
                if (kq >= m && P.isint[kq - m] && fabs(delta_k - floor(delta_k + 0.5)) > 1e-3)
                    delta_k = delta_k > 0.0 ? ceil(delta_k) : floor(delta_k);
                dz[kase] = fabs(dk * delta_k);   // Tomlin's estimate: choice only
            }
        }
        if (threadIdx.x == 0) {
            if (sh_degrad < dz[0] || sh_degrad < dz[1]) {
                sh_jj = j + 1;
                sh_dn = dzb[0];
                sh_up = dzb[1];
                if (dz[0] < dz[1]) { sh_next = -1; sh_degrad = dz[1]; }
                else { sh_next = +1; sh_degrad = dz[0]; }
                if (sh_degrad == DBL_MAX) sh_brk = 1;
            }
        }
        __syncthreads();
        if (sh_brk) break;
    }
    if (threadIdx.x == 0) {
        int jj = sh_jj, next = sh_next;
        double dn = sh_dn, up = sh_up;
        if (any_frac && sh_degrad < 1e-6 * (1.0 + 0.001 * fabs(z))) {
            // branch_mostf (glpios09.js:62): value closest to floor + 1/2
            double most = DBL_MAX;
            jj = 0;
            for (int j = 0; j < n; ++j) {
                const int k = m + j;
                if (stat[k] != BS || !P.isint[j]) continue;
                const double beta = x[k];
                if (fabs(beta - floor(beta + 0.5)) <= P.tol_int) continue;
                const double temp = floor(beta) + 0.5;
                if (most > fabs(beta - temp)) {
                    jj = j + 1;
                    most = fabs(beta - temp);
                    next = beta < temp ? -1 : +1;
                }
            }
            dn = 0.0;
            up = 0.0;
        }
        io.status[b] = NODE_OPT;
        io.obj[b] = z;
        io.pivots[b] = it;
        io.jj[b] = any_frac ? jj : 0;
        io.next[b] = next;
        io.dz[2 * b] = dn;
        io.dz[2 * b + 1] = up;
    }
#undef T_
}

size_t node_lp_lds(int m, int n)
{
    const size_t N = (size_t)m + n;
    return sizeof(double) * ((size_t)m * (2 * m + n) + 4 * N + m) + sizeof(int) * m + N + 16;
}

constexpr size_t NODE_LDS_MAX = 64 * 1024;

void launch_node_lp(hipStream_t s, const NodeProb &P, const NodeIO &io, int nb)
{
    const size_t lds = node_lp_lds(P.m, P.n);
    if (lds <= NODE_LDS_MAX) hipLaunchKernelGGL(k_node_lp<0>, dim3(nb), dim3(256), lds, s, P, io);
    else hipLaunchKernelGGL(k_node_lp<1>, dim3(nb), dim3(256), 0, s, P, io);
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

// an open node: its bound and creation order in the queue, its structural
// bounds and warm-start basis in a slot of the node pool
struct NodeRec {
    double bound;                 // local bound, minimisation form
    long long seq;                // creation order (tie-break: older first)
    int slot;
};

struct NodeCmp {
    bool operator()(const NodeRec &a, const NodeRec &b) const
    {
        if (a.bound != b.bound) return a.bound > b.bound;
        return a.seq > b.seq;
    }
};

// slots of 2 n doubles (lb | ub of the structurals) and m + n statuses,
// recycled through a free list (no per-node heap allocation)
struct NodePool {
    int n = 0, N = 0;
    std::vector<double> bnd;
    std::vector<signed char> st;
    std::vector<int> freel;
    int alloc()
    {
        if (!freel.empty()) {
            const int sl = freel.back();
            freel.pop_back();
            return sl;
        }
        const int sl = (int)(st.size() / (size_t)N);
        bnd.resize(bnd.size() + 2 * (size_t)n);
        st.resize(st.size() + (size_t)N);
        return sl;
    }
    void release(int sl) { freel.push_back(sl); }
    double *lb(int sl) { return bnd.data() + (size_t)sl * 2 * n; }
    double *ub(int sl) { return bnd.data() + (size_t)sl * 2 * n + n; }
    signed char *stat(int sl) { return st.data() + (size_t)sl * N; }
};

// one batch in flight: packed inputs / outputs (one copy each way)
struct BatchBuf {
    DevArr<char> din, dout;
    HostArr<char> hin, hout;
    hipEvent_t done = nullptr;
    std::vector<NodeRec> nodes;
    int nb = 0;
    ~BatchBuf()
    {
        if (done) (void)hipEventDestroy(done);
    }
};

}  // namespace

struct MipSolver {
    int m = 0, n = 0, N = 0;
    double sign = 1.0, c0 = 0.0;
    std::vector<double> A, c, rlb, rub, clb, cub, coef;
    std::vector<signed char> isint, fixed_col;
    DevArr<double> dA, dc, dscratch;
    DevArr<signed char> dint;
    BatchBuf bufs[2];
    NodePool pool;
    int bmax = 0;
    size_t in_bytes(int nb) const { return (size_t)nb * (2 * (size_t)N + 1) * sizeof(double) + (size_t)nb * N; }
    size_t out_bytes(int nb) const
    {
        return (size_t)nb * (3 + (size_t)N) * sizeof(double) + 4 * (size_t)nb * sizeof(int) + (size_t)nb * N;
    }
    bool alloc_batch(int B)
    {
        bmax = B;
        for (auto &bf : bufs) {
            bf.din.ensure(in_bytes(B) + 64); bf.dout.ensure(out_bytes(B) + 64);
            bf.hin.ensure(in_bytes(B) + 64); bf.hout.ensure(out_bytes(B) + 64);
            if (!bf.done && hipEventCreateWithFlags(&bf.done, hipEventDisableTiming) != hipSuccess) return false;
            if (!bf.din.p || !bf.dout.p || !bf.hin.p || !bf.hout.p) return false;
        }
        return true;
    }
    // ios_round_bound (glpios01.js:730): objective integrality
    bool round_ok = false;
    double round_s = 0.0, round_d = 1.0;

    // min-form bound -> rounded min-form bound
    double round_bound(double z) const
    {
        if (!round_ok) return z;
        // the reference rounds in the original direction; in minimisation
        // form both cases are "round up" of (bound - s) / d
        const double s = sign * (round_s - c0), d = round_d;
        const double h = (z - s) / d;
        if (h >= std::floor(h) + 0.001) return d * std::ceil(h) + s;
        return z;
    }
};

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

}  // namespace gk

using namespace gk;

int gk_ctx_device(gk_ctx *);
hipStream_t gk_ctx_stream(gk_ctx *);

extern "C" int gk_ios_driver(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm)
{
    return gk_ios_driver_sharded(ctx, mip, parm, nullptr);
}

extern "C" int gk_ios_driver_sharded(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, const gk_ios_shard *shard)
{
    if (!ctx || !mip || !parm) { set_err("gk_ios_driver: null argument"); return GK_EABI; }
    const int rank = shard ? shard->rank : 0, size = shard ? shard->size : 1;
    if (size < 1 || rank < 0 || rank >= size || (size > 1 && !shard->exchange)) {
        set_err("gk_ios_driver: invalid shard %d of %d", rank, size);
        return GK_EABI;
    }
    const int ramp = (shard && shard->ramp_nodes > 0) ? shard->ramp_nodes : 8;
    const int sync_every = (shard && shard->sync_every > 0) ? shard->sync_every : 4;
    const gk_lp &L = mip->lp;
    const int m = L.m, n = L.n;
    if (m < 1 || n < 1) { set_err("gk_ios_driver: m = %d, n = %d; invalid dimensions", m, n); return GK_EABI; }
    if (L.pbs_stat != 2 || L.dbs_stat != 2) {
        set_err("gk_ios_driver: optimal basis to initial LP relaxation not provided");
        return GK_EABI;
    }
    // node LPs up to 64 KiB keep their tableau in LDS; larger ones work in a
    // per-node slice of HBM, batches sized to at most 8 GiB of work area
    const size_t lds = node_lp_lds(m, n);
    const size_t SCRATCH_MAX = (size_t)8 << 30;
    if (lds > SCRATCH_MAX) {
        set_err("gk_ios_driver: node LP %d x %d needs %zu bytes of work area; at most %zu", m, n, lds, SCRATCH_MAX);
        return GK_EABI;
    }
    if (hipSetDevice(gk_ctx_device(ctx)) != hipSuccess) { set_err("gk_ios_driver: hipSetDevice failed"); return GK_EABI; }
    hipStream_t s = gk_ctx_stream(ctx);
    const auto t0 = std::chrono::steady_clock::now();
    MipSolver S;
    S.m = m; S.n = n; S.N = m + n;
    S.sign = (L.dir == 1) ? 1.0 : -1.0;                   // GLP_MIN = 1
    S.c0 = L.c0;
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
    S.A.assign((size_t)m * n, 0.0);
    for (int j = 1; j <= n; j++)
        for (int t = L.A_ptr[j]; t < L.A_ptr[j + 1]; t++) {
            const int i = L.A_ind[t];
            if (i < 1 || i > m) { set_err("gk_ios_driver: A_ind[%d] = %d; out of range", t, i); return GK_EABI; }
            S.A[(size_t)(j - 1) * m + (i - 1)] += L.A_val[t];
        }
    S.c.assign(S.N, 0.0);
    S.isint.assign(n, 0);
    for (int j = 0; j < n; j++) {
        S.c[m + j] = S.sign * L.col_coef[j + 1];
        S.isint[j] = (mip->col_kind[j + 1] == 2) ? 1 : 0;
    }
    setup_rounding(S, mip);
    // device problem
    S.dA.ensure(S.A.size()); S.dc.ensure(S.N); S.dint.ensure(n);
    const int BMAX = (lds <= NODE_LDS_MAX) ? 1024 : (int)std::max<size_t>(1, std::min<size_t>(1024, SCRATCH_MAX / lds));
    const size_t stride = (lds + 255) / 256 * 32;          // doubles, 256-byte aligned slices
    if (lds > NODE_LDS_MAX) {
        S.dscratch.ensure(stride * BMAX);
        if (!S.dscratch.p) { set_err("gk_ios_driver: out of memory (node work area)"); return GK_EABI; }
    }
    if (!S.alloc_batch(BMAX) || !S.dA.p || !S.dc.p || !S.dint.p) {
        set_err("gk_ios_driver: out of memory");
        return GK_EABI;
    }
    (void)hipMemcpyAsync(S.dA.p, S.A.data(), S.A.size() * sizeof(double), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(S.dc.p, S.c.data(), S.N * sizeof(double), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(S.dint.p, S.isint.data(), n, hipMemcpyHostToDevice, s);
    NodeProb P;
    P.m = m; P.n = n; P.ld = S.N; P.A = S.dA.p; P.c = S.dc.p; P.isint = S.dint.p; P.tol_int = parm->tol_int;
    NodePool &pool = S.pool;
    pool.n = n; pool.N = S.N;
    // root node: the optimal basis of the initial LP relaxation
    std::priority_queue<NodeRec, std::vector<NodeRec>, NodeCmp> open;
    long long seq = 0;
    {
        const int sl = pool.alloc();
        std::memcpy(pool.lb(sl), S.clb.data(), n * sizeof(double));
        std::memcpy(pool.ub(sl), S.cub.data(), n * sizeof(double));
        signed char *st = pool.stat(sl);
        for (int i = 0; i < m; i++) st[i] = L.row_stat[i + 1];
        for (int j = 0; j < n; j++) st[m + j] = L.col_stat[j + 1];
        open.push(NodeRec{-INF, seq++, sl});
    }
    bool have = false;                                    // incumbent of this rank (with x)
    double best = INF;                                    // its objective, minimisation form
    double gbest = INF;                                   // best over all ranks (sharded runs)
    std::vector<double> xbest(S.N, 0.0);
    long long lp_solves = 0, pivots = 0, created = 1, failed = 0;
    auto bestall = [&]() { return std::min(best, gbest); };
    auto hopeful = [&](double bound) {
        const double b = bestall();
        if (b == INF) return true;
        const double eps = parm->tol_obj * (1.0 + std::fabs(S.c0 + S.sign * b));
        return bound < b - eps;
    };
    // the preferred child of every branched node of a batch is evaluated in
    // the next batch assembled (parallel dives, as BLB dives into its chosen
    // child, glpios12.js); the other children wait in the best-bound queue
    std::vector<NodeRec> dive, next_dive;
    // single GPU: two batches in flight — the host assembles and launches
    // batch k + 1 before it processes the results of batch k (more
    // speculative nodes, the GPU never waits for the host)
    const int depth = (size == 1) ? 2 : 1;
    int inflight[2] = {0, 0}, cur = 0;
    bool fail_sync = false;
    auto launch = [&](BatchBuf &bf) {
        const int nb = (int)bf.nodes.size();
        bf.nb = nb;
        const double ball = bestall();
        const double cut = ball < INF ? ball - parm->tol_obj * (1.0 + std::fabs(S.c0 + S.sign * ball)) : INF;
        const size_t NB = (size_t)nb * S.N;
        double *hl = (double *)bf.hin.p, *hu = hl + NB, *hc = hu + NB;
        signed char *hs = (signed char *)(hc + nb);
        for (int b = 0; b < nb; b++) {
            const int sl = bf.nodes[b].slot;
            double *l = hl + (size_t)b * S.N, *u = hu + (size_t)b * S.N;
            std::memcpy(l, S.rlb.data(), m * sizeof(double));
            std::memcpy(u, S.rub.data(), m * sizeof(double));
            std::memcpy(l + m, pool.lb(sl), n * sizeof(double));
            std::memcpy(u + m, pool.ub(sl), n * sizeof(double));
            std::memcpy(hs + (size_t)b * S.N, pool.stat(sl), S.N);
            hc[b] = cut;
        }
        (void)hipMemcpyAsync(bf.din.p, bf.hin.p, S.in_bytes(nb), hipMemcpyHostToDevice, s);
        double *dl = (double *)bf.din.p, *du = dl + NB, *dc = du + NB;
        double *dobj = (double *)bf.dout.p, *ddz = dobj + nb, *dx = ddz + 2 * (size_t)nb;
        int *dstat = (int *)(dx + NB), *dpiv = dstat + nb, *djj = dpiv + nb, *dnext = djj + nb;
        NodeIO io;
        io.lb = dl; io.ub = du; io.stat_in = (const signed char *)(dc + nb); io.cutoff = dc;
        io.status = dstat; io.pivots = dpiv; io.jj = djj; io.next = dnext;
        io.obj = dobj; io.x = dx; io.dz = ddz; io.stat_out = (signed char *)(dnext + nb);
        io.it_lim = 10000;
        io.scratch = S.dscratch.p;
        io.scratch_stride = stride;
        launch_node_lp(s, P, io, nb);
        (void)hipMemcpyAsync(bf.hout.p, bf.dout.p, S.out_bytes(nb), hipMemcpyDeviceToHost, s);
        (void)hipEventRecord(bf.done, s);
    };
    auto process = [&](BatchBuf &bf) {
        if (hipEventSynchronize(bf.done) != hipSuccess) { fail_sync = true; return; }
        const int nb = bf.nb;
        const size_t NB = (size_t)nb * S.N;
        const double *hobj = (const double *)bf.hout.p, *hdz = hobj + nb, *hx = hdz + 2 * (size_t)nb;
        const int *hstat = (const int *)(hx + NB), *hpiv = hstat + nb, *hjj = hpiv + nb, *hnext = hjj + nb;
        const signed char *hso = (const signed char *)(hnext + nb);
        for (int b = 0; b < nb; b++) {
            const NodeRec nd = bf.nodes[b];
            lp_solves++;
            pivots += hpiv[b];
            const int st = hstat[b];
            if (st == NODE_FAIL) { failed++; continue; }
            if (st != NODE_OPT) continue;                  // infeasible or cut off
            const double z = hobj[b];
            const double bound = S.round_bound(z);
            if (!hopeful(bound)) continue;
            const double *x = hx + (size_t)b * S.N;
            const int jj = hjj[b];
            if (jj == 0) {                                 // integer feasible
                if (!have || z < best) {
                    have = true;
                    best = z;
                    std::memcpy(xbest.data(), x, S.N * sizeof(double));
                }
                continue;
            }
            const int j = jj - 1;
            const double beta = x[m + j];
            const double dz[2] = {hdz[2 * b], hdz[2 * b + 1]};
            const int first = hnext[b] < 0 ? 0 : 1;      // preferred child gets the older seq
            bool dived = false;
            for (int r = 0; r < 2; r++) {
                const int kase = (r == 0) ? first : 1 - first;
                if (dz[kase] == DBL_MAX) continue;        // that branch has no feasible point
                const int sl = pool.alloc();
                std::memcpy(pool.lb(sl), pool.lb(nd.slot), n * sizeof(double));
                std::memcpy(pool.ub(sl), pool.ub(nd.slot), n * sizeof(double));
                if (kase == 0) pool.ub(sl)[j] = std::floor(beta);
                else pool.lb(sl)[j] = std::ceil(beta);
                signed char *cs = pool.stat(sl);
                std::memcpy(cs, hso + (size_t)b * S.N, S.N);
                // a fixed bound pair makes a non-basic column NS
                if (cs[m + j] != BS && pool.lb(sl)[j] == pool.ub(sl)[j]) cs[m + j] = NS;
                const NodeRec c{S.round_bound(z + dz[kase]), seq++, sl};
                if (!dived) {
                    next_dive.push_back(c);
                    dived = true;
                } else
                    open.push(c);
                created++;
            }
        }
        for (const NodeRec &nd : bf.nodes) pool.release(nd.slot);
        bf.nodes.clear();
        for (const NodeRec &c : next_dive) dive.push_back(c);
        next_dive.clear();
    };
    auto drain = [&]() {
        for (int k = 0; k < 2; k++) {
            const int sb = (cur + k) & 1;
            if (inflight[sb]) { process(S.bufs[sb]); inflight[sb] = 0; }
        }
    };
    // sharded runs: every rank evaluates the same first
    // batches (deterministic, identical on every GPU) until the frontier holds
    // ramp * size nodes, then keeps the nodes i = rank (mod size) of the
    // frontier in (bound, creation) order; the incumbent value is exchanged
    // every sync_every batches (exchange() is collective: an idle rank keeps
    // calling it until no rank has work left)
    bool split_done = (size == 1), timed_out = false;
    int since_sync = 0;
    for (;;) {
        if (fail_sync) break;
        const bool any_inflight = inflight[0] || inflight[1];
        bool have_work = !open.empty() || !dive.empty() || any_inflight;
        if (have_work && parm->tm_lim < 0x7fffffff &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1000.0 >= parm->tm_lim) {
            timed_out = true;
            drain();
            while (!open.empty()) { pool.release(open.top().slot); open.pop(); }
            for (const NodeRec &d : dive) pool.release(d.slot);
            dive.clear();
            have_work = false;
        }
        if (!split_done) {
            if (!have_work) break;                        // the tree ended during the ramp-up: same on every rank
            if ((long long)open.size() + (long long)dive.size() >= (long long)ramp * size) {
                std::vector<NodeRec> front(dive.begin(), dive.end());
                while (!open.empty()) { front.push_back(open.top()); open.pop(); }
                dive.clear();
                std::sort(front.begin(), front.end(), [](const NodeRec &a, const NodeRec &b) {
                    return a.bound != b.bound ? a.bound < b.bound : a.seq < b.seq;
                });
                for (size_t i = 0; i < front.size(); i++) {
                    if ((int)(i % size) == rank) open.push(front[i]);
                    else pool.release(front[i].slot);
                }
                split_done = true;
                continue;
            }
        }
        if (split_done && size > 1 && (since_sync >= sync_every || !have_work)) {
            double b = best;
            const int active = shard->exchange(shard->info, &b, have_work ? 1 : 0);
            if (b < gbest) gbest = b;
            since_sync = 0;
            if (active == 0) break;
            if (!have_work) continue;
        }
        if (!have_work) break;
        since_sync++;
        // assemble the next batch into the free buffer set
        BatchBuf &bf = S.bufs[cur];
        if (inflight[cur]) { process(bf); inflight[cur] = 0; }
        bf.nodes.clear();
        {
            std::vector<NodeRec> keep;
            for (const NodeRec &nd : dive) {
                if (!hopeful(nd.bound)) { pool.release(nd.slot); continue; }
                if ((int)bf.nodes.size() < BMAX) bf.nodes.push_back(nd);
                else open.push(nd);
            }
            dive.clear();
        }
        while (!open.empty() && (int)bf.nodes.size() < BMAX) {
            const NodeRec nd = open.top();
            open.pop();
            if (!hopeful(nd.bound)) { pool.release(nd.slot); continue; }
            bf.nodes.push_back(nd);
        }
        if (!bf.nodes.empty()) {
            launch(bf);
            inflight[cur] = 1;
        }
        const int prev = cur ^ 1;
        if (depth == 1 || bf.nodes.empty()) {
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
    mip->lp_solves = lp_solves;
    mip->nodes_created = created;
    mip->pivots = pivots;
    if (failed) {
        set_err("gk_ios_driver: %lld node LP(s) could not be solved by the batched kernel", failed);
        return GK_EABI;
    }
    if (have) {
        mip->mip_stat = timed_out ? 2 : 5;                // GLP_FEAS / GLP_OPT
        mip->mip_obj = S.c0 + S.sign * best;
        for (int i = 0; i < m; i++) mip->row_mipx[i + 1] = xbest[i];
        for (int j = 0; j < n; j++)
            mip->col_mipx[j + 1] = S.isint[j] ? std::floor(xbest[m + j] + 0.5) : xbest[m + j];
    } else {
        mip->mip_stat = timed_out ? 1 : 4;                // GLP_UNDEF / GLP_NOFEAS
        mip->mip_obj = 0.0;
    }
    return timed_out ? 0x09 : 0;                          // GLP_ETMLIM
}
