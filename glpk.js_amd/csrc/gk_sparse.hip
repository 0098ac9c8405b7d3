// Sparse basis factor for large sparse LPs (SURVEY.md §8(a) rows luf_* /
// fhv_* / lpf_* / scf_*): B0 = L U by a Markowitz elimination with threshold
// pivoting on the host (the role of luf_factorize, glpluf.js:1105), the
// triangular solves on the device as level-scheduled sweeps (the role of
// luf_f_solve / luf_v_solve, glpluf.js:1227 / :1268), and the updates of the
// basis between refactorizations in Schur-complement form (the reference's
// lpf / scf factor of GLP_BF_BG / GR, glplpf.js:331, glpscf.js:217):
//
//   B_k = B0 + D S'   (S = the unit columns of the k replaced positions,
//                      D = new column - column of B0 at that position)
//   Y   = inv(B0) D = [inv(B0) a_t - e_{p_t}]            (m x k, dense)
//   M   = I + S' Y                                       (k x k, inverse kept)
//   inv(B_k) b  = z - Y (inv(M) z[P]),     z = inv(B0) b
//   inv(B_k)' e = inv(B0)' (e - S inv(M)' (Y' e))
//
// An update is one new (or replaced) column of Y, the inv(B0) a_q the pivot's
// FTRAN already formed, and a bordered / rank-1 update of inv(M): O(m + k^2)
// — no dependent chain over the updates, unlike an eta file or the
// Forrest–Tomlin row eliminations (glpfhv.js:148-447), whose steps each need
// the previous one's result.  k <= nfs_max (<= SP_KMAX) updates, then B0 is
// refactorized, as the reference's LPF_ELIMIT (glplpf.js:359).
//
// Why this shape on the MI355X: the explicit dense inverse the engine uses
// for dense and mid-size LPs (gk_reinvert.hip) costs 8 m^2 bytes and a rank-1
// pass over m x nr entries per pivot; at m = 100,000 that is 80 GB and
// ~10 ms per pivot.  The sparse LU of an LP basis is a few entries per row,
// so a solve is O(nnz(L + U)) traffic; its dependency depth (levels) is what
// bounds it, and each level is one barrier of a single workgroup whose
// working vector stays in the L2.  Basis factor CPU parity is not claimed
// bit-for-bit (the reference's FT-LU rounds differently); the objective,
// statuses and KKT conditions are (tests/test_gpu_sparse.py).
#include "gk_internal.h"
#include "gk_device.h"
#include "gk_hostprof.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace gk {

#define SPCHK(x)                                                                              \
    do {                                                                                      \
        hipError_t e__ = (x);                                                                 \
        if (e__ != hipSuccess) throw std::runtime_error(std::string("sparse factor: ") + #x + \
                                                        ": " + hipGetErrorString(e__));       \
    } while (0)

static double sp_now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

template <typename T>
struct SBuf {
    T *p = nullptr;
    size_t n = 0;
    void ensure(size_t cnt)
    {
        cnt = std::max<size_t>(cnt, 1);
        if (cnt <= n && p) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        SPCHK(hipMalloc((void **)&p, cnt * sizeof(T)));
        n = cnt;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// L U of B0: step k pivots row pr[k] (constraint row) and position pc[k]
struct SpLU {
    int m = 0;
    std::vector<int> pr, pc;
    std::vector<int> Lptr, Lrow;          // eta of step k: multipliers of the rows it eliminated
    std::vector<double> Lval;
    std::vector<int> Uptr, Ucol;          // row of step k without its diagonal (positions)
    std::vector<double> Uval, Udiag;
};

// one triangular sweep in gather form, steps in level order
struct SpTriHost {
    int nlev = 0;
    std::vector<int> lvptr, lvlong, iin, iout, eptr, eidx;   // lvlong[l]: first step of level l with > TRI_LONG entries
    std::vector<double> diag, eval;
    // LDS segments (sp_plan_sweep): entries [eptr[s], emid[s]) read the
    // sweep's vectors (external), [emid[s], eptr[s+1]) the outputs of steps
    // of the same segment, by their index within it (internal); aord: the
    // segment's steps (local indices) for its external pass, the ones of at
    // most TRI_LONG external entries first
    std::vector<int> emid, aord;
    std::vector<int> lvch;                        // level of one step of at most 64 internal entries (a chain link)
    // per step of an LDS segment, its first SP_RECN internal entries as one
    // record (srx: local indices two per int; srn: the internal count; srv:
    // the coefficients, zero-padded; srd: the reciprocal of the diagonal),
    // so that the internal pass loads a level's metadata by step index alone
    std::vector<int> srx, srn;                    // SP_RECN local indices (two per int) / the internal count
    std::vector<double> srv, srd;                 // SP_RECN coefficients / 1 / diag
};

struct SpSolves {
    SpTriHost fl, fu, bu, bl;
};

struct SpTriDevBufs {
    SBuf<int> lvptr, lvlong, iin, iout, eptr, eidx, emid, aord, srx, srn, lvch;
    SBuf<double> diag, eval, srv, srd;
    void release()
    {
        lvptr.release(); lvlong.release(); iin.release(); iout.release(); eptr.release(); eidx.release(); diag.release();
        eval.release(); emid.release(); aord.release(); srx.release(); srv.release(); srn.release(); srd.release();
        lvch.release();
    }
};

struct SpHost;

struct SpFactor {
    int m = -1;
    SpTriDevBufs fl, fu, bu, bl;
    SBuf<double> Y, Minv, zq, tpart, bt, scr, scr2, hh, bz, sacc;   // sacc: an LDS segment's external sums (k_sp_seg_a)
    SBuf<double> upd;                     // k_sp_update's rank-1 factors of inv(M), applied by k_sp_ycol
    SBuf<int> P, hdr;                     // hdr: nlev of fl, fu, bu, bl; k (updates in the chain); Y column of the last update
    long long nnz_l = 0, nnz_u = 0;
    int levels[4] = {0, 0, 0, 0};
    // the launch plan of each sweep (fl, fu, bu, bl): wide levels (>= SP_WIDE
    // steps) as grid launches (k_sp_level), the runs of narrow levels
    // between them in one workgroup (k_sp_sweep); wide[i] = 0: the whole
    // sweep in the fused one-workgroup kernels
    // grid: 1 a wide level on the grid (k_sp_level), 0 a run of narrow
    // levels in k_sp_sweep, 2 an LDS segment (k_sp_seg: steps sb .. sb+ns-1,
    // nas of them short in the external pass; pre: that pass on the grid
    // first, k_sp_seg_a with ablocks blocks)
    struct Seg {
        int grid, l0, l1, blocks;
        int sb = 0, ns = 0, nas = 0, pre = 0, ablocks = 0;
    };
    std::vector<Seg> plan[4];
    int wide[4] = {0, 0, 0, 0};
    SBuf<unsigned long long> stamps;      // GK_SP_STAMPS: 4 x SP_STAMP_MAX level stamps of the last solves
    std::vector<int> lv_host[4];          // (with stamps) the level sizes, for the dump
    double t_lu = 0.0, t_total = 0.0;
    // the pivots of the current chain, in order (p, entering variable), and
    // the look-ahead: the LU of an earlier basis of the chain factorized on
    // a host thread (sp_ahead_start), installed at the next refactorization
    // with the chain's later pivots replayed onto it (sp_ahead_install)
    SBuf<int> plog, prep;
    SBuf<char> rst;                       // the replay's DState (p, kq, refact_pending)
    struct SpHost *cur = nullptr, *nxt = nullptr;
    std::thread ahead;
    int ahead_mark = -1;
    ~SpFactor();
};

constexpr int TRI_LONG = 32;   // sweep steps with more entries run on a whole wave
// a level of at least this many steps runs on the grid (k_sp_level): below
// it the extra launch costs more than the workgroup's trips.  By the factor's
// order m (GK_SP_WIDE overrides): 2,048 for 16,384 <= m < 65,536 (the m =
// 20,020 mid-solve window 2,217 -> 2,351 pivots/s against 4,096), 4,096
// otherwise (m = 100,050: 878 against 818 pivots/s at 2,048; m = 4,005 keeps
// its one-workgroup sweeps)
static int sp_wide_min(int m)
{
    static const int w = [] {
        const char *e = std::getenv("GK_SP_WIDE");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    if (w > 0) return w;
    return (m >= 16384 && m < 65536) ? 2048 : 4096;
}

// ---------------------------------------------------------------------------
// host: Markowitz LU with threshold pivoting
// ---------------------------------------------------------------------------
// The active submatrix is kept by rows (column index, value) and by columns
// (row patterns); rows and columns sit in count buckets.  A pivot is a column
// singleton, else a row singleton, else the candidate of least Markowitz cost
// (r - 1)(c - 1) among the elements passing the threshold |a_ij| >= piv_tol
// max_j |a_ij| in the columns and rows of smallest count (at most piv_lim
// candidates, the search order of luf's find_pivot, glpluf.js:437-628).
// Elimination forms the multipliers of the pivot column (an L eta), updates
// the other rows with fill-in and drops entries below eps_tol
// (eliminate, glpluf.js:637-812); the pivot row goes to U.
namespace {

struct Buckets {
    std::vector<int> head, next, prev, cnt;
    void init(int n, int maxc)
    {
        head.assign(maxc + 2, -1);
        next.assign(n, -1);
        prev.assign(n, -1);
        cnt.assign(n, 0);
    }
    void add(int i, int c)
    {
        cnt[i] = c;
        prev[i] = -1;
        next[i] = head[c];
        if (head[c] >= 0) prev[head[c]] = i;
        head[c] = i;
    }
    void del(int i)
    {
        const int c = cnt[i];
        if (prev[i] >= 0) next[prev[i]] = next[i];
        else head[c] = next[i];
        if (next[i] >= 0) prev[next[i]] = prev[i];
        next[i] = prev[i] = -1;
    }
    void move(int i, int c)
    {
        del(i);
        add(i, c);
    }
};

}  // namespace

// the elimination's working storage, kept from one factorization to the next
// (the per-row / per-column vectors keep their capacity: a factorization of
// m = 100k allocated some 10^6 small vectors otherwise)
struct SpLUWork {
    std::vector<std::vector<int>> rc, cr;
    std::vector<std::vector<double>> rv;
    std::vector<double> rmax;
    std::vector<char> ract, cact;
    std::vector<int> wpos, rows, rsing;
    std::vector<char> cdone;
    Buckets R, C;
    std::vector<int> lid;                  // long rows: their slot in lmap (-1: short)
    std::vector<std::vector<int>> lmap;    // per long row: column -> index in the row (-1: none)
};

// the host products of one factorization (LU, the four sweeps, their
// plans) before they go to the device; the working storage stays with it
struct SpHost {
    SpLU lu;
    SpLUWork wk;
    SpSolves S;
    std::vector<SpFactor::Seg> plan[4];
    int wide[4] = {0, 0, 0, 0};
    int m = 0, ret = 1;
    double t_lu = 0.0;
    std::vector<int> cptr, crow;          // the look-ahead's copy of B's columns
    std::vector<double> cval;
};

SpFactor::~SpFactor()
{
    if (ahead.joinable()) ahead.join();
    delete cur;
    delete nxt;
    fl.release(); fu.release(); bu.release(); bl.release();
    Y.release(); Minv.release(); zq.release(); tpart.release(); bt.release(); scr.release(); scr2.release();
    hh.release(); bz.release(); stamps.release(); sacc.release(); plog.release(); prep.release(); rst.release();
    P.release();
    hdr.release();
}

// rows longer than this keep a dense position map (the linking rows of a
// block-angular basis: every elimination that touches one would rescan it)
constexpr int LU_LONG = 64;

// returns 0, or 1 when B0 is singular (BFD_ESING); rank in *rank
static int sp_lu_factor(SpLU &F, SpLUWork &Wk, int m, const std::vector<int> &cptr, const std::vector<int> &crow,
                 const std::vector<double> &cval, double piv_tol, int piv_lim, double eps_tol, int *rank)
{
    F.m = m;
    F.pr.assign(m, -1);
    F.pc.assign(m, -1);
    F.Lptr.assign(1, 0);
    F.Lrow.clear(); F.Lval.clear();
    F.Uptr.assign(1, 0);
    F.Ucol.clear(); F.Uval.clear(); F.Udiag.assign(m, 0.0);
    std::vector<std::vector<int>> &rc = Wk.rc;     // row i: columns
    std::vector<std::vector<double>> &rv = Wk.rv;  // row i: values
    std::vector<std::vector<int>> &cr = Wk.cr;     // column j: rows
    if ((int)rc.size() < m) { rc.resize(m); rv.resize(m); cr.resize(m); }
    for (int i = 0; i < m; i++) { rc[i].clear(); rv[i].clear(); cr[i].clear(); }
    // the column singletons of B (the slack columns of an LP basis, most of
    // the columns of a late one) pivot first, each on its own row, before
    // the active matrix exists: their rows go to U as they are, their L etas
    // are empty, and the elimination below starts on the rest (the pivots
    // the loop would take first anyway, without its pattern upkeep)
    std::vector<int> &rsing = Wk.rsing;            // row -> its singleton pivot (-1: none)
    rsing.assign(m, -1);
    std::vector<char> &cdone = Wk.cdone;
    cdone.assign(m, 0);
    int k0 = 0;
    for (int j = 0; j < m; j++) {
        int nz = 0, ti = -1;
        for (int t = cptr[j]; t < cptr[j + 1]; t++)
            if (cval[t] != 0.0) { nz++; ti = t; }
        if (nz != 1 || rsing[crow[ti]] >= 0) continue;
        rsing[crow[ti]] = k0;
        cdone[j] = 1;
        F.pr[k0] = crow[ti];
        F.pc[k0] = j;
        F.Udiag[k0] = cval[ti];
        k0++;
    }
    {
        // U rows of the singleton pivots: the other entries of their rows
        std::vector<int> &cnt = Wk.wpos;
        cnt.assign(k0 + 1, 0);
        for (int j = 0; j < m; j++)
            if (!cdone[j])
                for (int t = cptr[j]; t < cptr[j + 1]; t++)
                    if (cval[t] != 0.0 && rsing[crow[t]] >= 0) cnt[rsing[crow[t]] + 1]++;
        for (int q = 0; q < k0; q++) cnt[q + 1] += cnt[q];
        F.Uptr.assign(cnt.begin(), cnt.end());
        F.Ucol.assign(cnt[k0], 0);
        F.Uval.assign(cnt[k0], 0.0);
        for (int j = 0; j < m; j++)
            if (!cdone[j])
                for (int t = cptr[j]; t < cptr[j + 1]; t++) {
                    const int i = crow[t];
                    if (cval[t] == 0.0) continue;
                    if (rsing[i] >= 0) {
                        const int f = cnt[rsing[i]]++;
                        F.Ucol[f] = j;
                        F.Uval[f] = cval[t];
                    } else {
                        rc[i].push_back(j);
                        rv[i].push_back(cval[t]);
                        cr[j].push_back(i);
                    }
                }
        F.Lptr.assign(k0 + 1, 0);
    }
    Buckets &R = Wk.R, &C = Wk.C;
    R.init(m, m);
    C.init(m, m);
    std::vector<int> &lid = Wk.lid;
    std::vector<std::vector<int>> &lmap = Wk.lmap;
    lid.assign(m, -1);
    int nlong = 0;
    auto make_long = [&](int i) {
        if (lid[i] >= 0) return;
        if (nlong == (int)lmap.size()) lmap.emplace_back();
        std::vector<int> &mp = lmap[nlong];
        if ((int)mp.size() != m) mp.assign(m, -1);          // (slots come back all -1)
        lid[i] = nlong++;
        for (size_t t = 0; t < rc[i].size(); t++) mp[rc[i][t]] = (int)t;
    };
    // swap-remove entry t of row i (the map follows)
    auto row_remove = [&](int i, size_t t) {
        const int j = rc[i][t];
        const int last = rc[i].back();
        rc[i][t] = last; rc[i].pop_back();
        rv[i][t] = rv[i].back(); rv[i].pop_back();
        if (lid[i] >= 0) {
            std::vector<int> &mp = lmap[lid[i]];
            mp[j] = -1;
            if (t < rc[i].size()) mp[last] = (int)t;
        }
    };
    for (int i = 0; i < m; i++)
        if ((int)rc[i].size() > LU_LONG) make_long(i);
    for (int i = 0; i < m; i++)
        if (rsing[i] < 0) R.add(i, (int)rc[i].size());
    for (int j = 0; j < m; j++)
        if (!cdone[j]) C.add(j, (int)cr[j].size());
    std::vector<char> &ract = Wk.ract, &cact = Wk.cact;
    ract.assign(m, 1);
    cact.assign(m, 1);
    for (int i = 0; i < m; i++)
        if (rsing[i] >= 0) ract[i] = 0;
    for (int j = 0; j < m; j++)
        if (cdone[j]) cact[j] = 0;
    std::vector<double> &rmax = Wk.rmax;           // cached max |a_ij| of row i (< 0: stale)
    rmax.assign(m, -1.0);
    auto row_max = [&](int i) {
        if (rmax[i] < 0.0) {
            double b = 0.0;
            for (double v : rv[i]) b = std::max(b, std::fabs(v));
            rmax[i] = b;
        }
        return rmax[i];
    };
    auto find_in_row = [&](int i, int j) {
        if (lid[i] >= 0) return lmap[lid[i]][j];
        const std::vector<int> &r = rc[i];
        for (size_t t = 0; t < r.size(); t++)
            if (r[t] == j) return (int)t;
        return -1;
    };
    std::vector<int> &wpos = Wk.wpos;              // column -> index in the row being updated
    wpos.assign(m, -1);
    static const bool tdiag = std::getenv("GK_SP_TIMES") != nullptr;
    double t_search = 0.0, t_elim = 0.0, tt = 0.0;
    long long n_cs = 0, n_rs = 0, n_mk = 0, n_rows = 0, n_upd = 0, n_cand = 0;
    int k;
    n_cs = k0;
    for (k = k0; k < m; k++) {
        if (tdiag) tt = sp_now();
        int pi = -1, pj = -1;
        // column singleton, then row singleton
        if (C.head[1] >= 0) {
            pj = C.head[1];
            pi = cr[pj][0];
            n_cs++;
        } else if (R.head[1] >= 0) {
            pi = R.head[1];
            pj = rc[pi][0];
            n_rs++;
        } else {
            n_mk++;
            long long best = -1;
            double bestv = 0.0;
            int ncand = 0;
            for (int c = 2; c <= m && ncand < piv_lim; c++) {
                for (int j = C.head[c]; j >= 0 && ncand < piv_lim; j = C.next[j]) {
                    for (int i : cr[j]) {
                        const int t = find_in_row(i, j);
                        const double v = std::fabs(rv[i][t]);
                        if (v < piv_tol * row_max(i) || v == 0.0) continue;
                        const long long cost = (long long)(rc[i].size() - 1) * (c - 1);
                        if (best < 0 || cost < best || (cost == best && v > bestv)) {
                            best = cost; bestv = v; pi = i; pj = j;
                        }
                    }
                    ncand++;
                }
                for (int i = R.head[c]; i >= 0 && ncand < piv_lim; i = R.next[i]) {
                    const double big = row_max(i);
                    for (size_t t = 0; t < rc[i].size(); t++) {
                        const double v = std::fabs(rv[i][t]);
                        if (v < piv_tol * big || v == 0.0) continue;
                        const int j = rc[i][t];
                        const long long cost = (long long)(c - 1) * (cr[j].size() - 1);
                        if (best < 0 || cost < best || (cost == best && v > bestv)) {
                            best = cost; bestv = v; pi = i; pj = j;
                        }
                    }
                    ncand++;
                }
                if (best >= 0 && best <= (long long)(c - 1) * (c - 1)) break;
            }
            if (best < 0) {
                // no element passes the threshold: the largest element of
                // any active row (a rank test of the rest)
                double bv = 0.0;
                for (int i = 0; i < m; i++)
                    if (ract[i])
                        for (size_t t = 0; t < rc[i].size(); t++)
                            if (std::fabs(rv[i][t]) > bv) { bv = std::fabs(rv[i][t]); pi = i; pj = rc[i][t]; }
                if (bv == 0.0) break;   // the rest of the active matrix is zero: singular
            }
        }
        if (pi < 0 || pj < 0) break;
        if (tdiag) {
            const double t1 = sp_now();
            t_search += t1 - tt;
            tt = t1;
        }
        // the pivot
        const int tp = find_in_row(pi, pj);
        const double vp = rv[pi][tp];
        if (vp == 0.0) break;
        F.pr[k] = pi;
        F.pc[k] = pj;
        F.Udiag[k] = vp;
        // U row: the pivot row's other entries
        for (size_t t = 0; t < rc[pi].size(); t++)
            if ((int)t != tp) {
                F.Ucol.push_back(rc[pi][t]);
                F.Uval.push_back(rv[pi][t]);
            }
        F.Uptr.push_back((int)F.Ucol.size());
        // the pivot row leaves the column patterns
        for (int j : rc[pi]) {
            std::vector<int> &cj = cr[j];
            for (size_t t = 0; t < cj.size(); t++)
                if (cj[t] == pi) { cj[t] = cj.back(); cj.pop_back(); break; }
            if (j != pj) C.move(j, (int)cj.size());
        }
        R.del(pi);
        ract[pi] = 0;
        // eliminate the pivot column from the other rows
        std::vector<int> &rows = Wk.rows;
        rows.assign(cr[pj].begin(), cr[pj].end());
        C.del(pj);
        cact[pj] = 0;
        cr[pj].clear();
        n_rows += (long long)rows.size();
        n_upd += (long long)rows.size() * (long long)rc[pi].size();
        for (int i : rows) {
            const int ti = find_in_row(i, pj);
            const double f = rv[i][ti] / vp;
            F.Lrow.push_back(i);
            F.Lval.push_back(f);
            // remove a_{i,pj}
            row_remove(i, ti);
            if (lid[i] >= 0) {
                // a long row: its map finds the pivot row's columns; only the
                // entries the update touched can have cancelled
                std::vector<int> &mp = lmap[lid[i]];
                for (size_t t = 0; t < rc[pi].size(); t++) {
                    const int j = rc[pi][t];
                    if (j == pj) continue;
                    const double d = f * rv[pi][t];
                    const int pos = mp[j];
                    if (pos >= 0) rv[i][pos] -= d;
                    else {
                        mp[j] = (int)rc[i].size();
                        rc[i].push_back(j);
                        rv[i].push_back(-d);
                        cr[j].push_back(i);
                        C.move(j, (int)cr[j].size());
                    }
                }
                for (size_t t = 0; t < rc[pi].size(); t++) {
                    const int j = rc[pi][t];
                    if (j == pj) continue;
                    const int pos = mp[j];
                    if (pos < 0 || std::fabs(rv[i][pos]) >= eps_tol) continue;
                    std::vector<int> &cj = cr[j];
                    for (size_t u = 0; u < cj.size(); u++)
                        if (cj[u] == i) { cj[u] = cj.back(); cj.pop_back(); break; }
                    C.move(j, (int)cj.size());
                    row_remove(i, pos);
                }
            } else {
                for (size_t t = 0; t < rc[i].size(); t++) wpos[rc[i][t]] = (int)t;
                for (size_t t = 0; t < rc[pi].size(); t++) {
                    const int j = rc[pi][t];
                    if (j == pj) continue;
                    const double d = f * rv[pi][t];
                    if (wpos[j] >= 0) rv[i][wpos[j]] -= d;
                    else {
                        wpos[j] = (int)rc[i].size();
                        rc[i].push_back(j);
                        rv[i].push_back(-d);
                        cr[j].push_back(i);
                        C.move(j, (int)cr[j].size());
                    }
                }
                // drop what cancelled (|a| < eps_tol)
                for (size_t t = 0; t < rc[i].size();) {
                    if (std::fabs(rv[i][t]) < eps_tol) {
                        const int j = rc[i][t];
                        std::vector<int> &cj = cr[j];
                        for (size_t u = 0; u < cj.size(); u++)
                            if (cj[u] == i) { cj[u] = cj.back(); cj.pop_back(); break; }
                        C.move(j, (int)cj.size());
                        wpos[j] = -1;
                        rc[i][t] = rc[i].back(); rc[i].pop_back();
                        rv[i][t] = rv[i].back(); rv[i].pop_back();
                    } else t++;
                }
                for (int j : rc[i]) wpos[j] = -1;
                if ((int)rc[i].size() > LU_LONG) make_long(i);
            }
            rmax[i] = -1.0;
            R.move(i, (int)rc[i].size());
        }
        F.Lptr.push_back((int)F.Lrow.size());
        if (lid[pi] >= 0)
            for (int j : rc[pi]) lmap[lid[pi]][j] = -1;      // the slot goes back all -1
        rc[pi].clear();
        rv[pi].clear();
        if (tdiag) t_elim += sp_now() - tt;
    }
    if (tdiag)
        fprintf(stderr, "[gk sp times] LU search %.2f ms, elimination %.2f ms; pivots: %lld column / %lld row singletons, "
                "%lld Markowitz; %lld row updates, %lld update entries\n", 1e3 * t_search, 1e3 * t_elim, n_cs, n_rs, n_mk,
                n_rows, n_upd);
    (void)n_cand;
    *rank = k;
    // (singular: rows left active keep entries in their maps)
    for (int i = 0; i < m; i++)
        if (lid[i] >= 0)
            for (int j : rc[i]) lmap[lid[i]][j] = -1;
    if (k < m) return 1;
    return 0;
}

// the four gather-form triangular sweeps of a factor, each in level order
// (a step's level is one more than the deepest step it reads):
//   FTRAN L   z[r_k] = b[r_k] - sum_{t<k, r_k in L_t} l * z[r_t]   (in place)
//   FTRAN U   x[c_k] = (z[r_k] - sum_{(j, u) in U_k} u x[j]) / u_kk
//   BTRAN U'  w[k]   = (e[c_k] - sum_{t<k, c_k in U_t} u w[t]) / u_kk
//   BTRAN L'  y[r_k] = w[k] - sum_{(i, l) in L_k} l y[i]
// the dependences of every step of a sweep, in CSR form (ptr over the
// steps; idx / val the entries read and their coefficients; step the step
// that produces each entry read)
struct SpDeps {
    std::vector<int> ptr, idx, step;
    std::vector<double> val;
};

// inplace: the sweep writes the vector it reads (FTRAN L), so a step with
// no entries, iin = iout and a unit diagonal leaves its entry as it is and is
// dropped from the schedule (most steps of a slack-heavy basis: the
// single-workgroup sweep no longer walks them)
static void sp_build_tri(SpTriHost &T, int nsteps, const std::vector<int> &iin, const std::vector<int> &iout,
                         const std::vector<double> &diag, const SpDeps &D, bool reverse, bool inplace = false)
{
    thread_local std::vector<int> lev, cnt, pos, order;
    lev.assign(nsteps, 0);
    int nlev = 0, nkeep = 0;
    for (int s = 0; s < nsteps; s++) {
        const int k = reverse ? nsteps - 1 - s : s;
        if (inplace && D.ptr[k + 1] == D.ptr[k] && iin[k] == iout[k] && diag[k] == 1.0) {
            lev[k] = -1;
            continue;
        }
        int l = 0;
        for (int e = D.ptr[k]; e < D.ptr[k + 1]; e++) l = std::max(l, lev[D.step[e]] + 1);
        lev[k] = l;
        nlev = std::max(nlev, l + 1);
        nkeep++;
    }
    cnt.assign(nlev + 1, 0);
    for (int k = 0; k < nsteps; k++)
        if (lev[k] >= 0) cnt[lev[k] + 1]++;
    for (int l = 0; l < nlev; l++) cnt[l + 1] += cnt[l];
    T.lvptr.assign(cnt.begin(), cnt.end());
    T.nlev = nlev;
    pos.assign(nlev, 0);
    order.resize(nkeep);
    for (int k = 0; k < nsteps; k++)
        if (lev[k] >= 0) order[T.lvptr[lev[k]] + pos[lev[k]]++] = k;
    nsteps = nkeep;
    // within a level: the steps of at most TRI_LONG entries (one thread each)
    // first, the longer ones (one wave each) after them
    T.lvlong.assign(nlev, 0);
    for (int l = 0; l < nlev; l++) {
        auto b = order.begin() + T.lvptr[l], e = order.begin() + T.lvptr[l + 1];
        auto mid = std::stable_partition(b, e, [&](int k) { return D.ptr[k + 1] - D.ptr[k] <= TRI_LONG; });
        T.lvlong[l] = (int)(mid - order.begin());
    }
    static const bool lvlog = std::getenv("GK_SP_LEVELS") != nullptr;
    if (lvlog) {
        std::string line = "[gk sp levels]";
        long long tot = 0;
        for (int l = 0; l < nlev; l++) {
            long long ent = 0;
            for (int q = T.lvptr[l]; q < T.lvptr[l + 1]; q++) ent += D.ptr[order[q] + 1] - D.ptr[order[q]];
            tot += ent;
            line += " " + std::to_string(T.lvptr[l + 1] - T.lvptr[l]) + "/" + std::to_string(ent) + "/" +
                    std::to_string(T.lvptr[l + 1] - T.lvlong[l]);
        }
        fprintf(stderr, "%s (steps/entries/long per level; %lld entries)\n", line.c_str(), tot);
    }
    T.iin.resize(nsteps); T.iout.resize(nsteps); T.diag.resize(nsteps); T.eptr.assign(nsteps + 1, 0);
    T.eidx.resize(D.idx.size()); T.eval.resize(D.idx.size());
    int ne = 0;
    for (int s = 0; s < nsteps; s++) {
        const int k = order[s];
        T.iin[s] = iin[k];
        T.iout[s] = iout[k];
        T.diag[s] = diag[k];
        for (int e = D.ptr[k]; e < D.ptr[k + 1]; e++) {
            T.eidx[ne] = D.idx[e];
            T.eval[ne] = D.val[e];
            ne++;
        }
        T.eptr[s + 1] = ne;
    }
}

// the transposed dependences (a step reads the entries other steps' lists
// point at): for src = 0..m-1 in order, every entry e of src's list goes to
// the step key(e), recording (idx(src), val[e], src) — the same order as
// pushing them one by one
template <typename Key, typename Idx>
static void sp_deps_transposed(SpDeps &D, int m, const std::vector<int> &sptr, const std::vector<double> &sval,
                               Key key, Idx idx)
{
    D.ptr.assign(m + 1, 0);
    for (int t = 0; t < m; t++)
        for (int e = sptr[t]; e < sptr[t + 1]; e++) D.ptr[key(e) + 1]++;
    for (int k = 0; k < m; k++) D.ptr[k + 1] += D.ptr[k];
    const size_t nz = (size_t)D.ptr[m];
    D.idx.resize(nz); D.val.resize(nz); D.step.resize(nz);
    thread_local std::vector<int> fill;
    fill.assign(D.ptr.begin(), D.ptr.end() - 1);
    for (int t = 0; t < m; t++)
        for (int e = sptr[t]; e < sptr[t + 1]; e++) {
            const int k = key(e), f = fill[k]++;
            D.idx[f] = idx(t);
            D.val[f] = sval[e];
            D.step[f] = t;
        }
}

// the direct dependences (a step reads its own list)
template <typename Idx, typename Step>
static void sp_deps_direct(SpDeps &D, int m, const std::vector<int> &sptr, const std::vector<int> &sidx,
                           const std::vector<double> &sval, Idx idx, Step step)
{
    D.ptr.assign(sptr.begin(), sptr.begin() + m + 1);
    const size_t nz = (size_t)sptr[m];
    D.idx.resize(nz); D.val.resize(nz); D.step.resize(nz);
    for (size_t e = 0; e < nz; e++) {
        D.idx[e] = idx(sidx[e]);
        D.val[e] = sval[e];
        D.step[e] = step(sidx[e]);
    }
}

static void sp_plan_sweep(SpTriHost &T, std::vector<SpFactor::Seg> &plan, int &wide, int m);

// the four sweeps and their launch plans, one host thread each
static void sp_build_solves(const SpLU &F, SpSolves &S, std::vector<SpFactor::Seg> *plan, int *wide)
{
    const int m = F.m;
    std::vector<int> step_of_row(m), step_of_pos(m);
    for (int k = 0; k < m; k++) { step_of_row[F.pr[k]] = k; step_of_pos[F.pc[k]] = k; }
    auto sweep = [&](int which) {
        thread_local std::vector<int> in, out;
        thread_local std::vector<double> ones;
        thread_local SpDeps D;
        in.resize(m);
        out.resize(m);
        switch (which) {
        case 0:
            // FTRAN L: deps of step k' = (z index r_t, l) for every eta t < k' holding row r_k'
            sp_deps_transposed(D, m, F.Lptr, F.Lval, [&](int e) { return step_of_row[F.Lrow[e]]; },
                               [&](int t) { return F.pr[t]; });
            for (int k = 0; k < m; k++) in[k] = F.pr[k];
            ones.assign(m, 1.0);
            sp_build_tri(S.fl, m, in, in, ones, D, false, true);
            sp_plan_sweep(S.fl, plan[0], wide[0], m);
            break;
        case 1:
            // FTRAN U: deps of step k = (x index c_t, u) for the entries of U row k
            sp_deps_direct(D, m, F.Uptr, F.Ucol, F.Uval, [](int c) { return c; },
                           [&](int c) { return step_of_pos[c]; });
            for (int k = 0; k < m; k++) { in[k] = F.pr[k]; out[k] = F.pc[k]; }
            sp_build_tri(S.fu, m, in, out, F.Udiag, D, true);
            sp_plan_sweep(S.fu, plan[1], wide[1], m);
            break;
        case 2:
            // BTRAN U': deps of step k = (w index t, u) for every U row t < k holding column c_k
            sp_deps_transposed(D, m, F.Uptr, F.Uval, [&](int e) { return step_of_pos[F.Ucol[e]]; },
                               [](int t) { return t; });
            for (int k = 0; k < m; k++) { in[k] = F.pc[k]; out[k] = k; }
            sp_build_tri(S.bu, m, in, out, F.Udiag, D, false);
            sp_plan_sweep(S.bu, plan[2], wide[2], m);
            break;
        default:
            // BTRAN L': deps of step k = (y index i, l) for the entries of eta k
            sp_deps_direct(D, m, F.Lptr, F.Lrow, F.Lval, [](int i) { return i; },
                           [&](int i) { return step_of_row[i]; });
            for (int k = 0; k < m; k++) { in[k] = k; out[k] = F.pr[k]; }
            ones.assign(m, 1.0);
            sp_build_tri(S.bl, m, in, out, ones, D, true);
            sp_plan_sweep(S.bl, plan[3], wide[3], m);
            break;
        }
    };
    static const bool lvlog = std::getenv("GK_SP_LEVELS") != nullptr;   // (its lines in sweep order)
    if (m < 4096 || lvlog) {
        for (int w = 0; w < 4; w++) sweep(w);
        return;
    }
    std::thread th[3];
    for (int w = 1; w < 4; w++) th[w - 1] = std::thread(sweep, w);
    sweep(0);
    for (auto &t : th) t.join();
}

// ---------------------------------------------------------------------------
// LDS segments.  A run of narrow levels costs one barrier per level in the
// single workgroup, and on the m = 100k late basis about 6 us of it is the
// trip to the L2 for the entries the level gathers from the level before.
// A segment of consecutive narrow levels (at most SP_SEG_MAX steps) is
// solved in two passes instead: the external pass sums, for every step at
// once, the entries that read values produced before the segment (one
// parallel gather, on the grid when it is large); the internal pass then
// walks the segment's levels with the segment's own outputs in LDS — a level
// is LDS reads and a barrier, its metadata loaded a level ahead.
// ---------------------------------------------------------------------------
constexpr int SP_SEG_MAX = 8192;
constexpr int SP_SEG_LEVELS = 256;                // levels per LDS segment
// internal entries per step record: 8 measured slower (k_sp_seg<2> spilled
// at 128 VGPRs with two records in flight per thread)
constexpr int SP_RECN = 4;

static bool sp_seg_on()
{
    static const bool on = [] {
        const char *e = std::getenv("GK_SP_SEG");
        return !e || atoi(e) != 0;
    }();
    return on;
}

// GK_SP_LDS=0: the small factors' fused sweeps keep their outputs in global
// memory (the round-5 layout before lds_sweep)
static bool sp_lds_on()
{
    static const bool on = [] {
        const char *e = std::getenv("GK_SP_LDS");
        return !e || atoi(e) != 0;
    }();
    return on;
}

// entries from which a level runs on the grid (with LDS segments; a level
// of many steps, sp_wide_min, does in any case)
static int sp_wide_entries()
{
    static const int w = [] {
        const char *e = std::getenv("GK_SP_WIDE_E");
        return e ? std::max(1, atoi(e)) : 8192;
    }();
    return w;
}

// external entries from which a segment's external pass runs on the grid
// (2,048; 8,192 before round 6: m = 20,020 window +6 %, m = 100,050 +5 %)
static int sp_ga_min()
{
    static const int g = [] {
        const char *e = std::getenv("GK_SP_GA");
        return e ? std::max(0, atoi(e)) : 2048;
    }();
    return g;
}

// the launch plan of one sweep, and the re-encoding of its LDS segments:
// within a segment's levels the steps of at most TRI_LONG internal entries
// first, every step's external entries before its internal ones (each class
// in its original order), internal entries by the producing step's index in
// the segment.  wide: 1 when the sweep runs by its plan (not the fused
// one-workgroup kernels)
static void sp_plan_sweep(SpTriHost &T, std::vector<SpFactor::Seg> &plan, int &wide, int m)
{
    plan.clear();
    wide = 0;
    const int nlev = T.nlev, nst = nlev ? T.lvptr[nlev] : 0;
    // LDS segments for the large factors: a sweep with a level of
    // sp_wide_min steps or more, or of many steps in all; a small one keeps
    // the fused one-workgroup kernels (one launch per sweep pair)
    static const int seg_min = [] {                  // GK_SP_SEG_MIN: steps from which a sweep is segmented
        const char *e = std::getenv("GK_SP_SEG_MIN");
        return e ? std::max(1, atoi(e)) : 4096;    // (16384 before round 6: m = 20k FTRAN L +4 %)
    }();
    bool big = nst >= seg_min;
    for (int l = 0; l < nlev && !big; l++) big = T.lvptr[l + 1] - T.lvptr[l] >= sp_wide_min(m);
    const bool seg = sp_seg_on() && big;
    int run = -1;                            // first level of the current narrow run
    // a tail level: a few long steps (the linking rows of a block-angular
    // basis, one per level at the end of FTRAN L); a segment holds tail
    // levels or none, so that a tail step's entries into the levels before
    // the tail are external (the grid gathers them) and only the dense
    // triangle among the tail steps stays internal
    auto tail = [&](int l) {
        const int ns = T.lvptr[l + 1] - T.lvptr[l];
        return ns <= 16 && T.eptr[T.lvptr[l + 1]] - T.eptr[T.lvptr[l]] >= 512 * ns;
    };
    auto close_run = [&](int l1) {
        if (run < 0) return;
        if (!seg) plan.push_back({0, run, l1, 1});
        else
            for (int a = run; a < l1;) {     // greedy: levels while the steps fit
                int b = a + 1;
                while (b < l1 && b - a < SP_SEG_LEVELS && T.lvptr[b + 1] - T.lvptr[a] <= SP_SEG_MAX &&
                       tail(b) == tail(a))
                    b++;
                SpFactor::Seg g{2, a, b, 1};
                g.sb = T.lvptr[a];
                g.ns = T.lvptr[b] - T.lvptr[a];
                plan.push_back(g);
                a = b;
            }
        run = -1;
    };
    for (int l = 0; l < nlev; l++) {
        const int nshort = T.lvlong[l] - T.lvptr[l], nlong = T.lvptr[l + 1] - T.lvlong[l];
        const int nent = T.eptr[T.lvptr[l + 1]] - T.eptr[T.lvptr[l]];
        // (a level of a few long steps stays narrow: its entries into the
        // levels before go to its segment's external pass)
        if (nshort + nlong >= sp_wide_min(m) || (seg && nent >= sp_wide_entries() && nshort + nlong >= 64)) {
            close_run(l);
            plan.push_back({1, l, l + 1, std::max(1, (nshort + 255) / 256 + nlong)});   // (k_sp_level: a long step a block)
            wide = 1;
        } else if (run < 0)
            run = l;
    }
    close_run(nlev);
    T.emid.assign(T.eptr.begin() + 1, T.eptr.end());
    T.aord.assign(std::max(nst, 1), 0);
    if (!seg) return;
    wide = 1;
    // producing step of every index the sweep writes; segment of every step
    int M = 0;
    for (int s = 0; s < nst; s++) M = std::max(M, T.iout[s] + 1);
    for (int x : T.eidx) M = std::max(M, x + 1);
    std::vector<int> prod(M, -1), segof(nst, -1), nint(nst, 0), next(nst, 0), order(nst), newpos(nst);
    for (int s = 0; s < nst; s++) prod[T.iout[s]] = s;
    for (size_t g = 0; g < plan.size(); g++)
        if (plan[g].grid == 2)
            for (int s = plan[g].sb; s < plan[g].sb + plan[g].ns; s++) segof[s] = (int)g;
    auto internal = [&](int s, int e) {
        const int p = prod[T.eidx[e]];
        return segof[s] >= 0 && p >= 0 && segof[p] == segof[s];
    };
    for (int s = 0; s < nst; s++)
        for (int e = T.eptr[s]; e < T.eptr[s + 1]; e++) {
            if (internal(s, e)) nint[s]++;
            else next[s]++;
        }
    for (int s = 0; s < nst; s++) order[s] = s;
    for (const auto &g : plan)
        if (g.grid == 2)
            for (int l = g.l0; l < g.l1; l++) {
                auto b = order.begin() + T.lvptr[l], e = order.begin() + T.lvptr[l + 1];
                auto mid = std::stable_partition(b, e, [&](int k) { return nint[k] <= TRI_LONG; });
                T.lvlong[l] = (int)(mid - order.begin());
            }
    for (int s = 0; s < nst; s++) newpos[order[s]] = s;
    SpTriHost R;
    R.iin.resize(nst); R.iout.resize(nst); R.diag.resize(nst); R.eptr.assign(nst + 1, 0); R.emid.assign(nst, 0);
    R.eidx.resize(T.eidx.size()); R.eval.resize(T.eval.size());
    int ne = 0;
    for (int s = 0; s < nst; s++) {
        const int k = order[s];
        R.iin[s] = T.iin[k]; R.iout[s] = T.iout[k]; R.diag[s] = T.diag[k];
        for (int pass = 0; pass < 2; pass++) {
            for (int e = T.eptr[k]; e < T.eptr[k + 1]; e++) {
                const bool in = internal(k, e);
                if (in != (pass == 1)) continue;
                R.eidx[ne] = in ? newpos[prod[T.eidx[e]]] - plan[segof[k]].sb : T.eidx[e];
                R.eval[ne] = T.eval[e];
                ne++;
            }
            if (pass == 0) R.emid[s] = ne;
        }
        R.eptr[s + 1] = ne;
    }
    T.iin.swap(R.iin); T.iout.swap(R.iout); T.diag.swap(R.diag); T.eptr.swap(R.eptr); T.emid.swap(R.emid);
    T.eidx.swap(R.eidx); T.eval.swap(R.eval);
    for (auto &g : plan) {
        if (g.grid != 2) continue;
        int nas = 0;
        long long ext = 0;
        for (int i = 0; i < g.ns; i++) {
            const int s = g.sb + i, x = T.emid[s] - T.eptr[s];
            ext += x;
            if (x <= TRI_LONG) T.aord[g.sb + nas++] = i;
        }
        g.nas = nas;
        for (int i = 0, t = nas; i < g.ns; i++)
            if (T.emid[g.sb + i] - T.eptr[g.sb + i] > TRI_LONG) T.aord[g.sb + t++] = i;
        g.pre = ext >= sp_ga_min();
        g.ablocks = std::max(1, (nas + 255) / 256 + (g.ns - nas));      // (k_sp_seg_a: a long step a block)
    }
    T.lvch.assign(std::max(nlev, 1), 0);
    for (const auto &g : plan)
        if (g.grid == 2)
            for (int l = g.l0; l < g.l1; l++)
                T.lvch[l] = T.lvptr[l + 1] - T.lvptr[l] == 1 && T.eptr[T.lvptr[l] + 1] - T.emid[T.lvptr[l]] <= 64;
    T.srx.assign((size_t)(SP_RECN / 2) * std::max(nst, 1), 0);
    T.srn.assign(std::max(nst, 1), 0);
    T.srv.assign((size_t)SP_RECN * std::max(nst, 1), 0.0);
    T.srd.assign(std::max(nst, 1), 1.0);
    for (const auto &g : plan) {
        if (g.grid != 2) continue;
        for (int st = g.sb; st < g.sb + g.ns; st++) {
            const int eb = T.emid[st], n = T.eptr[st + 1] - eb;
            int ix[SP_RECN] = {};
            for (int u = 0; u < SP_RECN && u < n; u++) {
                ix[u] = T.eidx[eb + u];
                T.srv[(size_t)SP_RECN * st + u] = T.eval[eb + u];
            }
            for (int u = 0; u < SP_RECN / 2; u++) T.srx[(size_t)(SP_RECN / 2) * st + u] = ix[2 * u] | (ix[2 * u + 1] << 16);
            T.srn[st] = n;
            T.srd[st] = 1.0 / T.diag[st];
        }
    }
}

// ---------------------------------------------------------------------------
// device: level-scheduled sweeps (one workgroup; each level is one barrier,
// the vectors stay in L2), two right-hand sides at once for the pivot FTRAN
// ---------------------------------------------------------------------------
struct TriDev {
    const int *lvptr, *lvlong, *iin, *iout, *eptr, *eidx, *emid, *aord;
    const double *diag, *eval;
    const int *nlev;                              // device word: levels of the current factor
    unsigned long long *stamps;                   // GK_SP_STAMPS: device clock after each level (null: off)
    const int *lvch;                              // LDS segments: chain-link levels (SpTriHost::lvch)
    const int2 *srx;                              // LDS segments: step records (SpTriHost::srx / srn / srv / srd)
    const int *srn;
    const double2 *srv;
    const double *srd;
};
constexpr int SP_STAMP_MAX = 2048;                // levels stamped per sweep

// a -= sum over entries [eb, ee) of val[e] x[idx[e]], eight entries per
// trip: the index / value loads of a group are issued together (clamped
// into the range, so unconditional), then its gathers, then the products in
// entry order (a dropped entry subtracts 0).  A loop of one entry per
// iteration waited for each entry's own loads: one L2 round trip per entry
template <int NRHS, typename Get>
__device__ __forceinline__ void gather_sub8(const int *eidx, const double *eval, int eb, int ee, Get get, double &a0,
                                            double &a1)
{
    for (int e = eb; e < ee; e += 8) {
        int ix[8];
        double v[8], x0[8], x1[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int ec = min(e + u, ee - 1);
            ix[u] = eidx[ec];
            const double w = eval[ec];
            v[u] = (e + u < ee) ? w : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) get(ix[u], x0[u], x1[u]);
#pragma unroll
        for (int u = 0; u < 8; u++) {
            a0 -= v[u] * x0[u];
            if (NRHS == 2) a1 -= v[u] * x1[u];
        }
    }
}

// a wave's partial sums of val[e] x[idx[e]] over [eb, ee): each lane takes
// entries lane, lane + 64, ... four per trip (clamped, unconditional loads)
template <int NRHS, typename Get>
__device__ __forceinline__ void wave_dot4(const int *eidx, const double *eval, int eb, int ee, Get get, double &p0,
                                          double &p1)
{
    for (int e = eb + (int)(threadIdx.x & 63); e < ee; e += 256) {
        int ix[4];
        double v[4], x0[4], x1[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int ec = min(e + 64 * u, ee - 1);
            ix[u] = eidx[ec];
            const double w = eval[ec];
            v[u] = (e + 64 * u < ee) ? w : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) get(ix[u], x0[u], x1[u]);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            p0 += v[u] * x0[u];
            if (NRHS == 2) p1 += v[u] * x1[u];
        }
    }
}

// a long step's sum of val[e] x[idx[e]] over [eb, ee) by a whole block of
// 256 (four entries per thread per trip), reduced in a fixed order (wave
// sums, then the four waves in order); thread 0 returns it
template <int NRHS, typename Get>
__device__ __forceinline__ void block_dot4(const int *eidx, const double *eval, int eb, int ee, Get get, double &s0,
                                           double &s1)
{
    __shared__ double red[2][4];
    double p0 = 0.0, p1 = 0.0;
    for (int e = eb + (int)threadIdx.x; e < ee; e += 1024) {
        int ix[4];
        double v[4], x0[4], x1[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int ec = min(e + 256 * u, ee - 1);
            ix[u] = eidx[ec];
            const double w = eval[ec];
            v[u] = (e + 256 * u < ee) ? w : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) get(ix[u], x0[u], x1[u]);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            p0 += v[u] * x0[u];
            if (NRHS == 2) p1 += v[u] * x1[u];
        }
    }
    p0 = wsum(p0);
    if (NRHS == 2) p1 = wsum(p1);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = p0;
        red[1][w] = p1;
    }
    __syncthreads();
    s0 = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    s1 = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
}

// one step of a sweep: its metadata and right-hand side(s) do not depend on
// the sweep's own output, so they are loaded one level ahead (before the
// barrier that ends the previous level); after the barrier a level costs
// one trip — the gathers of the entries it reads — and its stores
template <int NRHS>
struct StepPre {
    int s, iout, eb, ee;
    double a0, a1, dg;
    int ix[4];
    double v[4];
};

template <int NRHS>
__device__ __forceinline__ void step_load(const TriDev &t, const double *in0, const double *in1, int s, int lim,
                                          StepPre<NRHS> &q)
{
    q.s = s;
    if (s >= lim) return;
    const int ii = t.iin[s];
    q.iout = t.iout[s];
    q.eb = t.eptr[s];
    q.ee = t.eptr[s + 1];
    q.dg = t.diag[s];
    q.a0 = in0[ii];
    q.a1 = (NRHS == 2) ? in1[ii] : 0.0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const bool ok = q.eb + u < q.ee;
        q.ix[u] = ok ? t.eidx[q.eb + u] : 0;
        q.v[u] = ok ? t.eval[q.eb + u] : 0.0;
    }
}

template <int NRHS>
__device__ __forceinline__ void step_run(const TriDev &t, const StepPre<NRHS> &q, double *out0, double *out1)
{
    double a0 = q.a0, a1 = q.a1;
    double x0[4], x1[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const bool ok = q.eb + u < q.ee;
        x0[u] = ok ? out0[q.ix[u]] : 0.0;
        x1[u] = (NRHS == 2 && ok) ? out1[q.ix[u]] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        a0 -= q.v[u] * x0[u];
        if (NRHS == 2) a1 -= q.v[u] * x1[u];
    }
    if (q.ee > q.eb + 4)
        gather_sub8<NRHS>(t.eidx, t.eval, q.eb + 4, q.ee, [&](int ix, double &x0, double &x1) {
            x0 = out0[ix];
            x1 = (NRHS == 2) ? out1[ix] : 0.0;
        }, a0, a1);
    out0[q.iout] = a0 / q.dg;
    if (NRHS == 2) out1[q.iout] = a1 / q.dg;
}

// a step of more than TRI_LONG entries: the calling wave strides them and
// reduces in a fixed order (deterministic), lane 0 stores
template <int NRHS>
__device__ __forceinline__ void step_wave(const TriDev &t, const double *in0, const double *in1, int s, double *out0,
                                          double *out1)
{
    const int lane = threadIdx.x & 63;
    const int ii = t.iin[s], io = t.iout[s], eb = t.eptr[s], ee = t.eptr[s + 1];
    const double dg = t.diag[s];
    const double b0 = in0[ii], b1 = (NRHS == 2) ? in1[ii] : 0.0;
    double a0 = 0.0, a1 = 0.0;
    (void)lane;
    wave_dot4<NRHS>(t.eidx, t.eval, eb, ee, [&](int ix, double &x0, double &x1) {
        x0 = out0[ix];
        x1 = (NRHS == 2) ? out1[ix] : 0.0;
    }, a0, a1);
    a0 = wsum(a0);
    if (NRHS == 2) a1 = wsum(a1);
    if (lane == 0) {
        out0[io] = (b0 - a0) / dg;
        if (NRHS == 2) out1[io] = (b1 - a1) / dg;
    }
}

// levels l0 .. nlev-1 (l0 = 1: level 0 ran on the whole grid, k_sp_level0)
// a level of few long steps, split over the workgroup's waves: this
// thread's first LPF entries of its step and (the step's leader) the step's
// metadata and right-hand side — none depends on the sweep's output, so they
// are loaded a level ahead like the short steps' (StepPre)
constexpr int LPF = 4;
template <int NRHS>
struct LongPre {
    int split, eb, ee, ii, io;
    double dg, a0, a1;
    int ix[LPF];
    double v[LPF];
};

template <int NRHS>
__device__ __forceinline__ void long_load(const TriDev &t, const double *in0, const double *in1, int ls, int le,
                                          LongPre<NRHS> &q)
{
    const int nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nl = le - ls;
    q.split = nl > 0 && 4 * nl <= nw;
    q.eb = q.ee = 0;
    if (!q.split) return;
    const int g = nw / nl, sidx = w / g, sub = w % g;
    if (sidx >= nl) return;
    q.eb = t.eptr[ls + sidx];
    q.ee = t.eptr[ls + sidx + 1];
#pragma unroll
    for (int u = 0; u < LPF; u++) {
        const int e = q.eb + (sub + u * g) * 64 + lane;
        const bool ok = e < q.ee;
        q.ix[u] = ok ? t.eidx[e] : 0;
        q.v[u] = ok ? t.eval[e] : 0.0;
    }
    if (sub == 0 && lane == 0) {
        q.ii = t.iin[ls + sidx];
        q.io = t.iout[ls + sidx];
        q.dg = t.diag[ls + sidx];
        q.a0 = in0[q.ii];
        q.a1 = (NRHS == 2) ? in1[q.ii] : 0.0;
    }
}

template <int NRHS>
__device__ void tri_sweep(const TriDev &t, const double *in0, const double *in1, double *out0, double *out1,
                          int l0 = 0, int l1 = -1)
{
    const int nlev = (l1 < 0) ? *t.nlev : l1;
    const int T = blockDim.x;
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __shared__ double red[2][16];
    if (nlev <= l0) return;
    int lb = t.lvptr[l0], le = t.lvptr[l0 + 1], ls = t.lvlong[l0];
    StepPre<NRHS> cur;
    step_load<NRHS>(t, in0, in1, lb + (int)threadIdx.x, ls, cur);
    LongPre<NRHS> lcur;
    long_load<NRHS>(t, in0, in1, ls, le, lcur);
    if (t.stamps && threadIdx.x == 0 && l0 < SP_STAMP_MAX) t.stamps[l0] = wall_clock64();
    for (int l = l0; l < nlev; l++) {
        // the next level's bounds and this thread's first (short) step of it
        const int nb = le, ne = (l + 1 < nlev) ? t.lvptr[l + 2] : le, nls = (l + 1 < nlev) ? t.lvlong[l + 1] : le;
        StepPre<NRHS> nxt;
        step_load<NRHS>(t, in0, in1, nb + (int)threadIdx.x, nls, nxt);
        LongPre<NRHS> lnxt;
        long_load<NRHS>(t, in0, in1, nls, ne, lnxt);
        if (cur.s < ls) step_run<NRHS>(t, cur, out0, out1);
        for (int s = cur.s + T; s < ls; s += T) {          // short steps beyond one per thread
            StepPre<NRHS> q;
            step_load<NRHS>(t, in0, in1, s, ls, q);
            step_run<NRHS>(t, q, out0, out1);
        }
        const int nl = le - ls;
        if (lcur.split) {
            // few long steps (a linking row's L step gathers thousands of
            // entries, alone on its level): nw / nl waves per step, their
            // partials summed in wave order by the step's first wave; the
            // first LPF entries per lane and the step's data came a level ahead
            const int g = nw / nl, sidx = w / g, sub = w % g;
            const int lane = threadIdx.x & 63;
            double a0 = 0.0, a1 = 0.0;
            const int eb = lcur.eb, ee = lcur.ee;
            if (sidx < nl) {
                double x0[LPF], x1[LPF];
#pragma unroll
                for (int u = 0; u < LPF; u++) {
                    const bool ok = eb + (sub + u * g) * 64 + lane < ee;
                    x0[u] = ok ? out0[lcur.ix[u]] : 0.0;
                    x1[u] = (NRHS == 2 && ok) ? out1[lcur.ix[u]] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < LPF; u++) {
                    a0 += lcur.v[u] * x0[u];
                    if (NRHS == 2) a1 += lcur.v[u] * x1[u];
                }
                for (int e = eb + (sub + LPF * g) * 64 + lane; e < ee; e += g * 64) {
                    const int ix = t.eidx[e];
                    a0 += t.eval[e] * out0[ix];
                    if (NRHS == 2) a1 += t.eval[e] * out1[ix];
                }
            }
            a0 = wsum(a0);
            if (NRHS == 2) a1 = wsum(a1);
            if (lane == 0) {
                red[0][w] = a0;
                red[1][w] = a1;
            }
            __syncthreads();
            if (sidx < nl && sub == 0 && lane == 0) {
                double s0 = 0.0, s1 = 0.0;
                for (int u = 0; u < g; u++) {
                    s0 += red[0][w + u];
                    s1 += red[1][w + u];
                }
                out0[lcur.io] = (lcur.a0 - s0) / lcur.dg;
                if (NRHS == 2) out1[lcur.io] = (lcur.a1 - s1) / lcur.dg;
            }
        } else
            for (int s = ls + w; s < le; s += nw) step_wave<NRHS>(t, in0, in1, s, out0, out1);
        __syncthreads();
        if (t.stamps && threadIdx.x == 0 && l + 1 < SP_STAMP_MAX) t.stamps[l + 1] = wall_clock64();
        cur = nxt;
        lcur = lnxt;
        lb = nb;
        le = ne;
        ls = nls;
    }
    (void)lb;
}

struct WoodDev {
    double *Y;                                    // m x SP_KMAX, row-major by position
    int *P;                                       // replaced positions (0-based)
    double *Minv;                                 // SP_KMAX x SP_KMAX, row-major
    int *k;                                       // device word: updates in the chain
    double *zq;                                   // inv(B0) h of the last pivot's FTRAN
    double *tpart;                                // Y' e partials of a general BTRAN (SP_KMAX per block)
    double *bt;                                   // BTRAN scratch (positions), FTRAN scratch z (2 x m)
    double *scr2;                                 // BTRAN step-space scratch (2 x m)
    double *hh;                                   // inv(M) z[P] of the FTRAN (2 x SP_KMAX)
    int *ycol;                                    // device word: Y column the last update wrote (-1: none)
    double *bz;                                   // e_p of the pivot's BTRAN (m; zero between uses)
    int *log, *nlog;                              // the chain's pivots (p, kq) and their count
    double *upd;                                  // inv(M)'s rank-1 update: a (SP_KMAX) | r (SP_KMAX) | divisor | sign
    int *nupd;                                    // device word: its order (0: none this pivot)
};

struct SpDev {
    TriDev fl, fu, bu, bl;
    WoodDev w;
    int m;
};

// gate of the pivot's kernels: 0 none, 1 the stop word, 2 stop or no
// leaving row (the BTRAN of e_p)
__device__ __forceinline__ bool sp_gated(const DState *st, int gate)
{
    return gate && (st->stop || (gate == 2 && st->p <= 0));
}

// level 0 of a sweep on the whole grid: its steps read no other step's
// output, so a level of SP_WIDE or more steps (the slack part of the basis)
// runs as a gather at HBM rate instead of m / 1024 dependent trips of the
// single workgroup; the workgroup's sweep then starts at level 1
template <int NRHS>
__global__ void __launch_bounds__(256) k_sp_level(TriDev t, const DState *st, int gate, const double *in0,
                                                  const double *in1, double *out0, double *out1, int l)
{
    if (sp_gated(st, gate)) return;
    const int lb = t.lvptr[l], ls = t.lvlong[l], le = t.lvptr[l + 1];
    const int nsb = (ls - lb + 255) / 256;                 // blocks of the short steps
    if ((int)blockIdx.x < nsb) {
        const int g = blockIdx.x * blockDim.x + threadIdx.x;
        if (lb + g < ls) {
            StepPre<NRHS> q;
            step_load<NRHS>(t, in0, in1, lb + g, ls, q);
            step_run<NRHS>(t, q, out0, out1);
        }
        return;
    }
    // a long step a block (blockDim 256)
    const int s = ls + (int)blockIdx.x - nsb;
    if (s >= le) return;
    double a0, a1;
    block_dot4<NRHS>(t.eidx, t.eval, t.eptr[s], t.eptr[s + 1], [&](int ix, double &x0, double &x1) {
        x0 = out0[ix];
        x1 = (NRHS == 2) ? out1[ix] : 0.0;
    }, a0, a1);
    if (threadIdx.x == 0) {
        const int ii = t.iin[s], io = t.iout[s];
        const double dg = t.diag[s];
        out0[io] = (in0[ii] - a0) / dg;
        if (NRHS == 2) out1[io] = (in1[ii] - a1) / dg;
    }
}

template <int NRHS>
__device__ void ftran_hh(const SpDev &sp);

// FTRAN part 1 (one workgroup): z = inv(B0) [h, work]; L in place, U into
// the scratch; the z of h is kept (zq) for the update of this pivot.
// parts: bit 0 the L sweep (from level l0l), bit 1 the U sweep (from l0u)
// a small factor's sweep with its output vector in LDS (lds_sweep): the
// output copied in (an in-place sweep reads the entries no step writes),
// the levels' gathers from LDS instead of the L2, the vector copied back
// after the last level.  The same arithmetic in the same order.
extern __shared__ double sp_lds[];
template <int NRHS>
__device__ void lds_sweep(const TriDev &t, int m, const double *in0, const double *in1, double *out0, double *out1,
                          double *s0, int l0)
{
    double *s1 = s0 + m;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        s0[i] = out0[i];
        if (NRHS == 2) s1[i] = out1[i];
    }
    __syncthreads();
    tri_sweep<NRHS>(t, in0, in1, s0, NRHS == 2 ? s1 : nullptr, l0);
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        out0[i] = s0[i];
        if (NRHS == 2) out1[i] = s1[i];
    }
    __syncthreads();
}

// the sweeps of factors up to this m keep their output vectors in LDS
// (NRHS = 2 FTRAN: 16 m bytes; the BTRAN's two sweeps: 16 m bytes)
constexpr int SP_LDS_M = 6144;

template <int NRHS>
__global__ void __launch_bounds__(1024) k_sp_ftran_lu(SpDev sp, const DState *st, double *h0, double *h1, int gated,
                                                      int parts, int l0l, int l0u, int lds)
{
    if (gated && st->stop) return;
    const int m = sp.m;
    if (parts & 1) {                                                   // in place: z[r] (row space)
        if (lds) lds_sweep<NRHS>(sp.fl, m, h0, h1, h0, h1, sp_lds, l0l);
        else tri_sweep<NRHS>(sp.fl, h0, h1, h0, h1, l0l);
    }
    double *x0 = sp.w.bt, *x1 = sp.w.bt + m;
    if (!(parts & 2)) return;
    if (lds) lds_sweep<NRHS>(sp.fu, m, h0, h1, x0, x1, sp_lds, l0u);   // positions
    else tri_sweep<NRHS>(sp.fu, h0, h1, x0, x1, l0u);
    ftran_hh<NRHS>(sp);
}

// hh = inv(M) z[P] for k_sp_ftran_wood, once per FTRAN: one wave per row of
// inv(M), its lanes along the row (coalesced), fixed-order reduction
template <int NRHS>
__device__ void ftran_hh(const SpDev &sp)
{
    const int m = sp.m;
    const double *x0 = sp.w.bt, *x1 = sp.w.bt + m;
    const int k = *sp.w.k;
    if (k == 0) return;
    __shared__ double g[2][SP_KMAX];
    for (int t = threadIdx.x; t < k; t += blockDim.x) {
        const int p = sp.w.P[t];
        g[0][t] = x0[p];
        if (NRHS == 2) g[1][t] = x1[p];
    }
    __syncthreads();
    // a wave per row of inv(M), four rows in flight at once (each row's sum
    // in the order of one row at a time)
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int t0 = threadIdx.x >> 6; t0 < k; t0 += 4 * nw) {
        double mv[4][SP_KMAX / 64];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int t = min(t0 + r * nw, k - 1);
#pragma unroll
            for (int q = 0; q < SP_KMAX / 64; q++) {
                const int u = lane + 64 * q;
                mv[r][q] = (u < k) ? sp.w.Minv[(size_t)t * SP_KMAX + u] : 0.0;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int q = 0; q < SP_KMAX / 64; q++) {
                const int u = lane + 64 * q;
                if (u < k) {
                    a0 += mv[r][q] * g[0][u];
                    if (NRHS == 2) a1 += mv[r][q] * g[1][u];
                }
            }
            a0 = wsum(a0);
            if (NRHS == 2) a1 = wsum(a1);
            const int t = t0 + r * nw;
            if (lane == 0 && t < k) {
                sp.w.hh[t] = a0;
                if (NRHS == 2) sp.w.hh[SP_KMAX + t] = a1;
            }
        }
    }
}

// FTRAN part 2 (grid): x = z - Y inv(M) z[P] for each right-hand side
// (inv(M) z[P] formed once by k_sp_ftran_lu's tail)
template <int NRHS>
__global__ void __launch_bounds__(256) k_sp_ftran_wood(SpDev sp, const DState *st, double *out0, double *out1,
                                                       int gated, int keep)
{
    if (gated && st->stop) return;
    const int m = sp.m;
    const int k = *sp.w.k;
    const double *z0 = sp.w.bt, *z1 = sp.w.bt + m;
    __shared__ double hh[2][SP_KMAX];
    for (int t = threadIdx.x; t < k; t += blockDim.x) {
        hh[0][t] = sp.w.hh[t];
        if (NRHS == 2) hh[1][t] = sp.w.hh[SP_KMAX + t];
    }
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double *yr = sp.w.Y + (size_t)i * SP_KMAX;
    double a0 = z0[i], a1 = (NRHS == 2) ? z1[i] : 0.0;
    for (int t = 0; t < k; t++) {
        const double y = yr[t];
        a0 -= y * hh[0][t];
        if (NRHS == 2) a1 -= y * hh[1][t];
    }
    if (keep) sp.w.zq[i] = z0[i];
    out0[i] = a0;
    if (NRHS == 2) out1[i] = a1;
}

// BTRAN of a general right-hand side, part 1 (grid): partials of Y' e
__global__ void __launch_bounds__(256) k_sp_btran_part(SpDev sp, const double *e)
{
    const int m = sp.m, k = *sp.w.k;
    __shared__ double red[SP_KMAX];
    const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5;   // 8 groups of 32 threads
    const int i0 = blockIdx.x * 256;
    for (int t = grp; t < k; t += 8) {
        double a = 0.0;
        for (int i = i0 + lane; i < min(i0 + 256, m); i += 32) a += sp.w.Y[(size_t)i * SP_KMAX + t] * e[i];
        for (int o = 16; o > 0; o >>= 1) a += __shfl_xor(a, o, 32);
        if (lane == 0) red[t] = a;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < k; t += blockDim.x) sp.w.tpart[(size_t)blockIdx.x * SP_KMAX + t] = red[t];
}

// BTRAN part 2 (one workgroup): e' = e - S inv(M)' (Y' e), then y = inv(B0)' e'
// mode 0: e general (partials from k_sp_btran_part over nparts blocks);
// mode 1: e = e_p of the pivot (st->p): Y' e_p is row p of Y;
// mode 2: both — e_p into y, e1 (general, partials) into y1 (the primal's
//         rho and update_gamma's u = inv(B)' v in one sweep pair)
// back to zero: the entries of bz the BTRAN of e_p set (the U' sweep that
// read them has finished: its last level ended with a barrier)
__device__ __forceinline__ void bz_clear(const SpDev &sp, int p, int k)
{
    if (threadIdx.x == 0) sp.w.bz[p] = 0.0;
    for (int t = threadIdx.x; t < k; t += blockDim.x) sp.w.bz[sp.w.P[t]] = 0.0;
}

// one workgroup: levels [l0, l1) of sweep t
// between the grid launches of the wide levels; clr: the BTRAN of e_p ends
// here (bz back to zero)
template <int NRHS>
__global__ void __launch_bounds__(1024) k_sp_sweep(SpDev sp, TriDev t, const DState *st, int gate,
                                                   const double *in0, const double *in1, double *out0,
                                                   double *out1, int l0, int l1, int clr)
{
    // (the sweep's TriDev is its own argument: one selected from sp by a
    // run-time index would be copied to scratch and every level's metadata
    // read through it)
    if (sp_gated(st, gate)) return;
    tri_sweep<NRHS>(t, in0, in1, out0, out1, l0, l1);
    if (clr) {
        __syncthreads();
        bz_clear(sp, st->p - 1, *sp.w.k);
    }
}

// ---- LDS segments (sp_plan_sweep) ---------------------------------------
// the external sum of a step of few external entries: its right-hand side
// less them, in entry order, four gathers in flight per trip
template <int NRHS>
__device__ __forceinline__ void seg_ext_thread(const TriDev &t, const double *in0, const double *in1,
                                               const double *out0, const double *out1, int s, double &a0, double &a1)
{
    const int ii = t.iin[s], ee = t.emid[s];
    int e = t.eptr[s];
    a0 = in0[ii];
    a1 = (NRHS == 2) ? in1[ii] : 0.0;
    if (ee > e)
        gather_sub8<NRHS>(t.eidx, t.eval, e, ee, [&](int ix, double &x0, double &x1) {
            x0 = out0[ix];
            x1 = (NRHS == 2) ? out1[ix] : 0.0;
        }, a0, a1);
}

// the external sum of a step of many: one wave, lanes strided, fixed-order
// reduction; every lane returns it
template <int NRHS>
__device__ __forceinline__ void seg_ext_wave(const TriDev &t, const double *in0, const double *in1,
                                             const double *out0, const double *out1, int s, double &a0, double &a1)
{
    const int eb = t.eptr[s], ee = t.emid[s];
    double p0 = 0.0, p1 = 0.0;
    wave_dot4<NRHS>(t.eidx, t.eval, eb, ee, [&](int ix, double &x0, double &x1) {
        x0 = out0[ix];
        x1 = (NRHS == 2) ? out1[ix] : 0.0;
    }, p0, p1);
    p0 = wsum(p0);
    if (NRHS == 2) p1 = wsum(p1);
    const int ii = t.iin[s];
    a0 = in0[ii] - p0;
    a1 = (NRHS == 2) ? in1[ii] - p1 : 0.0;
}

// the external pass of a segment by nthr threads (thread g; the grid or one
// workgroup, a multiple of 64): acc[local step] = the step's external sum
template <int NRHS>
__device__ void seg_ext(const TriDev &t, const double *in0, const double *in1, const double *out0, const double *out1,
                        int sb, int ns, int nas, double *acc0, double *acc1, int g, int nthr)
{
    for (int i = g; i < nas; i += nthr) {
        const int li = t.aord[sb + i];
        double a0, a1;
        seg_ext_thread<NRHS>(t, in0, in1, out0, out1, sb + li, a0, a1);
        acc0[li] = a0;
        if (NRHS == 2) acc1[li] = a1;
    }
    const int lane = g & 63;
    for (int i = nas + (g >> 6); i < ns; i += nthr >> 6) {
        const int li = t.aord[sb + i];
        double a0, a1;
        seg_ext_wave<NRHS>(t, in0, in1, out0, out1, sb + li, a0, a1);
        if (lane == 0) {
            acc0[li] = a0;
            if (NRHS == 2) acc1[li] = a1;
        }
    }
}

// the external pass on the grid (a segment of many external entries): into
// acc (2 x SP_SEG_MAX), which k_sp_seg then stages in LDS
template <int NRHS>
__global__ void __launch_bounds__(256) k_sp_seg_a(TriDev t, const DState *st, int gate, const double *in0,
                                                  const double *in1, const double *out0, const double *out1, int sb,
                                                  int ns, int nas, double *acc)
{
    if (sp_gated(st, gate)) return;
    const int nsb = (nas + 255) / 256;                     // blocks of the short steps
    if ((int)blockIdx.x < nsb) {
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        if (i < nas) {
            const int li = t.aord[sb + i];
            double a0, a1;
            seg_ext_thread<NRHS>(t, in0, in1, out0, out1, sb + li, a0, a1);
            acc[li] = a0;
            if (NRHS == 2) acc[SP_SEG_MAX + li] = a1;
        }
        return;
    }
    // a step of many external entries a block (blockDim 256)
    const int i = nas + (int)blockIdx.x - nsb;
    if (i >= ns) return;
    const int li = t.aord[sb + i], sx = sb + li;
    double a0, a1;
    block_dot4<NRHS>(t.eidx, t.eval, t.eptr[sx], t.emid[sx], [&](int ix, double &x0, double &x1) {
        x0 = out0[ix];
        x1 = (NRHS == 2) ? out1[ix] : 0.0;
    }, a0, a1);
    if (threadIdx.x == 0) {
        const int ii = t.iin[sx];
        acc[li] = in0[ii] - a0;
        if (NRHS == 2) acc[SP_SEG_MAX + li] = in1[ii] - a1;
    }
}

// a short step of the internal pass: its first internal entries and
// diagonal, loaded a level ahead (none depends on the sweep's values)
struct SegPre {
    int s, n;
    double rd;
    int ix[SP_RECN];
    double v[SP_RECN];
};

// one record load per step, unconditional (an index past the level reads a
// valid record and is dropped by n = 0): the compiler can count the loads in
// flight and the prefetch stays in flight across the level's barrier
__device__ __forceinline__ void segpre_load(const TriDev &t, int s, int lim, SegPre &q)
{
    static_assert(SP_RECN == 4, "segpre_load reads records of four entries");
    const int sc = max(min(s, lim - 1), 0);
    const int2 r = t.srx[sc];
    const double2 a = t.srv[2 * sc], b = t.srv[2 * sc + 1];
    const int n = t.srn[sc];
    q.rd = t.srd[sc];
    q.s = s;
    q.n = (s < lim) ? n : 0;
    q.ix[0] = r.x & 0xffff; q.ix[1] = (unsigned)r.x >> 16;
    q.ix[2] = r.y & 0xffff; q.ix[3] = (unsigned)r.y >> 16;
    q.v[0] = a.x; q.v[1] = a.y; q.v[2] = b.x; q.v[3] = b.y;
}

template <int NRHS>
__device__ __forceinline__ void segpre_run(const TriDev &t, const SegPre &q, int sb, double *L)
{
    const int li = q.s - sb;
    double a0 = L[li], a1 = (NRHS == 2) ? L[SP_SEG_MAX + li] : 0.0;
#pragma unroll
    for (int u = 0; u < SP_RECN; u++) {
        if (u < q.n) {
            a0 -= q.v[u] * L[q.ix[u]];
            if (NRHS == 2) a1 -= q.v[u] * L[SP_SEG_MAX + q.ix[u]];
        }
    }
    if (q.n > SP_RECN) {
        const int eb = t.emid[q.s];
        gather_sub8<NRHS>(t.eidx, t.eval, eb + SP_RECN, eb + q.n, [&](int ix, double &x0, double &x1) {
            x0 = L[ix];
            x1 = (NRHS == 2) ? L[SP_SEG_MAX + ix] : 0.0;
        }, a0, a1);
    }
    L[li] = a0 * q.rd;
    if (NRHS == 2) L[SP_SEG_MAX + li] = a1 * q.rd;
}

// the barrier between two levels of the internal pass: the level's LDS
// writes done, the next levels' metadata loads left in flight (a
// __syncthreads() may wait for them); the clobber keeps the compiler's LDS
// accesses on their side of it
__device__ __forceinline__ void seg_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// one level of the internal pass: the short steps (the first one of this
// thread prefetched in q), then the long ones — split over the waves when
// there are at most a quarter as many as waves, else a wave each
template <int NRHS>
__device__ __forceinline__ void seg_level(const TriDev &t, const SegPre &q, int sb, int ls, int le, double *L,
                                          double *red)
{
    const int T = blockDim.x, w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = threadIdx.x & 63;
    if (q.s < ls) segpre_run<NRHS>(t, q, sb, L);
    for (int s = q.s + T; s < ls; s += T) {              // short steps beyond one per thread
        SegPre r;
        segpre_load(t, s, ls, r);
        segpre_run<NRHS>(t, r, sb, L);
    }
    const int nl = le - ls;
    if (nl <= 0) return;
    if (4 * nl <= nw) {
        const int g = nw / nl, sidx = w / g, sub = w % g;
        double p0 = 0.0, p1 = 0.0;
        if (sidx < nl) {
            // the step's entries in chunks of 256, chunk c to wave sub + c g
            const int st = ls + sidx, eb = t.emid[st], ee = t.eptr[st + 1];
            for (int c = eb + 256 * sub; c < ee; c += 256 * g)
                wave_dot4<NRHS>(t.eidx, t.eval, c, min(c + 256, ee), [&](int ix, double &x0, double &x1) {
                    x0 = L[ix];
                    x1 = (NRHS == 2) ? L[SP_SEG_MAX + ix] : 0.0;
                }, p0, p1);
        }
        p0 = wsum(p0);
        if (NRHS == 2) p1 = wsum(p1);
        if (lane == 0) {
            red[w] = p0;
            red[16 + w] = p1;
        }
        seg_barrier();
        if (sidx < nl && sub == 0 && lane == 0) {
            double s0 = 0.0, s1 = 0.0;
            for (int u = 0; u < g; u++) {
                s0 += red[w + u];
                s1 += red[16 + w + u];
            }
            const int st = ls + sidx, li = st - sb;
            const double dg = t.diag[st];
            L[li] = (L[li] - s0) / dg;
            if (NRHS == 2) L[SP_SEG_MAX + li] = (L[SP_SEG_MAX + li] - s1) / dg;
        }
        return;
    }
    for (int st = ls + w; st < le; st += nw) {
        const int eb = t.emid[st], ee = t.eptr[st + 1];
        double p0 = 0.0, p1 = 0.0;
        wave_dot4<NRHS>(t.eidx, t.eval, eb, ee, [&](int ix, double &x0, double &x1) {
            x0 = L[ix];
            x1 = (NRHS == 2) ? L[SP_SEG_MAX + ix] : 0.0;
        }, p0, p1);
        p0 = wsum(p0);
        if (NRHS == 2) p1 = wsum(p1);
        if (lane == 0) {
            const int li = st - sb;
            const double dg = t.diag[st];
            L[li] = (L[li] - p0) / dg;
            if (NRHS == 2) L[SP_SEG_MAX + li] = (L[SP_SEG_MAX + li] - p1) / dg;
        }
    }
}

// one LDS segment: levels l0 .. l1-1 (at most SP_SEG_LEVELS), steps sb ..
// sb+ns-1 (one workgroup of 1024); pre: the external pass ran on the grid
// (acc).  The levels' bounds are staged in LDS; a level's short-step
// metadata is loaded while the level before runs; the outputs go to the
// sweep's vector once, after the last level.  A chain — consecutive levels
// of one step of at most 64 internal entries each, the dense triangle of a
// block-angular basis's linking rows — runs in wave 0 alone, 16 links per
// round, their entries staged in LDS by the whole workgroup first: a link
// is then an LDS gather, a wave reduction and one store, with no barrier.
// clr as k_sp_sweep
constexpr int SP_CHAIN = 16;                      // chain links staged per round (64 entries each)

template <int NRHS>
__global__ void __launch_bounds__(1024) k_sp_seg(SpDev sp, TriDev t, const DState *st, int gate, const double *in0,
                                                 const double *in1, double *out0, double *out1, int sb, int ns,
                                                 int nas, int l0, int l1, int pre, const double *acc, int clr)
{
    if (sp_gated(st, gate)) return;
    __shared__ double L[NRHS * SP_SEG_MAX];
    __shared__ int lvb[SP_SEG_LEVELS + 2], lvl[SP_SEG_LEVELS + 2], lch[SP_SEG_LEVELS + 2];
    __shared__ double red[32];
    __shared__ int chx[SP_CHAIN * 64], chn[SP_CHAIN];
    __shared__ double chv[SP_CHAIN * 64], chd[SP_CHAIN];
    const int T = blockDim.x, nlv = l1 - l0, lane = threadIdx.x & 63;
    // (two empty levels past the last: the prefetch runs unconditionally)
    for (int l = threadIdx.x; l < nlv + 2; l += T) {
        const int e = t.lvptr[l0 + min(l, nlv)];
        lvb[l] = e;
        lvl[l] = (l < nlv) ? t.lvlong[l0 + l] : e;
        lch[l] = (l < nlv) ? t.lvch[l0 + l] : 0;
    }
    SegPre A;
    segpre_load(t, t.lvptr[l0] + (int)threadIdx.x, t.lvlong[l0], A);
    if (pre)
        for (int i = threadIdx.x; i < ns; i += T) {
            L[i] = acc[i];
            if (NRHS == 2) L[SP_SEG_MAX + i] = acc[SP_SEG_MAX + i];
        }
    else
        seg_ext<NRHS>(t, in0, in1, out0, out1, sb, ns, nas, L, L + SP_SEG_MAX, threadIdx.x, T);
    __syncthreads();
    const bool stamp = t.stamps && threadIdx.x == 0;
    if (stamp && l0 < SP_STAMP_MAX) t.stamps[l0] = wall_clock64();
    for (int l = 0; l < nlv;) {
        int c = 0;
        while (c < SP_CHAIN && l + c < nlv && lch[l + c]) c++;
        if (c >= 2) {
            {
                const int j = threadIdx.x >> 6;
                if (j < c) {
                    const int s0 = lvb[l + j], eb = t.emid[s0], n = t.eptr[s0 + 1] - eb;
                    if (lane < n) {
                        chx[64 * j + lane] = t.eidx[eb + lane];
                        chv[64 * j + lane] = t.eval[eb + lane];
                    }
                    if (lane == 0) {
                        chn[j] = n;
                        chd[j] = t.srd[s0];
                    }
                }
            }
            __syncthreads();
            if (threadIdx.x < 64)
                for (int j = 0; j < c; j++) {
                    const int li = lvb[l + j] - sb, n = chn[j];
                    double p0 = 0.0, p1 = 0.0;
                    if (lane < n) {
                        const int ix = chx[64 * j + lane];
                        const double v = chv[64 * j + lane];
                        p0 = v * L[ix];
                        if (NRHS == 2) p1 = v * L[SP_SEG_MAX + ix];
                    }
                    p0 = wsum(p0);
                    if (NRHS == 2) p1 = wsum(p1);
                    if (lane == 0) {
                        L[li] = (L[li] - p0) * chd[j];
                        if (NRHS == 2) L[SP_SEG_MAX + li] = (L[SP_SEG_MAX + li] - p1) * chd[j];
                        if (stamp && l0 + l + j + 1 < SP_STAMP_MAX) t.stamps[l0 + l + j + 1] = wall_clock64();
                    }
                }
            __syncthreads();
            l += c;
            segpre_load(t, lvb[l] + (int)threadIdx.x, lvl[l], A);
            continue;
        }
        SegPre B;
        segpre_load(t, lvb[l + 1] + (int)threadIdx.x, lvl[l + 1], B);
        seg_level<NRHS>(t, A, sb, lvl[l], lvb[l + 1], L, red);
        seg_barrier();
        if (stamp && l0 + l + 1 < SP_STAMP_MAX) t.stamps[l0 + l + 1] = wall_clock64();
        A = B;
        l++;
    }
    for (int i = threadIdx.x; i < ns; i += T) {
        const int io = t.iout[sb + i];
        out0[io] = L[i];
        if (NRHS == 2) out1[io] = L[SP_SEG_MAX + i];
    }
    if (clr) {
        __syncthreads();
        bz_clear(sp, st->p - 1, *sp.w.k);
    }
}

// the FTRAN's inv(M) z[P] (k_sp_ftran_lu's tail) as its own launch, after a
// U sweep that ended on the grid or in a k_sp_sweep
template <int NRHS>
__global__ void __launch_bounds__(1024) k_sp_hh(SpDev sp, const DState *st, int gated)
{
    if (gated && st->stop) return;
    ftran_hh<NRHS>(sp);
}

// parts: bit 0 the Schur correction into b, bit 1 the U' sweep (from level
// l0u), bit 2 the L' sweep (from l0l)
template <int NRHS>
__global__ void __launch_bounds__(1024) k_sp_btran(SpDev sp, DState *st, const double *e, double *y, int mode,
                                                   int nparts, const double *e1, double *y1, int parts, int l0u,
                                                   int l0l, int lds)
{
    if (mode >= 1 && (st->stop || st->p <= 0)) return;
    const int m = sp.m, k = *sp.w.k;
    const int p = (mode >= 1) ? st->p - 1 : -1;
    __shared__ double tv[2][SP_KMAX], sv[2][SP_KMAX], svp[4][2][SP_KMAX];
    // mode 1: e_p lives in bz, zero everywhere but the k + 1 entries this
    // BTRAN sets (p and P) and clears again at its end — no O(m) fill
    double *b0 = (mode == 1) ? sp.w.bz : sp.w.bt, *b1 = sp.w.bt + m;      // positions
    double *w0 = sp.w.scr2, *w1 = sp.w.scr2 + m;  // step space
    if (!(parts & 1)) {
        if (parts & 2) tri_sweep<NRHS>(sp.bu, b0, b1, w0, w1, l0u);
        if (parts & 4) {
            tri_sweep<NRHS>(sp.bl, w0, w1, y, y1, l0l);
            if (mode == 1) bz_clear(sp, p, k);
        }
        return;
    }
    for (int t = threadIdx.x; t < k; t += blockDim.x) {
        double a = 0.0, a1 = 0.0;
        if (mode >= 1) a = sp.w.Y[(size_t)p * SP_KMAX + t];
        else
            for (int q = 0; q < nparts; q++) a += sp.w.tpart[(size_t)q * SP_KMAX + t];
        if (NRHS == 2)
            for (int q = 0; q < nparts; q++) a1 += sp.w.tpart[(size_t)q * SP_KMAX + t];
        tv[0][t] = a;
        tv[1][t] = a1;
    }
    if (mode == 1) {
        if (threadIdx.x == 0) b0[p] = 1.0;
    } else
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            b0[i] = (mode >= 1) ? (i == p ? 1.0 : 0.0) : e[i];
            if (NRHS == 2) b1[i] = e1[i];
        }
    __syncthreads();
    // sv = inv(M)' tv: four quarters of u per column t (coalesced along t),
    // partials summed in quarter order
    {
        const int q = threadIdx.x >> 8, t = threadIdx.x & 255;
        const int ub = q * ((k + 3) / 4), ue = min(k, ub + (k + 3) / 4);
        double a = 0.0, a1 = 0.0;
        if (t < k && q < 4) {
            // (eight entries of the column loaded before their products: the
            // same order of accumulation as one by one)
            int u = ub;
            for (; u + 8 <= ue; u += 8) {
                double mv[8];
#pragma unroll
                for (int r = 0; r < 8; r++) mv[r] = sp.w.Minv[(size_t)(u + r) * SP_KMAX + t];    // inv(M)'
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    a += mv[r] * tv[0][u + r];
                    if (NRHS == 2) a1 += mv[r] * tv[1][u + r];
                }
            }
            for (; u < ue; u++) {
                const double mi = sp.w.Minv[(size_t)u * SP_KMAX + t];
                a += mi * tv[0][u];
                if (NRHS == 2) a1 += mi * tv[1][u];
            }
        }
        if (t < k && q < 4) {
            svp[q][0][t] = a;
            svp[q][1][t] = a1;
        }
        __syncthreads();
        for (int t2 = threadIdx.x; t2 < k; t2 += blockDim.x) {
            sv[0][t2] = ((svp[0][0][t2] + svp[1][0][t2]) + svp[2][0][t2]) + svp[3][0][t2];
            sv[1][t2] = ((svp[0][1][t2] + svp[1][1][t2]) + svp[2][1][t2]) + svp[3][1][t2];
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < k; t += blockDim.x) {   // P holds distinct positions (k_sp_update)
        b0[sp.w.P[t]] -= sv[0][t];
        if (NRHS == 2) b1[sp.w.P[t]] -= sv[1][t];
    }
    __syncthreads();
    if (lds && (parts & 6) == 6) {
        // both sweeps with their outputs in LDS (the U' output, the L'
        // sweep's input, stays there; the step space is written back too)
        double *sa = sp_lds, *sb = sp_lds + NRHS * m;
        double *sa1 = sa + m, *sb1 = sb + m;
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            sa[i] = w0[i];
            sb[i] = y[i];
            if (NRHS == 2) {
                sa1[i] = w1[i];
                sb1[i] = y1[i];
            }
        }
        __syncthreads();
        tri_sweep<NRHS>(sp.bu, b0, b1, sa, NRHS == 2 ? sa1 : nullptr, l0u);
        __syncthreads();
        tri_sweep<NRHS>(sp.bl, sa, NRHS == 2 ? sa1 : nullptr, sb, NRHS == 2 ? sb1 : nullptr, l0l);
        __syncthreads();
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            w0[i] = sa[i];
            y[i] = sb[i];
            if (NRHS == 2) {
                w1[i] = sa1[i];
                y1[i] = sb1[i];
            }
        }
        __syncthreads();
        if (mode == 1) bz_clear(sp, p, k);
        return;
    }
    if (parts & 2) tri_sweep<NRHS>(sp.bu, b0, b1, w0, w1, l0u);
    if (parts & 4) {
        tri_sweep<NRHS>(sp.bl, w0, w1, y, y1, l0l);
        if (mode == 1) bz_clear(sp, p, k);
    }
}

// the update of this pivot (one workgroup, after the commit): the column
// entering at position p is N_q = -h, so inv(B0) N_q = -zq and
// y = -zq - e_p; a new position borders inv(M), a repeated one replaces
// its column (Sherman-Morrison).  A Schur pivot too small for a stable
// inverse ends the chain (refact_pending), as the growth check does for the
// dense inverse.
// out[t] = sum_u M[t][u] c[u] for t < k (M row-major, stride SP_KMAX): one
// wave per row, lanes along it (coalesced), fixed-order reduction; ends
// with a barrier
__device__ __forceinline__ void rows_dot(const double *M, const double *c, int k, double *out)
{
    // a wave per row, four rows of the wave in flight at once (the row sums
    // in the same order as one row at a time: lane u, u + 64, ... then wsum)
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int t0 = threadIdx.x >> 6; t0 < k; t0 += 4 * nw) {
        double mv[4][SP_KMAX / 64];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int t = min(t0 + r * nw, k - 1);
#pragma unroll
            for (int q = 0; q < SP_KMAX / 64; q++) {
                const int u = lane + 64 * q;
                mv[r][q] = (u < k) ? M[(size_t)t * SP_KMAX + u] : 0.0;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            double a = 0.0;
#pragma unroll
            for (int q = 0; q < SP_KMAX / 64; q++) {
                const int u = lane + 64 * q;
                if (u < k) a += mv[r][q] * c[u];
            }
            a = wsum(a);
            const int t = t0 + r * nw;
            if (lane == 0 && t < k) out[t] = a;
        }
    }
    __syncthreads();
}

__global__ void __launch_bounds__(1024) k_sp_update(SpDev sp, DState *st)
{
    if (st->stop || st->p <= 0) return;          // (primal: p = -1 is a bound flip, no basis change)
    const int k = *sp.w.k;
    const int p = st->p - 1;
    __shared__ int slot;
    __shared__ double c[SP_KMAX], r[SP_KMAX], ac[SP_KMAX], ra[SP_KMAX], col_old[SP_KMAX];
    __shared__ double sch;
    if (threadIdx.x == 0) {
        // the pivot log (the look-ahead's replay): every basis change of the chain
        const int nl = *sp.w.nlog;
        if (nl < SP_KMAX) {
            sp.w.log[2 * nl] = p;
            sp.w.log[2 * nl + 1] = st->kq;
        }
        *sp.w.nlog = nl + 1;
        slot = -1;
        *sp.w.ycol = -1;
        *sp.w.nupd = 0;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < k; t += blockDim.x)
        if (sp.w.P[t] == p) slot = t;                // at most one: positions are distinct
    __syncthreads();
    const int t0 = slot;
    double *Y = sp.w.Y, *Mi = sp.w.Minv;
    if (t0 < 0) {
        if (k >= SP_KMAX) {
            if (threadIdx.x == 0) st->refact_pending = 1;
            return;
        }
        // border: c_i = y[P_i], r_t = Y[p, t], d = 1 + y[p]
        for (int t = threadIdx.x; t < k; t += blockDim.x) {
            c[t] = -sp.w.zq[sp.w.P[t]] - (sp.w.P[t] == p ? 1.0 : 0.0);
            r[t] = Y[(size_t)p * SP_KMAX + t];
        }
        __syncthreads();
        rows_dot(Mi, c, k, ac);                          // inv(M) c
        for (int t = threadIdx.x; t < k; t += blockDim.x) {
            // r inv(M): the column's entries eight at a time, loaded before
            // their products (the same order of accumulation as one by one)
            double b = 0.0;
            int u = 0;
            for (; u + 8 <= k; u += 8) {
                double mv[8];
#pragma unroll
                for (int q = 0; q < 8; q++) mv[q] = Mi[(size_t)(u + q) * SP_KMAX + t];
#pragma unroll
                for (int q = 0; q < 8; q++) b += r[u + q] * mv[q];
            }
            for (; u < k; u++) b += r[u] * Mi[(size_t)u * SP_KMAX + t];
            ra[t] = b;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = 1.0 + (-sp.w.zq[p] - 1.0);
            for (int u = 0; u < k; u++) s -= r[u] * ac[u];
            sch = s;
        }
        __syncthreads();
        const double s = sch;
        double dmax = 0.0;                                // (a wave maximum: exact, any order)
        for (int u = (int)(threadIdx.x & 63); u < k; u += 64) dmax = fmax(dmax, fabs(ac[u]));
        dmax = wmax(dmax);
        if (!(fabs(s) > 1e-11 * (1.0 + dmax))) {
            if (threadIdx.x == 0) st->refact_pending = 1;
            return;
        }
        // the k x k block's rank-1 update inv(M) += a r / s: by k_sp_ycol's
        // grid (one workgroup streamed the k^2 entries through one CU)
        for (int t = threadIdx.x; t < k; t += blockDim.x) {
            sp.w.upd[t] = ac[t];
            sp.w.upd[SP_KMAX + t] = ra[t];
        }
        for (int t = threadIdx.x; t < k; t += blockDim.x) {
            Mi[(size_t)t * SP_KMAX + k] = -ac[t] / s;
            Mi[(size_t)k * SP_KMAX + t] = -ra[t] / s;
        }
        if (threadIdx.x == 0) {
            Mi[(size_t)k * SP_KMAX + k] = 1.0 / s;
            sp.w.P[k] = p;
            *sp.w.k = k + 1;
            *sp.w.ycol = k;                              // k_sp_ycol writes the column
            sp.w.upd[2 * SP_KMAX] = s;
            sp.w.upd[2 * SP_KMAX + 1] = +1.0;
            *sp.w.nupd = k;
        }
        return;
    }
    // replace column t0: M' = M + u e_t0', u_i = ynew[P_i] - Yold[P_i, t0]
    for (int t = threadIdx.x; t < k; t += blockDim.x) {
        const int pi = sp.w.P[t];
        col_old[t] = Y[(size_t)pi * SP_KMAX + t0];
        c[t] = (-sp.w.zq[pi] - (pi == p ? 1.0 : 0.0)) - col_old[t];
    }
    __syncthreads();
    rows_dot(Mi, c, k, ac);                          // inv(M) u
    for (int t = threadIdx.x; t < k; t += blockDim.x) ra[t] = Mi[(size_t)t0 * SP_KMAX + t];   // row t0 of inv(M)
    __syncthreads();
    const double den = 1.0 + ac[t0];
    double amax = 0.0;
    for (int u = (int)(threadIdx.x & 63); u < k; u += 64) amax = fmax(amax, fabs(ac[u]));
    amax = wmax(amax);
    if (!(fabs(den) > 1e-11 * (1.0 + amax))) {
        if (threadIdx.x == 0) st->refact_pending = 1;
        return;
    }
    __syncthreads();
    // inv(M) -= a r / den on k_sp_ycol's grid
    for (int t = threadIdx.x; t < k; t += blockDim.x) {
        sp.w.upd[t] = ac[t];
        sp.w.upd[SP_KMAX + t] = ra[t];
    }
    if (threadIdx.x == 0) {
        *sp.w.ycol = t0;
        sp.w.upd[2 * SP_KMAX] = den;
        sp.w.upd[2 * SP_KMAX + 1] = -1.0;
        *sp.w.nupd = k;
    }
}

// the column of Y the update of this pivot bordered or replaced (grid; the
// single-workgroup update would need m / 1024 trips of strided stores):
// y = -zq - e_p
__global__ void __launch_bounds__(256) k_sp_ycol(SpDev sp, const DState *st)
{
    if (st->stop || st->p <= 0) return;
    const int c = *sp.w.ycol;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    // k_sp_update's rank-1 update of inv(M)'s k x k block, spread over the
    // grid (the same expression per entry: m + (a_t r_u) / d, or minus)
    const int kk = *sp.w.nupd;
    if (kk > 0) {
        const double *a = sp.w.upd, *r = sp.w.upd + SP_KMAX;
        const double dv = sp.w.upd[2 * SP_KMAX];
        const bool plus = sp.w.upd[2 * SP_KMAX + 1] > 0.0;
        double *Mi = sp.w.Minv;
        for (int e = i; e < kk * kk; e += gridDim.x * blockDim.x) {
            const int t = e / kk, u = e % kk;
            double &x = Mi[(size_t)t * SP_KMAX + u];
            if (plus) x += a[t] * r[u] / dv;
            else x -= a[t] * r[u] / dv;
        }
    }
    if (c < 0 || i >= sp.m) return;
    sp.w.Y[(size_t)i * SP_KMAX + c] = -sp.w.zq[i] - (i == st->p - 1 ? 1.0 : 0.0);
}

// ---------------------------------------------------------------------------
// host side: upload of a factor, the solves between batches, the pivot hooks
// ---------------------------------------------------------------------------
static void up_tri(hipStream_t s, SpTriDevBufs &B, const SpTriHost &T, int *d_nlev)
{
    B.lvptr.ensure(T.lvptr.size());
    B.lvlong.ensure(std::max<size_t>(T.lvlong.size(), 1));
    B.iin.ensure(std::max<size_t>(T.iin.size(), 1));
    B.iout.ensure(std::max<size_t>(T.iout.size(), 1));
    B.eptr.ensure(T.eptr.size());
    B.eidx.ensure(std::max<size_t>(T.eidx.size(), 1));
    B.diag.ensure(std::max<size_t>(T.diag.size(), 1));
    B.eval.ensure(std::max<size_t>(T.eval.size(), 1));
    B.emid.ensure(std::max<size_t>(T.emid.size(), 1));
    B.aord.ensure(std::max<size_t>(T.aord.size(), 1));
    B.lvch.ensure(std::max<size_t>(T.lvch.size(), 1));
    if (!T.lvch.empty())
        SPCHK(hipMemcpyAsync(B.lvch.p, T.lvch.data(), T.lvch.size() * sizeof(int), hipMemcpyHostToDevice, s));
    B.srx.ensure(std::max<size_t>(T.srx.size(), SP_RECN / 2));
    B.srn.ensure(std::max<size_t>(T.srn.size(), 1));
    B.srv.ensure(std::max<size_t>(T.srv.size(), SP_RECN));
    B.srd.ensure(std::max<size_t>(T.srd.size(), 1));
    if (!T.srx.empty()) {
        SPCHK(hipMemcpyAsync(B.srx.p, T.srx.data(), T.srx.size() * sizeof(int), hipMemcpyHostToDevice, s));
        SPCHK(hipMemcpyAsync(B.srn.p, T.srn.data(), T.srn.size() * sizeof(int), hipMemcpyHostToDevice, s));
        SPCHK(hipMemcpyAsync(B.srv.p, T.srv.data(), T.srv.size() * sizeof(double), hipMemcpyHostToDevice, s));
        SPCHK(hipMemcpyAsync(B.srd.p, T.srd.data(), T.srd.size() * sizeof(double), hipMemcpyHostToDevice, s));
    }
    if (!T.emid.empty())
        SPCHK(hipMemcpyAsync(B.emid.p, T.emid.data(), T.emid.size() * sizeof(int), hipMemcpyHostToDevice, s));
    if (!T.aord.empty())
        SPCHK(hipMemcpyAsync(B.aord.p, T.aord.data(), T.aord.size() * sizeof(int), hipMemcpyHostToDevice, s));
    SPCHK(hipMemcpyAsync(B.lvptr.p, T.lvptr.data(), T.lvptr.size() * sizeof(int), hipMemcpyHostToDevice, s));
    if (!T.lvlong.empty())
        SPCHK(hipMemcpyAsync(B.lvlong.p, T.lvlong.data(), T.lvlong.size() * sizeof(int), hipMemcpyHostToDevice, s));
    SPCHK(hipMemcpyAsync(B.iin.p, T.iin.data(), T.iin.size() * sizeof(int), hipMemcpyHostToDevice, s));
    SPCHK(hipMemcpyAsync(B.iout.p, T.iout.data(), T.iout.size() * sizeof(int), hipMemcpyHostToDevice, s));
    SPCHK(hipMemcpyAsync(B.eptr.p, T.eptr.data(), T.eptr.size() * sizeof(int), hipMemcpyHostToDevice, s));
    if (!T.eidx.empty()) {
        SPCHK(hipMemcpyAsync(B.eidx.p, T.eidx.data(), T.eidx.size() * sizeof(int), hipMemcpyHostToDevice, s));
        SPCHK(hipMemcpyAsync(B.eval.p, T.eval.data(), T.eval.size() * sizeof(double), hipMemcpyHostToDevice, s));
    }
    SPCHK(hipMemcpyAsync(B.diag.p, T.diag.data(), T.diag.size() * sizeof(double), hipMemcpyHostToDevice, s));
    SPCHK(hipMemcpyAsync(d_nlev, &T.nlev, sizeof(int), hipMemcpyHostToDevice, s));
}

static TriDev tri_dev(const SpTriDevBufs &B, const int *nlev, unsigned long long *stamps)
{
    TriDev t;
    t.lvptr = B.lvptr.p; t.lvlong = B.lvlong.p; t.iin = B.iin.p; t.iout = B.iout.p; t.eptr = B.eptr.p; t.eidx = B.eidx.p;
    t.diag = B.diag.p; t.eval = B.eval.p; t.nlev = nlev; t.stamps = stamps; t.emid = B.emid.p; t.aord = B.aord.p;
    t.lvch = B.lvch.p;
    t.srx = (const int2 *)B.srx.p; t.srn = B.srn.p; t.srv = (const double2 *)B.srv.p; t.srd = B.srd.p;
    return t;
}

static const char *sp_stamps_path()
{
    static const char *p = std::getenv("GK_SP_STAMPS");
    return p;
}

static SpDev sp_dev(SpFactor &F)
{
    SpDev d;
    d.m = F.m;
    unsigned long long *sb = F.stamps.p;
    d.fl = tri_dev(F.fl, F.hdr.p + 0, sb ? sb + 0 * SP_STAMP_MAX : nullptr);
    d.fu = tri_dev(F.fu, F.hdr.p + 1, sb ? sb + 1 * SP_STAMP_MAX : nullptr);
    d.bu = tri_dev(F.bu, F.hdr.p + 2, sb ? sb + 2 * SP_STAMP_MAX : nullptr);
    d.bl = tri_dev(F.bl, F.hdr.p + 3, sb ? sb + 3 * SP_STAMP_MAX : nullptr);
    d.w.Y = F.Y.p; d.w.P = F.P.p; d.w.Minv = F.Minv.p; d.w.k = F.hdr.p + 4; d.w.zq = F.zq.p;
    d.w.tpart = F.tpart.p; d.w.bt = F.bt.p; d.w.scr2 = F.scr2.p; d.w.hh = F.hh.p; d.w.ycol = F.hdr.p + 5; d.w.bz = F.bz.p;
    d.w.log = F.plog.p; d.w.nlog = F.hdr.p + 6;
    d.w.upd = F.upd.p; d.w.nupd = F.hdr.p + 7;
    return d;
}

SpFactor *sp_create() { return new SpFactor; }
void sp_destroy(SpFactor *F) { delete F; }

void sp_info(const SpFactor *F, long long *nnz_lu, int *levels, double *t_lu)
{
    *nnz_lu = F->nnz_l + F->nnz_u;
    for (int i = 0; i < 4; i++) levels[i] = F->levels[i];
    *t_lu = F->t_lu;
}

// B0 from the basis header of (I | -A) (head 1-based; A in CSC, 0-based
// rows, the engine's scaled copy): factorize on the host, upload
static int sp_factorize_cols(SpFactor &F, hipStream_t s, int m, const std::vector<int> &cptr,
                             const std::vector<int> &crow, const std::vector<double> &cval, double piv_tol,
                             int piv_lim, double eps_tol, double t0);

int sp_factorize(SpFactor &F, hipStream_t s, int m, const int *head1, const int *Aptr, const int *Aind,
                 const double *Aval, double piv_tol, int piv_lim, double eps_tol)
{
    const double t0 = sp_now();
    std::vector<int> cptr(m + 1, 0), crow;
    std::vector<double> cval;
    crow.reserve((size_t)4 * m);
    cval.reserve((size_t)4 * m);
    for (int i = 1; i <= m; i++) {
        const int k = head1[i];
        if (k <= m) {
            crow.push_back(k - 1);
            cval.push_back(1.0);
        } else {
            const int j = k - m - 1;
            for (int t = Aptr[j]; t < Aptr[j + 1]; t++) {
                crow.push_back(Aind[t]);
                cval.push_back(-Aval[t]);
            }
        }
        cptr[i] = (int)crow.size();
    }
    return sp_factorize_cols(F, s, m, cptr, crow, cval, piv_tol, piv_lim, eps_tol, t0);
}

// B given by its columns (1-based CSC as gk_bfd_factorize_csc takes it:
// ptr[1..m+1], 1-based rows) — glp_factorize of a basis beyond the explicit
// inverse's limit
int sp_factorize_csc(SpFactor &F, hipStream_t s, int m, const int *ptr, const int *ind, const double *val,
                     double piv_tol, int piv_lim, double eps_tol)
{
    const double t0 = sp_now();
    std::vector<int> cptr(m + 1, 0), crow((size_t)(ptr[m + 1] - ptr[1]));
    std::vector<double> cval(crow.size());
    for (int j = 1; j <= m; j++) {
        for (int t = ptr[j]; t < ptr[j + 1]; t++) {
            crow[t - ptr[1]] = ind[t] - 1;
            cval[t - ptr[1]] = val[t];
        }
        cptr[j] = ptr[j + 1] - ptr[1];
    }
    return sp_factorize_cols(F, s, m, cptr, crow, cval, piv_tol, piv_lim, eps_tol, t0);
}

// the host part of a factorization (any thread)
static void sp_prepare(SpHost &H, int m, const std::vector<int> &cptr, const std::vector<int> &crow,
                       const std::vector<double> &cval, double piv_tol, int piv_lim, double eps_tol)
{
    const double t0 = sp_now();
    int rank = 0;
    H.m = m;
    H.ret = sp_lu_factor(H.lu, H.wk, m, cptr, crow, cval, piv_tol > 0.0 ? piv_tol : 0.1, piv_lim > 0 ? piv_lim : 4,
                         eps_tol > 0.0 ? eps_tol : 1e-15, &rank);
    H.t_lu = sp_now() - t0;
    if (H.ret) return;
    sp_build_solves(H.lu, H.S, H.plan, H.wide);
}

// the device part: buffers, the sweeps' upload, an empty chain
static void sp_install(SpFactor &F, hipStream_t s, SpHost &H, double t0)
{
    const int m = H.m;
    const SpSolves &S = H.S;
    for (int i = 0; i < 4; i++) {
        F.plan[i] = H.plan[i];
        F.wide[i] = H.wide[i];
    }
    F.t_lu = H.t_lu;
    F.nnz_l = (long long)H.lu.Lrow.size();
    F.nnz_u = (long long)H.lu.Ucol.size() + m;
    F.levels[0] = S.fl.nlev; F.levels[1] = S.fu.nlev; F.levels[2] = S.bu.nlev; F.levels[3] = S.bl.nlev;
    const SpTriHost *T4[4] = {&S.fl, &S.fu, &S.bu, &S.bl};
    if (F.m != m) {
        F.m = m;
        F.Y.ensure((size_t)m * SP_KMAX);
        F.zq.ensure(m);
        F.bt.ensure((size_t)2 * m);
        F.scr.ensure(m);
        F.scr2.ensure((size_t)2 * m);
        F.tpart.ensure((size_t)SP_KMAX * ((m + 255) / 256 + 1));
        F.bz.ensure(m);
        SPCHK(hipMemsetAsync(F.bz.p, 0, (size_t)m * sizeof(double), s));
    }
    F.P.ensure(SP_KMAX);
    F.hh.ensure((size_t)2 * SP_KMAX);
    F.upd.ensure((size_t)2 * SP_KMAX + 2);
    F.sacc.ensure((size_t)2 * SP_SEG_MAX);
    F.Minv.ensure((size_t)SP_KMAX * SP_KMAX);
    F.plog.ensure((size_t)2 * SP_KMAX);
    F.prep.ensure((size_t)2 * SP_KMAX);
    F.rst.ensure(sizeof(DState));
    F.hdr.ensure(8);
    if (sp_stamps_path()) {
        F.stamps.ensure((size_t)4 * SP_STAMP_MAX);
        SPCHK(hipMemsetAsync(F.stamps.p, 0, (size_t)4 * SP_STAMP_MAX * sizeof(unsigned long long), s));
        for (int i = 0; i < 4; i++) {
            const SpTriHost &T = *T4[i];
            F.lv_host[i].clear();
            for (int l = 0; l < T.nlev; l++) {
                F.lv_host[i].push_back(T.lvptr[l + 1] - T.lvptr[l]);
                F.lv_host[i].push_back(T.eptr[T.lvptr[l + 1]] - T.eptr[T.lvptr[l]]);
            }
        }
    }
    up_tri(s, F.fl, S.fl, F.hdr.p + 0);
    up_tri(s, F.fu, S.fu, F.hdr.p + 1);
    up_tri(s, F.bu, S.bu, F.hdr.p + 2);
    up_tri(s, F.bl, S.bl, F.hdr.p + 3);
    SPCHK(hipMemsetAsync(F.hdr.p + 4, 0, sizeof(int), s));          // k: no updates
    SPCHK(hipMemsetAsync(F.hdr.p + 6, 0, sizeof(int), s));          // the pivot log: empty
    SPCHK(hipStreamSynchronize(s));          // (pageable uploads of H's vectors)
    F.t_total = sp_now() - t0;
}

static int sp_factorize_cols(SpFactor &F, hipStream_t s, int m, const std::vector<int> &cptr,
                             const std::vector<int> &crow, const std::vector<double> &cval, double piv_tol,
                             int piv_lim, double eps_tol, double t0)
{
    sp_ahead_cancel(F);
    if (!F.cur) F.cur = new SpHost;
    sp_prepare(*F.cur, m, cptr, crow, cval, piv_tol, piv_lim, eps_tol);
    F.t_lu = F.cur->t_lu;
    if (F.cur->ret) return 1;
    sp_install(F, s, *F.cur, t0);
    return 0;
}

template <int NRHS>
static void ftran_lu(SpFactor &F, hipStream_t s, const SpDev &d, const DState *st, int gated, double *h0, double *h1);

// ---- the look-ahead ------------------------------------------------------
void sp_ahead_cancel(SpFactor &F)
{
    if (F.ahead.joinable()) F.ahead.join();
    F.ahead_mark = -1;
}

int sp_ahead_mark(const SpFactor &F) { return F.ahead_mark; }

// the pivots the current chain logged (synchronizes the stream)
int sp_log_count(SpFactor &F, hipStream_t s)
{
    int c = 0;
    if (!F.hdr.p) return 0;
    SPCHK(hipMemcpyAsync(&c, F.hdr.p + 6, sizeof(int), hipMemcpyDeviceToHost, s));
    SPCHK(hipStreamSynchronize(s));
    return c;
}

// B of the basis header head1 (as sp_factorize) factorized on a host thread;
// mark: the chain's pivot count at this basis
void sp_ahead_start(SpFactor &F, int m, const int *head1, const int *Aptr, const int *Aind, const double *Aval,
                    double piv_tol, int piv_lim, double eps_tol, int mark)
{
    sp_ahead_cancel(F);
    if (!F.nxt) F.nxt = new SpHost;
    SpHost *H = F.nxt;
    H->cptr.assign(m + 1, 0);
    H->crow.clear();
    H->cval.clear();
    for (int i = 1; i <= m; i++) {
        const int k = head1[i];
        if (k <= m) {
            H->crow.push_back(k - 1);
            H->cval.push_back(1.0);
        } else
            for (int t = Aptr[k - m - 1]; t < Aptr[k - m]; t++) {
                H->crow.push_back(Aind[t]);
                H->cval.push_back(-Aval[t]);
            }
        H->cptr[i] = (int)H->crow.size();
    }
    H->ret = 1;
    F.ahead_mark = mark;
    F.ahead = std::thread([H, m, piv_tol, piv_lim, eps_tol] {
        // (an exception must not leave the thread: std::terminate would end
        // a process that holds the GPU; a failed look-ahead is ret != 0 and
        // the caller factorizes synchronously)
        try {
            sp_prepare(*H, m, H->cptr, H->crow, H->cval, piv_tol, piv_lim, eps_tol);
        } catch (...) {
            H->ret = 1;
        }
    });
}

// h = -N_kq of the logged pivot j (the column the pivot brought in, as
// build_hq forms it) and the replay's state (p, kq, no stop); h was zeroed
__global__ void __launch_bounds__(256) k_sp_replay_col(double *h, int m, const int *cptr, const int *cind,
                                                       const double *cval, const int *log, int j, DState *rst)
{
    const int p = log[2 * j], kq = log[2 * j + 1];
    if (kq <= m) {
        if (threadIdx.x == 0) h[kq - 1] = -1.0;
    } else {
        const int c = kq - m - 1;
        for (int t = cptr[c] + threadIdx.x; t < cptr[c + 1]; t += blockDim.x) h[cind[t]] = cval[t];
    }
    if (threadIdx.x == 0) {
        rst->stop = 0;
        rst->p = p + 1;
        rst->kq = kq;
    }
}

// the look-ahead's factor installed in place of the current one, and the
// chain's pivots from its mark to cnt (the current chain length) replayed
// onto it: an FTRAN of each entering column and its Schur-complement update,
// in the pivots' order.  Returns the replayed count, or -1 when there was
// no look-ahead, its LU failed or a replayed update asked for a fresh
// factorization (the caller factorizes the current basis then).  A (CSC,
// the engine's device copy, 0-based) supplies the columns; h: m doubles of
// scratch; *t_wait: the time the join waited for the thread
int sp_ahead_install(SpFactor &F, hipStream_t s, int cnt, const int *Acptr, const int *Acind, const double *Acval,
                     double *h, double *t_wait)
{
    const int mark = F.ahead_mark;
    *t_wait = 0.0;
    if (mark < 0 || !F.ahead.joinable()) return -1;
    const double t0 = sp_now();
    F.ahead.join();
    F.ahead_mark = -1;
    *t_wait = sp_now() - t0;
    if (cnt < 0) cnt = sp_log_count(F, s);
    // (cnt > SP_KMAX: k_sp_update logs only the first SP_KMAX pivots of a
    // chain, so a longer one cannot be replayed from the log)
    if (F.nxt->ret || F.nxt->m != F.m || cnt < mark || cnt > SP_KMAX || cnt - mark > SP_KMAX) return -1;
    const int nrep = cnt - mark;
    if (nrep > 0)
        SPCHK(hipMemcpyAsync(F.prep.p, F.plog.p + 2 * mark, (size_t)2 * nrep * sizeof(int), hipMemcpyDeviceToDevice, s));
    std::swap(F.cur, F.nxt);
    sp_install(F, s, *F.cur, t0);
    const int m = F.m;
    DState *rst = (DState *)F.rst.p;
    SPCHK(hipMemsetAsync(rst, 0, sizeof(DState), s));
    SpDev d = sp_dev(F);
    for (int j = 0; j < nrep; j++) {
        SPCHK(hipMemsetAsync(h, 0, (size_t)m * sizeof(double), s));
        hipLaunchKernelGGL(k_sp_replay_col, dim3(1), dim3(256), 0, s, h, m, Acptr, Acind, Acval, (const int *)F.prep.p,
                           j, rst);
        ftran_lu<1>(F, s, d, nullptr, 0, h, nullptr);
        hipLaunchKernelGGL((k_sp_ftran_wood<1>), dim3((m + 255) / 256), dim3(256), 0, s, d, (const DState *)nullptr,
                           F.scr.p, (double *)nullptr, 0, 1);
        hipLaunchKernelGGL(k_sp_update, dim3(1), dim3(1024), 0, s, d, rst);
        hipLaunchKernelGGL(k_sp_ycol, dim3((m + 255) / 256), dim3(256), 0, s, d, (const DState *)rst);
    }
    int pend = 0;
    SPCHK(hipMemcpyAsync(&pend, &rst->refact_pending, sizeof(int), hipMemcpyDeviceToHost, s));
    SPCHK(hipStreamSynchronize(s));
    return pend ? -1 : nrep;
}

// one sweep by its plan; clr: the last launch clears bz (BTRAN of e_p)
template <int NRHS>
static void run_plan(const SpFactor &F, int which, const SpDev &d, hipStream_t s, const DState *st, int gate,
                     const double *in0, const double *in1, double *out0, double *out1, int clr)
{
    const TriDev &t = which == 0 ? d.fl : which == 1 ? d.fu : which == 2 ? d.bu : d.bl;
    const auto &pl = F.plan[which];
    for (size_t q = 0; q < pl.size(); q++) {
        const int last = clr && q + 1 == pl.size();
        if (pl[q].grid == 2) {
            const auto &g = pl[q];
            if (g.pre)
                hipLaunchKernelGGL((k_sp_seg_a<NRHS>), dim3(g.ablocks), dim3(256), 0, s, t, st, gate, in0, in1,
                                   (const double *)out0, (const double *)out1, g.sb, g.ns, g.nas, F.sacc.p);
            hipLaunchKernelGGL((k_sp_seg<NRHS>), dim3(1), dim3(1024), 0, s, d, t, st, gate, in0, in1, out0, out1, g.sb,
                               g.ns, g.nas, g.l0, g.l1, g.pre, (const double *)F.sacc.p, last);
        } else if (pl[q].grid) {
            hipLaunchKernelGGL((k_sp_level<NRHS>), dim3(pl[q].blocks), dim3(256), 0, s, t, st, gate, in0, in1, out0,
                               out1, pl[q].l0);
            if (last)
                hipLaunchKernelGGL((k_sp_sweep<NRHS>), dim3(1), dim3(1024), 0, s, d, t, st, gate, in0, in1, out0,
                                   out1, 0, 0, 1);
        } else
            hipLaunchKernelGGL((k_sp_sweep<NRHS>), dim3(1), dim3(1024), 0, s, d, t, st, gate, in0, in1, out0,
                               out1, pl[q].l0, pl[q].l1, last);
    }
    if (pl.empty() && clr)
        hipLaunchKernelGGL((k_sp_sweep<NRHS>), dim3(1), dim3(1024), 0, s, d, t, st, gate, in0, in1, out0, out1, 0,
                           0, 1);
}

// the fused sweep kernels may take up to 2 * 8 * SP_LDS_M bytes of dynamic LDS
static void sp_lds_attrs()
{
    static const bool done = [] {
        const int bytes = 2 * 8 * SP_LDS_M;
        (void)hipFuncSetAttribute((const void *)k_sp_ftran_lu<1>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        (void)hipFuncSetAttribute((const void *)k_sp_ftran_lu<2>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        (void)hipFuncSetAttribute((const void *)k_sp_btran<1>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        (void)hipFuncSetAttribute((const void *)k_sp_btran<2>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        return true;
    }();
    (void)done;
}

// z = inv(L U) [h0, h1] (L in place, U into bt) and inv(M) z[P]: one fused
// workgroup launch, or with wide levels the plans of both sweeps
template <int NRHS>
static void ftran_lu(SpFactor &F, hipStream_t s, const SpDev &d, const DState *st, int gated, double *h0, double *h1)
{
    if (!F.wide[0] && !F.wide[1]) {
        sp_lds_attrs();
        const int lds = sp_lds_on() && F.m <= SP_LDS_M;
        hipLaunchKernelGGL((k_sp_ftran_lu<NRHS>), dim3(1), dim3(1024), lds ? (size_t)NRHS * F.m * sizeof(double) : 0, s,
                           d, st, h0, h1, gated, 3, 0, 0, lds);
        return;
    }
    double *x0 = F.bt.p, *x1 = F.bt.p + F.m;
    run_plan<NRHS>(F, 0, d, s, st, gated, h0, h1, h0, h1, 0);
    run_plan<NRHS>(F, 1, d, s, st, gated, h0, h1, x0, x1, 0);
    hipLaunchKernelGGL((k_sp_hh<NRHS>), dim3(1), dim3(1024), 0, s, d, st, gated);
}

// the BTRAN (Schur correction, U', L'): one fused workgroup launch, or the
// correction alone and then the plans of both sweeps
template <int NRHS>
static void btran_seq(SpFactor &F, hipStream_t s, const SpDev &d, DState *st, const double *e, double *y, int mode,
                      int nparts, const double *e1, double *y1)
{
    if (!F.wide[2] && !F.wide[3]) {
        sp_lds_attrs();
        const int lds = sp_lds_on() && F.m <= SP_LDS_M && (NRHS == 1 || F.m <= SP_LDS_M / 2);
        hipLaunchKernelGGL((k_sp_btran<NRHS>), dim3(1), dim3(1024), lds ? (size_t)2 * NRHS * F.m * sizeof(double) : 0,
                           s, d, st, e, y, mode, nparts, e1, y1, 7, 0, 0, lds);
        return;
    }
    const int gate = mode >= 1 ? 2 : 0, m = F.m;
    double *b0 = (mode == 1) ? F.bz.p : F.bt.p, *b1 = F.bt.p + m, *w0 = F.scr2.p, *w1 = F.scr2.p + m;
    hipLaunchKernelGGL((k_sp_btran<NRHS>), dim3(1), dim3(1024), 0, s, d, st, e, y, mode, nparts, e1, y1, 1, 0, 0, 0);
    run_plan<NRHS>(F, 2, d, s, st, gate, b0, b1, w0, w1, 0);
    run_plan<NRHS>(F, 3, d, s, st, gate, w0, w1, y, y1, mode == 1);
}

// y = inv(B) x (positions), x untouched (device vectors)
void sp_ftran(SpFactor &F, hipStream_t s, const double *x, double *y)
{
    const int m = F.m;
    double *scratch = F.scr.p;
    SpDev d = sp_dev(F);
    SPCHK(hipMemcpyAsync(scratch, x, (size_t)m * sizeof(double), hipMemcpyDeviceToDevice, s));
    ftran_lu<1>(F, s, d, nullptr, 0, scratch, nullptr);
    hipLaunchKernelGGL((k_sp_ftran_wood<1>), dim3((m + 255) / 256), dim3(256), 0, s, d, (const DState *)nullptr, y,
                       (double *)nullptr, 0, 0);
}

// y = inv(B)' x (rows)
void sp_btran(SpFactor &F, hipStream_t s, const double *x, double *y)
{
    const int m = F.m;
    SpDev d = sp_dev(F);
    const int nb = (m + 255) / 256;
    hipLaunchKernelGGL(k_sp_btran_part, dim3(nb), dim3(256), 0, s, d, x);
    btran_seq<1>(F, s, d, nullptr, x, y, 0, nb, nullptr, nullptr);
}

// the pivot's hooks (gated on the stop word, captured with the rest)
void sp_pivot_btran(SpFactor &F, hipStream_t s, DState *st, double *rho)
{
    SpDev d = sp_dev(F);
    btran_seq<1>(F, s, d, st, nullptr, rho, 1, 0, nullptr, nullptr);
}

// the primal's BTRANs of a pivot (p > 0 only): rho = inv(B)' e_p and
// update_gamma's u = inv(B)' v in one sweep pair
void sp_pivot_btran2(SpFactor &F, hipStream_t s, DState *st, const double *v, double *rho, double *u)
{
    const int m = F.m;
    SpDev d = sp_dev(F);
    const int nb = (m + 255) / 256;
    hipLaunchKernelGGL(k_sp_btran_part, dim3(nb), dim3(256), 0, s, d, v);
    btran_seq<2>(F, s, d, st, nullptr, rho, 2, nb, v, u);
}

void sp_pivot_ftran(SpFactor &F, hipStream_t s, const DState *st, double *h, double *work, double *tcol, double *u,
                    int pse)
{
    const int m = F.m;
    SpDev d = sp_dev(F);
    if (pse) {
        ftran_lu<2>(F, s, d, st, 1, h, work);
        hipLaunchKernelGGL((k_sp_ftran_wood<2>), dim3((m + 255) / 256), dim3(256), 0, s, d, st, tcol, u, 1, 1);
    } else {
        ftran_lu<1>(F, s, d, st, 1, h, nullptr);
        hipLaunchKernelGGL((k_sp_ftran_wood<1>), dim3((m + 255) / 256), dim3(256), 0, s, d, st, tcol,
                           (double *)nullptr, 1, 1);
    }
}

void sp_pivot_update(SpFactor &F, hipStream_t s, DState *st)
{
    SpDev d = sp_dev(F);
    hipLaunchKernelGGL(k_sp_update, dim3(1), dim3(1024), 0, s, d, st);
    hipLaunchKernelGGL(k_sp_ycol, dim3((F.m + 255) / 256), dim3(256), 0, s, d, (const DState *)st);
}

// GK_SP_STAMPS=<file>: the device-clock duration of every level of the four
// sweeps in the last pivot (stamped by tri_sweep's thread 0 after each level
// barrier; levels that ran on the grid are not stamped), with the level's
// steps and entries; one line per sweep, appended to the file
void sp_stamps_dump(SpFactor &F, hipStream_t s, int wall_khz)
{
    const char *path = sp_stamps_path();
    if (!path || !F.stamps.p) return;
    std::vector<unsigned long long> h((size_t)4 * SP_STAMP_MAX);
    SPCHK(hipMemcpyAsync(h.data(), F.stamps.p, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    SPCHK(hipStreamSynchronize(s));
    FILE *fp = std::fopen(path, "a");
    if (!fp) return;
    static const char *names[4] = {"ftran_L", "ftran_U", "btran_U'", "btran_L'"};
    for (int i = 0; i < 4; i++) {
        const int nl = (int)F.lv_host[i].size() / 2;
        std::fprintf(fp, "%s levels %d:", names[i], nl);
        for (int l = 0; l < nl && l + 1 < SP_STAMP_MAX; l++) {
            const unsigned long long a = h[(size_t)i * SP_STAMP_MAX + l], b = h[(size_t)i * SP_STAMP_MAX + l + 1];
            const double us = (a && b > a) ? 1e3 * (double)(b - a) / wall_khz : -1.0;
            std::fprintf(fp, " %d/%d:%.2f", F.lv_host[i][2 * l], F.lv_host[i][2 * l + 1], us);
        }
        std::fprintf(fp, "\n");
    }
    std::fclose(fp);
}

// ---------------------------------------------------------------------------
// diagnostics (host only, no device): the factor of a basis given as CSC
// (1-based like gk_bfd_factorize_csc: ptr[1..m+1], ind 1-based) and the four
// sweeps run on the host in the same level order the device runs them:
// x = inv(B) b, y = inv(B)' e.  Returns 0, 1 (singular) or -1 (bad input);
// stats[0..5] = nnz(L), nnz(U) incl. diagonal, levels FTRAN L / U,
// BTRAN U' / L'.  Lets the CPU tests pin the elimination and the level
// schedules against numpy without a GPU.
// ---------------------------------------------------------------------------
// a sweep by its plan (the LDS segments' two passes, as k_sp_seg runs them)
static void host_sweep_plan(const SpTriHost &t, const std::vector<SpFactor::Seg> &plan, const double *in, double *out)
{
    std::vector<double> acc;
    for (const auto &g : plan) {
        if (g.grid != 2) {
            for (int l = g.l0; l < g.l1; l++)
                for (int s = t.lvptr[l]; s < t.lvptr[l + 1]; s++) {
                    double a = in[t.iin[s]];
                    for (int e = t.eptr[s]; e < t.eptr[s + 1]; e++) a -= t.eval[e] * out[t.eidx[e]];
                    out[t.iout[s]] = a / t.diag[s];
                }
            continue;
        }
        acc.assign(g.ns, 0.0);
        for (int i = 0; i < g.ns; i++) {
            const int li = t.aord[g.sb + i], s = g.sb + li;
            double a = in[t.iin[s]];
            for (int e = t.eptr[s]; e < t.emid[s]; e++) a -= t.eval[e] * out[t.eidx[e]];
            acc[li] = a;
        }
        for (int l = g.l0; l < g.l1; l++)
            for (int s = t.lvptr[l]; s < t.lvptr[l + 1]; s++) {
                double a = acc[s - g.sb];
                const int n = t.srn[s];
                if (n != t.eptr[s + 1] - t.emid[s]) throw std::runtime_error("sparse factor: step record count");
                for (int u = 0; u < SP_RECN && u < n; u++) {    // the record, as k_sp_seg reads it
                    const int w = t.srx[(size_t)(SP_RECN / 2) * s + u / 2];
                    const int ix = (u & 1) ? (int)((unsigned)w >> 16) : (w & 0xffff);
                    a -= t.srv[(size_t)SP_RECN * s + u] * acc[ix];
                }
                for (int e = t.emid[s] + SP_RECN; e < t.eptr[s + 1]; e++) a -= t.eval[e] * acc[t.eidx[e]];
                acc[s - g.sb] = (s < t.lvlong[l]) ? a * t.srd[s] : a / t.diag[s];
                out[t.iout[s]] = acc[s - g.sb];
            }
    }
}

}  // namespace gk

extern "C" int gk_sp_selftest(int m, const int *ptr, const int *ind, const double *val, const double *b,
                              const double *e, double *x, double *y, long long *stats)
{
    using namespace gk;
    HostProf host_prof_;                      // GK_HOST_PROF (diagnostics)
    if (m < 1 || !ptr || !ind || !val) return -1;
    std::vector<int> cptr(m + 1, 0), crow;
    std::vector<double> cval;
    for (int j = 1; j <= m; j++) {
        for (int t = ptr[j]; t < ptr[j + 1]; t++) {
            if (ind[t] < 1 || ind[t] > m) return -1;
            crow.push_back(ind[t] - 1);
            cval.push_back(val[t]);
        }
        cptr[j] = (int)crow.size();
    }
    SpLU lu;
    SpLUWork wk;
    int rank = 0;
    if (std::getenv("GK_SP_TIMES")) sp_lu_factor(lu, wk, m, cptr, crow, cval, 0.1, 4, 1e-15, &rank);   // warm storage
    const double t0 = sp_now();
    if (sp_lu_factor(lu, wk, m, cptr, crow, cval, 0.1, 4, 1e-15, &rank)) return 1;
    const double t1 = sp_now();
    SpSolves S;
    std::vector<SpFactor::Seg> pl[4];
    int wd[4];
    sp_build_solves(lu, S, pl, wd);
    const double t2 = sp_now();
    if (stats) {
        stats[0] = (long long)lu.Lrow.size();
        stats[1] = (long long)lu.Ucol.size() + m;
        stats[2] = S.fl.nlev; stats[3] = S.fu.nlev; stats[4] = S.bu.nlev; stats[5] = S.bl.nlev;
    }
    // the sweeps as the device runs them: re-encoded for LDS segments
    // (GK_SP_SEG, sp_plan_sweep) and solved by their plans
    if (std::getenv("GK_SP_TIMES"))
        fprintf(stderr, "[gk sp times] LU %.2f ms, solves and plans %.2f ms\n", 1e3 * (t1 - t0), 1e3 * (t2 - t1));
    if (std::getenv("GK_SP_LEVELS")) {
        const SpTriHost *T4[4] = {&S.fl, &S.fu, &S.bu, &S.bl};
        for (int i = 0; i < 4; i++) {
            std::string line = "[gk sp plan]";
            for (const auto &g : pl[i]) {
                char b[160];
                if (g.grid == 2) {
                    long long ext = 0, in = 0;
                    int mx = 0;
                    for (int st = g.sb; st < g.sb + g.ns; st++) {
                        ext += T4[i]->emid[st] - T4[i]->eptr[st];
                        in += T4[i]->eptr[st + 1] - T4[i]->emid[st];
                        mx = std::max(mx, T4[i]->eptr[st + 1] - T4[i]->emid[st]);
                    }
                    snprintf(b, sizeof b, " seg[%d,%d) ns %d ext %lld%s int %lld max %d;", g.l0, g.l1, g.ns, ext,
                             g.pre ? "(grid)" : "", in, mx);
                } else
                    snprintf(b, sizeof b, " %s[%d,%d);", g.grid ? "grid" : "run", g.l0, g.l1);
                line += b;
            }
            fprintf(stderr, "%s\n", line.c_str());
        }
    }
    std::vector<double> z(b, b + m), w(m);
    host_sweep_plan(S.fl, pl[0], z.data(), z.data());
    host_sweep_plan(S.fu, pl[1], z.data(), x);
    host_sweep_plan(S.bu, pl[2], e, w.data());
    host_sweep_plan(S.bl, pl[3], w.data(), y);
    return 0;
}
