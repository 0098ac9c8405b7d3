// Internal interfaces of libglpk_mi355x: device state layout, kernel
// launchers (gk_kernels.hip) and the engine structures (gk_engine.hip).
//
// Device layout (all 0-based in HBM; the reference's 1-based variable
// numbers k = 1..m+n are kept as *values* in head[]):
//   type/lb/ub/coef[k-1]            working bounds and objective, scaled as init_csa
//   head[pos-1] = k                 basis header, pos 1..m basic, m+1..m+n non-basic
//   bind[k-1]   = pos               inverse of head
//   stat[j-1]                       status of non-basic xN[j]
//   bbar[i-1], cbar[j-1]            values of basic variables / reduced costs
//   gamma[]                         steepest-edge weights (m for dual, n for primal)
//   A                               dense column-major (lda) or CSC + CSR copies
//   Binv[(i-1) + (r-1)*ldb]         explicit inverse of the basis matrix:
//                                   row i = basis position, column r = row of (I|-A)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <vector>

struct gk_comm;                     // the library's collective (gk_comm.hip, include/glpk_mi355x.h)

namespace gk {

enum : int {  // GLP_* (glpk.js:7-141)
    FR = 1, LO = 2, UP = 3, DB = 4, FX = 5,
    BS = 1, NL = 2, NU = 3, NF = 4, NS = 5,
    PT_STD = 0x11, PT_PSE = 0x22, RT_STD = 0x11, RT_HAR = 0x22,
};

// why a device batch of pivots stopped (the reference main-loop branch the
// host resumes at; glpspx02.js:1614-1966, glpspx01.js:1705-2056)
enum : int {
    ST_RUN = 0,
    ST_BATCH = 1,     // iteration budget of the batch used up
    ST_PHASE = 2,     // phase I reached feasibility: switch to phase II
    ST_OBJLIM = 3,    // obj_ll / obj_ul reached (dual, phase II)
    ST_P0 = 4,        // no basic variable chosen (dual: optimal / primal: unbounded ray)
    ST_Q0 = 5,        // no non-basic variable chosen
    ST_SMALLPIV = 6,  // pivot below 1e-5 (1 + 0.01 max) and not in rigorous mode
    ST_PIVCHK = 7,    // tcol[p] and trow[q] disagree
    ST_DCHK = 8,      // primal: cbar[q] disagrees with re-evaluated d_q
    ST_REFACT = 9,    // update limit reached: re-invert before the next pivot
    ST_REFSP = 10,    // PSE reference space must be reset (refct == 0)
};
// the gate mode of the end-of-call epilogue's kernels (GATE, gk_device.h)
constexpr int EPI_GATE = 0x100;


struct DState {
    int stop, p, q, p_stat;
    int phase, it_cnt, npiv, iter_left;
    int refct, upd_cnt, upd_lim, rigorous;
    int binv_fresh, cbar_fresh, pricing, rtest;
    int refact_pending, nr, ns, nw;        // nr: dense columns of inv(B); ns: support of rho; nw: nonzeros of A w
    int ce, pend, dinf, nwl;                // ce: column of inv(B) that becomes e_p (-1: none); pend: change_basis
                                            // pending; dinf: phase-I dual infeasibility seen; nwl: entries of wlist
    int need2, q1, pad0, pad1;              // Harris pass 2 needed; pass-1 choice
    double delta, teta, new_dq, cbar_q_new;
    double gamma_pq, eta_pq, pivot, xnq;
    double zeta, tol_bnd, tol_dj, tol_piv;
    double obj_ll, obj_ul, obj, tcol_max;
    double cbar_q_old, bytes;               // bytes: algorithmic HBM bytes of the pivots so far
    double teta1, bytes_trow;               // bytes_trow: algorithmic bytes of the pivot-row kernels
    unsigned long long tk_start, tk_end;    // device wall clock around the last pivot-row kernel
    unsigned long long tk_next, tk_pad;     // entry of the kernel after it
    double trow_ticks, trow_n;              // accumulated execution span of the pivot-row kernels (row path)
    double trow_ticks_b, trow_pad;          // same, entry to the next kernel's entry (dispatch included)
    unsigned long long trow_max_bits, tcol_max_bits;
    int kp, kq, fxp, rclr;                  // dual: leaving / entering variable of the pivot; x_kp fixed;
                                            // refsp[kp] to clear at change_basis
    int kq1, echk, page, pad4;              // variable of the pass-1 choice; echk: growth re-inversions requested;
                                            // page: product-form updates the pricing panel's rows went through
    double alfa1;                           // |trow| of the pass-1 choice
    unsigned long long grow_bits;           // max |tcol_i / alpha_p| (as double bits) of the product-form updates since
                                            // the last re-inversion, recorded when it exceeds 100
    unsigned long long tk_prev, tk_pad2;    // last block exit of the kernel before the pivot-row kernel
    double trow_ticks_r, trow_nr;           // pivot-row kernels, previous kernel's last exit to their last
                                            // exit (the bracket of a profiler's per-dispatch record)
    unsigned long long tk_upd0, tk_pad3;    // entry of the last k_dual_update (block 0)
    double upd_ticks, upd_n;                // k_dual_update spans (entry of block 0 to the last block exit)
    double bytes_upd, upd_tol;              // algorithmic bytes of the k_dual_update launches; bfcp upd_tol
    // MFMA panel pricing (gk_panel.hip): rows in the panel, slot of this
    // pivot's row, 1 when this pivot refilled the panel, 0 until the first
    // fill of the batch; hits and refills so far
    int pk, pcur, pmiss, pvalid;
    double phits, pmisses;
    // the entry gate of the multi-block pivot kernels (gk_device.h,
    // gate_arrive / gate_wait): arrivals per XCD slot of blockIdx, 0 between
    // launches
    int gate[8], gate_top, gate_pad;
    // the outbox of k_dual_row: the pivot it chose (p, kp, delta, ns) and the
    // reference-space reset, stored by its last block where no block of the
    // launch reads them; k_dual_ratio's block 0 applies them (and the pending
    // change of basis' counters) before any later kernel reads the state
    int ob_p, ob_kp, ob_ns, ob_reset;
    double ob_delta;
    // primal: the reduced cost of xN[q] after k_primal_ratio's d_q check (the
    // value it stores in cbar[q]); k_primal_commit reads it here, since the
    // commit thread owning cbar[q] overwrites that entry while other blocks
    // still need the old value
    double dq_ratio;
};

// ---- dense GEMV helpers ---------------------------------------------------
struct GemvPlan {
    int rows, cols, ld;
    int tiles, splits, cols_per_split;
};
GemvPlan gemv_plan(int rows, int cols, int ld);

// y = beta*base + alpha * M x  (M col-major rows x cols, zero entries of x skipped)
void gemv_n(hipStream_t s, const double *M, int rows, int cols, int ld, const double *x,
            double *partial, size_t partial_cap, double *y, double alpha, const double *base, double beta);
// y[l] = alpha * M[:,l] . x   for l < cols
void gemv_t(hipStream_t s, const double *M, int rows, int cols, int ld, const double *x, double *y, double alpha);

// ---- the (I | -A) column passes -------------------------------------------
// rows of a CSR matrix longer than this are summed by a whole wave (or, in
// k_dual_ratio's A w, a whole block) instead of by their own thread
constexpr int CSR_LONG = 32;
struct MatDev {
    int m, n, nnz;
    int dense;                    // 1: A dense column-major
    const double *A; int lda;     // dense
    const int *cptr, *cind; const double *cval;   // CSC, 0-based rows
    const int *rptr, *rcol; const double *rval;   // CSR, 0-based cols
    const double *AT; int ldt;    // dense: row-major copy (AT[r*ldt + c] = A[r, c]) for row-wise pivot rows
    int lpc;                      // lanes per column for CSC passes (1, 8 or 64)
    const int *lrow; int nlr;     // sparse: the rows longer than CSR_LONG (k_dual_ratio's A w: a block each)
};

enum : int { CP_TROW = 0, CP_CBAR = 1, CP_RESID = 2, CP_TROW_S = 3, CP_DOT = 4 };
// For positions pos = off+1 .. off+cnt: k = head[pos-1], N = column k of (I|-A):
//   CP_TROW   out1[i] = -(N . x), 0 if stat[i] == NS; atomic max |out1| into *maxbits
//   CP_CBAR   out1[i] = coef[k-1] - N . x
//   CP_RESID  out1[i] = h[i] - N . x
//   CP_TROW_S out1[i] = -(N . x), out2[i] = N . y  (0, 0 if NS)
//   CP_DOT    out1[i] = N . x
void colpass(hipStream_t s, const MatDev &A, int mode, int off, int cnt, const int *head, const signed char *stat,
             const double *coef, const double *h, const double *x, const double *y, double *out1, double *out2,
             unsigned long long *maxbits);

// y = base - A w  over structural columns (w dense over columns, zeros skipped);
// used for sums of (I|-A) columns (slack parts are added into base by the caller)
// glp_eval_tab_row for a batch (gk_tabrow.hip): out[t * (m + n) + k - 1]
void tab_rows(hipStream_t s, const double *Binv, int ldb, const MatDev &A, int nk, const int *pos, double *G,
              const double *aux, const double *cs, const double *rs, double *out, int use_mfma);
// (from, dense A only: y = from - (base - A w), the residual of eval_beta's refinement in one pass)
void aprod_neg_gated(hipStream_t s, const MatDev &A, const double *w, const double *base, double *y,
                     double *partial, size_t cap, const DState *st, int need_p, const double *from = nullptr);
void aprod_neg(hipStream_t s, const MatDev &A, const double *w, const double *base, double *y,
               double *partial, size_t partial_cap);

// scatter weights of positions off+1..off+cnt: w[pos] -> slack part ys[k-1] += w,
// structural part wc[c-1] = w  (ys, wc must be zeroed by the caller)
void scatter_pos(hipStream_t s, int m, int off, int cnt, const int *head, const double *w, double *ys, double *wc);

// ---- simplex pivot kernels --------------------------------------------------
// ---- sparse basis factor (gk_sparse.hip): B0 = L U on the host, level-
// scheduled sweeps on the device, Schur-complement updates (k <= SP_KMAX)
constexpr int SP_KMAX = 256;
struct SpFactor;
SpFactor *sp_create();
void sp_destroy(SpFactor *F);
void sp_info(const SpFactor *F, long long *nnz_lu, int *levels, double *t_lu);
// a sparse dual pivot's chain-independent algorithmic bytes (gk_dual.hip)
double sp_pivot_bytes(const struct SpxDev &d);
// 0, or 1 when B0 is singular; head1 1-based over (I | -A); A CSC, 0-based rows
int sp_factorize(SpFactor &F, hipStream_t s, int m, const int *head1, const int *Aptr, const int *Aind,
                 const double *Aval, double piv_tol, int piv_lim, double eps_tol);
int sp_factorize_csc(SpFactor &F, hipStream_t s, int m, const int *ptr, const int *ind, const double *val,
                     double piv_tol, int piv_lim, double eps_tol);
void sp_ftran(SpFactor &F, hipStream_t s, const double *x, double *y);   // y = inv(B) x
void sp_btran(SpFactor &F, hipStream_t s, const double *x, double *y);   // y = inv(B)' x
struct DState;
void sp_pivot_btran(SpFactor &F, hipStream_t s, DState *st, double *rho);
void sp_pivot_ftran(SpFactor &F, hipStream_t s, const DState *st, double *h, double *work, double *tcol, double *u,
                    int pse);
void sp_pivot_update(SpFactor &F, hipStream_t s, DState *st);
void sp_pivot_btran2(SpFactor &F, hipStream_t s, DState *st, const double *v, double *rho, double *u);
void sp_stamps_dump(SpFactor &F, hipStream_t s, int wall_khz);
// the look-ahead factorization (gk_sparse.hip): started on a host thread at
// a basis of the chain (mark: the chain's pivot count there), installed at
// the next refactorization with the later pivots replayed (returns their
// count, or -1: factorize the current basis instead)
void sp_ahead_start(SpFactor &F, int m, const int *head1, const int *Aptr, const int *Aind, const double *Aval,
                    double piv_tol, int piv_lim, double eps_tol, int mark);
void sp_ahead_cancel(SpFactor &F);
int sp_ahead_mark(const SpFactor &F);
int sp_log_count(SpFactor &F, hipStream_t s);
int sp_ahead_install(SpFactor &F, hipStream_t s, int cnt, const int *Acptr, const int *Acind, const double *Acval,
                     double *h, double *t_wait);   // GK_SP_STAMPS (diagnostics)

struct SpxDev {
    int m, n;
    MatDev A;
    signed char *type, *orig_type, *stat, *refsp;
    double *lb, *ub, *coef, *orig_lb, *orig_ub, *obj;
    int *head, *bind;
    double *bbar, *cbar, *gamma;
    double *tcol, *trow, *rho, *rowp, *u, *s, *h, *wcol, *ys, *work, *r1, *r2;
    double *Binv; int ldb;
    double *partial; size_t partial_cap;
    DState *st;
    // columns of inv(B) that are not unit vectors: inv(B) e_c = e_{bind[c]} for every
    // basic slack c, so only the nr columns rlist[0..nr) (the non-basic slacks) are dense
    int *rlist, *rpos;
    int *rho_idx; double *rho_val;          // rho in compact form, ns entries
    double *gpart;                           // per-block partial sums of the pivot-row pass
    // structural columns in the PSE reference space that are non-basic (the
    // columns A w of update_gamma runs over), maintained like rlist
    int *wlist, *wpos;
    double *cand;                            // per-block candidates: chuzr | pass 1 | pass 2
    double *awpart;                          // partial sums of A w
    size_t awpart_cap;
    int *awcnt;                              // per 512-row tile: arrivals of the A w splits (the last one reduces)
    unsigned long long *tslots;              // per-block end stamps of the pivot-row kernel
    unsigned long long *xslots;              // per-block exit stamps of the commit / update kernel
    unsigned long long *trace;               // profiling only: per-kernel, per-block entry / exit clock
    // MFMA panel pricing (gk_panel.hip): PANEL_MAX tableau rows over the
    // structural columns (pnl[t * ldp + j]), the rows of inv(B) they were
    // formed from (pnl_src[t * m + i]), the basis position of every slot
    // (ppos, 1-based) and the slot of every position (pslot, validated
    // against ppos)
    double *pnl, *pnl_src;
    int *pslot, *ppos;
    int ldp;
    SpFactor *sp;                            // host pointer: the sparse factor (nullptr: explicit inverse)
    struct LpShard *shard;                   // host pointer: column-sharded pricing (gk_bfd_set_comm), or nullptr
};

// column-sharded pricing of one LP (gk_bfd_set_comm): every rank
// holds the whole problem and factor and takes the same pivots; the pivot
// row's column pass runs over this rank's slice of the non-basic positions
// [rank L, rank L + L), L = ceil(n / size), and with PSE so does
// update_gamma's A w (the members of W in the slice); the slices (with each
// slice's max |trow|) and the A w partials are all-gathered before the ratio
// test (L + 1 + m doubles per rank)
struct LpShard {
    ::gk_comm *comm = nullptr;
    int rank = 0, size = 1, L = 0, n = 0, m = 0;
    // GK_SHARD_SIM = G with one rank (GK_SHARD_ONE_RANK): the G ranks' slices
    // formed one after another by this process, packed straight into the
    // receive blocks (no exchange) — the G-rank run's results, and per-slice
    // kernel times as one rank of G on its own GPU would see them
    int vsize = 0;
    double *dsend = nullptr, *drecv = nullptr;  // device: L + 1 + m | max(size, vsize) (L + 1 + m) doubles
    std::vector<double> hsend, hrecv;           // host staging (TCP transport)
    long long exchanges = 0;
    bool failed = false;
    ~LpShard();
};
// the all-gather of device blocks on stream s: RCCL on the stream itself,
// TCP through the host staging (synchronizes s); 0 on success
int gk_comm_allgather_dev(::gk_comm *c, const void *dsend, size_t bytes, void *drecv, hipStream_t s,
                          void *hsend, void *hrecv);
int gk_comm_size_rank(const ::gk_comm *c, int *rank);
void gk_comm_abort(::gk_comm *c);
void lp_shard_trow(hipStream_t s, const SpxDev &d, int pse);
void lp_shard_sim(hipStream_t s, const SpxDev &d, int pse);     // the pivot row of vsize simulated ranks
// a host decision every rank of the shard takes together: true when any
// rank's flag is set (one all-gather of a byte); throws if the exchange fails
bool shard_any(LpShard &sh, bool flag);
// a rank-local failure of the sharded LP: the communicator is aborted so
// that the peers' exchanges fail instead of waiting (gk_comm_abort)
void shard_abort(LpShard &sh);
bool lp_force_colpass();                     // GK_FORCE_COLPASS: the sharded plan on one GPU (comparisons)
constexpr int PANEL_MAX = 32;
constexpr int TRACE_KERNELS = 8, TRACE_BLOCKS = 2048;   // trace[(kid * TRACE_BLOCKS + block) * 2 + {0, 1}]
constexpr int TRACE_PHASES = 8;   // then phase stamps of wave 0: [TRACE_KERNELS * TRACE_BLOCKS * 2 + (kid * TRACE_BLOCKS + block) * 8 + ph]
constexpr size_t TRACE_LEN = (size_t)TRACE_KERNELS * TRACE_BLOCKS * (2 + TRACE_PHASES);

// launch geometry of one device batch, fixed on the host from nr at batch start
struct DualPlan {
    int pse, rigorous;
    int rowpath;                  // 1: pivot row by rows of AT over the support of rho
    int fused;                    // 1: dense A — h and A w read inside the FTRAN kernels
    int tsplits;                  // row path: splits over the support of rho (timing utility)
    int twaves;                   // row path: waves per 64-column block of k_trow_rows
    int fsplits;                  // FTRAN over the dense columns of inv(B): splits
    int uchunks;                  // rank-1 update: column chunks
    int awsplits;                 // A w over wlist: splits
    int nr_cap, ns_cap;           // upper bounds of nr / ns over the batch (speculative list loads)
    int fone, fwaves;             // 1: FTRAN in one kernel (k_dual_ftran1), fwaves waves per 64-row block
    int lpsu;                     // rank-1 update: list entries per chunk
    int colpath;                  // 1: sparse A — k_dual_col, CSR A w in k_dual_ratio, sparse k_dual_ftran1
    int fupd;                     // 1: FTRAN + commit in one kernel (k_dual_update)
    int ugm, uwaves;              // k_dual_update: inv(B) entries per thread, waves per block
    int gm;                       // chuzr candidate slots (4 per 256 rows, or one per 16 rows with fupd)
    int awone;                    // dense A w in one pass over 64-row tiles: the cap of nwl (0: split path)
    int panel;                    // rows of the MFMA pricing panel (0: the pivot row is a column pass over A)
    int panel_age;                // product-form updates a panel row may go through before a refill
    int sparse;                   // 1: sparse factor (gk_sparse.hip): BTRAN / FTRAN / update hooks
};
void dual_batch_begin(hipStream_t s, const SpxDev &d, const DualPlan &pl);
void dual_batch_end(hipStream_t s, const SpxDev &d, const DualPlan &pl);
DualPlan dual_plan(const SpxDev &d, int nr_max, int nwl_max, int pse, int rigorous);
// ev0/ev1, ev2/ev3 (optional, eager launches only): the start / stop events
// of the pivot-row kernel and of the fused update kernel (hipExtLaunchKernelGGL:
// the command processor's timestamps of the dispatch itself, as a profiler's)
void dual_iteration2(hipStream_t s, const SpxDev &d, const DualPlan &pl, hipEvent_t ev0 = nullptr,
                     hipEvent_t ev1 = nullptr, hipEvent_t ev2 = nullptr, hipEvent_t ev3 = nullptr);
void transpose_dense(hipStream_t s, const double *A, int m, int n, int lda, double *AT, int ldt);
// primal pivot pipeline (gk_primal.hip); the plan reuses DualPlan's fields
DualPlan primal_plan(const SpxDev &d, int nr_max, int pse);
bool primal_fast_ok(const SpxDev &d);
void primal_batch_begin(hipStream_t s, const SpxDev &d);
void primal_iteration2(hipStream_t s, const SpxDev &d, const DualPlan &pl);
// the primal pivot on the sparse factor (gk_sparse.hip hooks)
void primal_iteration_sparse(hipStream_t s, const SpxDev &d, int pse);
// coalesced host->device uploads: segment g of a staged region goes to g.dst
struct UpSeg {
    size_t off;
    void *dst;
    size_t bytes;
};
void scatter_segments(hipStream_t s, const char *src, const UpSeg *segs, int nseg);
// dual, dense A: CP_CBAR / CP_RESID of eval_cbar over the rows of AT in rlist
// (eg: the epilogue's form — gated on eg, nr read from eg->nr, the argument
// an upper bound of it; the same sums in the same order)
void rowpass_pi(hipStream_t s, const SpxDev &d, int mode, int nr, const double *pi, const double *h, double *out,
                const int *extra, int nextra, const DState *eg = nullptr, const double *pi2 = nullptr);
// MFMA panel pricing (gk_panel.hip), column-pass path on dense A: the chosen
// row from the panel (refilled on a miss) in place of the column pass, and
// the panel's update after the commit; panel_wanted: the plan's panel size
int panel_wanted(const SpxDev &d, const DualPlan &pl);
int panel_age_max();
void panel_trow(hipStream_t s, const SpxDev &d, const DualPlan &pl, bool picked = false);
void panel_update(hipStream_t s, const SpxDev &d, const DualPlan &pl);
// timing hook: the row-path pivot-row kernel alone (returns algorithmic bytes)
double launch_trow_rows(hipStream_t s, const SpxDev &d, const DualPlan &pl, int ns);
// y = inv(B) x and y = inv(B)' x over the nr dense columns of rlist and the
// unit columns of the basic slacks (valid while rlist is maintained: dual path)
// (acc: y += inv(B) x, the refinement step's update in the same pass)
void binv_ftran_list(hipStream_t s, const SpxDev &d, int nr, const double *x, double *y, const DState *eg = nullptr,
                     int acc = 0);
void binv_btran_list(hipStream_t s, const SpxDev &d, int nr, const double *x, double *y, const DState *eg = nullptr);

void primal_iteration(hipStream_t s, const SpxDev &d, int pse, int rigorous);
void launch_reset_refsp(hipStream_t s, const SpxDev &d, int dual);

// ---- factor (explicit inverse) kernels ------------------------------------------
void binv_rank1(hipStream_t s, double *Binv, int m, int ldb, const double *rho, const double *tcol, int p);
void fill_d(hipStream_t s, double *x, double v, size_t n);
void set_identity(hipStream_t s, double *M, int m, int ld);
// gather dense C = B[R, J] and S-part BS = B[S, J] of the basis into dense buffers
void gather_basis_blocks(hipStream_t s, const MatDev &A, int m, int k, const int *colsJ, const int *rowR,
                         double *C, double *BS, int ms, const int *rowS);
void gather_basis_blocks_csc(hipStream_t s, int m, int k, const int *bptr, const int *bind_rows, const double *bval,
                             const int *posJ, const int *rowR, const int *rowS, double *C, double *BS, int ms);
// Gauss-Jordan inversion with partial pivoting of the k x k matrix in X (k x 2k,
// [C | I] ping-pong in X/Y); returns number of steps completed (k on success)
int gauss_jordan(hipStream_t s, double *X, double *Y, int k, int *piv_step, int *piv, int *flag, double tiny,
                 double **result);
void extract_inverse_rowmajor(hipStream_t s, const double *X, int k, const int *piv, double *CinvR);
// blocked Gauss-Jordan (gk_reinvert.hip): C column-major in X (2 k^2 doubles),
// returns the buffer holding the inverted M = C' (see gk_reinvert.hip)
int gj_blocked_max();
size_t gj_blocked_scratch(int k);
// look-ahead side streams of the blocked inversion (owned by a gk_ctx)
struct GjSide {
    hipStream_t crit = nullptr, side = nullptr;
    hipEvent_t ev_in = nullptr, ev_main = nullptr, ev_side = nullptr;
};
GjSide *gj_side_create(int device);
void gj_side_destroy(GjSide *g);
bool gj_lookahead(int k);
double *gauss_jordan_blocked(hipStream_t s, double *X, double *scratch, int k, int *piv_step, int *piv, int *flag,
                             double tiny, GjSide *side = nullptr);
void extract_inverse_blocked(hipStream_t s, const double *M, int k, const int *piv, const int *piv_step,
                             double *CinvR);
// G (ms x k, col-major) = BS (ms x k col-major) * CinvR (k x k row-major)
void gemm_bs_cinv(hipStream_t s, const double *BS, int ms, int k, const double *CinvR, double *G, int use_mfma);
void assemble_binv(hipStream_t s, double *Binv, int m, int ldb, int k, int ms, const int *posJ, const int *rowR,
                   const int *posS, const int *rowS, const double *CinvR, const double *G);
// scheduled re-inversion by Newton refinement of the updated inverse
// (gk_newton.hip): C column-major in C, X0 / R / X1 / Xc k x k scratch; returns
// the buffer holding inv(C) in the CinvR layout, or nullptr (use Gauss-Jordan)
struct NewtonInfo {
    int steps = 0;
    double resid = 0.0;          // max |I - C X0| of the updated inverse
    double final_bound = 0.0;    // (k max |R|)^2 of the last step
};
int newton_min_k();
const double *newton_refine(hipStream_t s, int k, const double *C, const double *Binv, int ldb, const int *posJ,
                            const int *rowR, double *X0, double *R, double *X1, double *Xc,
                            unsigned long long *rbits, NewtonInfo *info);

// basic helpers
void vec_axpy(hipStream_t s, double *y, const double *x, double a, int n, const DState *st = nullptr, int need_p = 0);
void vec_copy(hipStream_t s, double *y, const double *x, int n);
void gather_row(hipStream_t s, const double *Binv, int ldb, int m, int p, double *rho);
void cb_vector(hipStream_t s, int m, const int *head, const double *coef, double *cB, const DState *st = nullptr,
               int need_p = 0);
void neg_xn_weights(hipStream_t s, const SpxDev &d, double *w);
// eval_beta's right-hand sides by variable: mode 0 -N xN, mode 1 B beta (see gk_kernels.hip)
void split_pos(hipStream_t s, const SpxDev &d, int mode, const double *beta, double *ys, double *wc,
               const DState *st = nullptr, int need_p = 0);

}  // namespace gk
