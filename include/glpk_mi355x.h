/*
 * glpk_mi355x.h — C-ABI of the MI355X-native simplex / branch-and-bound core.
 *
 * Drop-in boundary for the reference Cyame/glpk.js (GLPK 4.49 in JS).  The
 * JS host keeps glpapi*.js / glpcpx.js / glpmpl*.js and rebinds the closure
 * names of the hot path to these entry points through a thin N-API addon
 * (js/gk_addon.c, js/gk_shim.js).
 *
 *   entry point            replaces (reference file:line)
 *   ---------------------  ------------------------------------------------
 *   gk_spx_primal          spx_primal(lp, parm)            glpspx01.js:1
 *   gk_spx_dual            spx_dual(lp, parm)              glpspx02.js:1
 *   gk_bfd_create          bfd_create_it()                 glpbfd.js:10
 *   gk_bfd_set_parm        bfd_set_parm(bfd, parm)         glpbfd.js:31
 *   gk_bfd_factorize       bfd_factorize(bfd,m,bh,col,info) glpbfd.js:47
 *   gk_bfd_factorize_csc   (same, columns passed as CSC instead of a callback)
 *   gk_bfd_ftran           bfd_ftran(bfd, x)               glpbfd.js:148
 *   gk_bfd_btran           bfd_btran(bfd, x)               glpbfd.js:159
 *   gk_bfd_update          bfd_update_it(bfd,j,bh,len,ind,idx,val) glpbfd.js:170
 *   gk_bfd_get_count       bfd_get_count(bfd)              glpbfd.js:225
 *   gk_ios_driver          ios_driver(T) with cb_func == null (glpios03.js:1),
 *                          run from glp_intopt's solve_mip (glpapi09.js:62-79)
 *
 * Conventions (identical to the reference's typed arrays): every vector is
 * 1-based with element 0 unused; auxiliary variable k = 1..m is row k,
 * structural k = m+1..m+n is column k-m.  Return codes are the reference's
 * GLP_E* / BFD_E* values.  No entry point throws: on a contract violation
 * (the reference's xerror/xassert) it returns GK_EABI and gk_last_error()
 * holds the message; the N-API layer rethrows it as a JS Error.
 *
 * Every call is synchronous on the calling thread.  Internally a call may
 * use several HIP streams on the context's device.  There is no CPU
 * fallback: if no MI355X (gfx950) device is usable, gk_ctx_create fails and
 * returns NULL.
 */
#ifndef GLPK_MI355X_H
#define GLPK_MI355X_H

#ifdef __cplusplus
extern "C" {
#endif

#define GK_ABI_VERSION 11
#include <stddef.h>
#define GK_EABI (-1)          /* contract violation; see gk_last_error() */

typedef struct gk_ctx gk_ctx; /* one HIP device + stream(s)                */
typedef struct gk_bfd gk_bfd; /* replaces lp.bfd: device-resident factor   */

/* ---- context ------------------------------------------------------------ */
int         gk_abi_version(void);
int         gk_device_count(void);
gk_ctx     *gk_ctx_create(int device);          /* NULL on failure          */
void        gk_ctx_destroy(gk_ctx *ctx);       /* factors made on it keep it alive until they are destroyed */
/* profiling aid: enqueue an empty kernel (k_gk_mark) on the context stream,
 * so that a kernel trace can be windowed on a region of the host program */
int         gk_ctx_mark(gk_ctx *ctx, int tag);
const char *gk_last_error(void);                 /* thread-local message     */

/* ---- basis factorization (glpbfd.js) -------------------------------------
 * The factor of B is held on the device as an explicit dense inverse,
 * refreshed by re-inversion after nfs_max product-form updates (the
 * reference refactorizes after nfs_max Forrest–Tomlin updates,
 * glpfhv.js:182).  Field meanings follow glp_bfcp (glpapi12.js:108-121). */
typedef struct {
    int    type;       /* GLP_BF_FT (1) / GLP_BF_BG (2) / GLP_BF_GR (3): all three are served
                          by the same explicit-inverse factor (the update is exact product
                          form, so the Bartels-Golub / Givens variants coincide with it);
                          any other value: gk_bfd_set_parm fails with the reference's
                          "glp_set_bfcp: type = %d; invalid parameter" */
    int    lu_size;
    double piv_tol;
    int    piv_lim, suhl;
    double eps_tol, max_gro;
    int    nfs_max;    /* updates between re-inversions                      */
    double upd_tol;
    int    nrs_max, rs_size;
} gk_bfcp;

typedef int (*gk_col_fn)(void *info, int j, int *ind, double *val);

gk_bfd *gk_bfd_create(gk_ctx *ctx);
void    gk_bfd_destroy(gk_bfd *bfd);
int     gk_bfd_set_parm(gk_bfd *bfd, const gk_bfcp *parm);   /* 0 | GK_EABI (invalid field) */
/* glp_set_bfcp(lp, NULL) / copy_bfcp of a problem without a bfcp of its own
 * (glpapi12.js:127-139): the glp_get_bfcp defaults, with the re-inversion
 * interval left to the engine (up to min(1000, m / 4) updates while the
 * drift measured at each re-inversion stays below tol / 200; the first
 * drift above tol / 20 drops it to nfs_max = 100, and it lengthens again
 * only over two clean chains).  gk_bfd_set_parm marks its values
 * explicit: nfs_max / nrs_max then hold exactly, 100 included — on the
 * explicit inverse; the sparse factor's Schur-complement chain holds at most
 * 256 updates, so there an explicit value above 256 is capped at 256.  A new
 * factor starts in the default state.  (ABI 8) */
int     gk_bfd_reset_parm(gk_bfd *bfd);
/* diagnostics of the sparse factor (gk_sparse.hip; ABI 8), host only: the
 * Markowitz L U of a basis given as CSC (as gk_bfd_factorize_csc: ptr[1..m+1],
 * 1-based ind) and its four level-scheduled sweeps run on the host in the
 * order the device runs them: x = inv(B) b, y = inv(B)' e ([0..m), 0-based).
 * stats[0..5]: nnz(L), nnz(U) with its diagonal, levels of FTRAN L / U and
 * BTRAN U' / L'.  0 | 1 (singular) | -1 (invalid input). */
int     gk_sp_selftest(int m, const int *ptr, const int *ind, const double *val, const double *b,
                       const double *e, double *x, double *y, long long *stats);
/* 0 | BFD_ESING(1) | BFD_ECOND(2); col(info, j, ind, val) fills column j of B
 * exactly like b_col/inv_col (glpapi12.js:7, glpspx01.js:147). */
int     gk_bfd_factorize(gk_bfd *bfd, int m, gk_col_fn col, void *info);
/* same with B given as CSC: column j occupies [ptr[j], ptr[j+1]) of ind/val
 * (positions 1-based, ptr[1..m+1]); ind holds 1-based row numbers. */
int     gk_bfd_factorize_csc(gk_bfd *bfd, int m, const int *ptr, const int *ind, const double *val);
void    gk_bfd_ftran(gk_bfd *bfd, double *x);            /* x[1..m] := inv(B) x  */
void    gk_bfd_btran(gk_bfd *bfd, double *x);            /* x[1..m] := inv(B') x */
/* replace column j of B by (ind[idx+1..idx+len], val[1..len]) — the
 * reference's (odd but exact) indexing convention of fhv_update_it. */
int     gk_bfd_update(gk_bfd *bfd, int j, int len, const int *ind, int idx, const double *val);
int     gk_bfd_get_count(const gk_bfd *bfd);
int     gk_bfd_valid(const gk_bfd *bfd);

/* ---- simplex (glpspx01.js / glpspx02.js) --------------------------------- */
/* The factor behind gk_spx_* and gk_bfd_factorize* is chosen by a cost
 * model: the explicit inverse inv(B) (dense, 8 m^2 bytes of
 * HBM, m <= 65535) for dense A and small or dense-column sparse bases; a
 * sparse LU with Schur-complement updates (at most SP_KMAX = 256 updates
 * per chain) for sparse A with m >= 2048 and 16 nnz(A)/n <= m, and always
 * beyond m = 65535.  GK_SPARSE=1 / 0 forces either; gk_spx_stats.factor_sparse
 * reports the choice. */
typedef struct {                /* glp_smcp, SMCP (glpapi06.js:359-375)       */
    int    msg_lev, meth, pricing, r_test;
    double tol_bnd, tol_dj, tol_piv, obj_ll, obj_ul;
    int    it_lim, tm_lim, out_frq, out_dly, presolve;
} gk_smcp;

typedef struct {
    /* problem (read; the fields init_csa reads, glpspx01.js:42-145) */
    int m, n, nnz, dir;
    double c0;
    const signed char *row_type;             /* [1..m] GLP_FR..GLP_FX */
    const double *row_lb, *row_ub, *rii;     /* [1..m] unscaled bounds, row scale */
    const signed char *col_type;             /* [1..n] */
    const double *col_lb, *col_ub, *col_coef, *sjj;   /* [1..n] */
    const int *A_ptr;                        /* [1..n+1] positions into A_ind/A_val */
    const int *A_ind;                        /* [1..nnz] 1-based row numbers, list order */
    const double *A_val;                     /* [1..nnz] unscaled values */
    unsigned long long a_version;            /* !=0: A/scale unchanged since the last call
                                                with this version => reuse the device copy */
    /* basis (read/write) */
    int *head;                               /* [1..m] basis header (lp.head) */
    signed char *row_stat, *col_stat;        /* [1..m], [1..n] */
    /* solution (write; store_sol, glpspx01.js:1591) */
    int *row_bind, *col_bind;
    double *row_prim, *row_dual, *col_prim, *col_dual;
    int it_cnt;                              /* in/out: lp.it_cnt */
    int pbs_stat, dbs_stat, some;            /* out */
    double obj_val;                          /* out */
    int valid;                               /* out: lp.valid */
    unsigned long long b_version;            /* !=0: bounds, types, costs, dir, c0 and the scale
                                                factors unchanged since the last call with this
                                                version (and a_version) => init_csa's rebuild and
                                                its comparison with the resident working set are
                                                skipped; 0: always rebuilt and compared (ABI 8) */
} gk_lp;

/* The factor handle must be valid for lp->head (as after glp_factorize);
 * on return it is valid for the new lp->head (store_sol semantics), or on
 * GLP_EFAIL left as the reference leaves it. Returns 0 | GLP_EFAIL |
 * GLP_EOBJLL | GLP_EOBJUL | GLP_EITLIM | GLP_ETMLIM | GK_EABI. */
int gk_spx_primal(gk_ctx *ctx, gk_lp *lp, gk_bfd *bfd, const gk_smcp *parm);
int gk_spx_dual(gk_ctx *ctx, gk_lp *lp, gk_bfd *bfd, const gk_smcp *parm);

/* The reference's terminal output of the simplex (display, glpspx01.js:
 * 1550-1589 / glpspx02.js:1452-1497, and the messages of the main loops),
 * reported instead of printed: the host formats each line with its own
 * number printing (the reference's are JavaScript conversions of doubles),
 * in call order, on the calling thread, during the gk_spx_* call.  Reports
 * follow parm->msg_lev and out_frq / out_dly as the reference's do (a device
 * batch ends at every multiple of out_frq when progress lines are on).
 *   kind GK_RPT_PROGRESS: code 1 primal / 2 dual, it_cnt, phase, obj (primal;
 *     dual phase II), infeas (the sum of primal / dual infeasibilities), aux =
 *     the number of basic fixed variables:
 *       primal  (phase 1 ? ' ' : '*') it ": obj = " obj "  infeas = " inf " (" aux ")"
 *       dual I  " " it ":  infeas = " inf " (" aux ")"
 *       dual II "|" it ": obj = " obj "  infeas = " inf " (" aux ")"
 *   kind GK_RPT_MSG: code GK_MSG_*, phase, aux (GK_MSG_INSTAB: 1 primal /
 *     2 dual; GK_MSG_FACTERR: the factorization's return code) */
#define GK_RPT_PROGRESS 1
#define GK_RPT_MSG 2
#define GK_MSG_OPTIMAL 1    /* "OPTIMAL SOLUTION FOUND" */
#define GK_MSG_NODFS 2      /* "PROBLEM HAS NO DUAL FEASIBLE SOLUTION" */
#define GK_MSG_NOPFS 3      /* "PROBLEM HAS NO FEASIBLE SOLUTION" */
#define GK_MSG_UNBND 4      /* "PROBLEM HAS UNBOUNDED SOLUTION" */
#define GK_MSG_ITLIM 5      /* "ITERATION LIMIT EXCEEDED; SEARCH TERMINATED" */
#define GK_MSG_TMLIM 6      /* "TIME LIMIT EXCEEDED; SEARCH TERMINATED" */
#define GK_MSG_OBJLL 7      /* "OBJECTIVE LOWER LIMIT REACHED; SEARCH TERMINATED" */
#define GK_MSG_OBJUL 8      /* "OBJECTIVE UPPER LIMIT REACHED; SEARCH TERMINATED" */
#define GK_MSG_INSTAB 9     /* "Warning: numerical instability (primal|dual simplex, phase I|II)" */
#define GK_MSG_NOCHOICE 10  /* "Error: unable to choose basic variable on phase I" */
#define GK_MSG_FACTERR 11   /* "Error: unable to factorize the basis matrix (aux)",
                               "Sorry, basis recovery procedure not implemented yet" */
typedef void (*gk_report_fn)(void *ud, int kind, int code, int it_cnt, int phase, double obj, double infeas,
                             int aux);
void gk_bfd_set_report(gk_bfd *bfd, gk_report_fn fn, void *ud);

/* engine counters of the last gk_spx_* call on this handle (for benches) */
typedef struct {
    long long pivots, reinversions, batches, host_syncs;
    double seconds_total, seconds_reinvert;
    double bytes_pivots;        /* algorithmic HBM bytes the pivots had to move */
    long long graphs_built;     /* device batches captured as HIP graphs */
    double seconds_init, seconds_eval, seconds_batches;   /* host wall time split */
    double trow_ms;             /* with gk_bfd_profile: HIP-event time of the pivot-row kernels */
    long long trow_launches;
    double trow_bytes;          /* algorithmic bytes of those kernels (all pivots of the call) */
    double trow_dev_ms;         /* device wall-clock execution span of the row-path pivot-row kernels */
    long long trow_dev_launches;
    double trow_dev_ms_b;       /* same, from their entry to the next kernel's entry (dispatch included) */
    double trow_dev_ms_r;       /* same, from the last block exit of the kernel before them to their
                                   own last block exit (a profiler's per-dispatch bracket) */
    long long trow_dev_launches_r;
    double upd_dev_ms;          /* (profiling) device span of the k_dual_update launches: entry of
                                   block 0 to the last block exit, summed (gk_bfd_profile 3 / 4); with
                                   gk_bfd_profile 1 / 2 the kernels' start / stop events instead */
    long long upd_dev_launches;
    double upd_bytes;           /* (profiling) algorithmic bytes of every k_dual_update launch */
    int resident;               /* 1: the call found its working set resident (no re-upload) */
    int evals_skipped;          /* eval_cbar / eval_bbar calls whose result was already resident */
    long long panel_hits;       /* dual pivots whose pivot row came from the MFMA pricing panel */
    long long panel_refills;    /* MFMA refills of the panel (one pass over A for up to 32 rows) */
    long long refine_tries;     /* scheduled re-inversions offered to Newton refinement (k >= GK_NEWTON_MIN_K) */
    long long refinements;      /* ... served by it (two MFMA GEMMs per step; the rest: Gauss-Jordan) */
    long long refine_steps;     /* Newton steps taken by those */
    double refine_resid_max;    /* largest max|I - C X| of an updated inverse offered to it */
    /* ABI 9: the factor the call ran on (gk_bfd_factor_kind), the host
     * Markowitz LU time of its sparse refactorizations, and how many of
     * those were factored ahead on a host thread while the device pivoted */
    int factor_sparse;          /* 1: the sparse LU (gk_sparse.hip), 0: the explicit inverse */
    int lu_ahead;               /* sparse refactorizations taken from the look-ahead thread */
    double seconds_lu;          /* host wall time of the Markowitz LU factorizations (all threads) */
    /* ABI 11: column-sharded pricing (gk_bfd_set_comm) */
    long long shard_exchanges;  /* pivot-row all-gathers of the call (0 when not sharded) */
} gk_spx_stats;
void gk_bfd_last_stats(const gk_bfd *bfd, gk_spx_stats *st);
/* record HIP events around the pivot-row kernel of every dual pivot (benches) */
/* 1: events, eager; 2: + block clock stamps; 3: block stamps only, graphs
 * kept; 4: kernel-span stamps and byte accounting only, graphs kept.  With 0
 * (the default) the pivot kernels keep no clocks and no byte counts: the
 * trow_* / upd_* / bytes_pivots statistics are filled only in modes 1-4 */
void gk_bfd_profile(gk_bfd *bfd, int enable);
/* profiling aid (enable == 2 above): copies the per-kernel, per-block device
 * clock stamps of the last pivot, trace[(kernel * 2048 + block) * 2 + {0 entry,
 * 1 exit}], kernels 0 top, 1 pivot row, 2 ratio, 3 FTRAN (one kernel), 4 commit,
 * 5 row finish (column path), 6 FTRAN (split), 7 FTRAN reduce; returns the
 * number of entries copied (0 when tracing was never enabled) */
int gk_bfd_trace(gk_bfd *bfd, unsigned long long *out, size_t cnt);

/* measurement hook for bench.py (not part of the reference interface):
 * launch one engine kernel `reps` times on the problem left resident by the
 * last gk_spx_* call, bracketed by two HIP events on the engine's stream,
 * and return the average milliseconds per launch (or < 0 on error).
 *   which 0: pivot-row pass trow = -rho' N as the engine runs it at the
 *            current basis (rows of A in the support of rho when that is
 *            at most m/2 rows and A is dense, else the column pass)
 *         1: A w product of the dual steepest-edge update
 *         2: inv(B) x product (FTRAN)
 *         3: rank-1 update of inv(B) (on a scratch copy)
 * *bytes receives the algorithmic bytes one launch must move. */
double gk_bfd_time_kernel(gk_bfd *bfd, int which, int reps, double *bytes);

/* ---- tableau rows (glp_eval_tab_row, glpapi12.js:401) --------------------
 * Rows of the simplex tableau of the basic variables k[0..nk) (1..m+n, each
 * basic in lp->head) on the current factor of bfd, all in one pass:
 *   alfa[t * (m + n) + j - 1] = alfa_{k_t, j} for every non-basic variable j
 * (rho' A_j for a structural, -rho_j for an auxiliary, rho = glp_btran(e_i),
 * the problem's scaling applied as glp_btran does), 0 for basic j.  The
 * reference returns the non-zeros as (ind, val) lists; the host compacts.
 * On dense A the batch is one GEMM on the matrix cores; flags & 1 forces the
 * per-row CSC path.  A is taken from lp (uploaded when lp->a_version is new).
 * 0 | GK_EABI (no valid factor, k out of range or non-basic). */
int gk_bfd_eval_tab_rows(gk_bfd *bfd, gk_lp *lp, int nk, const int *k, double *alfa, int flags);

/* ---- branch and bound (glpios03.js, glpapi09.js) -------------------------
 * gk_ios_driver serves glp_intopt with cb_func == null, presolve off and no
 * cut generators.  Every br_tech (FFV, LFV, MFV, DTH, PCH; glpios09.js:1) and
 * bt_tech (DFS, BFS, BLB, BPH; glpios12.js:2) is native; pp_tech NONE / ROOT
 * / ALL runs ios_preprocess_node (glpios02.js:1) inside the node kernel.
 * Node LPs are solved in batches, one workgroup per node; a node the batched
 * kernel cannot finish is re-solved by the full engine (ios_solve_node's
 * glp_simplex, GLP_DUALP); GLP_EFAIL (5) only when that fails too, as the
 * reference's ios_driver (glpios03.js:669-673). */
typedef struct {                /* glp_iocp, IOCP (glpapi09.js:392-414)       */
    int    msg_lev, br_tech, bt_tech;
    double tol_int, tol_obj;
    int    tm_lim, out_frq, out_dly, pp_tech;
    double mip_gap;
    int    presolve;
} gk_iocp;

typedef struct {
    gk_lp lp;                                 /* root problem, solved to optimality */
    const signed char *col_kind;              /* [1..n] GLP_CV / GLP_IV */
    /* out */
    int mip_stat;
    double mip_obj;
    double *col_mipx, *row_mipx;              /* [1..n], [1..m] */
    long long lp_solves, nodes_created, pivots;
    long long node_fallbacks;   /* node LPs re-solved by the full engine (gk_spx_*) after the
                                   batched kernel gave up (iteration limit, singular basis) */
    long long probe_lps;        /* PCH pseudocost probes (eval_degrad, glpios09.js:337) */
    long long pp_fathomed;      /* nodes fathomed by ios_preprocess_node (no LP solved) */
    long long nodes_moved;      /* sharded runs: open nodes received from other ranks */
} gk_mip;

int gk_ios_driver(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm);

/* The reference's search progress lines (show_progress, glpios03.js:2-48,
 * printed at :607, :780 and :943), reported instead of printed, on the
 * calling thread during gk_ios_driver(_sharded) on this context, when
 * parm->msg_lev >= GLP_MSG_ON: once at the start (the root), at every new
 * incumbent, every out_frq milliseconds of search, and at the end.  Record
 * kind GK_RPT_MIP:
 *   code    bit 0: a new incumbent (">>>>>" instead of "mip ="), bit 1: an
 *           incumbent exists, bit 2: no active subproblem ("tree is empty")
 *   it_cnt  simplex iterations so far (the root LP's it_cnt plus every node LP)
 *   phase   active subproblems (T.a_cnt)
 *   obj     incumbent objective (original sense)
 *   infeas  best local bound over the active subproblems (original sense;
 *           +-DBL_MAX print as "+inf" / "-inf")
 *   aux     subproblems fathomed so far (T.t_cnt - T.n_cnt; the driver keeps
 *           no inactive nodes, so this is created minus active)
 * The host formats "+it: mip = obj >= bound gap (a; d)" as glpios03.js:45. */
#define GK_RPT_MIP 3
void gk_ios_set_report(gk_ctx *ctx, gk_report_fn fn, void *ud);

/* one GPU's share of a branch-and-bound run over several GPUs (one process
 * per GPU).  All ranks call gk_ios_driver_sharded on the same problem; they
 * evaluate the first batches identically, split the frontier round-robin
 * (node i -> rank i mod size), and every sync_every batches run one epoch of
 * the exchange.  The main path is allgather (gk_comm_allgather of this
 * library, through gk_ios_driver_comm below, or a host's own): every epoch
 * all-gathers {incumbent, best open bound, open nodes, active} and hands open
 * nodes (bounds + warm-start basis) from the ranks with the most to idle
 * ranks.  Without allgather, exchange() is the
 * incumbent-only protocol: it receives this rank's best objective (internal
 * minimisation form; DBL_MAX if none) and whether it still has open nodes,
 * and must return the minimum over ranks in *best and the number of ranks
 * with work (0 ends the run).  On return each rank holds its own incumbent
 * (mip_stat GLP_OPT with a solution, else GLP_NOFEAS); gk_ios_driver_comm
 * agrees on the best over ranks, a caller of this entry point picks it. */
typedef struct {
    int rank, size;
    int ramp_nodes;                 /* frontier per rank before the split (0: 8) */
    int sync_every;                 /* batches between exchanges (0: 4) */
    int (*exchange)(void *info, double *best, int active);
    void *info;
    /* optional (preferred when set): all-gather of `bytes` bytes from every
     * rank into recv (size * bytes, rank order); returns 0 on success.  With
     * it every sync epoch exchanges {incumbent, best bound, open nodes,
     * active} and hands open nodes (bounds + warm-start basis) from the ranks
     * with the most to idle ranks; exchange is then unused */
    int (*allgather)(void *info, const void *send, size_t bytes, void *recv);
} gk_ios_shard;
int gk_ios_driver_sharded(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, const gk_ios_shard *shard);

/* ---- collective of the sharded branch and bound --------
 * One process per GPU, each with a gk_comm.  Rank 0 listens on addr
 * ("host:port"; the others connect to it: the bootstrap).  The epoch
 * exchange of the sharded driver is an all-gather of fixed-size byte
 * blocks: over RCCL (ncclAllGather, xGMI) when every rank drives a device of
 * its own (GK_COMM_AUTO) or when asked (GK_COMM_RCCL), through rank 0 over
 * TCP otherwise (ranks sharing a device, hosts without a device: ctx may be
 * NULL for GK_COMM_TCP).  Blocking; every rank must call the collectives in
 * the same order. */
typedef struct gk_comm gk_comm;
#define GK_COMM_AUTO 0
#define GK_COMM_TCP 1
#define GK_COMM_RCCL 2
gk_comm *gk_comm_create(gk_ctx *ctx, int rank, int size, const char *addr, int backend);   /* NULL on failure */
void     gk_comm_destroy(gk_comm *comm);
int      gk_comm_backend(const gk_comm *comm);          /* GK_COMM_TCP | GK_COMM_RCCL */
int      gk_comm_rank(const gk_comm *comm);
int      gk_comm_size(const gk_comm *comm);
/* recv[r * bytes .. (r + 1) * bytes) = rank r's send block; 0 on success.
 * The signature of gk_ios_shard.allgather (info = the gk_comm). */
int      gk_comm_allgather(void *comm, const void *send, size_t bytes, void *recv);
/* the incumbent shared by the ranks between the exchange epochs: when every
 * rank of comm runs on one host, one word of shared memory holds the best
 * objective published so far (an atomic min on an order-preserving image of
 * the double).  gk_comm_incumbent publishes mine and returns the best over
 * the ranks (mine itself without a shared word); the sharded search calls it
 * before every batch (internal minimisation form, DBL_MAX: none).  Each
 * gk_ios_driver_comm search of comm has a word of its own: a later search on
 * the same communicator starts from DBL_MAX, not from an earlier one's best.
 * gk_comm_shared_incumbent: 1 when the word exists. */
double   gk_comm_incumbent(gk_comm *comm, double mine);
int      gk_comm_shared_incumbent(const gk_comm *comm);
/* options of the sharded search run through gk_ios_driver_comm:
 * GK_COMM_OPT_RAMP  the frontier per rank before the split (gk_ios_shard.ramp_nodes;
 *                   0 the default, < 0 split the root alone: rank 0 starts with all the work)
 * GK_COMM_OPT_SYNC  batches between exchange epochs (gk_ios_shard.sync_every; 0 the default) */
#define GK_COMM_OPT_RAMP 1
#define GK_COMM_OPT_SYNC 2
int      gk_comm_set_option(gk_comm *comm, int opt, int value);
/* glp_intopt on every rank of comm: gk_ios_driver_sharded with this
 * library's all-gather, then an all-gather of the ranks' incumbents so that
 * every rank returns the same winner (best objective, lowest rank on ties),
 * mip_stat GLP_OPT when the search finished on every rank.  With a
 * one-rank comm it is gk_ios_driver. */
int gk_ios_driver_comm(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, gk_comm *comm);

/* column-sharded pricing of one LP: gk_spx_dual on this
 * factor forms each pivot row from this rank's slice of the non-basic
 * positions (a column pass over 1/size of A) and all-gathers the slices over
 * comm — RCCL on the engine's stream between distinct GPUs, TCP otherwise —
 * so every rank takes the pivots the single-GPU column pass takes.  Every
 * rank of comm makes the same gk_spx_dual calls on the same problem.  Dense
 * A, dual simplex; comm = NULL turns it off (so does a one-rank comm, unless
 * GK_SHARD_ONE_RANK=1 — a test knob that runs the exchange with one rank).
 * Stops are collective: tm_lim is decided by all-gathering every rank's
 * time-limit flag at each batch boundary (any rank's stops all); a failure
 * on one rank (GK_EABI) aborts comm, so the peers' next exchange fails and
 * they return GK_EABI too instead of waiting.  0 or GK_EABI. */
int gk_bfd_set_comm(gk_bfd *bfd, gk_comm *comm);

/* the source stamp the library was built from (16 hex digits of a hash of
 * its HIP / C++ sources and headers, glpk.js_amd/stamp.py); the Python host
 * refuses a library whose stamp is not its sources' */
const char *gk_build_stamp(void);

/* glp_scale_prob (glpscl.js:1-225) on the device: the
 * row and column scale factors of A (CSC: ptr[0..n] 0-based offsets, ind[]
 * 1-based row numbers, val[]) after glp_unscale_prob and the flags'
 * geometric-mean / equilibration / power-of-two steps, bit-identical to the
 * reference.  rii[m], sjj[n] receive the factors; report[13] receives
 * (min|aij|, max|aij|, ratio) after the stages A, GM, EQ, 2N (the numbers
 * the reference prints) and report[12] the stage bits (1 well scaled, 2 GM,
 * 4 EQ, 8 2N, 16 skipped as well scaled).  Returns 0, 1 for invalid flags
 * (the reference's xerror "invalid scaling options"), or GK_EABI. */
int gk_scale_prob(gk_ctx *ctx, int m, int n, const int *ptr, const int *ind, const double *val, int flags,
                  double *rii, double *sjj, double *report);
/* the same, also returning the device time of the sweeps (ms, HIP events)
 * and their algorithmic bytes (bench.py) */
int gk_scale_prob_timed(gk_ctx *ctx, int m, int n, const int *ptr, const int *ind, const double *val, int flags,
                        double *rii, double *sjj, double *report, double *sweep_ms, double *sweep_bytes);

/* ---- advanced initial basis (glpini01.js) ---------------------------------
 * Replaces adv_basis (glpini01.js:268-354, called by glp_adv_basis(lp, 0)):
 * the basis of the maximal lower triangular part of (I | -A) found by triang
 * (:2-212), columns of fixed variables removed, completed with auxiliary
 * variables; non-basic statuses by type (double-bounded: the bound of
 * smaller magnitude).  Reads m, n, row/col type and bounds, A_ptr / A_ind
 * (list order) of lp; writes lp->row_stat[1..m], lp->col_stat[1..n].  With
 * m == 0 or n == 0 it is glp_std_basis (glpapi05.js:49).  Host code (no
 * context, no device).  Returns the size of the triangular part, or GK_EABI. */
int gk_adv_basis(gk_lp *lp);

/* ---- LP / MIP presolver (glpnpp01.js .. glpnpp05.js) ----------------------
 * The preprocessor glp_simplex (glpapi06.js:41 preprocess_and_solve_lp) and
 * glp_intopt (glpapi09.js:111 preprocess_and_solve_mip) run with presolve =
 * GLP_ON.  Host code (no context, no device): the reduced problem is solved
 * by gk_spx_* / gk_ios_driver like any other.  Sequence (each step replaces
 * the reference routine named):
 *   gk_npp_create                          npp_create_wksp  glpnpp01.js:2
 *   gk_npp_load(npp, P, kind, sol)         npp_load_prob    :262 (names and
 *       scaling off; P's problem arrays in list order; kind [1..n] for
 *       sol = GLP_MIP (3), NULL for GLP_SOL (1))
 *   gk_npp_simplex / gk_npp_integer        npp_simplex      glpnpp05.js:430
 *                                          npp_integer      :437
 *       -> 0 | GLP_ENOPFS (10) | GLP_ENODFS (11) | GK_EABI; msg[7] (or
 *       NULL) gets the counts npp_integer prints: variables binarized,
 *       binaries made, rows added, binarization failures, hidden packing,
 *       hidden covering, reduced coefficients
 *   gk_npp_build_size, gk_npp_build        npp_build_prob   glpnpp01.js:396
 *       (arrays 1-based as gk_lp's; A by columns in the order the
 *       reference's glp_set_mat_col leaves them; row_ref / col_ref map each
 *       reduced row / column to the original one; *c0 the constant term)
 *   gk_npp_postprocess(npp, s1, s2, ...)   npp_postprocess  :474
 *       (GLP_SOL: s1 / s2 = pbs / dbs status, the reduced problem's row
 *       statuses and duals, column statuses and primal values; GLP_MIP: s1 =
 *       mip_stat, col_prim = mipx, the rest NULL)
 *   gk_npp_unload_sol / gk_npp_unload_mip  npp_unload_sol   :572
 *   gk_npp_destroy
 * The transformations, their order and their arithmetic are the reference's
 * (gk_npp.cc), so the reduced problem equals the reference's bit for bit. */
typedef struct gk_npp gk_npp;
gk_npp *gk_npp_create(void);
void    gk_npp_destroy(gk_npp *npp);
int     gk_npp_load(gk_npp *npp, const gk_lp *P, const signed char *col_kind, int sol);
int     gk_npp_simplex(gk_npp *npp);
int     gk_npp_integer(gk_npp *npp, int binarize, int *msg);
int     gk_npp_build_size(gk_npp *npp, int *m, int *n, int *nnz);
int     gk_npp_build(gk_npp *npp, signed char *row_type, double *row_lb, double *row_ub,
                     signed char *col_type, double *col_lb, double *col_ub, double *col_coef,
                     signed char *col_kind, int *A_ptr, int *A_ind, double *A_val,
                     int *row_ref, int *col_ref, double *c0);
int     gk_npp_postprocess(gk_npp *npp, int stat1, int stat2, const signed char *row_stat,
                           const double *row_dual, const signed char *col_stat, const double *col_prim);
int     gk_npp_unload_sol(gk_npp *npp, gk_lp *P);
int     gk_npp_unload_mip(gk_npp *npp, const gk_lp *P, const signed char *col_kind, double *row_mipx,
                          double *col_mipx, int *mip_stat, double *mip_obj);

#ifdef __cplusplus
}
#endif
#endif /* GLPK_MI355X_H */
