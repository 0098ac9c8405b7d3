/* ORACLE (test infrastructure only): restatement of glp_scale_prob
 * (glpscl.js:1-225) and round2n (glplib03.js:26) on a CSC matrix, for the
 * parity tests of the device scaling (gk_scale.hip).  Every quantity the
 * reference forms is a min / max of |a_ij| * (r_i * s_j), a product of two
 * such values, a quotient or a correctly rounded square root, so the
 * restatement reproduces the reference's factors bit for bit.
 *
 *   A: n columns, ptr[0..n] 0-based offsets, ind[] 1-based row numbers.
 *   report[0..11]: (min, max, ratio) after the stages A, GM, EQ, 2N;
 *   report[12]: bit 0 well scaled, bit 1 GM done, bit 2 EQ done, bit 3 2N
 *   done, bit 4 returned after the well-scaled skip.
 * Returns 0, or 1 for invalid flags (glp_scale_prob's xerror). */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SF_GM 0x01
#define SF_EQ 0x10
#define SF_2N 0x20
#define SF_SKIP 0x40
#define SF_AUTO 0x80

typedef struct {
    int m, n;
    const int *ptr, *ind;
    const double *val;
    int *rptr, *rcol;           /* rows: CSR built once */
    double *rval;
    double *rii, *sjj;          /* 1-based */
} Scl;

/* min / max over row i (glpscl.js:2-28): the first entry initialises; an
 * empty row gives 1 */
static void row_mm(const Scl *S, int i, double *mn, double *mx)
{
    double lo = 1.0, hi = 1.0;
    for (int t = S->rptr[i]; t < S->rptr[i + 1]; t++) {
        double temp = fabs(S->rval[t]) * (S->rii[i] * S->sjj[S->rcol[t]]);
        if (t == S->rptr[i] || lo > temp) lo = temp;
        if (t == S->rptr[i] || hi < temp) hi = temp;
    }
    *mn = lo;
    *mx = hi;
}

static void col_mm(const Scl *S, int j, double *mn, double *mx)
{
    double lo = 1.0, hi = 1.0;
    for (int t = S->ptr[j - 1]; t < S->ptr[j]; t++) {
        double temp = fabs(S->val[t]) * (S->rii[S->ind[t]] * S->sjj[j]);
        if (t == S->ptr[j - 1] || lo > temp) lo = temp;
        if (t == S->ptr[j - 1] || hi < temp) hi = temp;
    }
    *mn = lo;
    *mx = hi;
}

/* min_mat_aij / max_mat_aij (:58-80): over the rows only */
static void mat_mm(const Scl *S, double *mn, double *mx)
{
    double lo = 1.0, hi = 1.0, a, b;
    for (int i = 1; i <= S->m; i++) {
        row_mm(S, i, &a, &b);
        if (i == 1 || lo > a) lo = a;
        if (i == 1 || hi < b) hi = b;
    }
    *mn = lo;
    *mx = hi;
}

static double max_row_ratio(const Scl *S)
{
    double ratio = 1.0, a, b;
    for (int i = 1; i <= S->m; i++) {
        row_mm(S, i, &a, &b);
        double temp = b / a;
        if (i == 1 || ratio < temp) ratio = temp;
    }
    return ratio;
}

static double max_col_ratio(const Scl *S)
{
    double ratio = 1.0, a, b;
    for (int j = 1; j <= S->n; j++) {
        col_mm(S, j, &a, &b);
        double temp = b / a;
        if (j == 1 || ratio < temp) ratio = temp;
    }
    return ratio;
}

/* one gm_scaling (:98-117, gm = 1) or eq_scaling (:82-96, gm = 0) sweep:
 * rows first when flag == 0, columns first when flag == 1 */
static void sweep(Scl *S, int flag, int gm)
{
    double a, b;
    for (int pass = 0; pass <= 1; pass++) {
        if (pass == flag) {
            for (int i = 1; i <= S->m; i++) {
                row_mm(S, i, &a, &b);
                S->rii[i] = gm ? S->rii[i] / sqrt(a * b) : S->rii[i] / b;
            }
        } else {
            for (int j = 1; j <= S->n; j++) {
                col_mm(S, j, &a, &b);
                S->sjj[j] = gm ? S->sjj[j] / sqrt(a * b) : S->sjj[j] / b;
            }
        }
    }
}

/* round2n (glplib03.js:26): the nearest power of two, ties (f = 0.75) down */
static double round2n(double x)
{
    int e;
    double f = frexp(x, &e);        /* x = f 2^e, 0.5 <= f < 1 */
    return ldexp(1.0, f <= 0.75 ? e - 1 : e);
}

static void report_stage(const Scl *S, double *rep)
{
    mat_mm(S, &rep[0], &rep[1]);
    rep[2] = rep[1] / rep[0];
}

int orc_scale_prob(int m, int n, const int *ptr, const int *ind, const double *val, int flags, double *rii_out,
                   double *sjj_out, double *report)
{
    if (flags & ~(SF_GM | SF_EQ | SF_2N | SF_SKIP | SF_AUTO)) return 1;
    if (flags & SF_AUTO) flags = SF_GM | SF_EQ | SF_SKIP;
    Scl S;
    S.m = m;
    S.n = n;
    S.ptr = ptr;
    S.ind = ind;
    S.val = val;
    int nnz = ptr[n];
    S.rptr = calloc((size_t)m + 2, sizeof(int));
    S.rcol = malloc(sizeof(int) * (size_t)(nnz + 1));
    S.rval = malloc(sizeof(double) * (size_t)(nnz + 1));
    S.rii = malloc(sizeof(double) * (size_t)(m + 1));
    S.sjj = malloc(sizeof(double) * (size_t)(n + 1));
    for (int t = 0; t < nnz; t++) S.rptr[ind[t] + 1]++;
    for (int i = 1; i <= m + 1; i++) S.rptr[i] += S.rptr[i - 1];
    {
        int *fill = malloc(sizeof(int) * (size_t)(m + 2));
        memcpy(fill, S.rptr, sizeof(int) * (size_t)(m + 2));
        for (int j = 1; j <= n; j++)
            for (int t = ptr[j - 1]; t < ptr[j]; t++) {
                int p = fill[ind[t]]++;
                S.rcol[p] = j;
                S.rval[p] = val[t];
            }
        free(fill);
    }
    /* glp_unscale_prob */
    for (int i = 0; i <= m; i++) S.rii[i] = 1.0;
    for (int j = 0; j <= n; j++) S.sjj[j] = 1.0;
    memset(report, 0, sizeof(double) * 13);
    int bits = 0;
    report_stage(&S, report);
    if (report[0] >= 0.10 && report[1] <= 10.0) {
        bits |= 1;
        if (flags & SF_SKIP) {
            bits |= 16;
            goto done;
        }
    }
    if (flags & SF_GM) {
        /* gm_iterate (:143-160), it_max 15, tau 0.90 */
        int flag = max_row_ratio(&S) > max_col_ratio(&S);
        double ratio = 0.0, r_old, a, b;
        for (int k = 1; k <= 15; k++) {
            r_old = ratio;
            mat_mm(&S, &a, &b);
            ratio = b / a;
            if (k > 1 && ratio > 0.90 * r_old) break;
            sweep(&S, flag, 1);
        }
        report_stage(&S, report + 3);
        bits |= 2;
    }
    if (flags & SF_EQ) {
        sweep(&S, max_row_ratio(&S) > max_col_ratio(&S), 0);
        report_stage(&S, report + 6);
        bits |= 4;
    }
    if (flags & SF_2N) {
        for (int i = 1; i <= m; i++) S.rii[i] = round2n(S.rii[i]);
        for (int j = 1; j <= n; j++) S.sjj[j] = round2n(S.sjj[j]);
        report_stage(&S, report + 9);
        bits |= 8;
    }
done:
    report[12] = bits;
    for (int i = 1; i <= m; i++) rii_out[i - 1] = S.rii[i];
    for (int j = 1; j <= n; j++) sjj_out[j - 1] = S.sjj[j];
    free(S.rptr);
    free(S.rcol);
    free(S.rval);
    free(S.rii);
    free(S.sjj);
    return 0;
}
