/* ORACLE (test infrastructure only) — two-phase primal revised simplex with
 * projected steepest edge and Harris' two-pass ratio test.  Restates
 * glpspx01.js (GLPK 4.49) function by function; line numbers are cited at
 * each routine. */
#include <math.h>
#include <string.h>
#include "orc.h"

static const double kappa = 0.10;                 /* glpspx01.js:3 */

typedef struct {
    int m, n;
    signed char *type; double *lb, *ub, *coef, *obj;
    int *A_ptr, *A_ind; double *A_val;
    int *head; signed char *stat;
    int *N_ptr, *N_len, *N_ind; double *N_val;
    int valid; orc_bfd *bfd;
    double zeta; int phase; double tm_beg; int it_beg, it_cnt, it_dpy;
    double *bbar, *cbar;
    int refct; signed char *refsp; double *gamma;
    int q; int tcol_nnz; int *tcol_ind; double *tcol_vec; double tcol_max; int tcol_num;
    int p, p_stat; double teta;
    int trow_nnz; int *trow_ind; double *trow_vec;
    double *work1, *work2, *work3, *work4;
} csa_t;

#define D(n) ((double *)orc_alloc((size_t)(n), sizeof(double)))
#define I(n) ((int *)orc_alloc((size_t)(n), sizeof(int)))
#define C(n) ((signed char *)orc_alloc((size_t)(n), 1))

static csa_t *alloc_csa(orc_prob *lp)                       /* :5 */
{
    int m = lp->m, n = lp->n, nnz = lp->nnz;
    csa_t *csa = (csa_t *)orc_alloc(1, sizeof(csa_t));
    ORC_ASSERT(m > 0 && n > 0);
    csa->m = m; csa->n = n;
    csa->type = C(1 + m + n); csa->lb = D(1 + m + n); csa->ub = D(1 + m + n); csa->coef = D(1 + m + n);
    csa->obj = D(1 + n);
    csa->A_ptr = I(1 + n + 1); csa->A_ind = I(1 + nnz); csa->A_val = D(1 + nnz);
    csa->head = I(1 + m + n); csa->stat = C(1 + n);
    csa->N_ptr = I(1 + m + 1); csa->N_len = I(1 + m);
    csa->bbar = D(1 + m); csa->cbar = D(1 + n);
    csa->refsp = C(1 + m + n); csa->gamma = D(1 + n);
    csa->tcol_ind = I(1 + m); csa->tcol_vec = D(1 + m);
    csa->trow_ind = I(1 + n); csa->trow_vec = D(1 + n);
    csa->work1 = D(1 + m); csa->work2 = D(1 + m); csa->work3 = D(1 + m); csa->work4 = D(1 + m);
    return csa;
}

static void free_csa(csa_t *csa)
{
    orc_free(csa->type); orc_free(csa->lb); orc_free(csa->ub); orc_free(csa->coef); orc_free(csa->obj);
    orc_free(csa->A_ptr); orc_free(csa->A_ind); orc_free(csa->A_val);
    orc_free(csa->head); orc_free(csa->stat);
    orc_free(csa->N_ptr); orc_free(csa->N_len); orc_free(csa->N_ind); orc_free(csa->N_val);
    orc_free(csa->bbar); orc_free(csa->cbar); orc_free(csa->refsp); orc_free(csa->gamma);
    orc_free(csa->tcol_ind); orc_free(csa->tcol_vec); orc_free(csa->trow_ind); orc_free(csa->trow_vec);
    orc_free(csa->work1); orc_free(csa->work2); orc_free(csa->work3); orc_free(csa->work4);
    orc_free(csa);
}

static void alloc_N(csa_t *csa);
static void build_N(csa_t *csa);

static void init_csa(csa_t *csa, orc_prob *lp)              /* :42 */
{
    int m = csa->m, n = csa->n, i, j, k, loc, ptr;
    double cmax;
    for (i = 1; i <= m; i++) {
        csa->type[i] = lp->row_type[i];
        csa->lb[i] = lp->row_lb[i] * lp->rii[i];
        csa->ub[i] = lp->row_ub[i] * lp->rii[i];
        csa->coef[i] = 0.0;
    }
    for (j = 1; j <= n; j++) {
        csa->type[m + j] = lp->col_type[j];
        csa->lb[m + j] = lp->col_lb[j] / lp->sjj[j];
        csa->ub[m + j] = lp->col_ub[j] / lp->sjj[j];
        csa->coef[m + j] = lp->col_coef[j] * lp->sjj[j];
    }
    csa->obj[0] = lp->c0;
    memcpy(&csa->obj[1], &csa->coef[m + 1], (size_t)n * sizeof(double));
    cmax = 0.0;
    for (j = 1; j <= n; j++)
        if (cmax < fabs(csa->obj[j])) cmax = fabs(csa->obj[j]);
    if (cmax == 0.0) cmax = 1.0;
    switch (lp->dir) {
    case GLP_MIN: csa->zeta = +1.0 / cmax; break;
    case GLP_MAX: csa->zeta = -1.0 / cmax; break;
    default: ORC_ASSERT(0);
    }
    if (fabs(csa->zeta) < 1.0) csa->zeta *= 1000.0;
    loc = 1;
    for (j = 1; j <= n; j++) {
        csa->A_ptr[j] = loc;
        for (ptr = lp->A_ptr[j]; ptr < lp->A_ptr[j + 1]; ptr++) {
            i = lp->A_ind[ptr];
            csa->A_ind[loc] = i;
            csa->A_val[loc] = lp->rii[i] * lp->A_val[ptr] * lp->sjj[j];
            loc++;
        }
    }
    csa->A_ptr[n + 1] = loc;
    ORC_ASSERT(loc == lp->nnz + 1);
    ORC_ASSERT(lp->valid);
    memcpy(&csa->head[1], &lp->head[1], (size_t)m * sizeof(int));
    k = 0;
    for (i = 1; i <= m; i++) {
        if (lp->row_stat[i] != GLP_BS) {
            k++;
            ORC_ASSERT(k <= n);
            csa->head[m + k] = i;
            csa->stat[k] = lp->row_stat[i];
        }
    }
    for (j = 1; j <= n; j++) {
        if (lp->col_stat[j] != GLP_BS) {
            k++;
            ORC_ASSERT(k <= n);
            csa->head[m + k] = m + j;
            csa->stat[k] = lp->col_stat[j];
        }
    }
    ORC_ASSERT(k == n);
    csa->valid = 1; lp->valid = 0;
    csa->bfd = lp->bfd; lp->bfd = NULL;
    alloc_N(csa);
    build_N(csa);
    csa->phase = 0;
    csa->tm_beg = orc_time();
    csa->it_beg = csa->it_cnt = lp->it_cnt;
    csa->it_dpy = -1;
    csa->refct = 0;
    memset(&csa->refsp[1], 0, (size_t)(m + n));
    for (j = 1; j <= n; j++) csa->gamma[j] = 1.0;
}

static int inv_col(void *info, int i, int *ind, double *val)   /* :147 */
{
    csa_t *csa = (csa_t *)info;
    int m = csa->m, k, len, ptr, t;
    k = csa->head[i];
    if (k <= m) {
        len = 1;
        ind[1] = k;
        val[1] = 1.0;
    } else {
        ptr = csa->A_ptr[k - m];
        len = csa->A_ptr[k - m + 1] - ptr;
        memcpy(&ind[1], &csa->A_ind[ptr], (size_t)len * sizeof(int));
        memcpy(&val[1], &csa->A_val[ptr], (size_t)len * sizeof(double));
        for (t = 1; t <= len; t++) val[t] = -val[t];
    }
    return len;
}

static int invert_B(csa_t *csa)                              /* :177 */
{
    int ret = bfd_factorize(csa->bfd, csa->m, NULL, inv_col, csa);
    csa->valid = (ret == 0);
    return ret;
}

static int update_B(csa_t *csa, int i, int k)                 /* :183 */
{
    int m = csa->m, ret;
    if (k <= m) {
        int ind[2]; double val[2];
        ind[1] = k;
        val[1] = 1.0;
        ORC_ASSERT(csa->valid);
        ret = bfd_update_it(csa->bfd, i, 0, 1, ind, 0, val);
    } else {
        double *val = csa->work1;
        int beg = csa->A_ptr[k - m], end = csa->A_ptr[k - m + 1], ptr, len = 0;
        for (ptr = beg; ptr < end; ptr++) val[++len] = -csa->A_val[ptr];
        ORC_ASSERT(csa->valid);
        ret = bfd_update_it(csa->bfd, i, 0, len, csa->A_ind, beg - 1, val);
    }
    csa->valid = (ret == 0);
    return ret;
}

static void error_ftran(csa_t *csa, const double *h, const double *x, double *r)   /* :219 */
{
    int m = csa->m, i, k, beg, end, ptr;
    double temp;
    memcpy(&r[1], &h[1], (size_t)m * sizeof(double));
    for (i = 1; i <= m; i++) {
        temp = x[i];
        if (temp == 0.0) continue;
        k = csa->head[i];
        if (k <= m)
            r[k] -= temp;
        else {
            beg = csa->A_ptr[k - m];
            end = csa->A_ptr[k - m + 1];
            for (ptr = beg; ptr < end; ptr++) r[csa->A_ind[ptr]] += csa->A_val[ptr] * temp;
        }
    }
}

static void refine_ftran(csa_t *csa, const double *h, double *x)   /* :251 */
{
    int m = csa->m, i;
    double *r = csa->work1, *d = csa->work1;
    error_ftran(csa, h, x, r);
    ORC_ASSERT(csa->valid);
    bfd_ftran(csa->bfd, d);
    for (i = 1; i <= m; i++) x[i] += d[i];
}

static void error_btran(csa_t *csa, const double *h, const double *x, double *r)   /* :265 */
{
    int m = csa->m, i, k, beg, end, ptr;
    double temp;
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        temp = h[i];
        if (k <= m)
            temp -= x[k];
        else {
            beg = csa->A_ptr[k - m];
            end = csa->A_ptr[k - m + 1];
            for (ptr = beg; ptr < end; ptr++) temp += csa->A_val[ptr] * x[csa->A_ind[ptr]];
        }
        r[i] = temp;
    }
}

static void refine_btran(csa_t *csa, const double *h, double *x)   /* :295 */
{
    int m = csa->m, i;
    double *r = csa->work1, *d = csa->work1;
    error_btran(csa, h, x, r);
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, d);
    for (i = 1; i <= m; i++) x[i] += d[i];
}

static void alloc_N(csa_t *csa)                               /* :309 */
{
    int m = csa->m, n = csa->n, i, j, ptr;
    int *N_ptr = csa->N_ptr, *N_len = csa->N_len;
    for (i = 1; i <= m; i++) N_len[i] = 1;
    for (j = 1; j <= n; j++)
        for (ptr = csa->A_ptr[j]; ptr < csa->A_ptr[j + 1]; ptr++) N_len[csa->A_ind[ptr]]++;
    N_ptr[1] = 1;
    for (i = 1; i <= m; i++) {
        if (N_len[i] > n) N_len[i] = n;
        N_ptr[i + 1] = N_ptr[i] + N_len[i];
    }
    csa->N_ind = I(N_ptr[m + 1]);
    csa->N_val = D(N_ptr[m + 1]);
}

static void add_N_col(csa_t *csa, int j, int k)                /* :340 */
{
    int m = csa->m, pos, i, ptr;
    if (k <= m) {
        pos = csa->N_ptr[k] + (csa->N_len[k]++);
        csa->N_ind[pos] = j;
        csa->N_val[pos] = 1.0;
    } else {
        for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++) {
            i = csa->A_ind[ptr];
            pos = csa->N_ptr[i] + (csa->N_len[i]++);
            csa->N_ind[pos] = j;
            csa->N_val[pos] = -csa->A_val[ptr];
        }
    }
}

static void del_N_col(csa_t *csa, int j, int k)                /* :377 */
{
    int m = csa->m, pos, head, tail, i, ptr;
    if (k <= m) {
        head = csa->N_ptr[k];
        for (pos = head; csa->N_ind[pos] != j; pos++) {}
        tail = head + (--csa->N_len[k]);
        csa->N_ind[pos] = csa->N_ind[tail];
        csa->N_val[pos] = csa->N_val[tail];
    } else {
        for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++) {
            i = csa->A_ind[ptr];
            head = csa->N_ptr[i];
            for (pos = head; csa->N_ind[pos] != j; pos++) {}
            tail = head + (--csa->N_len[i]);
            csa->N_ind[pos] = csa->N_ind[tail];
            csa->N_val[pos] = csa->N_val[tail];
        }
    }
}

static void build_N(csa_t *csa)                                 /* :421 */
{
    int m = csa->m, n = csa->n, j;
    memset(&csa->N_len[1], 0, (size_t)m * sizeof(int));
    for (j = 1; j <= n; j++)
        if (csa->stat[j] != GLP_NS) add_N_col(csa, j, csa->head[m + j]);
}

static double get_xN(csa_t *csa, int j)                        /* :442 */
{
    int k = csa->head[csa->m + j];
    switch (csa->stat[j]) {
    case GLP_NL: return csa->lb[k];
    case GLP_NU: return csa->ub[k];
    case GLP_NF: return 0.0;
    case GLP_NS: return csa->lb[k];
    default: ORC_ASSERT(0);
    }
    return 0.0;
}

static void eval_beta(csa_t *csa, double *beta)                 /* :473 */
{
    int m = csa->m, n = csa->n, i, j, k, ptr;
    double *h = csa->work2, xN;
    for (i = 1; i <= m; i++) h[i] = 0.0;
    for (j = 1; j <= n; j++) {
        k = csa->head[m + j];
        xN = get_xN(csa, j);
        if (xN == 0.0) continue;
        if (k <= m)
            h[k] -= xN;
        else
            for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
                h[csa->A_ind[ptr]] += xN * csa->A_val[ptr];
    }
    memcpy(&beta[1], &h[1], (size_t)m * sizeof(double));
    ORC_ASSERT(csa->valid);
    bfd_ftran(csa->bfd, beta);
    refine_ftran(csa, h, beta);
}

static void eval_pi(csa_t *csa, double *pi)                     /* :514 */
{
    int m = csa->m, i;
    double *cB = csa->work2;
    for (i = 1; i <= m; i++) cB[i] = csa->coef[csa->head[i]];
    memcpy(&pi[1], &cB[1], (size_t)m * sizeof(double));
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, pi);
    refine_btran(csa, cB, pi);
}

static double eval_cost(csa_t *csa, const double *pi, int j)    /* :531 */
{
    int m = csa->m, k = csa->head[m + j], ptr;
    double dj = csa->coef[k];
    if (k <= m)
        dj -= pi[k];
    else
        for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
            dj += csa->A_val[ptr] * pi[csa->A_ind[ptr]];
    return dj;
}

static void eval_bbar(csa_t *csa) { eval_beta(csa, csa->bbar); }   /* :560 */

static void eval_cbar(csa_t *csa)                               /* :565 */
{
    int n = csa->n, j;
    double *pi = csa->work3;
    eval_pi(csa, pi);
    for (j = 1; j <= n; j++) csa->cbar[j] = eval_cost(csa, pi, j);
}

static void reset_refsp(csa_t *csa)                             /* :586 */
{
    int m = csa->m, n = csa->n, j;
    ORC_ASSERT(csa->refct == 0);
    csa->refct = 1000;
    memset(&csa->refsp[1], 0, (size_t)(m + n));
    for (j = 1; j <= n; j++) {
        csa->refsp[csa->head[m + j]] = 1;
        csa->gamma[j] = 1.0;
    }
}

static void chuzc(csa_t *csa, double tol_dj)                     /* :646 */
{
    int n = csa->n, j, q = 0;
    double dj, best = 0.0, temp;
    for (j = 1; j <= n; j++) {
        dj = csa->cbar[j];
        switch (csa->stat[j]) {
        case GLP_NL: if (dj >= -tol_dj) continue; break;
        case GLP_NU: if (dj <= +tol_dj) continue; break;
        case GLP_NF: if (-tol_dj <= dj && dj <= +tol_dj) continue; break;
        case GLP_NS: continue;
        default: ORC_ASSERT(0);
        }
        temp = (dj * dj) / csa->gamma[j];
        if (best < temp) { q = j; best = temp; }
    }
    csa->q = q;
}

/* right-hand side h = -N[q] (:702-719) */
static void neg_N_col(csa_t *csa, double *h)
{
    int m = csa->m, i, k = csa->head[m + csa->q], ptr;
    for (i = 1; i <= m; i++) h[i] = 0.0;
    if (k <= m)
        h[k] = -1.0;
    else
        for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++) h[csa->A_ind[ptr]] = csa->A_val[ptr];
}

static void tcol_pattern(csa_t *csa)
{
    int m = csa->m, i, nnz = 0;
    for (i = 1; i <= m; i++)
        if (csa->tcol_vec[i] != 0.0) csa->tcol_ind[++nnz] = i;
    csa->tcol_nnz = nnz;
}

static void eval_tcol(csa_t *csa)                                /* :690 */
{
    neg_N_col(csa, csa->tcol_vec);
    ORC_ASSERT(csa->valid);
    bfd_ftran(csa->bfd, csa->tcol_vec);
    tcol_pattern(csa);
}

static void refine_tcol(csa_t *csa)                              /* :732 */
{
    double *h = csa->work3;
    neg_N_col(csa, h);
    refine_ftran(csa, h, csa->tcol_vec);
    tcol_pattern(csa);
}

static void sort_tcol(csa_t *csa, double tol_piv)                 /* :773 */
{
    int nnz = csa->tcol_nnz, i, num, pos;
    int *ind = csa->tcol_ind; double *vec = csa->tcol_vec;
    double big = 0.0, eps, temp;
    for (pos = 1; pos <= nnz; pos++) {
        temp = fabs(vec[ind[pos]]);
        if (big < temp) big = temp;
    }
    csa->tcol_max = big;
    eps = tol_piv * (1.0 + 0.01 * big);
    for (num = 0; num < nnz;) {
        i = ind[nnz];
        if (fabs(vec[i]) < eps)
            nnz--;
        else {
            num++;
            ind[nnz] = ind[num];
            ind[num] = i;
        }
    }
    csa->tcol_num = num;
}

static void chuzr(csa_t *csa, double rtol)                        /* :808 */
{
    int m = csa->m, q = csa->q, phase = csa->phase;
    signed char *type = csa->type; double *lb = csa->lb, *ub = csa->ub, *coef = csa->coef;
    int *head = csa->head; double *bbar = csa->bbar;
    int i, i_stat = 0, k, p, p_stat, pos;
    double alfa, big, delta, s, t = 0.0, teta, tmax;
    s = (csa->cbar[q] > 0.0 ? -1.0 : +1.0);
    k = head[m + q];
    if (type[k] == GLP_DB) { p = -1; p_stat = 0; teta = ub[k] - lb[k]; big = 1.0; }
    else { p = 0; p_stat = 0; teta = DBL_MAX; big = 0.0; }
    for (pos = 1; pos <= csa->tcol_num; pos++) {
        i = csa->tcol_ind[pos];
        k = head[i];
        alfa = s * csa->tcol_vec[i];
        if (alfa > 0.0) {
            if (phase == 1 && coef[k] < 0.0) {
                delta = rtol * (1.0 + kappa * fabs(lb[k]));
                t = ((lb[k] + delta) - bbar[i]) / alfa;
                i_stat = GLP_NL;
            } else if (phase == 1 && coef[k] > 0.0)
                continue;
            else if (type[k] == GLP_UP || type[k] == GLP_DB || type[k] == GLP_FX) {
                delta = rtol * (1.0 + kappa * fabs(ub[k]));
                t = ((ub[k] + delta) - bbar[i]) / alfa;
                i_stat = GLP_NU;
            } else
                continue;
        } else {
            if (phase == 1 && coef[k] > 0.0) {
                delta = rtol * (1.0 + kappa * fabs(ub[k]));
                t = ((ub[k] - delta) - bbar[i]) / alfa;
                i_stat = GLP_NU;
            } else if (phase == 1 && coef[k] < 0.0)
                continue;
            else if (type[k] == GLP_LO || type[k] == GLP_DB || type[k] == GLP_FX) {
                delta = rtol * (1.0 + kappa * fabs(lb[k]));
                t = ((lb[k] - delta) - bbar[i]) / alfa;
                i_stat = GLP_NL;
            } else
                continue;
        }
        if (t < 0.0) t = 0.0;
        if (teta > t || (teta == t && big < fabs(alfa))) {
            p = i; p_stat = i_stat; teta = t; big = fabs(alfa);
        }
    }
    if (rtol == 0.0) goto done;
    if (p <= 0) goto done;
    if (teta == 0.0) goto done;
    tmax = teta;
    p = 0; p_stat = 0; teta = DBL_MAX; big = 0.0;
    for (pos = 1; pos <= csa->tcol_num; pos++) {
        i = csa->tcol_ind[pos];
        k = head[i];
        alfa = s * csa->tcol_vec[i];
        if (alfa > 0.0) {
            if (phase == 1 && coef[k] < 0.0) {
                t = (lb[k] - bbar[i]) / alfa;
                i_stat = GLP_NL;
            } else if (phase == 1 && coef[k] > 0.0)
                continue;
            else if (type[k] == GLP_UP || type[k] == GLP_DB || type[k] == GLP_FX) {
                t = (ub[k] - bbar[i]) / alfa;
                i_stat = GLP_NU;
            } else
                continue;
        } else {
            if (phase == 1 && coef[k] > 0.0) {
                t = (ub[k] - bbar[i]) / alfa;
                i_stat = GLP_NU;
            } else if (phase == 1 && coef[k] < 0.0)
                continue;
            else if (type[k] == GLP_LO || type[k] == GLP_DB || type[k] == GLP_FX) {
                t = (lb[k] - bbar[i]) / alfa;
                i_stat = GLP_NL;
            } else
                continue;
        }
        if (t < 0.0) t = 0.0;
        if (t <= tmax && big < fabs(alfa)) {
            p = i; p_stat = i_stat; teta = t; big = fabs(alfa);
        }
    }
    ORC_ASSERT(p != 0);
done:
    csa->p = p;
    if (p > 0 && type[head[p]] == GLP_FX)
        csa->p_stat = GLP_NS;
    else
        csa->p_stat = p_stat;
    csa->teta = s * teta;
}

static void eval_rho(csa_t *csa, double *rho)                     /* :1030 */
{
    int m = csa->m, i;
    for (i = 1; i <= m; i++) rho[i] = 0.0;
    rho[csa->p] = 1.0;
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, rho);
}

static void refine_rho(csa_t *csa, double *rho)                   /* :1044 */
{
    int m = csa->m, i;
    double *e = csa->work3;
    for (i = 1; i <= m; i++) e[i] = 0.0;
    e[csa->p] = 1.0;
    refine_btran(csa, e, rho);
}

static void eval_trow(csa_t *csa, const double *rho)              /* :1058 */
{
    int m = csa->m, n = csa->n, i, j, ptr, end, nnz;
    double *trow_vec = csa->trow_vec, temp;
    for (j = 1; j <= n; j++) trow_vec[j] = 0.0;
    for (i = 1; i <= m; i++) {
        temp = rho[i];
        if (temp == 0.0) continue;
        end = csa->N_ptr[i] + csa->N_len[i];
        for (ptr = csa->N_ptr[i]; ptr < end; ptr++) trow_vec[csa->N_ind[ptr]] -= temp * csa->N_val[ptr];
    }
    nnz = 0;
    for (j = 1; j <= n; j++)
        if (trow_vec[j] != 0.0) csa->trow_ind[++nnz] = j;
    csa->trow_nnz = nnz;
}

static void update_bbar(csa_t *csa)                                /* :1100 */
{
    int p = csa->p, i, pos;
    double teta = csa->teta;
    if (p > 0) csa->bbar[p] = get_xN(csa, csa->q) + teta;
    if (teta == 0.0) return;
    for (pos = 1; pos <= csa->tcol_nnz; pos++) {
        i = csa->tcol_ind[pos];
        if (i == p) continue;
        csa->bbar[i] += csa->tcol_vec[i] * teta;
    }
}

static double reeval_cost(csa_t *csa)                              /* :1133 */
{
    int m = csa->m, i, pos;
    double dq = csa->coef[csa->head[m + csa->q]];
    for (pos = 1; pos <= csa->tcol_nnz; pos++) {
        i = csa->tcol_ind[pos];
        dq += csa->coef[csa->head[i]] * csa->tcol_vec[i];
    }
    return dq;
}

static void update_cbar(csa_t *csa)                                /* :1154 */
{
    int q = csa->q, j, pos;
    double new_dq = (csa->cbar[q] /= csa->trow_vec[q]);
    for (pos = 1; pos <= csa->trow_nnz; pos++) {
        j = csa->trow_ind[pos];
        if (j == q) continue;
        csa->cbar[j] -= csa->trow_vec[j] * new_dq;
    }
}

static void update_gamma(csa_t *csa)                                /* :1178 */
{
    int m = csa->m, q = csa->q, p = csa->p, i, j, k, pos, ptr;
    int *head = csa->head; signed char *refsp = csa->refsp;
    double *gamma = csa->gamma, *u = csa->work3;
    double gamma_q, delta_q, pivot, s, t, t1, t2;
    ORC_ASSERT(csa->refct > 0);
    csa->refct--;
    gamma_q = delta_q = (refsp[head[m + q]] ? 1.0 : 0.0);
    for (i = 1; i <= m; i++) u[i] = 0.0;
    for (pos = 1; pos <= csa->tcol_nnz; pos++) {
        i = csa->tcol_ind[pos];
        if (refsp[head[i]]) {
            u[i] = t = csa->tcol_vec[i];
            gamma_q += t * t;
        } else
            u[i] = 0.0;
    }
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, u);
    pivot = csa->trow_vec[q];
    for (pos = 1; pos <= csa->trow_nnz; pos++) {
        j = csa->trow_ind[pos];
        if (j == q) continue;
        t = csa->trow_vec[j] / pivot;
        k = head[m + j];
        if (k <= m)
            s = u[k];
        else {
            s = 0.0;
            for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
                s -= csa->A_val[ptr] * u[csa->A_ind[ptr]];
        }
        t1 = gamma[j] + t * t * gamma_q + 2.0 * t * s;
        t2 = (refsp[k] ? 1.0 : 0.0) + delta_q * t * t;
        gamma[j] = (t1 >= t2 ? t1 : t2);
        if (gamma[j] < DBL_EPSILON) gamma[j] = DBL_EPSILON;
    }
    if (csa->type[head[p]] == GLP_FX)
        gamma[q] = 1.0;
    else {
        gamma[q] = gamma_q / (pivot * pivot);
        if (gamma[q] < DBL_EPSILON) gamma[q] = DBL_EPSILON;
    }
}

static void change_basis(csa_t *csa)                                /* :1310 */
{
    int m = csa->m, q = csa->q, p = csa->p, k;
    if (p < 0) {
        switch (csa->stat[q]) {
        case GLP_NL: csa->stat[q] = GLP_NU; break;
        case GLP_NU: csa->stat[q] = GLP_NL; break;
        default: ORC_ASSERT(0);
        }
    } else {
        k = csa->head[p];
        csa->head[p] = csa->head[m + q];
        csa->head[m + q] = k;
        csa->stat[q] = (signed char)csa->p_stat;
    }
}

static int set_aux_obj(csa_t *csa, double tol_bnd)                   /* :1373 */
{
    int m = csa->m, n = csa->n, i, k, cnt = 0;
    signed char *type = csa->type; double *lb = csa->lb, *ub = csa->ub, eps;
    tol_bnd *= 0.90;
    for (k = 1; k <= m + n; k++) csa->coef[k] = 0.0;
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        if (type[k] == GLP_LO || type[k] == GLP_DB || type[k] == GLP_FX) {
            eps = tol_bnd * (1.0 + kappa * fabs(lb[k]));
            if (csa->bbar[i] < lb[k] - eps) { csa->coef[k] = -1.0; cnt++; }
        }
        if (type[k] == GLP_UP || type[k] == GLP_DB || type[k] == GLP_FX) {
            eps = tol_bnd * (1.0 + kappa * fabs(ub[k]));
            if (csa->bbar[i] > ub[k] + eps) { csa->coef[k] = +1.0; cnt++; }
        }
    }
    return cnt;
}

static void set_orig_obj(csa_t *csa)                                 /* :1416 */
{
    int m = csa->m, n = csa->n, i, j;
    for (i = 1; i <= m; i++) csa->coef[i] = 0.0;
    for (j = 1; j <= n; j++) csa->coef[m + j] = csa->zeta * csa->obj[j];
}

static int check_stab(csa_t *csa, double tol_bnd)                     /* :1429 */
{
    int m = csa->m, phase = csa->phase, i, k;
    signed char *type = csa->type; double *lb = csa->lb, *ub = csa->ub, *coef = csa->coef, eps;
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        if (phase == 1 && coef[k] < 0.0) {
            eps = tol_bnd * (1.0 + kappa * fabs(lb[k]));
            if (csa->bbar[i] > lb[k] + eps) return 1;
        } else if (phase == 1 && coef[k] > 0.0) {
            eps = tol_bnd * (1.0 + kappa * fabs(ub[k]));
            if (csa->bbar[i] < ub[k] - eps) return 1;
        } else {
            if (type[k] == GLP_LO || type[k] == GLP_DB || type[k] == GLP_FX) {
                eps = tol_bnd * (1.0 + kappa * fabs(lb[k]));
                if (csa->bbar[i] < lb[k] - eps) return 1;
            }
            if (type[k] == GLP_UP || type[k] == GLP_DB || type[k] == GLP_FX) {
                eps = tol_bnd * (1.0 + kappa * fabs(ub[k]));
                if (csa->bbar[i] > ub[k] + eps) return 1;
            }
        }
    }
    return 0;
}

static int check_feas(csa_t *csa, double tol_bnd)                      /* :1483 */
{
    int m = csa->m, i, k;
    double *lb = csa->lb, *ub = csa->ub, *coef = csa->coef, eps;
    ORC_ASSERT(csa->phase == 1);
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        if (coef[k] < 0.0) {
            eps = tol_bnd * (1.0 + kappa * fabs(lb[k]));
            if (csa->bbar[i] < lb[k] - eps) return 1;
        } else if (coef[k] > 0.0) {
            eps = tol_bnd * (1.0 + kappa * fabs(ub[k]));
            if (csa->bbar[i] > ub[k] + eps) return 1;
        }
    }
    return 0;
}

static double eval_obj(csa_t *csa)                                       /* :1524 */
{
    int m = csa->m, n = csa->n, i, j, k;
    double sum = csa->obj[0];
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        if (k > m) sum += csa->obj[k - m] * csa->bbar[i];
    }
    for (j = 1; j <= n; j++) {
        k = csa->head[m + j];
        if (k > m) sum += csa->obj[k - m] * get_xN(csa, j);
    }
    return sum;
}

static void store_sol(csa_t *csa, orc_prob *lp, int p_stat, int d_stat, int ray)   /* :1591 */
{
    int m = csa->m, n = csa->n, i, j, k;
    double zeta = csa->zeta;
    lp->valid = 1; csa->valid = 0;
    lp->bfd = csa->bfd; csa->bfd = NULL;
    memcpy(&lp->head[1], &csa->head[1], (size_t)m * sizeof(int));
    lp->pbs_stat = p_stat;
    lp->dbs_stat = d_stat;
    lp->obj_val = eval_obj(csa);
    lp->it_cnt = csa->it_cnt;
    lp->some = ray;
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        if (k <= m) {
            lp->row_stat[k] = GLP_BS; lp->row_bind[k] = i;
            lp->row_prim[k] = csa->bbar[i] / lp->rii[k];
            lp->row_dual[k] = 0.0;
        } else {
            lp->col_stat[k - m] = GLP_BS; lp->col_bind[k - m] = i;
            lp->col_prim[k - m] = csa->bbar[i] * lp->sjj[k - m];
            lp->col_dual[k - m] = 0.0;
        }
    }
    for (j = 1; j <= n; j++) {
        k = csa->head[m + j];
        if (k <= m) {
            lp->row_stat[k] = csa->stat[j]; lp->row_bind[k] = 0;
            switch (csa->stat[j]) {
            case GLP_NL: lp->row_prim[k] = lp->row_lb[k]; break;
            case GLP_NU: lp->row_prim[k] = lp->row_ub[k]; break;
            case GLP_NF: lp->row_prim[k] = 0.0; break;
            case GLP_NS: lp->row_prim[k] = lp->row_lb[k]; break;
            default: ORC_ASSERT(0);
            }
            lp->row_dual[k] = (csa->cbar[j] * lp->rii[k]) / zeta;
        } else {
            int c = k - m;
            lp->col_stat[c] = csa->stat[j]; lp->col_bind[c] = 0;
            switch (csa->stat[j]) {
            case GLP_NL: lp->col_prim[c] = lp->col_lb[c]; break;
            case GLP_NU: lp->col_prim[c] = lp->col_ub[c]; break;
            case GLP_NF: lp->col_prim[c] = 0.0; break;
            case GLP_NS: lp->col_prim[c] = lp->col_lb[c]; break;
            default: ORC_ASSERT(0);
            }
            lp->col_dual[c] = (csa->cbar[j] / lp->sjj[c]) / zeta;
        }
    }
}

static int fail_return(csa_t *csa, orc_prob *lp)   /* :1715-1722 / :1943-1950 */
{
    ORC_ASSERT(!lp->valid && lp->bfd == NULL);
    lp->bfd = csa->bfd; csa->bfd = NULL;
    lp->pbs_stat = lp->dbs_stat = GLP_UNDEF;
    lp->obj_val = 0.0;
    lp->it_cnt = csa->it_cnt;
    lp->some = 0;
    return GLP_EFAIL;
}

static int time_exhausted(csa_t *csa, const orc_smcp *parm)
{
    return parm->tm_lim < ORC_INT_MAX && 1000.0 * (orc_time() - csa->tm_beg) >= parm->tm_lim;
}

int spx_primal(orc_prob *lp, const orc_smcp *parm)                 /* :1, loop :1705 */
{
    csa_t *csa;
    int binv_st = 2, bbar_st = 0, cbar_st = 0, rigorous = 0;
    int p_stat, d_stat, ret;
    csa = alloc_csa(lp);
    init_csa(csa, lp);
    for (;;) {
        if (binv_st == 0) {
            ret = invert_B(csa);
            if (ret != 0) { ret = fail_return(csa, lp); break; }
            csa->valid = 1;
            binv_st = 1;
            bbar_st = cbar_st = 0;
        }
        if (bbar_st == 0) {
            eval_bbar(csa);
            bbar_st = 1;
            if (csa->phase == 0) {
                if (set_aux_obj(csa, parm->tol_bnd) > 0)
                    csa->phase = 1;
                else {
                    set_orig_obj(csa);
                    csa->phase = 2;
                }
                ORC_ASSERT(check_stab(csa, parm->tol_bnd) == 0);
                cbar_st = 0;
            }
            if (check_stab(csa, parm->tol_bnd)) {
                orc_instab_events++; orc_instab_last_it = csa->it_cnt;
                csa->phase = 0;
                binv_st = 0;
                rigorous = 5;
                continue;
            }
        }
        ORC_ASSERT(csa->phase == 1 || csa->phase == 2);
        if (csa->phase == 1 && !check_feas(csa, parm->tol_bnd)) {
            csa->phase = 2;
            set_orig_obj(csa);
            cbar_st = 0;
        }
        if (cbar_st == 0) {
            eval_cbar(csa);
            cbar_st = 1;
        }
        if (parm->pricing == GLP_PT_PSE) {
            if (csa->refct == 0) reset_refsp(csa);
        } else
            ORC_ASSERT(parm->pricing == GLP_PT_STD);
        ORC_ASSERT(binv_st && bbar_st && cbar_st);
        if ((parm->it_lim < ORC_INT_MAX && csa->it_cnt - csa->it_beg >= parm->it_lim) ||
            time_exhausted(csa, parm)) {
            int is_it = (parm->it_lim < ORC_INT_MAX && csa->it_cnt - csa->it_beg >= parm->it_lim);
            if (bbar_st != 1 || (csa->phase == 2 && cbar_st != 1)) {
                if (bbar_st != 1) bbar_st = 0;
                if (csa->phase == 2 && cbar_st != 1) cbar_st = 0;
                continue;
            }
            switch (csa->phase) {
            case 1:
                p_stat = GLP_INFEAS;
                set_orig_obj(csa);
                eval_cbar(csa);
                break;
            default:
                p_stat = GLP_FEAS;
                break;
            }
            chuzc(csa, parm->tol_dj);
            d_stat = (csa->q == 0 ? GLP_FEAS : GLP_INFEAS);
            store_sol(csa, lp, p_stat, d_stat, 0);
            ret = is_it ? GLP_EITLIM : GLP_ETMLIM;
            break;
        }
        chuzc(csa, parm->tol_dj);
        if (csa->q == 0) {
            if (bbar_st != 1 || cbar_st != 1) {
                if (bbar_st != 1) bbar_st = 0;
                if (cbar_st != 1) cbar_st = 0;
                continue;
            }
            switch (csa->phase) {
            case 1:
                p_stat = GLP_NOFEAS;
                set_orig_obj(csa);
                eval_cbar(csa);
                chuzc(csa, parm->tol_dj);
                d_stat = (csa->q == 0 ? GLP_FEAS : GLP_INFEAS);
                break;
            default:
                p_stat = d_stat = GLP_FEAS;
                break;
            }
            store_sol(csa, lp, p_stat, d_stat, 0);
            ret = 0;
            break;
        }
        eval_tcol(csa);
        if (rigorous) refine_tcol(csa);
        sort_tcol(csa, parm->tol_piv);
        {
            double d1 = csa->cbar[csa->q], d2 = reeval_cost(csa);
            ORC_ASSERT(d1 != 0.0);
            if (fabs(d1 - d2) > 1e-5 * (1.0 + fabs(d2)) || !((d1 < 0.0 && d2 < 0.0) || (d1 > 0.0 && d2 > 0.0))) {
                if (cbar_st != 1 || !rigorous) {
                    if (cbar_st != 1) cbar_st = 0;
                    rigorous = 5;
                    continue;
                }
            }
            if (d1 > 0.0)
                csa->cbar[csa->q] = (d2 > 0.0 ? d2 : +DBL_EPSILON);
            else
                csa->cbar[csa->q] = (d2 < 0.0 ? d2 : -DBL_EPSILON);
        }
        if (parm->r_test == GLP_RT_STD)
            chuzr(csa, 0.0);
        else {
            ORC_ASSERT(parm->r_test == GLP_RT_HAR);
            chuzr(csa, 0.30 * parm->tol_bnd);
        }
        if (csa->p == 0) {
            if (bbar_st != 1 || cbar_st != 1 || !rigorous) {
                if (bbar_st != 1) bbar_st = 0;
                if (cbar_st != 1) cbar_st = 0;
                rigorous = 1;
                continue;
            }
            if (csa->phase == 1)
                ret = fail_return(csa, lp);
            else {
                store_sol(csa, lp, GLP_FEAS, GLP_NOFEAS, csa->head[csa->m + csa->q]);
                ret = 0;
            }
            break;
        }
        if (csa->p > 0) {
            double piv = csa->tcol_vec[csa->p];
            double eps = 1e-5 * (1.0 + 0.01 * csa->tcol_max);
            if (fabs(piv) < eps) {
                if (!rigorous) { rigorous = 5; continue; }
            }
        }
        if (csa->p > 0) {
            double *rho = csa->work4;
            eval_rho(csa, rho);
            if (rigorous) refine_rho(csa, rho);
            eval_trow(csa, rho);
        }
        if (csa->p > 0) {
            double piv1 = csa->tcol_vec[csa->p], piv2 = csa->trow_vec[csa->q];
            ORC_ASSERT(piv1 != 0.0);
            if (fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) || !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0))) {
                if (binv_st != 1 || !rigorous) {
                    if (binv_st != 1) binv_st = 0;
                    rigorous = 5;
                    continue;
                }
                if (csa->trow_vec[csa->q] == 0.0) {
                    csa->trow_nnz++;
                    ORC_ASSERT(csa->trow_nnz <= csa->n);
                    csa->trow_ind[csa->trow_nnz] = csa->q;
                }
                csa->trow_vec[csa->q] = piv1;
            }
        }
        update_bbar(csa);
        bbar_st = 2;
        if (csa->p > 0) {
            update_cbar(csa);
            cbar_st = 2;
            if (csa->phase == 1) {
                int k = csa->head[csa->p];
                csa->cbar[csa->q] -= csa->coef[k];
                csa->coef[k] = 0.0;
            }
        }
        if (csa->p > 0) {
            if (parm->pricing == GLP_PT_PSE) {
                if (csa->refct > 0) update_gamma(csa);
            }
        }
        if (csa->p > 0) {
            ret = update_B(csa, csa->p, csa->head[csa->m + csa->q]);
            if (ret == 0)
                binv_st = 2;
            else {
                csa->valid = 0;
                binv_st = 0;
            }
        }
        if (csa->p > 0) {
            del_N_col(csa, csa->q, csa->head[csa->m + csa->q]);
            if (csa->type[csa->head[csa->p]] != GLP_FX)
                add_N_col(csa, csa->q, csa->head[csa->p]);
        }
        if (orc_trace)
            orc_trace(orc_trace_ctx, 1, csa->it_cnt, csa->phase, csa->p, csa->q, csa->head[csa->m + csa->q],
                      csa->p > 0 ? csa->head[csa->p] : 0, csa->teta);
        change_basis(csa);
        csa->it_cnt++;
        if (rigorous > 0) rigorous--;
    }
    if (csa->bfd) { bfd_delete_it(csa->bfd); csa->bfd = NULL; }
    free_csa(csa);
    return ret;
}
