/* ORACLE (test infrastructure only) — two-phase dual revised simplex with
 * dual projected steepest edge and Harris' two-pass ratio test on the pivot
 * row.  Restates glpspx02.js (GLPK 4.49) function by function; line numbers
 * are cited at each routine. */
#include <math.h>
#include <string.h>
#include "orc.h"

static const double kappa = 0.10;                 /* glpspx02.js:3 */

typedef struct {
    int m, n;
    signed char *type; double *lb, *ub, *coef;
    signed char *orig_type; double *orig_lb, *orig_ub, *obj;
    int *A_ptr, *A_ind; double *A_val;
    int *AT_ptr, *AT_ind; double *AT_val;
    int *head, *bind; signed char *stat;
    int valid; orc_bfd *bfd;
    double zeta; int phase; double tm_beg; int it_beg, it_cnt, it_dpy;
    double *bbar, *cbar;
    int refct; signed char *refsp; double *gamma;
    int p; double delta;
    int trow_nnz; int *trow_ind; double *trow_vec; double trow_max; int trow_num;
    int q; double new_dq;
    int tcol_nnz; int *tcol_ind; double *tcol_vec;
    double *work1, *work2, *work3, *work4;
} csa_t;

#define D(n) ((double *)orc_alloc((size_t)(n), sizeof(double)))
#define I(n) ((int *)orc_alloc((size_t)(n), sizeof(int)))
#define C(n) ((signed char *)orc_alloc((size_t)(n), 1))

static csa_t *alloc_csa(orc_prob *lp)                                 /* :5 */
{
    int m = lp->m, n = lp->n, nnz = lp->nnz;
    csa_t *csa = (csa_t *)orc_alloc(1, sizeof(csa_t));
    ORC_ASSERT(m > 0 && n > 0);
    csa->m = m; csa->n = n;
    csa->type = C(1 + m + n); csa->lb = D(1 + m + n); csa->ub = D(1 + m + n); csa->coef = D(1 + m + n);
    csa->orig_type = C(1 + m + n); csa->orig_lb = D(1 + m + n); csa->orig_ub = D(1 + m + n);
    csa->obj = D(1 + n);
    csa->A_ptr = I(1 + n + 1); csa->A_ind = I(1 + nnz); csa->A_val = D(1 + nnz);
    csa->AT_ptr = I(1 + m + 1); csa->AT_ind = I(1 + nnz); csa->AT_val = D(1 + nnz);
    csa->head = I(1 + m + n); csa->bind = I(1 + m + n); csa->stat = C(1 + n);
    csa->bbar = D(1 + m); csa->cbar = D(1 + n);
    csa->refsp = C(1 + m + n); csa->gamma = D(1 + m);
    csa->trow_ind = I(1 + n); csa->trow_vec = D(1 + n);
    csa->tcol_ind = I(1 + m); csa->tcol_vec = D(1 + m);
    csa->work1 = D(1 + m); csa->work2 = D(1 + m); csa->work3 = D(1 + m); csa->work4 = D(1 + m);
    return csa;
}

static void free_csa(csa_t *csa)
{
    orc_free(csa->type); orc_free(csa->lb); orc_free(csa->ub); orc_free(csa->coef);
    orc_free(csa->orig_type); orc_free(csa->orig_lb); orc_free(csa->orig_ub); orc_free(csa->obj);
    orc_free(csa->A_ptr); orc_free(csa->A_ind); orc_free(csa->A_val);
    orc_free(csa->AT_ptr); orc_free(csa->AT_ind); orc_free(csa->AT_val);
    orc_free(csa->head); orc_free(csa->bind); orc_free(csa->stat);
    orc_free(csa->bbar); orc_free(csa->cbar); orc_free(csa->refsp); orc_free(csa->gamma);
    orc_free(csa->trow_ind); orc_free(csa->trow_vec); orc_free(csa->tcol_ind); orc_free(csa->tcol_vec);
    orc_free(csa->work1); orc_free(csa->work2); orc_free(csa->work3); orc_free(csa->work4);
    orc_free(csa);
}

static void init_csa(csa_t *csa, orc_prob *lp)                        /* :89 */
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
    memcpy(&csa->orig_type[1], &csa->type[1], (size_t)(m + n));
    memcpy(&csa->orig_lb[1], &csa->lb[1], (size_t)(m + n) * sizeof(double));
    memcpy(&csa->orig_ub[1], &csa->ub[1], (size_t)(m + n) * sizeof(double));
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
    for (j = 1; j <= n; j++) csa->coef[m + j] *= csa->zeta;
    /* chrome_workaround_1 (:45): A by columns */
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
    ORC_ASSERT(loc - 1 == lp->nnz);
    /* chrome_workaround_2 (:66): A by rows (only the per-row set matters
     * numerically, see eval_trow2) */
    loc = 1;
    for (i = 1; i <= m; i++) {
        csa->AT_ptr[i] = loc;
        for (ptr = lp->AT_ptr[i]; ptr < lp->AT_ptr[i + 1]; ptr++) {
            j = lp->AT_ind[ptr];
            csa->AT_ind[loc] = j;
            csa->AT_val[loc] = lp->rii[i] * lp->AT_val[ptr] * lp->sjj[j];
            loc++;
        }
    }
    csa->AT_ptr[m + 1] = loc;
    ORC_ASSERT(loc - 1 == lp->nnz);
    ORC_ASSERT(lp->valid);
    memcpy(&csa->head[1], &lp->head[1], (size_t)m * sizeof(int));
    k = 0;
    for (i = 1; i <= m; i++)
        if (lp->row_stat[i] != GLP_BS) {
            k++;
            ORC_ASSERT(k <= n);
            csa->head[m + k] = i;
            csa->stat[k] = lp->row_stat[i];
        }
    for (j = 1; j <= n; j++)
        if (lp->col_stat[j] != GLP_BS) {
            k++;
            ORC_ASSERT(k <= n);
            csa->head[m + k] = m + j;
            csa->stat[k] = lp->col_stat[j];
        }
    ORC_ASSERT(k == n);
    for (k = 1; k <= m + n; k++) csa->bind[csa->head[k]] = k;
    csa->valid = 1; lp->valid = 0;
    csa->bfd = lp->bfd; lp->bfd = NULL;
    csa->phase = 0;
    csa->tm_beg = orc_time();
    csa->it_beg = csa->it_cnt = lp->it_cnt;
    csa->it_dpy = -1;
    csa->refct = 0;
    memset(&csa->refsp[1], 0, (size_t)(m + n));
    for (i = 1; i <= m; i++) csa->gamma[i] = 1.0;
}

static int inv_col(void *info, int i, int *ind, double *val)            /* :192 */
{
    csa_t *csa = (csa_t *)info;
    int m = csa->m, k, len, ptr, t;
    k = csa->head[i];
    if (k <= m) {
        len = 1; ind[1] = k; val[1] = 1.0;
    } else {
        ptr = csa->A_ptr[k - m];
        len = csa->A_ptr[k - m + 1] - ptr;
        memcpy(&ind[1], &csa->A_ind[ptr], (size_t)len * sizeof(int));
        memcpy(&val[1], &csa->A_val[ptr], (size_t)len * sizeof(double));
        for (t = 1; t <= len; t++) val[t] = -val[t];
    }
    return len;
}

static int invert_B(csa_t *csa)                                          /* :222 */
{
    int ret = bfd_factorize(csa->bfd, csa->m, NULL, inv_col, csa);
    csa->valid = (ret == 0);
    return ret;
}

static int update_B(csa_t *csa, int i, int k)                             /* :228 */
{
    int m = csa->m, ret;
    if (k <= m) {
        int ind[2]; double val[2];
        ind[1] = k; val[1] = 1.0;
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

static void error_ftran(csa_t *csa, const double *h, const double *x, double *r)   /* :264 */
{
    int m = csa->m, i, k, ptr;
    double temp;
    memcpy(&r[1], &h[1], (size_t)m * sizeof(double));
    for (i = 1; i <= m; i++) {
        temp = x[i];
        if (temp == 0.0) continue;
        k = csa->head[i];
        if (k <= m)
            r[k] -= temp;
        else
            for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
                r[csa->A_ind[ptr]] += csa->A_val[ptr] * temp;
    }
}

static void refine_ftran(csa_t *csa, const double *h, double *x)          /* :296 */
{
    int m = csa->m, i;
    double *r = csa->work1, *d = csa->work1;
    error_ftran(csa, h, x, r);
    ORC_ASSERT(csa->valid);
    bfd_ftran(csa->bfd, d);
    for (i = 1; i <= m; i++) x[i] += d[i];
}

static void error_btran(csa_t *csa, const double *h, const double *x, double *r)   /* :310 */
{
    int m = csa->m, i, k, ptr;
    double temp;
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        temp = h[i];
        if (k <= m)
            temp -= x[k];
        else
            for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
                temp += csa->A_val[ptr] * x[csa->A_ind[ptr]];
        r[i] = temp;
    }
}

static void refine_btran(csa_t *csa, const double *h, double *x)          /* :340 */
{
    int m = csa->m, i;
    double *r = csa->work1, *d = csa->work1;
    error_btran(csa, h, x, r);
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, d);
    for (i = 1; i <= m; i++) x[i] += d[i];
}

static double get_xN(csa_t *csa, int j)                                   /* :354 */
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

static void eval_beta(csa_t *csa, double *beta)                            /* :385 */
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

static void eval_pi(csa_t *csa, double *pi)                                /* :426 */
{
    int m = csa->m, i;
    double *cB = csa->work2;
    for (i = 1; i <= m; i++) cB[i] = csa->coef[csa->head[i]];
    memcpy(&pi[1], &cB[1], (size_t)m * sizeof(double));
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, pi);
    refine_btran(csa, cB, pi);
}

static double eval_cost(csa_t *csa, const double *pi, int j)               /* :443 */
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

static void eval_bbar(csa_t *csa) { eval_beta(csa, csa->bbar); }              /* :472 */

static void eval_cbar(csa_t *csa)                                           /* :476 */
{
    int n = csa->n, j;
    double *pi = csa->work3;
    eval_pi(csa, pi);
    for (j = 1; j <= n; j++) csa->cbar[j] = eval_cost(csa, pi, j);
}

static void reset_refsp(csa_t *csa)                                         /* :497 */
{
    int m = csa->m, n = csa->n, i;
    ORC_ASSERT(csa->refct == 0);
    csa->refct = 1000;
    memset(&csa->refsp[1], 0, (size_t)(m + n));
    for (i = 1; i <= m; i++) {
        csa->refsp[csa->head[i]] = 1;
        csa->gamma[i] = 1.0;
    }
}

static void chuzr(csa_t *csa, double tol_bnd)                                /* :572 */
{
    int m = csa->m, i, k, p = 0;
    signed char *type = csa->type; double *lb = csa->lb, *ub = csa->ub;
    double delta = 0.0, best = 0.0, eps, ri, temp;
    for (i = 1; i <= m; i++) {
        k = csa->head[i];
        ri = 0.0;
        if (type[k] == GLP_LO || type[k] == GLP_DB || type[k] == GLP_FX) {
            eps = tol_bnd * (1.0 + kappa * fabs(lb[k]));
            if (csa->bbar[i] < lb[k] - eps) ri = lb[k] - csa->bbar[i];
        }
        if (type[k] == GLP_UP || type[k] == GLP_DB || type[k] == GLP_FX) {
            eps = tol_bnd * (1.0 + kappa * fabs(ub[k]));
            if (csa->bbar[i] > ub[k] + eps) ri = ub[k] - csa->bbar[i];
        }
        if (ri == 0.0) continue;
        temp = csa->gamma[i];
        if (temp < DBL_EPSILON) temp = DBL_EPSILON;
        temp = (ri * ri) / temp;
        if (best < temp) { p = i; delta = ri; best = temp; }
    }
    csa->p = p;
    csa->delta = delta;
}

static void eval_rho(csa_t *csa, double *rho)                                /* :627 */
{
    int m = csa->m, i;
    for (i = 1; i <= m; i++) rho[i] = 0.0;
    rho[csa->p] = 1.0;
    ORC_ASSERT(csa->valid);
    bfd_btran(csa->bfd, rho);
}

static void refine_rho(csa_t *csa, double *rho)                              /* :641 */
{
    int m = csa->m, i;
    double *e = csa->work3;
    for (i = 1; i <= m; i++) e[i] = 0.0;
    e[csa->p] = 1.0;
    refine_btran(csa, e, rho);
}

static void eval_trow1(csa_t *csa, const double *rho)                        /* :655 */
{
    int m = csa->m, n = csa->n, j, k, ptr, nnz = 0;
    double temp;
    for (j = 1; j <= n; j++) {
        if (csa->stat[j] == GLP_NS) { csa->trow_vec[j] = 0.0; continue; }
        k = csa->head[m + j];
        if (k <= m)
            temp = -rho[k];
        else {
            temp = 0.0;
            for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
                temp += rho[csa->A_ind[ptr]] * csa->A_val[ptr];
        }
        if (temp != 0.0) csa->trow_ind[++nnz] = j;
        csa->trow_vec[j] = temp;
    }
    csa->trow_nnz = nnz;
}

static void eval_trow2(csa_t *csa, const double *rho)                        /* :695 */
{
    int m = csa->m, n = csa->n, i, j, ptr, nnz;
    int *bind = csa->bind; signed char *stat = csa->stat;
    double *trow_vec = csa->trow_vec, temp;
    for (j = 1; j <= n; j++) trow_vec[j] = 0.0;
    for (i = 1; i <= m; i++) {
        temp = rho[i];
        if (temp == 0.0) continue;
        j = bind[i] - m;
        if (j >= 1 && stat[j] != GLP_NS) trow_vec[j] -= temp;
        for (ptr = csa->AT_ptr[i]; ptr < csa->AT_ptr[i + 1]; ptr++) {
            j = bind[m + csa->AT_ind[ptr]] - m;
            if (j >= 1 && stat[j] != GLP_NS) trow_vec[j] += temp * csa->AT_val[ptr];
        }
    }
    nnz = 0;
    for (j = 1; j <= n; j++)
        if (trow_vec[j] != 0.0) csa->trow_ind[++nnz] = j;
    csa->trow_nnz = nnz;
}

static void eval_trow(csa_t *csa, const double *rho)                         /* :735 */
{
    int m = csa->m, i, nnz = 0;
    double dens;
    for (i = 1; i <= m; i++)
        if (rho[i] != 0.0) nnz++;
    dens = (double)nnz / (double)m;
    if (dens >= 0.20) eval_trow1(csa, rho); else eval_trow2(csa, rho);
}

static void sort_trow(csa_t *csa, double tol_piv)                             /* :754 */
{
    int nnz = csa->trow_nnz, j, num, pos;
    int *ind = csa->trow_ind; double *vec = csa->trow_vec;
    double big = 0.0, eps, temp;
    for (pos = 1; pos <= nnz; pos++) {
        temp = fabs(vec[ind[pos]]);
        if (big < temp) big = temp;
    }
    csa->trow_max = big;
    eps = tol_piv * (1.0 + 0.01 * big);
    for (num = 0; num < nnz;) {
        j = ind[nnz];
        if (fabs(vec[j]) < eps)
            nnz--;
        else {
            num++;
            ind[nnz] = ind[num];
            ind[num] = j;
        }
    }
    csa->trow_num = num;
}

static void chuzc(csa_t *csa, double rtol)                                     /* :793 */
{
    signed char *stat = csa->stat; double *cbar = csa->cbar;
    int j, pos, q;
    double alfa, big, s, t = 0.0, teta, tmax;
    s = (csa->delta > 0.0 ? +1.0 : -1.0);
    q = 0; teta = DBL_MAX; big = 0.0;
    for (pos = 1; pos <= csa->trow_num; pos++) {
        j = csa->trow_ind[pos];
        alfa = s * csa->trow_vec[j];
        if (alfa > 0.0) {
            if (stat[j] == GLP_NL || stat[j] == GLP_NF)
                t = (cbar[j] + rtol) / alfa;
            else
                continue;
        } else {
            if (stat[j] == GLP_NU || stat[j] == GLP_NF)
                t = (cbar[j] - rtol) / alfa;
            else
                continue;
        }
        if (t < 0.0) t = 0.0;
        if (teta > t || (teta == t && big < fabs(alfa))) { q = j; teta = t; big = fabs(alfa); }
    }
    if (rtol == 0.0) goto done;
    if (q == 0) goto done;
    if (teta == 0.0) goto done;
    tmax = teta;
    q = 0; teta = DBL_MAX; big = 0.0;
    for (pos = 1; pos <= csa->trow_num; pos++) {
        j = csa->trow_ind[pos];
        alfa = s * csa->trow_vec[j];
        if (alfa > 0.0) {
            if (stat[j] == GLP_NL || stat[j] == GLP_NF)
                t = cbar[j] / alfa;
            else
                continue;
        } else {
            if (stat[j] == GLP_NU || stat[j] == GLP_NF)
                t = cbar[j] / alfa;
            else
                continue;
        }
        if (t < 0.0) t = 0.0;
        if (t <= tmax && big < fabs(alfa)) { q = j; teta = t; big = fabs(alfa); }
    }
    ORC_ASSERT(q != 0);
done:
    csa->q = q;
    csa->new_dq = s * teta;
}

static void neg_N_col(csa_t *csa, double *h)            /* h = -N[q], :947-966 */
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

static void eval_tcol(csa_t *csa)                                              /* :937 */
{
    neg_N_col(csa, csa->tcol_vec);
    ORC_ASSERT(csa->valid);
    bfd_ftran(csa->bfd, csa->tcol_vec);
    tcol_pattern(csa);
}

static void refine_tcol(csa_t *csa)                                            /* :979 */
{
    double *h = csa->work3;
    neg_N_col(csa, h);
    refine_ftran(csa, h, csa->tcol_vec);
    tcol_pattern(csa);
}

static void update_cbar(csa_t *csa)                                            /* :1020 */
{
    int q = csa->q, j, pos;
    double new_dq = csa->new_dq;
    csa->cbar[q] = new_dq;
    if (new_dq == 0.0) return;
    for (pos = 1; pos <= csa->trow_nnz; pos++) {
        j = csa->trow_ind[pos];
        if (j != q) csa->cbar[j] -= csa->trow_vec[j] * new_dq;
    }
}

static void update_bbar(csa_t *csa)                                            /* :1042 */
{
    int p = csa->p, i, pos;
    double teta = csa->delta / csa->tcol_vec[p];
    csa->bbar[p] = get_xN(csa, csa->q) + teta;
    if (teta == 0.0) return;
    for (pos = 1; pos <= csa->tcol_nnz; pos++) {
        i = csa->tcol_ind[pos];
        if (i != p) csa->bbar[i] += csa->tcol_vec[i] * teta;
    }
}

static void update_gamma(csa_t *csa)                                           /* :1075 */
{
    int m = csa->m, p = csa->p, q = csa->q, i, j, k, pos, ptr;
    signed char *type = csa->type, *refsp = csa->refsp;
    int *head = csa->head; double *gamma = csa->gamma, *u = csa->work3;
    double gamma_p, eta_p, pivot, t, t1, t2;
    ORC_ASSERT(csa->refct > 0);
    csa->refct--;
    gamma_p = eta_p = (refsp[head[p]] ? 1.0 : 0.0);
    for (i = 1; i <= m; i++) u[i] = 0.0;
    for (pos = 1; pos <= csa->trow_nnz; pos++) {
        j = csa->trow_ind[pos];
        k = head[m + j];
        if (!refsp[k]) continue;
        t = csa->trow_vec[j];
        gamma_p += t * t;
        if (k <= m)
            u[k] += t;
        else
            for (ptr = csa->A_ptr[k - m]; ptr < csa->A_ptr[k - m + 1]; ptr++)
                u[csa->A_ind[ptr]] -= t * csa->A_val[ptr];
    }
    ORC_ASSERT(csa->valid);
    bfd_ftran(csa->bfd, u);
    pivot = csa->tcol_vec[p];
    for (pos = 1; pos <= csa->tcol_nnz; pos++) {
        i = csa->tcol_ind[pos];
        k = head[i];
        if (i == p) continue;
        if (type[head[i]] == GLP_FR) continue;
        t = csa->tcol_vec[i] / pivot;
        t1 = gamma[i] + t * t * gamma_p + 2.0 * t * u[i];
        t2 = (refsp[k] ? 1.0 : 0.0) + eta_p * t * t;
        gamma[i] = (t1 >= t2 ? t1 : t2);
        if (gamma[i] < DBL_EPSILON) gamma[i] = DBL_EPSILON;
    }
    if (type[head[m + q]] == GLP_FR)
        gamma[p] = 1.0;
    else {
        gamma[p] = gamma_p / (pivot * pivot);
        if (gamma[p] < DBL_EPSILON) gamma[p] = DBL_EPSILON;
    }
    k = head[p];
    if (type[k] == GLP_FX && refsp[k]) {
        refsp[k] = 0;
        for (pos = 1; pos <= csa->tcol_nnz; pos++) {
            i = csa->tcol_ind[pos];
            if (i == p) {
                if (type[head[m + q]] == GLP_FR) continue;
                t = 1.0 / csa->tcol_vec[p];
            } else {
                if (type[head[i]] == GLP_FR) continue;
                t = csa->tcol_vec[i] / csa->tcol_vec[p];
            }
            gamma[i] -= t * t;
            if (gamma[i] < DBL_EPSILON) gamma[i] = DBL_EPSILON;
        }
    }
}

static void change_basis(csa_t *csa)                                           /* :1259 */
{
    int m = csa->m, p = csa->p, q = csa->q, k;
    k = csa->head[p]; csa->head[p] = csa->head[m + q]; csa->head[m + q] = k;
    csa->bind[csa->head[p]] = p; csa->bind[csa->head[m + q]] = m + q;
    if (csa->type[k] == GLP_FX)
        csa->stat[q] = GLP_NS;
    else if (csa->delta > 0.0)
        csa->stat[q] = GLP_NL;
    else
        csa->stat[q] = GLP_NU;
}

static int check_feas(csa_t *csa, double tol_dj)                               /* :1296 */
{
    int m = csa->m, n = csa->n, j, k;
    for (j = 1; j <= n; j++) {
        k = csa->head[m + j];
        if (csa->cbar[j] < -tol_dj)
            if (csa->orig_type[k] == GLP_LO || csa->orig_type[k] == GLP_FR) return 1;
        if (csa->cbar[j] > +tol_dj)
            if (csa->orig_type[k] == GLP_UP || csa->orig_type[k] == GLP_FR) return 1;
    }
    return 0;
}

static void set_aux_bnds(csa_t *csa)                                           /* :1317 */
{
    int m = csa->m, n = csa->n, j, k;
    for (k = 1; k <= m + n; k++) {
        switch (csa->orig_type[k]) {
        case GLP_FR: csa->type[k] = GLP_DB; csa->lb[k] = -1e3; csa->ub[k] = +1e3; break;
        case GLP_LO: csa->type[k] = GLP_DB; csa->lb[k] = 0.0; csa->ub[k] = +1.0; break;
        case GLP_UP: csa->type[k] = GLP_DB; csa->lb[k] = -1.0; csa->ub[k] = 0.0; break;
        case GLP_DB:
        case GLP_FX: csa->type[k] = GLP_FX; csa->lb[k] = csa->ub[k] = 0.0; break;
        default: ORC_ASSERT(0);
        }
    }
    for (j = 1; j <= n; j++) {
        k = csa->head[m + j];
        if (csa->type[k] == GLP_FX)
            csa->stat[j] = GLP_NS;
        else if (csa->cbar[j] >= 0.0)
            csa->stat[j] = GLP_NL;
        else
            csa->stat[j] = GLP_NU;
    }
}

static void set_orig_bnds(csa_t *csa)                                          /* :1361 */
{
    int m = csa->m, n = csa->n, j, k;
    memcpy(&csa->type[1], &csa->orig_type[1], (size_t)(m + n));
    memcpy(&csa->lb[1], &csa->orig_lb[1], (size_t)(m + n) * sizeof(double));
    memcpy(&csa->ub[1], &csa->orig_ub[1], (size_t)(m + n) * sizeof(double));
    for (j = 1; j <= n; j++) {
        k = csa->head[m + j];
        switch (csa->type[k]) {
        case GLP_FR: csa->stat[j] = GLP_NF; break;
        case GLP_LO: csa->stat[j] = GLP_NL; break;
        case GLP_UP: csa->stat[j] = GLP_NU; break;
        case GLP_DB:
            if (csa->cbar[j] >= +DBL_EPSILON)
                csa->stat[j] = GLP_NL;
            else if (csa->cbar[j] <= -DBL_EPSILON)
                csa->stat[j] = GLP_NU;
            else if (fabs(csa->lb[k]) <= fabs(csa->ub[k]))
                csa->stat[j] = GLP_NL;
            else
                csa->stat[j] = GLP_NU;
            break;
        case GLP_FX: csa->stat[j] = GLP_NS; break;
        default: ORC_ASSERT(0);
        }
    }
}

static int check_stab(csa_t *csa, double tol_dj)                                /* :1410 */
{
    int n = csa->n, j;
    for (j = 1; j <= n; j++) {
        if (csa->cbar[j] < -tol_dj)
            if (csa->stat[j] == GLP_NL || csa->stat[j] == GLP_NF) return 1;
        if (csa->cbar[j] > +tol_dj)
            if (csa->stat[j] == GLP_NU || csa->stat[j] == GLP_NF) return 1;
    }
    return 0;
}

static double eval_obj(csa_t *csa)                                              /* :1424 */
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

static void store_sol(csa_t *csa, orc_prob *lp, int p_stat, int d_stat, int ray)   /* :1499 */
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

static int fail_return(csa_t *csa, orc_prob *lp)
{
    ORC_ASSERT(!lp->valid && lp->bfd == NULL);
    lp->bfd = csa->bfd; csa->bfd = NULL;
    lp->pbs_stat = lp->dbs_stat = GLP_UNDEF;
    lp->obj_val = 0.0;
    lp->it_cnt = csa->it_cnt;
    lp->some = 0;
    return GLP_EFAIL;
}

int spx_dual(orc_prob *lp, const orc_smcp *parm)                     /* :1, loop :1614 */
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
        if (cbar_st == 0) {
            eval_cbar(csa);
            cbar_st = 1;
            if (csa->phase == 0) {
                if (check_feas(csa, 0.90 * parm->tol_dj) != 0) {
                    csa->phase = 1;
                    set_aux_bnds(csa);
                } else {
                    csa->phase = 2;
                    set_orig_bnds(csa);
                }
                ORC_ASSERT(check_stab(csa, parm->tol_dj) == 0);
                csa->refct = 0;
                bbar_st = 0;
            }
            if (check_stab(csa, parm->tol_dj) != 0) {
                orc_instab_events++; orc_instab_last_it = csa->it_cnt;
                if (parm->meth == GLP_DUALP) {
                    store_sol(csa, lp, GLP_UNDEF, GLP_UNDEF, 0);
                    ret = GLP_EFAIL;
                    break;
                }
                csa->phase = 0;
                binv_st = 0;
                rigorous = 5;
                continue;
            }
        }
        ORC_ASSERT(csa->phase == 1 || csa->phase == 2);
        if (csa->phase == 1 && check_feas(csa, parm->tol_dj) == 0) {
            csa->phase = 2;
            if (cbar_st != 1) {
                eval_cbar(csa);
                cbar_st = 1;
            }
            set_orig_bnds(csa);
            csa->refct = 0;
            bbar_st = 0;
        }
        if (bbar_st == 0) {
            eval_bbar(csa);
            if (csa->phase == 2) csa->bbar[0] = eval_obj(csa);
            bbar_st = 1;
        }
        if (parm->pricing == GLP_PT_PSE) {
            if (csa->refct == 0) reset_refsp(csa);
        } else
            ORC_ASSERT(parm->pricing == GLP_PT_STD);
        ORC_ASSERT(binv_st && bbar_st && cbar_st);
        if (csa->phase == 2 && csa->zeta < 0.0 && parm->obj_ll > -DBL_MAX && csa->bbar[0] <= parm->obj_ll) {
            if (bbar_st != 1 || cbar_st != 1) {
                if (bbar_st != 1) bbar_st = 0;
                if (cbar_st != 1) cbar_st = 0;
                continue;
            }
            store_sol(csa, lp, GLP_INFEAS, GLP_FEAS, 0);
            ret = GLP_EOBJLL;
            break;
        }
        if (csa->phase == 2 && csa->zeta > 0.0 && parm->obj_ul < +DBL_MAX && csa->bbar[0] >= parm->obj_ul) {
            if (bbar_st != 1 || cbar_st != 1) {
                if (bbar_st != 1) bbar_st = 0;
                if (cbar_st != 1) cbar_st = 0;
                continue;
            }
            store_sol(csa, lp, GLP_INFEAS, GLP_FEAS, 0);
            ret = GLP_EOBJUL;
            break;
        }
        {
            int it_hit = (parm->it_lim < ORC_INT_MAX && csa->it_cnt - csa->it_beg >= parm->it_lim);
            int tm_hit = !it_hit && parm->tm_lim < ORC_INT_MAX &&
                         1000.0 * (orc_time() - csa->tm_beg) >= parm->tm_lim;
            if (it_hit || tm_hit) {
                if ((csa->phase == 2 && bbar_st != 1) || cbar_st != 1) {
                    if (csa->phase == 2 && bbar_st != 1) bbar_st = 0;
                    if (cbar_st != 1) cbar_st = 0;
                    continue;
                }
                if (csa->phase == 1) {
                    d_stat = GLP_INFEAS;
                    set_orig_bnds(csa);
                    eval_bbar(csa);
                } else
                    d_stat = GLP_FEAS;
                store_sol(csa, lp, GLP_INFEAS, d_stat, 0);
                ret = it_hit ? GLP_EITLIM : GLP_ETMLIM;
                break;
            }
        }
        chuzr(csa, parm->tol_bnd);
        if (csa->p == 0) {
            if (bbar_st != 1 || cbar_st != 1) {
                if (bbar_st != 1) bbar_st = 0;
                if (cbar_st != 1) cbar_st = 0;
                continue;
            }
            if (csa->phase == 1) {
                set_orig_bnds(csa);
                eval_bbar(csa);
                p_stat = GLP_INFEAS; d_stat = GLP_NOFEAS;
            } else
                p_stat = d_stat = GLP_FEAS;
            store_sol(csa, lp, p_stat, d_stat, 0);
            ret = 0;
            break;
        }
        {
            double *rho = csa->work4;
            eval_rho(csa, rho);
            if (rigorous) refine_rho(csa, rho);
            eval_trow(csa, rho);
            sort_trow(csa, parm->tol_bnd);
        }
        if (parm->r_test == GLP_RT_STD)
            chuzc(csa, 0.0);
        else {
            ORC_ASSERT(parm->r_test == GLP_RT_HAR);
            chuzc(csa, 0.30 * parm->tol_dj);
        }
        if (csa->q == 0) {
            if (bbar_st != 1 || cbar_st != 1 || !rigorous) {
                if (bbar_st != 1) bbar_st = 0;
                if (cbar_st != 1) cbar_st = 0;
                rigorous = 1;
                continue;
            }
            if (csa->phase == 1)
                ret = fail_return(csa, lp);
            else {
                store_sol(csa, lp, GLP_NOFEAS, GLP_FEAS, csa->head[csa->p]);
                ret = 0;
            }
            break;
        }
        {
            double piv = csa->trow_vec[csa->q];
            double eps = 1e-5 * (1.0 + 0.01 * csa->trow_max);
            if (fabs(piv) < eps) {
                if (!rigorous) { rigorous = 5; continue; }
            }
        }
        eval_tcol(csa);
        if (rigorous) refine_tcol(csa);
        {
            double piv1 = csa->tcol_vec[csa->p], piv2 = csa->trow_vec[csa->q];
            ORC_ASSERT(piv1 != 0.0);
            if (fabs(piv1 - piv2) > 1e-8 * (1.0 + fabs(piv1)) || !((piv1 > 0.0 && piv2 > 0.0) || (piv1 < 0.0 && piv2 < 0.0))) {
                if (binv_st != 1 || !rigorous) {
                    if (binv_st != 1) binv_st = 0;
                    rigorous = 5;
                    continue;
                }
                if (csa->tcol_vec[csa->p] == 0.0) {
                    csa->tcol_nnz++;
                    ORC_ASSERT(csa->tcol_nnz <= csa->m);
                    csa->tcol_ind[csa->tcol_nnz] = csa->p;
                }
                csa->tcol_vec[csa->p] = piv2;
            }
        }
        update_bbar(csa);
        if (csa->phase == 2)
            csa->bbar[0] += (csa->cbar[csa->q] / csa->zeta) * (csa->delta / csa->tcol_vec[csa->p]);
        bbar_st = 2;
        update_cbar(csa);
        cbar_st = 2;
        if (parm->pricing == GLP_PT_PSE) {
            if (csa->refct > 0) update_gamma(csa);
        }
        ret = update_B(csa, csa->p, csa->head[csa->m + csa->q]);
        if (ret == 0)
            binv_st = 2;
        else {
            csa->valid = 0;
            binv_st = 0;
        }
        if (orc_trace)
            orc_trace(orc_trace_ctx, 2, csa->it_cnt, csa->phase, csa->p, csa->q, csa->head[csa->m + csa->q],
                      csa->head[csa->p], csa->delta);
        change_basis(csa);
        csa->it_cnt++;
        if (rigorous > 0) rigorous--;
    }
    if (csa->bfd) { bfd_delete_it(csa->bfd); csa->bfd = NULL; }
    free_csa(csa);
    return ret;
}
