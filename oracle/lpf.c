/* ORACLE (test infrastructure only) — LP basis factorization with a dense
 * Schur complement (Bartels–Golub / Givens updates).  Restates glpscf.js
 * (scf_create_it :14, bg_transform :52, givens :104, gr_transform :118,
 * estimate_rank :177, scf_update_exp :217, solve :282, tsolve :309,
 * scf_solve_it :337, scf_reset_it :346) and glplpf.js (lpf_create_it :10,
 * lpf_factorize :36, r_prod :126, rt_prod :145, s_prod :165, st_prod :185,
 * lpf_ftran :235, lpf_btran :275, enlarge_sva :316, lpf_update_it :331).
 *
 * Reproduced as the JS behaves, including lpf_update_it's idx = 0 calls of
 * s_prod/rt_prod (glplpf.js:420/:422), which accumulate the new Schur row and
 * column into the f/v part of the work arrays instead of the g/w part.
 * orc_lpf_fixed != 0 (orc_set_lpf_fix) applies the offsets of the C original
 * instead (idx = m0: the g = fg + m0 and w = vw + m0 parts that
 * scf_update_exp reads), the variant tests/golden/gen_golden.js --lpf-fix runs
 * through the reference. */
#include <math.h>
#include <string.h>
#include "orc.h"

#define SCF_EPS 1e-10

int orc_lpf_fixed = 0;
void orc_set_lpf_fix(int on) { orc_lpf_fixed = on != 0; }

orc_scf *scf_create_it(int n_max)
{
    orc_scf *scf;
    if (!(1 <= n_max && n_max <= 32767)) orc_fail("scf_create_it: n_max = %d; invalid parameter", n_max);
    scf = (orc_scf *)orc_alloc(1, sizeof(orc_scf));
    scf->n_max = n_max;
    scf->f = (double *)orc_alloc((size_t)(1 + n_max * n_max), sizeof(double));
    scf->u = (double *)orc_alloc((size_t)(1 + n_max * (n_max + 1) / 2), sizeof(double));
    scf->p = (int *)orc_alloc((size_t)(1 + n_max), sizeof(int));
    scf->t_opt = SCF_TBG;
    scf->w = (double *)orc_alloc((size_t)(1 + n_max), sizeof(double));
    return scf;
}

void scf_delete_it(orc_scf *scf)
{
    if (!scf) return;
    orc_free(scf->f); orc_free(scf->u); orc_free(scf->p); orc_free(scf->w); orc_free(scf);
}

static int f_loc(orc_scf *scf, int i, int j)
{
    ORC_ASSERT(1 <= i && i <= scf->n);
    ORC_ASSERT(1 <= j && j <= scf->n);
    return (i - 1) * scf->n_max + j;
}

static int u_loc(orc_scf *scf, int i, int j)
{
    ORC_ASSERT(1 <= i && i <= scf->n);
    ORC_ASSERT(i <= j && j <= scf->n);
    return (i - 1) * scf->n_max + j - i * (i - 1) / 2;
}

static void bg_transform(orc_scf *scf, int k, double *un)
{
    int n = scf->n, j, k1, kj, kk, n1, nj;
    double *f = scf->f, *u = scf->u, t;
    ORC_ASSERT(1 <= k && k <= n);
    for (; k < n; k++) {
        kk = u_loc(scf, k, k);
        k1 = f_loc(scf, k, 1);
        n1 = f_loc(scf, n, 1);
        if (fabs(u[kk]) < fabs(un[k])) {
            for (j = k, kj = kk; j <= n; j++, kj++) { t = u[kj]; u[kj] = un[j]; un[j] = t; }
            for (j = 1, kj = k1, nj = n1; j <= n; j++, kj++, nj++) { t = f[kj]; f[kj] = f[nj]; f[nj] = t; }
        }
        if (fabs(u[kk]) < SCF_EPS) u[kk] = un[k] = 0.0;
        if (un[k] == 0.0) continue;
        t = un[k] / u[kk];
        for (j = k + 1, kj = kk + 1; j <= n; j++, kj++) un[j] -= t * u[kj];
        for (j = 1, kj = k1, nj = n1; j <= n; j++, kj++, nj++) f[nj] -= t * f[kj];
    }
    if (fabs(un[n]) < SCF_EPS) un[n] = 0.0;
    u[u_loc(scf, n, n)] = un[n];
}

static void givens(double a, double b, double *c, double *s)
{
    double t;
    if (b == 0.0) { *c = 1.0; *s = 0.0; }
    else if (fabs(a) <= fabs(b)) { t = -a / b; *s = 1.0 / sqrt(1.0 + t * t); *c = *s * t; }
    else { t = -b / a; *c = 1.0 / sqrt(1.0 + t * t); *s = *c * t; }
}

static void gr_transform(orc_scf *scf, int k, double *un)
{
    int n = scf->n, j, k1, kj, kk, n1, nj;
    double *f = scf->f, *u = scf->u, c, s;
    ORC_ASSERT(1 <= k && k <= n);
    for (; k < n; k++) {
        kk = u_loc(scf, k, k);
        k1 = f_loc(scf, k, 1);
        n1 = f_loc(scf, n, 1);
        if (fabs(u[kk]) < SCF_EPS && fabs(un[k]) < SCF_EPS) u[kk] = un[k] = 0.0;
        if (un[k] == 0.0) continue;
        givens(u[kk], un[k], &c, &s);
        for (j = k, kj = kk; j <= n; j++, kj++) {
            double ukj = u[kj], unj = un[j];
            u[kj] = c * ukj - s * unj;
            un[j] = s * ukj + c * unj;
        }
        for (j = 1, kj = k1, nj = n1; j <= n; j++, kj++, nj++) {
            double fkj = f[kj], fnj = f[nj];
            f[kj] = c * fkj - s * fnj;
            f[nj] = s * fkj + c * fnj;
        }
    }
    if (fabs(un[n]) < SCF_EPS) un[n] = 0.0;
    u[u_loc(scf, n, n)] = un[n];
}

static int estimate_rank(orc_scf *scf)
{
    int n_max = scf->n_max, n = scf->n, i, ii, inc, rank = 0;
    for (i = 1, ii = u_loc(scf, i, i), inc = n_max; i <= n; i++, ii += inc, inc--)
        if (scf->u[ii] != 0.0) rank++;
    return rank;
}

int scf_update_exp(orc_scf *scf, const double *x, int idx, const double *y, int idy, double z)
{
    int n_max = scf->n_max, n = scf->n, i, ij, in_, j, k, nj, ret = 0;
    double *f = scf->f, *u = scf->u, *un = scf->w, t;
    int *p = scf->p;
    if (n == n_max) return SCF_ELIMIT;
    scf->n = ++n;
    for (i = 1, in_ = f_loc(scf, i, n); i < n; i++, in_ += n_max) f[in_] = 0.0;
    for (j = 1, nj = f_loc(scf, n, j); j < n; j++, nj++) f[nj] = 0.0;
    f[f_loc(scf, n, n)] = 1.0;
    for (i = 1; i < n; i++) {
        t = 0.0;
        for (j = 1, ij = f_loc(scf, i, 1); j < n; j++, ij++) t += f[ij] * x[j + idx];
        u[u_loc(scf, i, n)] = t;
    }
    for (j = 1; j < n; j++) un[j] = y[p[j] + idy];
    un[n] = z;
    p[n] = n;
    for (k = 1; k < n; k++)
        if (un[k] != 0.0) break;
    if (scf->t_opt == SCF_TBG) bg_transform(scf, k, un);
    else if (scf->t_opt == SCF_TGR) gr_transform(scf, k, un);
    else ORC_ASSERT(0);
    scf->rank = estimate_rank(scf);
    if (scf->rank != n) ret = SCF_ESING;
    return ret;
}

static void scf_solve(orc_scf *scf, double *x, int idx)
{
    int n = scf->n, i, j, ij;
    double *f = scf->f, *u = scf->u, *y = scf->w, t;
    int *p = scf->p;
    for (i = 1; i <= n; i++) {
        t = 0.0;
        for (j = 1, ij = f_loc(scf, i, 1); j <= n; j++, ij++) t += f[ij] * x[j + idx];
        y[i] = t;
    }
    for (i = n; i >= 1; i--) {
        t = y[i];
        for (j = n, ij = u_loc(scf, i, n); j > i; j--, ij--) t -= u[ij] * y[j];
        y[i] = t / u[ij];
    }
    for (i = 1; i <= n; i++) x[p[i] + idx] = y[i];
}

static void scf_tsolve(orc_scf *scf, double *x, int idx)
{
    int n = scf->n, i, j, ij;
    double *f = scf->f, *u = scf->u, *y = scf->w, t;
    int *p = scf->p;
    for (i = 1; i <= n; i++) y[i] = x[p[i] + idx];
    for (i = 1; i <= n; i++) {
        ij = u_loc(scf, i, i);
        t = (y[i] /= u[ij]);
        for (j = i + 1, ij++; j <= n; j++, ij++) y[j] -= u[ij] * t;
    }
    for (j = 1; j <= n; j++) x[j + idx] = 0.0;
    for (i = 1; i <= n; i++) {
        t = y[i];
        for (j = 1, ij = f_loc(scf, i, 1); j <= n; j++, ij++) x[j + idx] += f[ij] * t;
    }
}

void scf_solve_it(orc_scf *scf, int tr, double *x)
{
    (void)tr; (void)x;
    ORC_ASSERT(0);   /* use the idx form below */
}

static void scf_solve_idx(orc_scf *scf, int tr, double *x, int idx)
{
    if (scf->rank < scf->n) orc_fail("scf_solve_it: singular matrix");
    if (!tr) scf_solve(scf, x, idx); else scf_tsolve(scf, x, idx);
}

/* ---------------------------------------------------------------- lpf --- */
orc_lpf *lpf_create_it(void)
{
    orc_lpf *lpf = (orc_lpf *)orc_alloc(1, sizeof(orc_lpf));
    lpf->luf = luf_create_it();
    lpf->n_max = 50;
    lpf->v_size = 1000;
    return lpf;
}

void lpf_delete_it(orc_lpf *lpf)
{
    if (!lpf) return;
    luf_delete_it(lpf->luf);
    orc_free(lpf->R_ptr); orc_free(lpf->R_len); orc_free(lpf->S_ptr); orc_free(lpf->S_len);
    scf_delete_it(lpf->scf);
    orc_free(lpf->P_row); orc_free(lpf->P_col); orc_free(lpf->Q_row); orc_free(lpf->Q_col);
    orc_free(lpf->v_ind); orc_free(lpf->v_val); orc_free(lpf->work1); orc_free(lpf->work2);
    orc_free(lpf);
}

int lpf_factorize(orc_lpf *lpf, int m, const int *bh, orc_col_fn col, void *info)
{
    int k, ret, N;
    (void)bh;
    if (m < 1) orc_fail("lpf_factorize: m = %d; invalid parameter", m);
    lpf->m0 = lpf->m = m;
    lpf->valid = 0;
    if (lpf->R_ptr == NULL) lpf->R_ptr = (int *)orc_alloc((size_t)(1 + lpf->n_max), sizeof(int));
    if (lpf->R_len == NULL) lpf->R_len = (int *)orc_alloc((size_t)(1 + lpf->n_max), sizeof(int));
    if (lpf->S_ptr == NULL) lpf->S_ptr = (int *)orc_alloc((size_t)(1 + lpf->n_max), sizeof(int));
    if (lpf->S_len == NULL) lpf->S_len = (int *)orc_alloc((size_t)(1 + lpf->n_max), sizeof(int));
    if (lpf->scf == NULL) lpf->scf = scf_create_it(lpf->n_max);
    if (lpf->v_ind == NULL) lpf->v_ind = (int *)orc_alloc((size_t)(1 + lpf->v_size), sizeof(int));
    if (lpf->v_val == NULL) lpf->v_val = (double *)orc_alloc((size_t)(1 + lpf->v_size), sizeof(double));
    if (lpf->m0_max < m) {
        orc_free(lpf->P_row); orc_free(lpf->P_col); orc_free(lpf->Q_row); orc_free(lpf->Q_col);
        orc_free(lpf->work1); orc_free(lpf->work2);
        lpf->m0_max = m + 100;
        N = 1 + lpf->m0_max + lpf->n_max;
        lpf->P_row = (int *)orc_alloc((size_t)N, sizeof(int));
        lpf->P_col = (int *)orc_alloc((size_t)N, sizeof(int));
        lpf->Q_row = (int *)orc_alloc((size_t)N, sizeof(int));
        lpf->Q_col = (int *)orc_alloc((size_t)N, sizeof(int));
        lpf->work1 = (double *)orc_alloc((size_t)N, sizeof(double));
        lpf->work2 = (double *)orc_alloc((size_t)N, sizeof(double));
    }
    ret = luf_factorize(lpf->luf, m, col, info);
    if (ret == 1) return LPF_ESING;
    if (ret == 2) return LPF_ECOND;
    ORC_ASSERT(ret == 0);
    lpf->valid = 1;
    lpf->n = 0;
    lpf->scf->n = lpf->scf->rank = 0;
    for (k = 1; k <= m; k++) {
        lpf->P_row[k] = lpf->P_col[k] = k;
        lpf->Q_row[k] = lpf->Q_col[k] = k;
    }
    lpf->v_ptr = 1;
    return 0;
}

static void r_prod(orc_lpf *lpf, double *y, double a, const double *x, int idx)
{
    int j, beg, end, ptr;
    double t;
    for (j = 1; j <= lpf->n; j++) {
        if (x[j + idx] == 0.0) continue;
        t = a * x[j + idx];
        beg = lpf->R_ptr[j];
        end = beg + lpf->R_len[j];
        for (ptr = beg; ptr < end; ptr++) y[lpf->v_ind[ptr]] += t * lpf->v_val[ptr];
    }
}

static void rt_prod(orc_lpf *lpf, double *y, int idx, double a, const double *x)
{
    int j, beg, end, ptr;
    double t;
    for (j = 1; j <= lpf->n; j++) {
        t = 0.0;
        beg = lpf->R_ptr[j];
        end = beg + lpf->R_len[j];
        for (ptr = beg; ptr < end; ptr++) t += lpf->v_val[ptr] * x[lpf->v_ind[ptr]];
        y[j + idx] += a * t;
    }
}

static void s_prod(orc_lpf *lpf, double *y, int idx, double a, const double *x)
{
    int i, beg, end, ptr;
    double t;
    for (i = 1; i <= lpf->n; i++) {
        t = 0.0;
        beg = lpf->S_ptr[i];
        end = beg + lpf->S_len[i];
        for (ptr = beg; ptr < end; ptr++) t += lpf->v_val[ptr] * x[lpf->v_ind[ptr]];
        y[i + idx] += a * t;
    }
}

static void st_prod(orc_lpf *lpf, double *y, double a, const double *x, int idx)
{
    int i, beg, end, ptr;
    double t;
    for (i = 1; i <= lpf->n; i++) {
        if (x[i + idx] == 0.0) continue;
        t = a * x[i + idx];
        beg = lpf->S_ptr[i];
        end = beg + lpf->S_len[i];
        for (ptr = beg; ptr < end; ptr++) y[lpf->v_ind[ptr]] += t * lpf->v_val[ptr];
    }
}

void lpf_ftran(orc_lpf *lpf, double *x)
{
    int m0 = lpf->m0, m = lpf->m, n = lpf->n, i, ii;
    double *fg = lpf->work1;
    if (!lpf->valid) orc_fail("lpf_ftran: the factorization is not valid");
    ORC_ASSERT(0 <= m && m <= m0 + n);
    for (i = 1; i <= m0 + n; i++) fg[i] = ((ii = lpf->P_col[i]) <= m ? x[ii] : 0.0);
    luf_f_solve(lpf->luf, 0, fg);
    s_prod(lpf, fg, m0, -1.0, fg);
    scf_solve_idx(lpf->scf, 0, fg, m0);
    r_prod(lpf, fg, -1.0, fg, m0);
    luf_v_solve(lpf->luf, 0, fg);
    for (i = 1; i <= m; i++) x[i] = fg[lpf->Q_col[i]];
}

void lpf_btran(orc_lpf *lpf, double *x)
{
    int m0 = lpf->m0, m = lpf->m, n = lpf->n, i, ii;
    double *fg = lpf->work1;
    if (!lpf->valid) orc_fail("lpf_btran: the factorization is not valid");
    ORC_ASSERT(0 <= m && m <= m0 + n);
    for (i = 1; i <= m0 + n; i++) fg[i] = ((ii = lpf->Q_row[i]) <= m ? x[ii] : 0.0);
    luf_v_solve(lpf->luf, 1, fg);
    rt_prod(lpf, fg, m0, -1.0, fg);
    scf_solve_idx(lpf->scf, 1, fg, m0);
    st_prod(lpf, fg, -1.0, fg, m0);
    luf_f_solve(lpf->luf, 1, fg);
    for (i = 1; i <= m; i++) x[i] = fg[lpf->P_row[i]];
}

static void enlarge_sva(orc_lpf *lpf, int new_size)
{
    int v_size = lpf->v_size, used = lpf->v_ptr - 1;
    int *v_ind = lpf->v_ind; double *v_val = lpf->v_val;
    ORC_ASSERT(v_size < new_size);
    /* the reference loops forever here when v_size == 0 (glplpf.js:322) */
    if (v_size <= 0) orc_fail("lpf: enlarge_sva with v_size = 0 does not terminate in the reference");
    while (v_size < new_size) v_size += v_size;
    lpf->v_size = v_size;
    lpf->v_ind = (int *)orc_alloc((size_t)(1 + v_size), sizeof(int));
    lpf->v_val = (double *)orc_alloc((size_t)(1 + v_size), sizeof(double));
    ORC_ASSERT(used >= 0);
    memcpy(&lpf->v_ind[1], &v_ind[1], (size_t)used * sizeof(int));
    memcpy(&lpf->v_val[1], &v_val[1], (size_t)used * sizeof(double));
    orc_free(v_ind); orc_free(v_val);
}

int lpf_update_it(orc_lpf *lpf, int j, int bh, int len, const int *ind, int idx, const double *val)
{
    int m0 = lpf->m0, m = lpf->m, n = lpf->n, i, ii, k, v_ptr;
    double *a = lpf->work2, *fg = lpf->work1, *vw = lpf->work2, z;
    (void)bh;
    if (!lpf->valid) orc_fail("lpf_update_it: the factorization is not valid");
    if (!(1 <= j && j <= m)) orc_fail("lpf_update_it: j = %d; column number out of range", j);
    ORC_ASSERT(0 <= m && m <= m0 + n);
    if (n == lpf->n_max) { lpf->valid = 0; return LPF_ELIMIT; }
    for (i = 1; i <= m; i++) a[i] = 0.0;
    for (k = 1; k <= len; k++) {
        i = ind[idx + k];
        if (!(1 <= i && i <= m)) orc_fail("lpf_update_it: ind[%d] = %d; row number out of range", k, i);
        if (a[i] != 0.0) orc_fail("lpf_update_it: ind[%d] = %d; duplicate row index not allowed", k, i);
        if (val[k] == 0.0) orc_fail("lpf_update_it: val[%d]; zero element not allowed", k);
        a[i] = val[k];
    }
    for (i = 1; i <= m0 + n; i++) fg[i] = ((ii = lpf->P_col[i]) <= m ? a[ii] : 0.0);
    for (i = 1; i <= m0 + n; i++) vw[i] = 0.0;
    vw[lpf->Q_col[j]] = 1.0;
    luf_f_solve(lpf->luf, 0, fg);
    luf_v_solve(lpf->luf, 1, vw);
    v_ptr = lpf->v_ptr;
    if (lpf->v_size < v_ptr + m0 + m0) enlarge_sva(lpf, v_ptr + m0 + m0);
    lpf->R_ptr[n + 1] = v_ptr;
    for (i = 1; i <= m0; i++)
        if (fg[i] != 0.0) { lpf->v_ind[v_ptr] = i; lpf->v_val[v_ptr] = fg[i]; v_ptr++; }
    lpf->R_len[n + 1] = v_ptr - lpf->v_ptr;
    lpf->v_ptr = v_ptr;
    lpf->S_ptr[n + 1] = v_ptr;
    for (i = 1; i <= m0; i++)
        if (vw[i] != 0.0) { lpf->v_ind[v_ptr] = i; lpf->v_val[v_ptr] = vw[i]; v_ptr++; }
    lpf->S_len[n + 1] = v_ptr - lpf->v_ptr;
    lpf->v_ptr = v_ptr;
    s_prod(lpf, fg, orc_lpf_fixed ? m0 : 0, -1.0, fg);     /* glplpf.js:420, idx 0 as in the JS */
    rt_prod(lpf, vw, orc_lpf_fixed ? m0 : 0, -1.0, vw);    /* glplpf.js:422 */
    z = 0.0;
    for (i = 1; i <= m0; i++) z -= vw[i] * fg[i];
    switch (scf_update_exp(lpf->scf, fg, m0, vw, m0, z)) {
    case 0: break;
    case SCF_ESING: lpf->valid = 0; return LPF_ESING;
    default: ORC_ASSERT(0);
    }
    lpf->P_row[m0 + n + 1] = lpf->P_col[m0 + n + 1] = m0 + n + 1;
    lpf->Q_row[m0 + n + 1] = lpf->Q_col[m0 + n + 1] = m0 + n + 1;
    i = lpf->Q_col[j]; ii = lpf->Q_col[m0 + n + 1];
    lpf->Q_row[i] = m0 + n + 1; lpf->Q_col[m0 + n + 1] = i;
    lpf->Q_row[ii] = j; lpf->Q_col[j] = ii;
    lpf->n++;
    ORC_ASSERT(lpf->n <= lpf->n_max);
    return 0;
}
