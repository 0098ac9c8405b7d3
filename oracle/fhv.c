/* ORACLE (test infrastructure only) — B = F*H*V basis factorization with
 * Forrest–Tomlin row-eta updates.  Restates glpfhv.js (GLPK 4.49):
 * fhv_create_it :9, fhv_factorize :26, fhv_h_solve :77, fhv_ftran :114,
 * fhv_btran :131, fhv_update_it :148. */
#include <math.h>
#include <string.h>
#include "orc.h"

orc_fhv *fhv_create_it(void)
{
    orc_fhv *fhv = (orc_fhv *)orc_alloc(1, sizeof(orc_fhv));
    fhv->luf = luf_create_it();
    fhv->hh_max = 50;
    fhv->upd_tol = 1e-6;
    return fhv;
}

void fhv_delete_it(orc_fhv *fhv)
{
    if (!fhv) return;
    luf_delete_it(fhv->luf);
    orc_free(fhv->hh_ind); orc_free(fhv->hh_ptr); orc_free(fhv->hh_len);
    orc_free(fhv->p0_row); orc_free(fhv->p0_col); orc_free(fhv->cc_ind); orc_free(fhv->cc_val);
    orc_free(fhv);
}

int fhv_factorize(orc_fhv *fhv, int m, orc_col_fn col, void *info)   /* glpfhv.js:26 */
{
    int ret;
    if (m < 1) orc_fail("fhv_factorize: m = %d; invalid parameter", m);
    fhv->m = m;
    fhv->valid = 0;
    if (fhv->hh_ind == NULL) fhv->hh_ind = (int *)orc_alloc((size_t)(1 + fhv->hh_max), sizeof(int));
    if (fhv->hh_ptr == NULL) fhv->hh_ptr = (int *)orc_alloc((size_t)(1 + fhv->hh_max), sizeof(int));
    if (fhv->hh_len == NULL) fhv->hh_len = (int *)orc_alloc((size_t)(1 + fhv->hh_max), sizeof(int));
    if (fhv->m_max < m) {
        orc_free(fhv->p0_row); orc_free(fhv->p0_col); orc_free(fhv->cc_ind); orc_free(fhv->cc_val);
        fhv->m_max = m + 100;
        fhv->p0_row = (int *)orc_alloc((size_t)(1 + fhv->m_max), sizeof(int));
        fhv->p0_col = (int *)orc_alloc((size_t)(1 + fhv->m_max), sizeof(int));
        fhv->cc_ind = (int *)orc_alloc((size_t)(1 + fhv->m_max), sizeof(int));
        fhv->cc_val = (double *)orc_alloc((size_t)(1 + fhv->m_max), sizeof(double));
    }
    ret = luf_factorize(fhv->luf, m, col, info);
    if (ret == 1) return 1;                      /* FHV_ESING */
    if (ret == 2) return 2;                      /* FHV_ECOND */
    ORC_ASSERT(ret == 0);
    fhv->valid = 1;
    fhv->hh_nfs = 0;
    memcpy(&fhv->p0_row[1], &fhv->luf->pp_row[1], (size_t)m * sizeof(int));
    memcpy(&fhv->p0_col[1], &fhv->luf->pp_col[1], (size_t)m * sizeof(int));
    fhv->nnz_h = 0;
    return 0;
}

void fhv_h_solve(orc_fhv *fhv, int tr, double *x)            /* glpfhv.js:77 */
{
    int nfs = fhv->hh_nfs, i, k, beg, end, ptr;
    int *sv_ind = fhv->luf->sv_ind; double *sv_val = fhv->luf->sv_val;
    double temp;
    if (!fhv->valid) orc_fail("fhv_h_solve: the factorization is not valid");
    if (!tr) {
        for (k = 1; k <= nfs; k++) {
            i = fhv->hh_ind[k];
            temp = x[i];
            beg = fhv->hh_ptr[k];
            end = beg + fhv->hh_len[k] - 1;
            for (ptr = beg; ptr <= end; ptr++) temp -= sv_val[ptr] * x[sv_ind[ptr]];
            x[i] = temp;
        }
    } else {
        for (k = nfs; k >= 1; k--) {
            i = fhv->hh_ind[k];
            temp = x[i];
            if (temp == 0.0) continue;
            beg = fhv->hh_ptr[k];
            end = beg + fhv->hh_len[k] - 1;
            for (ptr = beg; ptr <= end; ptr++) x[sv_ind[ptr]] -= sv_val[ptr] * temp;
        }
    }
}

/* F is applied with the row permutation P0 saved at factorization time */
static void f_solve_p0(orc_fhv *fhv, int tr, double *x)
{
    int *pp_row = fhv->luf->pp_row, *pp_col = fhv->luf->pp_col;
    fhv->luf->pp_row = fhv->p0_row;
    fhv->luf->pp_col = fhv->p0_col;
    luf_f_solve(fhv->luf, tr, x);
    fhv->luf->pp_row = pp_row;
    fhv->luf->pp_col = pp_col;
}

void fhv_ftran(orc_fhv *fhv, double *x)                      /* glpfhv.js:114 */
{
    if (!fhv->valid) orc_fail("fhv_ftran: the factorization is not valid");
    f_solve_p0(fhv, 0, x);
    fhv_h_solve(fhv, 0, x);
    luf_v_solve(fhv->luf, 0, x);
}

void fhv_btran(orc_fhv *fhv, double *x)                      /* glpfhv.js:131 */
{
    if (!fhv->valid) orc_fail("fhv_btran: the factorization is not valid");
    luf_v_solve(fhv->luf, 1, x);
    fhv_h_solve(fhv, 1, x);
    f_solve_p0(fhv, 1, x);
}

/* glpfhv.js:148 — replace column j of B by (ind[idx+1..idx+len], val[1..len]) */
int fhv_update_it(orc_fhv *fhv, int j, int len, const int *ind, int idx, const double *val)
{
    int m = fhv->m;
    orc_luf *luf = fhv->luf;
    int *vr_ptr = luf->vr_ptr, *vr_len = luf->vr_len, *vr_cap = luf->vr_cap;
    double *vr_piv = luf->vr_piv;
    int *vc_ptr = luf->vc_ptr, *vc_len = luf->vc_len, *vc_cap = luf->vc_cap;
    int *pp_row = luf->pp_row, *pp_col = luf->pp_col, *qq_row = luf->qq_row, *qq_col = luf->qq_col;
    double *work = luf->work, eps_tol = luf->eps_tol;
    int *hh_ind = fhv->hh_ind, *hh_ptr = fhv->hh_ptr, *hh_len = fhv->hh_len;
    int *cc_ind = fhv->cc_ind; double *cc_val = fhv->cc_val;
    double upd_tol = fhv->upd_tol;
    int i, i_beg, i_end, i_ptr, j_beg, j_end, j_ptr, k, k1, k2, p, q, p_beg, p_end, p_ptr, ptr;
    double f, temp;
    int *sv_ind; double *sv_val;
    if (!fhv->valid) orc_fail("fhv_update_it: the factorization is not valid");
    if (!(1 <= j && j <= m)) orc_fail("fhv_update_it: j = %d; column number out of range", j);
    if (fhv->hh_nfs == fhv->hh_max) { fhv->valid = 0; return 4; }      /* FHV_ELIMIT */
    for (i = 1; i <= m; i++) cc_val[i] = 0.0;
    for (k = 1; k <= len; k++) {
        i = ind[idx + k];
        if (!(1 <= i && i <= m)) orc_fail("fhv_update_it: ind[%d] = %d; row number out of range", k, i);
        if (cc_val[i] != 0.0) orc_fail("fhv_update_it: ind[%d] = %d; duplicate row index not allowed", k, i);
        if (val[k] == 0.0) orc_fail("fhv_update_it: val[%d] = %g; zero element not allowed", k, val[k]);
        cc_val[i] = val[k];
    }
    f_solve_p0(fhv, 0, cc_val);
    fhv_h_solve(fhv, 0, cc_val);
    len = 0;
    for (i = 1; i <= m; i++) {
        temp = cc_val[i];
        if (temp == 0.0 || fabs(temp) < eps_tol) continue;
        len++; cc_ind[len] = i; cc_val[len] = temp;
    }
    sv_ind = luf->sv_ind; sv_val = luf->sv_val;
    j_beg = vc_ptr[j];
    j_end = j_beg + vc_len[j] - 1;
    for (j_ptr = j_beg; j_ptr <= j_end; j_ptr++) {
        i = sv_ind[j_ptr];
        i_beg = vr_ptr[i];
        i_end = i_beg + vr_len[i] - 1;
        for (i_ptr = i_beg; sv_ind[i_ptr] != j; i_ptr++) {}
        ORC_ASSERT(i_ptr <= i_end);
        sv_ind[i_ptr] = sv_ind[i_end];
        sv_val[i_ptr] = sv_val[i_end];
        vr_len[i]--;
    }
    luf->nnz_v -= vc_len[j];
    vc_len[j] = 0;
    k1 = qq_row[j]; k2 = 0;
    for (ptr = 1; ptr <= len; ptr++) {
        i = cc_ind[ptr];
        if (vr_len[i] + 1 > vr_cap[i]) {
            if (luf_enlarge_row(luf, i, vr_len[i] + 10)) {
                fhv->valid = 0;
                luf->new_sva = luf->sv_size + luf->sv_size;
                ORC_ASSERT(luf->new_sva > luf->sv_size);
                return 5;                                                  /* FHV_EROOM */
            }
        }
        i_ptr = vr_ptr[i] + vr_len[i];
        sv_ind[i_ptr] = j;
        sv_val[i_ptr] = cc_val[ptr];
        vr_len[i]++;
        if (k2 < pp_col[i]) k2 = pp_col[i];
    }
    if (vc_cap[j] < len) {
        if (luf_enlarge_col(luf, j, len)) {
            fhv->valid = 0;
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            return 5;
        }
    }
    j_ptr = vc_ptr[j];
    memmove(&sv_ind[j_ptr], &cc_ind[1], (size_t)len * sizeof(int));
    memmove(&sv_val[j_ptr], &cc_val[1], (size_t)len * sizeof(double));
    vc_len[j] = len;
    luf->nnz_v += len;
    if (k1 > k2) { fhv->valid = 0; return 1; }                           /* FHV_ESING */
    i = pp_row[k1]; j = qq_col[k1];
    for (k = k1; k < k2; k++) {
        pp_row[k] = pp_row[k + 1]; pp_col[pp_row[k]] = k;
        qq_col[k] = qq_col[k + 1]; qq_row[qq_col[k]] = k;
    }
    pp_row[k2] = i; pp_col[i] = k2;
    qq_col[k2] = j; qq_row[j] = k2;
    for (j = 1; j <= m; j++) work[j] = 0.0;
    i_beg = vr_ptr[i];
    i_end = i_beg + vr_len[i] - 1;
    for (i_ptr = i_beg; i_ptr <= i_end; i_ptr++) {
        j = sv_ind[i_ptr];
        work[j] = sv_val[i_ptr];
        j_beg = vc_ptr[j];
        j_end = j_beg + vc_len[j] - 1;
        for (j_ptr = j_beg; sv_ind[j_ptr] != i; j_ptr++) {}
        ORC_ASSERT(j_ptr <= j_end);
        sv_ind[j_ptr] = sv_ind[j_end];
        sv_val[j_ptr] = sv_val[j_end];
        vc_len[j]--;
    }
    luf->nnz_v -= vr_len[i];
    vr_len[i] = 0;
    fhv->hh_nfs++;
    hh_ind[fhv->hh_nfs] = i;
    hh_len[fhv->hh_nfs] = 0;
    if (luf->sv_end - luf->sv_beg < k2 - k1) {
        luf_defrag_sva(luf);
        if (luf->sv_end - luf->sv_beg < k2 - k1) {
            fhv->valid = luf->valid = 0;
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            return 5;
        }
    }
    for (k = k1; k < k2; k++) {
        p = pp_row[k]; q = qq_col[k];
        if (work[q] == 0.0) continue;
        f = work[q] / vr_piv[p];
        p_beg = vr_ptr[p];
        p_end = p_beg + vr_len[p] - 1;
        for (p_ptr = p_beg; p_ptr <= p_end; p_ptr++) work[sv_ind[p_ptr]] -= f * sv_val[p_ptr];
        luf->sv_end--;
        sv_ind[luf->sv_end] = p;
        sv_val[luf->sv_end] = f;
        hh_len[fhv->hh_nfs]++;
    }
    if (hh_len[fhv->hh_nfs] == 0)
        fhv->hh_nfs--;
    else {
        hh_ptr[fhv->hh_nfs] = luf->sv_end;
        fhv->nnz_h += hh_len[fhv->hh_nfs];
    }
    vr_piv[i] = work[qq_col[k2]];
    len = 0;
    for (k = k2 + 1; k <= m; k++) {
        j = qq_col[k];
        temp = work[j];
        if (fabs(temp) < eps_tol) continue;
        if (vc_len[j] + 1 > vc_cap[j]) {
            if (luf_enlarge_col(luf, j, vc_len[j] + 10)) {
                fhv->valid = 0;
                luf->new_sva = luf->sv_size + luf->sv_size;
                ORC_ASSERT(luf->new_sva > luf->sv_size);
                return 5;
            }
        }
        j_ptr = vc_ptr[j] + vc_len[j];
        sv_ind[j_ptr] = i;
        sv_val[j_ptr] = temp;
        vc_len[j]++;
        len++; cc_ind[len] = j; cc_val[len] = temp;
    }
    if (vr_cap[i] < len) {
        if (luf_enlarge_row(luf, i, len)) {
            fhv->valid = 0;
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            return 5;
        }
    }
    i_ptr = vr_ptr[i];
    memmove(&sv_ind[i_ptr], &cc_ind[1], (size_t)len * sizeof(int));
    memmove(&sv_val[i_ptr], &cc_val[1], (size_t)len * sizeof(double));
    vr_len[i] = len;
    luf->nnz_v += len;
    temp = 0.0;
    i = pp_row[k2];
    i_beg = vr_ptr[i];
    i_end = i_beg + vr_len[i] - 1;
    for (i_ptr = i_beg; i_ptr <= i_end; i_ptr++)
        if (temp < fabs(sv_val[i_ptr])) temp = fabs(sv_val[i_ptr]);
    j = qq_col[k2];
    j_beg = vc_ptr[j];
    j_end = j_beg + vc_len[j] - 1;
    for (j_ptr = j_beg; j_ptr <= j_end; j_ptr++)
        if (temp < fabs(sv_val[j_ptr])) temp = fabs(sv_val[j_ptr]);
    if (fabs(vr_piv[i]) < upd_tol * temp) { fhv->valid = 0; return 3; }   /* FHV_ECHECK */
    return 0;
}
