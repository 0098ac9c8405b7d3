/* ORACLE (test infrastructure only) — sparse Markowitz LU of the basis
 * matrix in a sparse vector area (SVA).  Restates glpluf.js (GLPK 4.49):
 * luf_create_it :6, luf_defrag_sva :40, luf_enlarge_row :96,
 * luf_enlarge_col :157, reallocate :218, initialize :251, find_pivot :437,
 * eliminate :637, build_v_cols :969, build_f_rows :1045,
 * luf_factorize :1105, luf_f_solve :1227, luf_v_solve :1268. */
#include <stdlib.h>
#include <string.h>
#include "orc.h"

#define NEWI(n) ((int *)orc_alloc((size_t)(n), sizeof(int)))
#define NEWD(n) ((double *)orc_alloc((size_t)(n), sizeof(double)))

orc_luf *luf_create_it(void)                                 /* glpluf.js:6 */
{
    orc_luf *luf = (orc_luf *)orc_alloc(1, sizeof(orc_luf));
    luf->piv_tol = 0.10;
    luf->piv_lim = 4;
    luf->suhl = 1;
    luf->eps_tol = 1e-15;
    luf->max_gro = 1e+10;
    return luf;
}

static void free_arrays(orc_luf *luf)
{
    orc_free(luf->fr_ptr); orc_free(luf->fr_len); orc_free(luf->fc_ptr); orc_free(luf->fc_len);
    orc_free(luf->vr_ptr); orc_free(luf->vr_len); orc_free(luf->vr_cap); orc_free(luf->vr_piv);
    orc_free(luf->vc_ptr); orc_free(luf->vc_len); orc_free(luf->vc_cap);
    orc_free(luf->pp_row); orc_free(luf->pp_col); orc_free(luf->qq_row); orc_free(luf->qq_col);
    orc_free(luf->sv_prev); orc_free(luf->sv_next); orc_free(luf->vr_max);
    orc_free(luf->rs_head); orc_free(luf->rs_prev); orc_free(luf->rs_next);
    orc_free(luf->cs_head); orc_free(luf->cs_prev); orc_free(luf->cs_next);
    orc_free(luf->flag); orc_free(luf->work);
}

void luf_delete_it(orc_luf *luf)
{
    if (!luf) return;
    free_arrays(luf);
    orc_free(luf->sv_ind); orc_free(luf->sv_val);
    orc_free(luf);
}

/* glpluf.js:40 — gather all unused SVA locations into one extent */
void luf_defrag_sva(orc_luf *luf)
{
    int n = luf->n, sv_beg = 1, k, i, j;
    int *vr_ptr = luf->vr_ptr, *vr_len = luf->vr_len, *vr_cap = luf->vr_cap;
    int *vc_ptr = luf->vc_ptr, *vc_len = luf->vc_len, *vc_cap = luf->vc_cap;
    int *sv_ind = luf->sv_ind, *sv_next = luf->sv_next; double *sv_val = luf->sv_val;
    for (k = luf->sv_head; k != 0; k = sv_next[k]) {
        if (k <= n) {
            i = k;
            if (vr_ptr[i] != sv_beg) break;
            vr_cap[i] = vr_len[i];
            sv_beg += vr_cap[i];
        } else {
            j = k - n;
            if (vc_ptr[j] != sv_beg) break;
            vc_cap[j] = vc_len[j];
            sv_beg += vc_cap[j];
        }
    }
    for (; k != 0; k = sv_next[k]) {
        if (k <= n) {
            i = k;
            memmove(&sv_ind[sv_beg], &sv_ind[vr_ptr[i]], (size_t)vr_len[i] * sizeof(int));
            memmove(&sv_val[sv_beg], &sv_val[vr_ptr[i]], (size_t)vr_len[i] * sizeof(double));
            vr_ptr[i] = sv_beg;
            vr_cap[i] = vr_len[i];
            sv_beg += vr_cap[i];
        } else {
            j = k - n;
            memmove(&sv_ind[sv_beg], &sv_ind[vc_ptr[j]], (size_t)vc_len[j] * sizeof(int));
            memmove(&sv_val[sv_beg], &sv_val[vc_ptr[j]], (size_t)vc_len[j] * sizeof(double));
            vc_ptr[j] = sv_beg;
            vc_cap[j] = vc_len[j];
            sv_beg += vc_cap[j];
        }
    }
    luf->sv_beg = sv_beg;
}

/* move node k (row k<=n, column k-n) to the tail of the SVA address list,
 * giving its old locations to the predecessor (glpluf.js:128-153) */
static void move_to_tail(orc_luf *luf, int k, int cur)
{
    int n = luf->n, kk;
    int *sv_prev = luf->sv_prev, *sv_next = luf->sv_next;
    if (sv_prev[k] == 0)
        luf->sv_head = sv_next[k];
    else {
        kk = sv_prev[k];
        if (kk <= n) luf->vr_cap[kk] += cur; else luf->vc_cap[kk - n] += cur;
        sv_next[sv_prev[k]] = sv_next[k];
    }
    if (sv_next[k] == 0)
        luf->sv_tail = sv_prev[k];
    else
        sv_prev[sv_next[k]] = sv_prev[k];
    sv_prev[k] = luf->sv_tail;
    sv_next[k] = 0;
    if (sv_prev[k] == 0)
        luf->sv_head = k;
    else
        sv_next[sv_prev[k]] = k;
    luf->sv_tail = k;
}

int luf_enlarge_row(orc_luf *luf, int i, int cap)            /* glpluf.js:96 */
{
    int cur;
    ORC_ASSERT(1 <= i && i <= luf->n);
    ORC_ASSERT(luf->vr_cap[i] < cap);
    if (luf->sv_end - luf->sv_beg < cap) {
        luf_defrag_sva(luf);
        if (luf->sv_end - luf->sv_beg < cap) return 1;
    }
    cur = luf->vr_cap[i];
    memmove(&luf->sv_ind[luf->sv_beg], &luf->sv_ind[luf->vr_ptr[i]], (size_t)luf->vr_len[i] * sizeof(int));
    memmove(&luf->sv_val[luf->sv_beg], &luf->sv_val[luf->vr_ptr[i]], (size_t)luf->vr_len[i] * sizeof(double));
    luf->vr_ptr[i] = luf->sv_beg;
    luf->vr_cap[i] = cap;
    luf->sv_beg += cap;
    move_to_tail(luf, i, cur);
    return 0;
}

int luf_enlarge_col(orc_luf *luf, int j, int cap)            /* glpluf.js:157 */
{
    int cur;
    ORC_ASSERT(1 <= j && j <= luf->n);
    ORC_ASSERT(luf->vc_cap[j] < cap);
    if (luf->sv_end - luf->sv_beg < cap) {
        luf_defrag_sva(luf);
        if (luf->sv_end - luf->sv_beg < cap) return 1;
    }
    cur = luf->vc_cap[j];
    memmove(&luf->sv_ind[luf->sv_beg], &luf->sv_ind[luf->vc_ptr[j]], (size_t)luf->vc_len[j] * sizeof(int));
    memmove(&luf->sv_val[luf->sv_beg], &luf->sv_val[luf->vc_ptr[j]], (size_t)luf->vc_len[j] * sizeof(double));
    luf->vc_ptr[j] = luf->sv_beg;
    luf->vc_cap[j] = cap;
    luf->sv_beg += cap;
    move_to_tail(luf, luf->n + j, cur);
    return 0;
}

static void reallocate(orc_luf *luf, int n)                  /* glpluf.js:218 */
{
    int N;
    luf->n = n;
    if (n <= luf->n_max) return;
    free_arrays(luf);
    luf->n_max = N = n + 100;
    luf->fr_ptr = NEWI(1 + N); luf->fr_len = NEWI(1 + N);
    luf->fc_ptr = NEWI(1 + N); luf->fc_len = NEWI(1 + N);
    luf->vr_ptr = NEWI(1 + N); luf->vr_len = NEWI(1 + N); luf->vr_cap = NEWI(1 + N);
    luf->vr_piv = NEWD(1 + N);
    luf->vc_ptr = NEWI(1 + N); luf->vc_len = NEWI(1 + N); luf->vc_cap = NEWI(1 + N);
    luf->pp_row = NEWI(1 + N); luf->pp_col = NEWI(1 + N);
    luf->qq_row = NEWI(1 + N); luf->qq_col = NEWI(1 + N);
    luf->sv_prev = NEWI(1 + N + N); luf->sv_next = NEWI(1 + N + N);
    luf->vr_max = NEWD(1 + N);
    luf->rs_head = NEWI(1 + N); luf->rs_prev = NEWI(1 + N); luf->rs_next = NEWI(1 + N);
    luf->cs_head = NEWI(1 + N); luf->cs_prev = NEWI(1 + N); luf->cs_next = NEWI(1 + N);
    luf->flag = NEWI(1 + N);
    luf->work = NEWD(1 + N);
}

/* glpluf.js:251 — V := A (rows and columns), F := I, P = Q = I, active lists */
static int initialize(orc_luf *luf, orc_col_fn col, void *info)
{
    int n = luf->n, i, j, k, len, nnz, sv_beg, sv_end, ptr, i_ptr, j_beg, j_end;
    int *fc_ptr = luf->fc_ptr, *fc_len = luf->fc_len;
    int *vr_ptr = luf->vr_ptr, *vr_len = luf->vr_len, *vr_cap = luf->vr_cap;
    int *vc_ptr = luf->vc_ptr, *vc_len = luf->vc_len, *vc_cap = luf->vc_cap;
    int *pp_row = luf->pp_row, *pp_col = luf->pp_col, *qq_row = luf->qq_row, *qq_col = luf->qq_col;
    int *sv_ind = luf->sv_ind, *sv_prev = luf->sv_prev, *sv_next = luf->sv_next;
    double *sv_val = luf->sv_val, *vr_max = luf->vr_max, *work = luf->work;
    int *rs_head = luf->rs_head, *rs_prev = luf->rs_prev, *rs_next = luf->rs_next;
    int *cs_head = luf->cs_head, *cs_prev = luf->cs_prev, *cs_next = luf->cs_next;
    int *flag = luf->flag;
    double big, val;
    sv_beg = 1;
    sv_end = luf->sv_size + 1;
    for (j = 1; j <= n; j++) { fc_ptr[j] = sv_end; fc_len[j] = 0; }
    for (i = 1; i <= n; i++) { vr_len[i] = vr_cap[i] = 0; flag[i] = 0; }
    nnz = 0;
    big = 0.0;
    for (j = 1; j <= n; j++) {
        int *rn = pp_row; double *aj = work;
        len = col(info, j, rn, aj);
        if (!(0 <= len && len <= n))
            orc_fail("luf_factorize: j = %d; len = %d; invalid column length", j, len);
        if (sv_end - sv_beg < len) return 1;
        vc_ptr[j] = sv_beg;
        vc_len[j] = vc_cap[j] = len;
        nnz += len;
        for (ptr = 1; ptr <= len; ptr++) {
            i = rn[ptr];
            val = aj[ptr];
            if (!(1 <= i && i <= n))
                orc_fail("luf_factorize: i = %d; j = %d; invalid row index", i, j);
            if (flag[i])
                orc_fail("luf_factorize: i = %d; j = %d; duplicate element not allowed", i, j);
            if (val == 0.0)
                orc_fail("luf_factorize: i = %d; j = %d; zero element not allowed", i, j);
            sv_ind[sv_beg] = i;
            sv_val[sv_beg] = val;
            sv_beg++;
            if (val < 0.0) val = -val;
            if (big < val) big = val;
            flag[i] = 1;
            vr_cap[i]++;
        }
        for (ptr = 1; ptr <= len; ptr++) flag[rn[ptr]] = 0;
    }
    for (i = 1; i <= n; i++) {
        len = vr_cap[i];
        if (sv_end - sv_beg < len) return 1;
        vr_ptr[i] = sv_beg;
        sv_beg += len;
    }
    for (j = 1; j <= n; j++) {
        j_beg = vc_ptr[j];
        j_end = j_beg + vc_len[j] - 1;
        for (k = j_beg; k <= j_end; k++) {
            i = sv_ind[k];
            val = sv_val[k];
            i_ptr = vr_ptr[i] + vr_len[i];
            sv_ind[i_ptr] = j;
            sv_val[i_ptr] = val;
            vr_len[i]++;
        }
    }
    for (k = 1; k <= n; k++) pp_row[k] = pp_col[k] = qq_row[k] = qq_col[k] = k;
    luf->sv_beg = sv_beg;
    luf->sv_end = sv_end;
    luf->sv_head = n + 1;
    luf->sv_tail = n;
    for (i = 1; i <= n; i++) { sv_prev[i] = i - 1; sv_next[i] = i + 1; }
    sv_prev[1] = n + n;
    sv_next[n] = 0;
    for (j = 1; j <= n; j++) { sv_prev[n + j] = n + j - 1; sv_next[n + j] = n + j + 1; }
    sv_prev[n + 1] = 0;
    sv_next[n + n] = 1;
    for (k = 1; k <= n; k++) { flag[k] = 0; work[k] = 0.0; }
    luf->nnz_a = nnz;
    luf->nnz_f = 0;
    luf->nnz_v = nnz;
    luf->max_a = big;
    luf->big_v = big;
    luf->rank = -1;
    for (i = 1; i <= n; i++) vr_max[i] = -1.0;
    for (len = 0; len <= n; len++) rs_head[len] = 0;
    for (i = 1; i <= n; i++) {
        len = vr_len[i];
        rs_prev[i] = 0;
        rs_next[i] = rs_head[len];
        if (rs_next[i] != 0) rs_prev[rs_next[i]] = i;
        rs_head[len] = i;
    }
    for (len = 0; len <= n; len++) cs_head[len] = 0;
    for (j = 1; j <= n; j++) {
        len = vc_len[j];
        cs_prev[j] = 0;
        cs_next[j] = cs_head[len];
        if (cs_next[j] != 0) cs_prev[cs_next[j]] = j;
        cs_head[len] = j;
    }
    return 0;
}

/* largest |v[i,*]| of an active row, cached in vr_max (glpluf.js:499-508) */
static double row_max(orc_luf *luf, int i)
{
    double big = luf->vr_max[i], temp;
    if (big < 0.0) {
        int i_beg = luf->vr_ptr[i], i_end = i_beg + luf->vr_len[i] - 1, p;
        for (p = i_beg; p <= i_end; p++) {
            temp = luf->sv_val[p];
            if (temp < 0.0) temp = -temp;
            if (big < temp) big = temp;
        }
        luf->vr_max[i] = big;
    }
    return big;
}

/* glpluf.js:437 — Markowitz pivot search with Suhl's column exclusion;
 * returns 1 if the active submatrix is exactly zero */
static int find_pivot(orc_luf *luf, int *pp, int *qq)
{
    int n = luf->n;
    int *vr_ptr = luf->vr_ptr, *vr_len = luf->vr_len, *vc_ptr = luf->vc_ptr, *vc_len = luf->vc_len;
    int *sv_ind = luf->sv_ind; double *sv_val = luf->sv_val;
    int *rs_head = luf->rs_head, *rs_next = luf->rs_next;
    int *cs_head = luf->cs_head, *cs_prev = luf->cs_prev, *cs_next = luf->cs_next;
    double piv_tol = luf->piv_tol; int piv_lim = luf->piv_lim, suhl = luf->suhl;
    int p, q, len, i, i_beg, i_end, i_ptr, j, j_beg, j_end, j_ptr, ncand, next_j, min_p, min_q, min_len;
    double best, cost, big, temp;
    p = q = 0; best = DBL_MAX; ncand = 0;
    j = cs_head[1];
    if (j != 0) {
        ORC_ASSERT(vc_len[j] == 1);
        p = sv_ind[vc_ptr[j]]; q = j;
        goto done;
    }
    i = rs_head[1];
    if (i != 0) {
        ORC_ASSERT(vr_len[i] == 1);
        p = i; q = sv_ind[vr_ptr[i]];
        goto done;
    }
    for (len = 2; len <= n; len++) {
        for (j = cs_head[len]; j != 0; j = next_j) {
            j_beg = vc_ptr[j];
            j_end = j_beg + vc_len[j] - 1;
            next_j = cs_next[j];
            min_p = min_q = 0; min_len = INT_MAX;
            for (j_ptr = j_beg; j_ptr <= j_end; j_ptr++) {
                i = sv_ind[j_ptr];
                i_beg = vr_ptr[i];
                i_end = i_beg + vr_len[i] - 1;
                if (vr_len[i] >= min_len) continue;
                big = row_max(luf, i);
                for (i_ptr = vr_ptr[i]; sv_ind[i_ptr] != j; i_ptr++) {}
                ORC_ASSERT(i_ptr <= i_end);
                temp = sv_val[i_ptr];
                if (temp < 0.0) temp = -temp;
                if (temp < piv_tol * big) continue;
                min_p = i; min_q = j; min_len = vr_len[i];
                if (min_len <= len) { p = min_p; q = min_q; goto done; }
            }
            if (min_p != 0) {
                ncand++;
                cost = (double)(min_len - 1) * (double)(len - 1);
                if (cost < best) { p = min_p; q = min_q; best = cost; }
                if (ncand == piv_lim) goto done;
            } else if (suhl) {
                if (cs_prev[j] == 0)
                    cs_head[len] = cs_next[j];
                else
                    cs_next[cs_prev[j]] = cs_next[j];
                if (cs_next[j] != 0)
                    cs_prev[cs_next[j]] = cs_prev[j];
                cs_prev[j] = cs_next[j] = j;
            }
        }
        for (i = rs_head[len]; i != 0; i = rs_next[i]) {
            i_beg = vr_ptr[i];
            i_end = i_beg + vr_len[i] - 1;
            big = row_max(luf, i);
            min_p = min_q = 0; min_len = INT_MAX;
            for (i_ptr = i_beg; i_ptr <= i_end; i_ptr++) {
                j = sv_ind[i_ptr];
                if (vc_len[j] >= min_len) continue;
                temp = sv_val[i_ptr];
                if (temp < 0.0) temp = -temp;
                if (temp < piv_tol * big) continue;
                min_p = i; min_q = j; min_len = vc_len[j];
                if (min_len <= len) { p = min_p; q = min_q; goto done; }
            }
            if (min_p != 0) {
                ncand++;
                cost = (double)(len - 1) * (double)(min_len - 1);
                if (cost < best) { p = min_p; q = min_q; best = cost; }
                if (ncand == piv_lim) goto done;
            } else
                ORC_ASSERT(min_p != min_p);
        }
    }
done:
    *pp = p; *qq = q;
    return p == 0;
}

static void rs_remove(orc_luf *luf, int i)
{
    if (luf->rs_prev[i] == 0)
        luf->rs_head[luf->vr_len[i]] = luf->rs_next[i];
    else
        luf->rs_next[luf->rs_prev[i]] = luf->rs_next[i];
    if (luf->rs_next[i] != 0)
        luf->rs_prev[luf->rs_next[i]] = luf->rs_prev[i];
}

static void cs_remove(orc_luf *luf, int j)
{
    if (luf->cs_prev[j] == 0)
        luf->cs_head[luf->vc_len[j]] = luf->cs_next[j];
    else
        luf->cs_next[luf->cs_prev[j]] = luf->cs_next[j];
    if (luf->cs_next[j] != 0)
        luf->cs_prev[luf->cs_next[j]] = luf->cs_prev[j];
}

/* glpluf.js:637 — gaussian elimination of the pivot column v[*,q] */
static int eliminate(orc_luf *luf, int p, int q)
{
    int n = luf->n;
    int *fc_len = luf->fc_len;
    int *vr_ptr = luf->vr_ptr, *vr_len = luf->vr_len, *vr_cap = luf->vr_cap;
    double *vr_piv = luf->vr_piv;
    int *vc_ptr = luf->vc_ptr, *vc_len = luf->vc_len, *vc_cap = luf->vc_cap;
    int *sv_prev = luf->sv_prev, *sv_next = luf->sv_next;
    int *rs_head = luf->rs_head, *rs_prev = luf->rs_prev, *rs_next = luf->rs_next;
    int *cs_head = luf->cs_head, *cs_prev = luf->cs_prev, *cs_next = luf->cs_next;
    int *flag = luf->flag; double *work = luf->work, *vr_max = luf->vr_max;
    double eps_tol = luf->eps_tol;
    int *ndx = luf->fr_len;
    int len, fill, i, i_beg, i_end, i_ptr, j, j_beg, j_end, j_ptr, k, p_beg, p_end, p_ptr, q_beg, q_end;
    double fip, val, vpq, temp;
    /* sv_ind/sv_val may move only through luf_enlarge_*, which do not
     * reallocate the SVA itself, so cached pointers stay valid */
    int *sv_ind = luf->sv_ind; double *sv_val = luf->sv_val;
    ORC_ASSERT(1 <= p && p <= n);
    ORC_ASSERT(1 <= q && q <= n);
    rs_remove(luf, p);
    cs_remove(luf, q);
    p_beg = vr_ptr[p];
    p_end = p_beg + vr_len[p] - 1;
    for (p_ptr = p_beg; sv_ind[p_ptr] != q; p_ptr++) {}
    ORC_ASSERT(p_ptr <= p_end);
    vpq = (vr_piv[p] = sv_val[p_ptr]);
    sv_ind[p_ptr] = sv_ind[p_end];
    sv_val[p_ptr] = sv_val[p_end];
    vr_len[p]--;
    p_end--;
    q_beg = vc_ptr[q];
    q_end = q_beg + vc_len[q] - 1;
    for (i_ptr = q_beg; sv_ind[i_ptr] != p; i_ptr++) {}
    ORC_ASSERT(i_ptr <= q_end);
    sv_ind[i_ptr] = sv_ind[q_end];
    vc_len[q]--;
    q_end--;
    for (p_ptr = p_beg; p_ptr <= p_end; p_ptr++) {
        j = sv_ind[p_ptr];
        flag[j] = 1;
        work[j] = sv_val[p_ptr];
        cs_remove(luf, j);
        j_beg = vc_ptr[j];
        j_end = j_beg + vc_len[j] - 1;
        for (j_ptr = j_beg; sv_ind[j_ptr] != p; j_ptr++) {}
        ORC_ASSERT(j_ptr <= j_end);
        sv_ind[j_ptr] = sv_ind[j_end];
        vc_len[j]--;
    }
    while (q_beg <= q_end) {
        i = sv_ind[q_beg];
        rs_remove(luf, i);
        i_beg = vr_ptr[i];
        i_end = i_beg + vr_len[i] - 1;
        for (i_ptr = i_beg; sv_ind[i_ptr] != q; i_ptr++) {}
        ORC_ASSERT(i_ptr <= i_end);
        fip = sv_val[i_ptr] / vpq;
        sv_ind[i_ptr] = sv_ind[i_end];
        sv_val[i_ptr] = sv_val[i_end];
        vr_len[i]--;
        i_end--;
        sv_ind[q_beg] = sv_ind[q_end];
        vc_len[q]--;
        q_end--;
        fill = vr_len[p];
        for (i_ptr = i_beg; i_ptr <= i_end; i_ptr++) {
            j = sv_ind[i_ptr];
            if (flag[j]) {
                temp = (sv_val[i_ptr] -= fip * work[j]);
                if (temp < 0.0) temp = -temp;
                flag[j] = 0;
                fill--;
                if (temp == 0.0 || temp < eps_tol) {
                    sv_ind[i_ptr] = sv_ind[i_end];
                    sv_val[i_ptr] = sv_val[i_end];
                    vr_len[i]--;
                    i_ptr--;
                    i_end--;
                    j_beg = vc_ptr[j];
                    j_end = j_beg + vc_len[j] - 1;
                    for (j_ptr = j_beg; sv_ind[j_ptr] != i; j_ptr++) {}
                    ORC_ASSERT(j_ptr <= j_end);
                    sv_ind[j_ptr] = sv_ind[j_end];
                    vc_len[j]--;
                } else {
                    if (luf->big_v < temp) luf->big_v = temp;
                }
            }
        }
        if (vr_len[i] + fill > vr_cap[i]) {
            if (luf_enlarge_row(luf, i, vr_len[i] + fill)) return 1;
            p_beg = vr_ptr[p];
            p_end = p_beg + vr_len[p] - 1;
            q_beg = vc_ptr[q];
            q_end = q_beg + vc_len[q] - 1;
        }
        len = 0;
        for (p_ptr = p_beg; p_ptr <= p_end; p_ptr++) {
            j = sv_ind[p_ptr];
            if (flag[j]) {
                temp = (val = -fip * work[j]);
                if (temp < 0.0) temp = -temp;
                if (temp == 0.0 || temp < eps_tol) {
                    /* ignore tiny fill-in */
                } else {
                    i_ptr = vr_ptr[i] + vr_len[i];
                    sv_ind[i_ptr] = j;
                    sv_val[i_ptr] = val;
                    vr_len[i]++;
                    ndx[++len] = j;
                    if (luf->big_v < temp) luf->big_v = temp;
                }
            } else
                flag[j] = 1;
        }
        for (k = 1; k <= len; k++) {
            j = ndx[k];
            if (vc_len[j] + 1 > vc_cap[j]) {
                if (luf_enlarge_col(luf, j, vc_len[j] + 10)) return 1;
                p_beg = vr_ptr[p];
                p_end = p_beg + vr_len[p] - 1;
                q_beg = vc_ptr[q];
                q_end = q_beg + vc_len[q] - 1;
            }
            j_ptr = vc_ptr[j] + vc_len[j];
            sv_ind[j_ptr] = i;
            vc_len[j]++;
        }
        rs_prev[i] = 0;
        rs_next[i] = rs_head[vr_len[i]];
        if (rs_next[i] != 0) rs_prev[rs_next[i]] = i;
        rs_head[vr_len[i]] = i;
        vr_max[i] = -1.0;
        if (luf->sv_end - luf->sv_beg < 1) {
            luf_defrag_sva(luf);
            if (luf->sv_end - luf->sv_beg < 1) return 1;
            p_beg = vr_ptr[p];
            p_end = p_beg + vr_len[p] - 1;
            q_beg = vc_ptr[q];
            q_end = q_beg + vc_len[q] - 1;
        }
        luf->sv_end--;
        sv_ind[luf->sv_end] = i;
        sv_val[luf->sv_end] = fip;
        fc_len[p]++;
    }
    ORC_ASSERT(vc_len[q] == 0);
    vc_cap[q] = 0;
    k = n + q;
    if (sv_prev[k] == 0)
        luf->sv_head = sv_next[k];
    else
        sv_next[sv_prev[k]] = sv_next[k];
    if (sv_next[k] == 0)
        luf->sv_tail = sv_prev[k];
    else
        sv_prev[sv_next[k]] = sv_prev[k];
    luf->fc_ptr[p] = luf->sv_end;
    for (p_ptr = p_beg; p_ptr <= p_end; p_ptr++) {
        j = sv_ind[p_ptr];
        flag[j] = 0;
        work[j] = 0.0;
        if (!(vc_len[j] != 1 && cs_prev[j] == j && cs_next[j] == j)) {
            cs_prev[j] = 0;
            cs_next[j] = cs_head[vc_len[j]];
            if (cs_next[j] != 0) cs_prev[cs_next[j]] = j;
            cs_head[vc_len[j]] = j;
        }
    }
    return 0;
}

static int build_v_cols(orc_luf *luf)                        /* glpluf.js:969 */
{
    int n = luf->n, i, i_beg, i_end, i_ptr, j, j_ptr, k, nnz;
    int *vr_ptr = luf->vr_ptr, *vr_len = luf->vr_len;
    int *vc_ptr = luf->vc_ptr, *vc_len = luf->vc_len, *vc_cap = luf->vc_cap;
    int *sv_ind = luf->sv_ind, *sv_prev = luf->sv_prev, *sv_next = luf->sv_next;
    double *sv_val = luf->sv_val;
    nnz = 0;
    for (i = 1; i <= n; i++) {
        i_beg = vr_ptr[i];
        i_end = i_beg + vr_len[i] - 1;
        for (i_ptr = i_beg; i_ptr <= i_end; i_ptr++) vc_cap[sv_ind[i_ptr]]++;
        nnz += vr_len[i];
    }
    luf->nnz_v = nnz;
    if (luf->sv_end - luf->sv_beg < nnz) return 1;
    for (j = 1; j <= n; j++) {
        vc_ptr[j] = luf->sv_beg;
        luf->sv_beg += vc_cap[j];
    }
    for (i = 1; i <= n; i++) {
        i_beg = vr_ptr[i];
        i_end = i_beg + vr_len[i] - 1;
        for (i_ptr = i_beg; i_ptr <= i_end; i_ptr++) {
            j = sv_ind[i_ptr];
            j_ptr = vc_ptr[j] + vc_len[j];
            sv_ind[j_ptr] = i;
            sv_val[j_ptr] = sv_val[i_ptr];
            vc_len[j]++;
        }
    }
    for (k = n + 1; k <= n + n; k++) { sv_prev[k] = k - 1; sv_next[k] = k + 1; }
    sv_prev[n + 1] = luf->sv_tail;
    sv_next[luf->sv_tail] = n + 1;
    sv_next[n + n] = 0;
    luf->sv_tail = n + n;
    return 0;
}

static int build_f_rows(orc_luf *luf)                        /* glpluf.js:1045 */
{
    int n = luf->n, i, j, j_beg, j_end, j_ptr, ptr, nnz;
    int *fr_ptr = luf->fr_ptr, *fr_len = luf->fr_len, *fc_ptr = luf->fc_ptr, *fc_len = luf->fc_len;
    int *sv_ind = luf->sv_ind; double *sv_val = luf->sv_val;
    for (i = 1; i <= n; i++) fr_len[i] = 0;
    nnz = 0;
    for (j = 1; j <= n; j++) {
        j_beg = fc_ptr[j];
        j_end = j_beg + fc_len[j] - 1;
        for (j_ptr = j_beg; j_ptr <= j_end; j_ptr++) fr_len[sv_ind[j_ptr]]++;
        nnz += fc_len[j];
    }
    luf->nnz_f = nnz;
    if (luf->sv_end - luf->sv_beg < nnz) return 1;
    for (i = 1; i <= n; i++) {
        fr_ptr[i] = luf->sv_end;
        luf->sv_end -= fr_len[i];
    }
    for (j = 1; j <= n; j++) {
        j_beg = fc_ptr[j];
        j_end = j_beg + fc_len[j] - 1;
        for (j_ptr = j_beg; j_ptr <= j_end; j_ptr++) {
            i = sv_ind[j_ptr];
            ptr = --fr_ptr[i];
            sv_ind[ptr] = j;
            sv_val[ptr] = sv_val[j_ptr];
        }
    }
    return 0;
}

int luf_factorize(orc_luf *luf, int n, orc_col_fn col, void *info)   /* glpluf.js:1105 */
{
    int i, j, k, p, q, t, ret = -1;
    if (n < 1) orc_fail("luf_factorize: n = %d; invalid parameter", n);
    luf->valid = 0;
    reallocate(luf, n);
    if (luf->sv_size == 0 && luf->new_sva == 0)
        luf->new_sva = 5 * (n + 10);
    for (;;) {                                   /* the more() loop, :1126-1204 */
        int *pp_row, *pp_col, *qq_row, *qq_col;
        if (luf->new_sva > 0) {
            orc_free(luf->sv_ind); orc_free(luf->sv_val);
            luf->sv_size = luf->new_sva;
            luf->sv_ind = NEWI(1 + luf->sv_size);
            luf->sv_val = NEWD(1 + luf->sv_size);
            luf->new_sva = 0;
        }
        if (initialize(luf, col, info)) {
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            continue;
        }
        pp_row = luf->pp_row; pp_col = luf->pp_col; qq_row = luf->qq_row; qq_col = luf->qq_col;
        for (k = 1; k <= n; k++) {
            if (find_pivot(luf, &p, &q)) {
                luf->rank = k - 1;
                ret = 1;                          /* LUF_ESING */
                break;
            }
            i = pp_col[p]; j = qq_row[q];
            ORC_ASSERT(k <= i && i <= n && k <= j && j <= n);
            t = pp_row[k];
            pp_row[i] = t; pp_col[t] = i;
            pp_row[k] = p; pp_col[p] = k;
            t = qq_col[k];
            qq_col[j] = t; qq_row[t] = j;
            qq_col[k] = q; qq_row[q] = k;
            if (eliminate(luf, p, q)) { ret = -2; break; }
            if (luf->big_v > luf->max_gro * luf->max_a) {
                luf->rank = k - 1;
                ret = 2;                          /* LUF_ECOND */
                break;
            }
        }
        if (ret == 1 || ret == 2) return ret;
        if (ret == -2) {
            ret = -1;
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            continue;
        }
        luf_defrag_sva(luf);
        if (build_v_cols(luf)) {
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            continue;
        }
        if (build_f_rows(luf)) {
            luf->new_sva = luf->sv_size + luf->sv_size;
            ORC_ASSERT(luf->new_sva > luf->sv_size);
            continue;
        }
        break;
    }
    luf->valid = 1;
    luf->rank = n;
    t = 3 * (n + luf->nnz_v) + 2 * luf->nnz_f;
    if (luf->sv_size < t) {
        luf->new_sva = luf->sv_size;
        while (luf->new_sva < t) {
            k = luf->new_sva;
            luf->new_sva = k + k;
            ORC_ASSERT(luf->new_sva > k);
        }
    }
    return 0;
}

void luf_f_solve(orc_luf *luf, int tr, double *x)            /* glpluf.js:1227 */
{
    int n = luf->n, i, j, k, beg, end, ptr;
    int *pp_row = luf->pp_row, *sv_ind = luf->sv_ind; double *sv_val = luf->sv_val;
    double xk;
    if (!luf->valid) orc_fail("luf_f_solve: LU-factorization is not valid");
    if (!tr) {
        for (j = 1; j <= n; j++) {
            k = pp_row[j];
            xk = x[k];
            if (xk != 0.0) {
                beg = luf->fc_ptr[k];
                end = beg + luf->fc_len[k] - 1;
                for (ptr = beg; ptr <= end; ptr++) x[sv_ind[ptr]] -= sv_val[ptr] * xk;
            }
        }
    } else {
        for (i = n; i >= 1; i--) {
            k = pp_row[i];
            xk = x[k];
            if (xk != 0.0) {
                beg = luf->fr_ptr[k];
                end = beg + luf->fr_len[k] - 1;
                for (ptr = beg; ptr <= end; ptr++) x[sv_ind[ptr]] -= sv_val[ptr] * xk;
            }
        }
    }
}

void luf_v_solve(orc_luf *luf, int tr, double *x)            /* glpluf.js:1268 */
{
    int n = luf->n, i, j, k, beg, end, ptr;
    int *pp_row = luf->pp_row, *qq_col = luf->qq_col, *sv_ind = luf->sv_ind;
    double *sv_val = luf->sv_val, *vr_piv = luf->vr_piv, *b = luf->work;
    double temp;
    if (!luf->valid) orc_fail("luf_v_solve: LU-factorization is not valid");
    for (k = 1; k <= n; k++) { b[k] = x[k]; x[k] = 0.0; }
    if (!tr) {
        for (k = n; k >= 1; k--) {
            i = pp_row[k]; j = qq_col[k];
            temp = b[i];
            if (temp != 0.0) {
                x[j] = (temp /= vr_piv[i]);
                beg = luf->vc_ptr[j];
                end = beg + luf->vc_len[j] - 1;
                for (ptr = beg; ptr <= end; ptr++) b[sv_ind[ptr]] -= sv_val[ptr] * temp;
            }
        }
    } else {
        for (k = 1; k <= n; k++) {
            i = pp_row[k]; j = qq_col[k];
            temp = b[j];
            if (temp != 0.0) {
                x[i] = (temp /= vr_piv[i]);
                beg = luf->vr_ptr[i];
                end = beg + luf->vr_len[i] - 1;
                for (ptr = beg; ptr <= end; ptr++) b[sv_ind[ptr]] -= sv_val[ptr] * temp;
            }
        }
    }
}
