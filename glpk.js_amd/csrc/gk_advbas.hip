// glp_adv_basis (glpini01.js:1-362): a starting basis from the maximal lower
// triangular part of the augmented matrix A~ = (I | -A), columns of fixed
// variables implicitly removed.  Host code: the algorithm is a greedy walk
// over doubly linked lists (one row singleton or one longest column per
// step, each step depending on the last), with no data-parallel work to
// offload; it runs once per problem on the JS host's request.  The list
// orders (LIFO buckets by length, the merge of the column buckets, the
// column patterns in the problem's list order) follow the reference
// exactly, so the chosen basis is the reference's.
#include "gk_internal.h"
#include "../../include/glpk_mi355x.h"
#include <cmath>
#include <vector>

namespace gk {
void set_err(const char *fmt, ...);
}

namespace {

using gk::FR;
using gk::LO;
using gk::UP;
using gk::DB;
using gk::FX;

// the pattern of A~ (mat, glpini01.js:214-266): column j (1..m+n) and row i
// (1..m), fixed variables' columns empty
struct AugPattern {
    int m = 0, n = 0;
    const gk_lp *lp = nullptr;
    std::vector<int> rptr, rcol;           // rows of A: structural column numbers (1..n)
    bool fixed_col(int j) const             // j in 1..m+n
    {
        return j <= m ? lp->row_type[j] == FX : lp->col_type[j - m] == FX;
    }
    // column j: its row numbers, in the problem's list order
    int col(int j, int *ndx) const
    {
        if (fixed_col(j)) return 0;
        if (j <= m) {
            ndx[1] = j;
            return 1;
        }
        const int c = j - m;
        int len = 0;
        for (int p = lp->A_ptr[c]; p < lp->A_ptr[c + 1]; p++) ndx[++len] = lp->A_ind[p];
        return len;
    }
    // row i: the non-fixed structural columns (as m + c) and the row's own
    // auxiliary column (order immaterial: used to count and to find the
    // single active column of a singleton)
    int row(int i, int *ndx) const
    {
        int len = 0;
        for (int t = rptr[i]; t < rptr[i + 1]; t++)
            if (lp->col_type[rcol[t]] != FX) ndx[++len] = m + rcol[t];
        if (lp->row_type[i] != FX) ndx[++len] = i;
        return len;
    }
};

// triang (glpini01.js:2-212): rn[1..m], cn[1..n] permutations such that the
// first `size` rows and columns of P A Q are lower triangular
int triang(int m, int n, const AugPattern &A, std::vector<int> &rn, std::vector<int> &cn)
{
    std::vector<int> ndx(1 + std::max(m, n)), rs_len(1 + m), rs_head(1 + n), rs_prev(1 + m), rs_next(1 + m),
        cs_prev(1 + n), cs_next(1 + n);
    int size = 0;
    // columns in buckets by length (rs_len as the bucket heads), LIFO
    std::vector<int> &head = rs_len;
    for (int j = 1; j <= n; j++) {
        const int len = A.col(j, ndx.data());
        cs_prev[j] = head[len];
        head[len] = j;
    }
    // one list, by descending length
    int cs_head = 0;
    for (int len = 0; len <= m; len++)
        for (int j = head[len]; j != 0; j = cs_prev[j]) {
            cs_next[j] = cs_head;
            cs_head = j;
        }
    int jj = 0;
    for (int j = cs_head; j != 0; j = cs_next[j]) {
        cs_prev[j] = jj;
        jj = j;
    }
    // rows in doubly linked buckets by active length
    for (int i = 1; i <= m; i++) {
        const int len = A.row(i, ndx.data());
        rs_len[i] = len;
        rs_prev[i] = 0;
        rs_next[i] = rs_head[len];
        if (rs_next[i] != 0) rs_prev[rs_next[i]] = i;
        rs_head[len] = i;
    }
    for (int i = 1; i <= m; i++) rn[i] = 0;
    for (int j = 1; j <= n; j++) cn[j] = 0;
    int k1 = 1, k2 = n;
    while (k1 <= k2) {
        int j;
        const int i = rs_head[1];
        if (i != 0) {
            // a row singleton: its only active column goes to b[k1, k1]
            j = 0;
            for (int t = A.row(i, ndx.data()); t >= 1; t--)
                if (cn[ndx[t]] == 0) j = ndx[t];
            if (j == 0) {
                gk::set_err("glp_adv_basis: triang: inconsistent row pattern");
                return -1;
            }
            rn[i] = cn[j] = k1;
            k1++;
            size++;
        } else {
            // no singleton: an active column of maximal length leaves
            j = cs_head;
            if (j == 0) {
                gk::set_err("glp_adv_basis: triang: empty column list");
                return -1;
            }
            cn[j] = k2;
            k2--;
        }
        // column j leaves the list and the active submatrix
        if (cs_prev[j] == 0) cs_head = cs_next[j];
        else cs_next[cs_prev[j]] = cs_next[j];
        if (cs_next[j] != 0) cs_prev[cs_next[j]] = cs_prev[j];
        for (int t = A.col(j, ndx.data()); t >= 1; t--) {
            const int r = ndx[t];
            int len = rs_len[r];
            if (rs_prev[r] == 0) rs_head[len] = rs_next[r];
            else rs_next[rs_prev[r]] = rs_next[r];
            if (rs_next[r] != 0) rs_prev[rs_next[r]] = rs_prev[r];
            rs_len[r] = --len;
            rs_prev[r] = 0;
            rs_next[r] = rs_head[len];
            if (rs_next[r] != 0) rs_prev[rs_next[r]] = r;
            rs_head[len] = r;
        }
    }
    for (int i = 1; i <= m; i++)
        if (rn[i] == 0) rn[i] = k1++;
    return size;
}

}  // namespace

extern "C" int gk_adv_basis(gk_lp *lp)
{
    using namespace gk;
    if (!lp || lp->m < 0 || lp->n < 0) {
        set_err("glp_adv_basis: invalid problem");
        return GK_EABI;
    }
    const int m = lp->m, n = lp->n;
    auto nonbasic = [](int type, double lb, double ub) -> signed char {
        switch (type) {
        case FR: return NF;
        case LO: return NL;
        case UP: return NU;
        case DB: return std::fabs(lb) <= std::fabs(ub) ? NL : NU;
        default: return NS;
        }
    };
    if (m == 0 || n == 0) {
        // glp_std_basis (glpapi05.js): every auxiliary basic, every
        // structural at its bound
        for (int i = 1; i <= m; i++) lp->row_stat[i] = BS;
        for (int j = 1; j <= n; j++) lp->col_stat[j] = nonbasic(lp->col_type[j], lp->col_lb[j], lp->col_ub[j]);
        return 0;
    }
    AugPattern A;
    A.m = m;
    A.n = n;
    A.lp = lp;
    // rows of A from the columns (the row patterns are only counted and
    // searched, so their order is free)
    A.rptr.assign(m + 2, 0);
    for (int c = 1; c <= n; c++)
        for (int p = lp->A_ptr[c]; p < lp->A_ptr[c + 1]; p++) {
            const int i = lp->A_ind[p];
            if (i < 1 || i > m) {
                set_err("glp_adv_basis: row index %d out of range", i);
                return GK_EABI;
            }
            A.rptr[i + 1]++;
        }
    for (int i = 1; i <= m + 1; i++) A.rptr[i] += A.rptr[i - 1];
    A.rcol.assign(A.rptr[m + 1] + 1, 0);
    {
        std::vector<int> fill(A.rptr.begin(), A.rptr.end());
        for (int c = 1; c <= n; c++)
            for (int p = lp->A_ptr[c]; p < lp->A_ptr[c + 1]; p++) A.rcol[fill[lp->A_ind[p]]++] = c;
    }
    std::vector<int> rn(1 + m), cn(1 + m + n);
    const int size = triang(m, m + n, A, rn, cn);
    if (size < 0) return GK_EABI;
    // adv_basis (glpini01.js:268-354)
    std::vector<int> rn_inv(1 + m), cn_inv(1 + m + n), tagx(1 + m + n, -1);
    for (int i = 1; i <= m; i++) rn_inv[rn[i]] = i;
    for (int j = 1; j <= m + n; j++) cn_inv[cn[j]] = j;
    for (int jj = 1; jj <= size; jj++) tagx[cn_inv[jj]] = BS;
    for (int jj = size + 1; jj <= m; jj++) {
        // the auxiliary variable of the jj-th row of P A~ Q completes the basis
        const int i = rn_inv[jj];
        tagx[i] = BS;
    }
    for (int k = 1; k <= m + n; k++)
        if (tagx[k] != BS)
            tagx[k] = k <= m ? nonbasic(lp->row_type[k], lp->row_lb[k], lp->row_ub[k])
                             : nonbasic(lp->col_type[k - m], lp->col_lb[k - m], lp->col_ub[k - m]);
    for (int i = 1; i <= m; i++) lp->row_stat[i] = (signed char)tagx[i];
    for (int j = 1; j <= n; j++) lp->col_stat[j] = (signed char)tagx[m + j];
    return size;
}
