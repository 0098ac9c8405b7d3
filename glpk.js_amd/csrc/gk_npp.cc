// LP / MIP presolver (glp_simplex / glp_intopt with presolve = GLP_ON):
// GLPK 4.49's preprocessor as glpk.js ships it (lib/glpnpp01.js ..
// glpnpp05.js).  Host code, like glp_adv_basis: the transformations are a
// sequential walk over doubly linked row and column lists (each one may
// re-activate the rows and columns it touches), run once per solve before the
// device simplex; postprocessing replays the transformation stack backwards
// over the device's solution of the reduced problem.
//
// Everything that decides the reduced problem is kept in the reference's
// order: the row / column list orders (activation moves to the front,
// deactivation to the back, glpnpp01.js:60-134), the element order inside
// each list (new elements at the front, :164), the order of the sums over
// them and the saved coefficient lists of each stack entry (walked in the
// reverse of their creation order, as the reference's singly linked lists
// are), so the reduced problem is the reference's bit for bit.
//
// Storage: rows, columns and elements in pools addressed by index; a list
// link of -1 is the reference's null.  Row p of the original problem is pool
// index p - 1 (rows and columns are only ever appended).
#include "gk_internal.h"
#include "../../include/glpk_mi355x.h"
#include <cfloat>
#include <cmath>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

namespace gk {
void set_err(const char *fmt, ...);
}

namespace {

using gk::BS;
using gk::DB;
using gk::FR;
using gk::FX;
using gk::LO;
using gk::NF;
using gk::NL;
using gk::NS;
using gk::NU;
using gk::UP;

constexpr double BIG = DBL_MAX;
constexpr int SOL = 1, IPT = 2, MIP = 3;         // GLP_SOL / GLP_IPT / GLP_MIP
constexpr int ENOPFS = 10, ENODFS = 11;           // GLP_ENOPFS / GLP_ENODFS

struct NppFail : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// the stack entry kinds: one per transformation with a recovery routine
enum Kind : int {
    T_FREE_ROW,       // npp_free_row        glpnpp02.js:2
    T_FIXED_COL,      // npp_fixed_col       :357
    T_MAKE_EQ,        // npp_make_equality   :394
    T_MAKE_FIXED,     // npp_make_fixed      :437
    T_EMPTY_COL,      // npp_empty_col       glpnpp03.js:16
    T_EQ_SINGLET,     // npp_eq_singlet      :121
    T_INEQ_SINGLET,   // npp_ineq_singlet    :291
    T_IMPL_SLACK,     // npp_implied_slack   :510
    T_IMPL_FREE,      // npp_implied_free    :594
    T_FORCING,        // npp_forcing_row     :861
    T_INACTIVE,       // npp_inactive_bound  :1098
    T_LBND_COL,       // npp_lbnd_col        glpnpp02.js:196
    T_BINARIZE,       // npp_binarize_prob   glpnpp04.js:2
};

// a linear form sum a[j] x[j] (copy_form, glpnpp04.js:101): the reference
// builds it by prepending, so it runs over the row in reverse list order
struct Term {
    double aj;
    int xj;
};

struct Row {
    double lb = -BIG, ub = +BIG;
    int ptr = -1;                 // first element of the row list
    int temp = 0;                 // active flag; the new row number while building
    int prev = -1, next = -1;
};

struct Col {
    int is_int = 0;
    double lb = 0.0, ub = 0.0, coef = 0.0;
    int ptr = -1;
    int temp = 0;
    int prev = -1, next = -1;
    double ll = 0.0, uu = 0.0;    // implied bounds (npp_implied_bounds)
};

struct Aij {
    int row, col;
    double val;
    int r_prev, r_next, c_prev, c_next;
};

struct Lfe {                      // saved coefficient: row or column number, value
    int ref;
    double val;
};

struct FCol {                     // a column of a forcing row (glpnpp03.js:974-981)
    int j, stat;
    double a, c;
    int lb, le;                   // its saved column, lfe[lb, le)
};

struct Tse {
    int kind;
    int p = 0, q = 0, stat = 0, lb_changed = 0, ub_changed = 0;
    double apq = 0.0, b = 0.0, c = 0.0, s = 0.0, lb = 0.0, ub = 0.0;
    int lb_ = 0, le_ = 0;         // saved coefficients lfe[lb_, le_), creation order
    int fb = 0, fe = 0;           // forcing-row columns fcol[fb, fe), creation order
    int j0 = 0, nb = 0;           // binarized variable: first added column, n
};

struct Npp {
    int orig_dir = 0, orig_m = 0, orig_n = 0, orig_nnz = 0;
    double c0 = 0.0;
    int sol = SOL;
    std::vector<Row> row;
    std::vector<Col> col;
    std::vector<Aij> a;
    int r_head = -1, r_tail = -1, c_head = -1, c_tail = -1;
    std::vector<Tse> tse;
    std::vector<Lfe> lfe;
    std::vector<FCol> fcol;
    // reduced problem
    bool built = false;
    int m = 0, n = 0, nnz = 0;
    std::vector<int> row_ref, col_ref;
    // recovered solution (npp_postprocess, glpnpp01.js:474)
    int p_stat = 0, d_stat = 0, i_stat = 0;
    std::vector<signed char> r_stat, c_stat;
    std::vector<double> c_value, r_pi;
    bool post = false;

    // ---- lists (glpnpp01.js:24-134) --------------------------------------
    void row_insert(int r, bool front)
    {
        Row &R = row[r];
        if (front) {
            R.prev = -1;
            R.next = r_head;
            if (R.next < 0) r_tail = r; else row[R.next].prev = r;
            r_head = r;
        } else {
            R.prev = r_tail;
            R.next = -1;
            if (R.prev < 0) r_head = r; else row[R.prev].next = r;
            r_tail = r;
        }
    }
    void row_unlink(int r)
    {
        const Row &R = row[r];
        if (R.prev < 0) r_head = R.next; else row[R.prev].next = R.next;
        if (R.next < 0) r_tail = R.prev; else row[R.next].prev = R.prev;
    }
    void col_insert(int c, bool front)
    {
        Col &C = col[c];
        if (front) {
            C.prev = -1;
            C.next = c_head;
            if (C.next < 0) c_tail = c; else col[C.next].prev = c;
            c_head = c;
        } else {
            C.prev = c_tail;
            C.next = -1;
            if (C.prev < 0) c_head = c; else col[C.prev].next = c;
            c_tail = c;
        }
    }
    void col_unlink(int c)
    {
        const Col &C = col[c];
        if (C.prev < 0) c_head = C.next; else col[C.prev].next = C.next;
        if (C.next < 0) c_tail = C.prev; else col[C.next].prev = C.prev;
    }
    void activate_row(int r)
    {
        if (!row[r].temp) {
            row[r].temp = 1;
            row_unlink(r);
            row_insert(r, true);
        }
    }
    void deactivate_row(int r)
    {
        if (row[r].temp) {
            row[r].temp = 0;
            row_unlink(r);
            row_insert(r, false);
        }
    }
    void activate_col(int c)
    {
        if (!col[c].temp) {
            col[c].temp = 1;
            col_unlink(c);
            col_insert(c, true);
        }
    }
    void deactivate_col(int c)
    {
        if (col[c].temp) {
            col[c].temp = 0;
            col_unlink(c);
            col_insert(c, false);
        }
    }
    int add_row()
    {
        row.emplace_back();
        const int r = (int)row.size() - 1;
        row_insert(r, false);
        return r;
    }
    int add_col()
    {
        col.emplace_back();
        const int c = (int)col.size() - 1;
        col_insert(c, false);
        return c;
    }
    // a new element goes to the front of its row and column lists (:164)
    int add_aij(int r, int c, double v)
    {
        a.push_back(Aij{r, c, v, -1, row[r].ptr, -1, col[c].ptr});
        const int e = (int)a.size() - 1;
        if (a[e].r_next >= 0) a[a[e].r_next].r_prev = e;
        if (a[e].c_next >= 0) a[a[e].c_next].c_prev = e;
        row[r].ptr = col[c].ptr = e;
        return e;
    }
    void del_row(int r)
    {
        // npp_erase_row + npp_remove_row (:209-228)
        while (row[r].ptr >= 0) {
            const Aij &e = a[row[r].ptr];
            row[r].ptr = e.r_next;
            if (e.c_prev < 0) col[e.col].ptr = e.c_next; else a[e.c_prev].c_next = e.c_next;
            if (e.c_next >= 0) a[e.c_next].c_prev = e.c_prev;
        }
        row_unlink(r);
    }
    void del_col(int c)
    {
        // :230
        while (col[c].ptr >= 0) {
            const Aij &e = a[col[c].ptr];
            col[c].ptr = e.c_next;
            if (e.r_prev < 0) row[e.row].ptr = e.r_next; else a[e.r_prev].r_next = e.r_next;
            if (e.r_next >= 0) a[e.r_next].r_prev = e.r_prev;
        }
        col_unlink(c);
    }
    Tse &push(int kind)
    {
        tse.push_back(Tse{});
        tse.back().kind = kind;
        return tse.back();
    }
    // the saved coefficient list of the entry being built, as lfe[beg, end)
    int lfe_mark() const { return (int)lfe.size(); }

    // ---- glpnpp02.js ----------------------------------------------------
    void free_row(int p)
    {
        if (!(row[p].lb == -BIG && row[p].ub == +BIG)) throw NppFail("npp_free_row: row is not free");
        Tse &t = push(T_FREE_ROW);
        t.p = p + 1;
        del_row(p);
    }
    // substitute x[q] = s into the objective and the rows of column q
    void substitute(int q, double s)
    {
        c0 += col[q].coef * s;
        for (int e = col[q].ptr; e >= 0; e = a[e].c_next) {
            Row &I = row[a[e].row];
            if (I.lb == I.ub)
                I.ub = (I.lb -= a[e].val * s);
            else {
                if (I.lb != -BIG) I.lb -= a[e].val * s;
                if (I.ub != +BIG) I.ub -= a[e].val * s;
            }
        }
    }
    void fixed_col(int q)
    {
        if (col[q].lb != col[q].ub) throw NppFail("npp_fixed_col: column is not fixed");
        Tse &t = push(T_FIXED_COL);
        t.q = q + 1;
        t.s = col[q].lb;
        substitute(q, col[q].lb);
        del_col(q);
    }
    int make_equality(int p)
    {
        Row &P = row[p];
        const double eps = 1e-9 + 1e-12 * std::fabs(P.lb);
        if (P.ub - P.lb > eps) return 0;
        Tse &t = push(T_MAKE_EQ);
        t.p = p + 1;
        double b = 0.5 * (P.ub + P.lb);
        const double nint = std::floor(b + 0.5);
        if (std::fabs(b - nint) <= eps) b = nint;
        P.lb = P.ub = b;
        return 1;
    }
    int make_fixed(int q)
    {
        Col &Q = col[q];
        const double eps = 1e-9 + 1e-12 * std::fabs(Q.lb);
        if (Q.ub - Q.lb > eps) return 0;
        const int lb = lfe_mark();
        if (sol == SOL)
            for (int e = Q.ptr; e >= 0; e = a[e].c_next) lfe.push_back(Lfe{a[e].row + 1, a[e].val});
        Tse &t = push(T_MAKE_FIXED);
        t.q = q + 1;
        t.c = Q.coef;
        t.lb_ = lb;
        t.le_ = lfe_mark();
        double s = 0.5 * (Q.ub + Q.lb);
        const double nint = std::floor(s + 0.5);
        if (std::fabs(s - nint) <= eps) s = nint;
        Q.lb = Q.ub = s;
        return 1;
    }

    // ---- glpnpp03.js ----------------------------------------------------
    int empty_row(int p)
    {
        const double eps = 1e-3;
        if (row[p].lb > +eps || row[p].ub < -eps) return 1;
        row[p].lb = -BIG;
        row[p].ub = +BIG;
        free_row(p);
        return 0;
    }
    int empty_col(int q)
    {
        const double eps = 1e-3;
        Col &Q = col[q];
        if (Q.coef > +eps && Q.lb == -BIG) return 1;
        if (Q.coef < -eps && Q.ub == +BIG) return 1;
        int stat;
        auto at_lb = [&] { stat = NL; Q.ub = Q.lb; };
        auto at_ub = [&] { stat = NU; Q.lb = Q.ub; };
        if (Q.lb == -BIG && Q.ub == +BIG) {
            stat = NF;
            Q.lb = Q.ub = 0.0;
        } else if (Q.ub == +BIG)
            at_lb();
        else if (Q.lb == -BIG)
            at_ub();
        else if (Q.lb != Q.ub) {
            if (Q.coef >= +DBL_EPSILON) at_lb();
            else if (Q.coef <= -DBL_EPSILON) at_ub();
            else if (std::fabs(Q.lb) <= std::fabs(Q.ub)) at_lb();
            else at_ub();
        } else
            stat = NS;
        Tse &t = push(T_EMPTY_COL);
        t.q = q + 1;
        t.stat = stat;
        fixed_col(q);
        return 0;
    }
    int implied_value(int q, double s)
    {
        Col &Q = col[q];
        if (Q.is_int) {
            const double nint = std::floor(s + 0.5);
            if (std::fabs(s - nint) <= 1e-5) s = nint;
            else return 2;
        }
        if (Q.lb != -BIG) {
            const double eps = Q.is_int ? 1e-5 : 1e-5 + 1e-8 * std::fabs(Q.lb);
            if (s < Q.lb - eps) return 1;
            if (s < Q.lb + 1e-3 * eps) {
                Q.ub = Q.lb;
                return 0;
            }
        }
        if (Q.ub != +BIG) {
            const double eps = Q.is_int ? 1e-5 : 1e-5 + 1e-8 * std::fabs(Q.ub);
            if (s > Q.ub + eps) return 1;
            if (s > Q.ub - 1e-3 * eps) {
                Q.lb = Q.ub;
                return 0;
            }
        }
        Q.lb = Q.ub = s;
        return 0;
    }
    int eq_singlet(int p)
    {
        const int e0 = row[p].ptr;
        const int q = a[e0].col;
        const double apq = a[e0].val;
        const int ret = implied_value(q, row[p].lb / apq);
        if (ret != 0) return ret;
        const int lb = lfe_mark();
        if (sol != MIP)
            for (int e = col[q].ptr; e >= 0; e = a[e].c_next)
                if (a[e].row != p) lfe.push_back(Lfe{a[e].row + 1, a[e].val});
        Tse &t = push(T_EQ_SINGLET);
        t.p = p + 1;
        t.q = q + 1;
        t.apq = apq;
        t.c = col[q].coef;
        t.lb_ = lb;
        t.le_ = lfe_mark();
        del_row(p);
        return 0;
    }
    int implied_lower(int q, double l)
    {
        Col &Q = col[q];
        if (Q.is_int) {
            const double nint = std::floor(l + 0.5);
            l = std::fabs(l - nint) <= 1e-5 ? nint : std::ceil(l);
        }
        if (Q.lb != -BIG) {
            const double eps = Q.is_int ? 1e-3 : 1e-3 + 1e-6 * std::fabs(Q.lb);
            if (l < Q.lb + eps) return 0;                       // redundant
        }
        if (Q.ub != +BIG) {
            const double eps = Q.is_int ? 1e-5 : 1e-5 + 1e-8 * std::fabs(Q.ub);
            if (l > Q.ub + eps) return 4;                       // infeasible
            if (l > Q.ub - 1e-3 * eps) {
                Q.lb = Q.ub;
                return 3;                                       // fixed
            }
        }
        int ret;
        if (Q.lb == -BIG) ret = 2;
        else if (Q.is_int && l > Q.lb + 0.5) ret = 2;
        else if (l > Q.lb + 0.30 * (1.0 + std::fabs(Q.lb))) ret = 2;
        else ret = 1;
        Q.lb = l;
        return ret;
    }
    int implied_upper(int q, double u)
    {
        Col &Q = col[q];
        if (Q.is_int) {
            const double nint = std::floor(u + 0.5);
            u = std::fabs(u - nint) <= 1e-5 ? nint : std::floor(u);
        }
        if (Q.ub != +BIG) {
            const double eps = Q.is_int ? 1e-3 : 1e-3 + 1e-6 * std::fabs(Q.ub);
            if (u > Q.ub - eps) return 0;
        }
        if (Q.lb != -BIG) {
            const double eps = Q.is_int ? 1e-5 : 1e-5 + 1e-8 * std::fabs(Q.lb);
            if (u < Q.lb - eps) return 4;
            if (u < Q.lb + 1e-3 * eps) {
                Q.ub = Q.lb;
                return 3;
            }
        }
        int ret;
        if (Q.ub == +BIG) ret = 2;
        else if (Q.is_int && u < Q.ub - 0.5) ret = 2;
        else if (u < Q.ub - 0.30 * (1.0 + std::fabs(Q.ub))) ret = 2;
        else ret = 1;
        Q.ub = u;
        return ret;
    }
    int ineq_singlet(int p)
    {
        const int e0 = row[p].ptr;
        const int q = a[e0].col;
        const double apq = a[e0].val;
        const Row &P = row[p];
        double ll, uu;
        if (apq > 0.0) {
            ll = P.lb == -BIG ? -BIG : P.lb / apq;
            uu = P.ub == +BIG ? +BIG : P.ub / apq;
        } else {
            ll = P.ub == +BIG ? -BIG : P.ub / apq;
            uu = P.lb == -BIG ? +BIG : P.lb / apq;
        }
        int lbc = 0, ubc = 0;
        if (ll != -BIG) {
            lbc = implied_lower(q, ll);
            if (lbc == 4) return 4;
        }
        if (uu != +BIG && lbc != 3) {
            ubc = implied_upper(q, uu);
            if (ubc == 4) return 4;
        }
        if (!lbc && !ubc) {
            row[p].lb = -BIG;
            row[p].ub = +BIG;
            free_row(p);
            return 0;
        }
        const int lb = lfe_mark();
        if (sol != MIP)
            for (int e = col[q].ptr; e >= 0; e = a[e].c_next)
                if (e != e0) lfe.push_back(Lfe{a[e].row + 1, a[e].val});
        Tse &t = push(T_INEQ_SINGLET);
        t.p = p + 1;
        t.q = q + 1;
        t.apq = apq;
        t.c = col[q].coef;
        t.lb = row[p].lb;
        t.ub = row[p].ub;
        t.lb_changed = lbc;
        t.ub_changed = ubc;
        t.lb_ = lb;
        t.le_ = lfe_mark();
        del_row(p);
        return lbc >= ubc ? lbc : ubc;
    }
    void implied_slack(int q)
    {
        const int e0 = col[q].ptr;
        const int p = a[e0].row;
        const double apq = a[e0].val, b = row[p].lb, c = col[q].coef;
        const int lb = lfe_mark();
        for (int e = row[p].ptr; e >= 0; e = a[e].r_next) {
            if (a[e].col == q) continue;
            lfe.push_back(Lfe{a[e].col + 1, a[e].val});
            col[a[e].col].coef -= c * (a[e].val / apq);
        }
        Tse &t = push(T_IMPL_SLACK);
        t.p = p + 1;
        t.q = q + 1;
        t.apq = apq;
        t.b = b;
        t.c = c;
        t.lb_ = lb;
        t.le_ = lfe_mark();
        c0 += c * (b / apq);
        const Col &Q = col[q];
        Row &P = row[p];
        if (apq > 0.0) {
            P.lb = Q.ub == +BIG ? -BIG : b - apq * Q.ub;
            P.ub = Q.lb == -BIG ? +BIG : b - apq * Q.lb;
        } else {
            P.lb = Q.lb == -BIG ? -BIG : b - apq * Q.lb;
            P.ub = Q.ub == +BIG ? +BIG : b - apq * Q.ub;
        }
        del_col(q);
    }
    int implied_free(int q)
    {
        const int e0 = col[q].ptr;
        const int p = a[e0].row;
        const double apq = a[e0].val;
        Row &P = row[p];
        double alfa = P.lb;
        if (alfa != -BIG)
            for (int e = P.ptr; e >= 0; e = a[e].r_next) {
                if (e == e0) continue;
                const Col &J = col[a[e].col];
                if (a[e].val > 0.0) {
                    if (J.ub == +BIG) { alfa = -BIG; break; }
                    alfa -= a[e].val * J.ub;
                } else {
                    if (J.lb == -BIG) { alfa = -BIG; break; }
                    alfa -= a[e].val * J.lb;
                }
            }
        double beta = P.ub;
        if (beta != +BIG)
            for (int e = P.ptr; e >= 0; e = a[e].r_next) {
                if (e == e0) continue;
                const Col &J = col[a[e].col];
                if (a[e].val > 0.0) {
                    if (J.lb == -BIG) { beta = +BIG; break; }
                    beta -= a[e].val * J.lb;
                } else {
                    if (J.ub == +BIG) { beta = +BIG; break; }
                    beta -= a[e].val * J.ub;
                }
            }
        double l, u;
        if (apq > 0.0) {
            l = alfa == -BIG ? -BIG : alfa / apq;
            u = beta == +BIG ? +BIG : beta / apq;
        } else {
            l = beta == +BIG ? -BIG : beta / apq;
            u = alfa == -BIG ? +BIG : alfa / apq;
        }
        Col &Q = col[q];
        if (Q.lb != -BIG) {
            const double eps = 1e-9 + 1e-12 * std::fabs(Q.lb);
            if (l < Q.lb - eps) return 1;
        }
        if (Q.ub != +BIG) {
            const double eps = 1e-9 + 1e-12 * std::fabs(Q.ub);
            if (u > Q.ub + eps) return 1;
        }
        Q.lb = -BIG;
        Q.ub = +BIG;
        const int ti = (int)tse.size();
        Tse &t0 = push(T_IMPL_FREE);
        t0.p = p + 1;
        t0.stat = -1;
        const double pi = Q.coef / apq;
        auto at_lb = [&] { tse[ti].stat = NL; P.ub = P.lb; };
        auto at_ub = [&] { tse[ti].stat = NU; P.lb = P.ub; };
        if (pi > +DBL_EPSILON) {
            if (P.lb != -BIG) at_lb();
            else {
                if (pi > +1e-5) return 2;
                at_ub();
            }
        } else if (pi < -DBL_EPSILON) {
            if (P.ub != +BIG) at_ub();
            else {
                if (pi < -1e-5) return 2;
                at_lb();
            }
        } else {
            if (P.ub == +BIG) at_lb();
            else if (P.lb == -BIG) at_ub();
            else if (std::fabs(P.lb) <= std::fabs(P.ub)) at_lb();
            else at_ub();
        }
        return 0;
    }
    int forcing_row(int p, int at)
    {
        double big = 1.0;
        for (int e = row[p].ptr; e >= 0; e = a[e].r_next)
            if (big < std::fabs(a[e].val)) big = std::fabs(a[e].val);
        for (int e = row[p].ptr; e >= 0; e = a[e].r_next)
            if (std::fabs(a[e].val) < 1e-7 * big) return 1;
        const int ti = (int)tse.size();
        {
            Tse &t = push(T_FORCING);
            t.p = p + 1;
            if (row[p].lb == row[p].ub) t.stat = NS;
            else if (at == 0) t.stat = NL;
            else t.stat = NU;
            t.fb = (int)fcol.size();
        }
        for (int e = row[p].ptr; e >= 0; e = a[e].r_next) {
            const int j = a[e].col;
            Col &J = col[j];
            FCol fc{j + 1, -1, a[e].val, J.coef, 0, 0};
            const bool lower = (at == 0 && a[e].val < 0.0) || (at != 0 && a[e].val > 0.0);
            if (lower) {
                fc.stat = NL;
                J.ub = J.lb;
            } else {
                fc.stat = NU;
                J.lb = J.ub;
            }
            if (sol != MIP) {
                fc.lb = lfe_mark();
                for (int f = J.ptr; f >= 0; f = a[f].c_next)
                    if (f != e) lfe.push_back(Lfe{a[f].row + 1, a[f].val});
                fc.le = lfe_mark();
                fcol.push_back(fc);
            }
        }
        tse[ti].fe = (int)fcol.size();
        row[p].lb = -BIG;
        row[p].ub = +BIG;
        return 0;
    }
    int analyze_row(int p)
    {
        const Row &P = row[p];
        double l = 0.0, u = 0.0;
        for (int e = P.ptr; e >= 0; e = a[e].r_next) {
            const Col &J = col[a[e].col];
            if (a[e].val > 0.0) {
                if (J.lb == -BIG) { l = -BIG; break; }
                l += a[e].val * J.lb;
            } else {
                if (J.ub == +BIG) { l = -BIG; break; }
                l += a[e].val * J.ub;
            }
        }
        for (int e = P.ptr; e >= 0; e = a[e].r_next) {
            const Col &J = col[a[e].col];
            if (a[e].val > 0.0) {
                if (J.ub == +BIG) { u = +BIG; break; }
                u += a[e].val * J.ub;
            } else {
                if (J.lb == -BIG) { u = +BIG; break; }
                u += a[e].val * J.lb;
            }
        }
        if (P.lb != -BIG && P.lb - (1e-3 + 1e-6 * std::fabs(P.lb)) > u) return 0x33;
        if (P.ub != +BIG && P.ub + (1e-3 + 1e-6 * std::fabs(P.ub)) < l) return 0x33;
        int ret = 0;
        if (P.lb != -BIG) {
            const double eps = 1e-9 + 1e-12 * std::fabs(P.lb);
            if (P.lb - eps > l) ret |= (P.lb + eps <= u) ? 0x01 : 0x02;
        }
        if (P.ub != +BIG) {
            const double eps = 1e-9 + 1e-12 * std::fabs(P.ub);
            if (P.ub + eps < u) ret |= (P.ub - eps >= l) ? 0x10 : 0x20;
        }
        return ret;
    }
    void inactive_bound(int p, int which)
    {
        Row &P = row[p];
        if (sol == SOL) {
            Tse &t = push(T_INACTIVE);
            t.p = p + 1;
            if (P.ub == +BIG) t.stat = NL;
            else if (P.lb == -BIG) t.stat = NU;
            else if (P.lb != P.ub) t.stat = which == 0 ? NU : NL;
            else t.stat = NS;
        }
        if (which == 0) P.lb = -BIG;
        else P.ub = +BIG;
    }
    void implied_bounds(int p)
    {
        const Row &P = row[p];
        double big = 1.0;
        for (int e = P.ptr; e >= 0; e = a[e].r_next) {
            col[a[e].col].ll = -BIG;
            col[a[e].col].uu = +BIG;
            if (big < std::fabs(a[e].val)) big = std::fabs(a[e].val);
        }
        const double eps = 1e-6 * big;
        // row lower bound (assumed active): the columns that can make the
        // activity unbounded above, at most one of them
        for (int side = 0; side < 2; side++) {
            const double bnd = side == 0 ? P.lb : P.ub;
            if (side == 0 ? bnd == -BIG : bnd == +BIG) continue;
            int k = -1;
            bool skip = false;
            for (int e = P.ptr; e >= 0; e = a[e].r_next) {
                const Col &J = col[a[e].col];
                const bool open = side == 0 ? ((a[e].val > 0.0 && J.ub == +BIG) || (a[e].val < 0.0 && J.lb == -BIG))
                                            : ((a[e].val > 0.0 && J.lb == -BIG) || (a[e].val < 0.0 && J.ub == +BIG));
                if (open) {
                    if (k < 0) k = e;
                    else { skip = true; break; }
                }
            }
            if (skip) continue;
            double temp = bnd;
            for (int e = P.ptr; e >= 0; e = a[e].r_next) {
                if (e == k) continue;
                const Col &J = col[a[e].col];
                if (side == 0) temp -= a[e].val * (a[e].val > 0.0 ? J.ub : J.lb);
                else temp -= a[e].val * (a[e].val > 0.0 ? J.lb : J.ub);
            }
            if (k < 0) {
                for (int e = P.ptr; e >= 0; e = a[e].r_next) {
                    Col &J = col[a[e].col];
                    if (side == 0) {
                        if (a[e].val >= +eps) J.ll = J.ub + temp / a[e].val;
                        else if (a[e].val <= -eps) J.uu = J.lb + temp / a[e].val;
                    } else {
                        if (a[e].val >= +eps) J.uu = J.lb + temp / a[e].val;
                        else if (a[e].val <= -eps) J.ll = J.ub + temp / a[e].val;
                    }
                }
            } else {
                Col &K = col[a[k].col];
                if (side == 0) {
                    if (a[k].val >= +eps) K.ll = temp / a[k].val;
                    else if (a[k].val <= -eps) K.uu = temp / a[k].val;
                } else {
                    if (a[k].val >= +eps) K.uu = temp / a[k].val;
                    else if (a[k].val <= -eps) K.ll = temp / a[k].val;
                }
            }
        }
    }

    // ---- glpnpp04.js (MIP) ----------------------------------------------
    void lbnd_col(int q)
    {
        Col &Q = col[q];
        Tse &t = push(T_LBND_COL);
        t.q = q + 1;
        t.s = Q.lb;
        c0 += Q.coef * Q.lb;
        for (int e = Q.ptr; e >= 0; e = a[e].c_next) {
            Row &I = row[a[e].row];
            if (I.lb == I.ub)
                I.ub = (I.lb -= a[e].val * Q.lb);
            else {
                if (I.lb != -BIG) I.lb -= a[e].val * Q.lb;
                if (I.ub != +BIG) I.ub -= a[e].val * Q.lb;
            }
        }
        if (Q.ub != +BIG) Q.ub -= Q.lb;
        Q.lb = 0.0;
    }
    // counts: nvars, nbins, nrows, nfails
    void binarize(int cnt[4])
    {
        int nfails = 0, nvars = 0, nbins = 0, nrows = 0;
        for (int c = c_tail; c >= 0; c = col[c].prev) {
            if (!col[c].is_int) continue;
            if (col[c].lb == col[c].ub) continue;
            if (col[c].lb == 0.0 && col[c].ub == 1.0) continue;
            if (col[c].lb < -1e6 || col[c].ub > +1e6 || col[c].ub - col[c].lb > 4095.0) {
                nfails++;
                continue;
            }
            nvars++;
            if (col[c].lb != 0.0) lbnd_col(c);
            const int u = (int)col[c].ub;
            if ((double)u != col[c].ub) throw NppFail("npp_binarize_prob: upper bound not integral");
            if (u == 1) continue;
            int nbit = 2;
            double temp = 4.0;
            while (u >= temp) {
                nbit++;
                temp += temp;
            }
            nbins += nbit;
            const int ti = (int)tse.size();
            {
                Tse &t = push(T_BINARIZE);
                t.q = c + 1;
                t.j0 = 0;
                t.nb = nbit;
            }
            int r = -1;
            if (u < temp - 1) {
                r = add_row();
                nrows++;
                row[r].lb = -BIG;
                row[r].ub = u;
            }
            col[c].ub = 1.0;
            if (r >= 0) add_aij(r, c, 1.0);
            double w = 2.0;
            for (int k = 1; k < nbit; k++, w += w) {
                const int b = add_col();
                col[b].is_int = 1;
                col[b].lb = 0.0;
                col[b].ub = 1.0;
                col[b].coef = w * col[c].coef;
                if (tse[ti].j0 == 0) tse[ti].j0 = b + 1;
                else if (tse[ti].j0 + (k - 1) != b + 1) throw NppFail("npp_binarize_prob: column numbering");
                for (int e = col[c].ptr; e >= 0; e = a[e].c_next) add_aij(a[e].row, b, w * a[e].val);
            }
        }
        cnt[0] = nvars;
        cnt[1] = nbins;
        cnt[2] = nrows;
        cnt[3] = nfails;
    }
    std::vector<Term> copy_form(int r, double sg) const
    {
        std::vector<Term> f;
        for (int e = row[r].ptr; e >= 0; e = a[e].r_next) f.push_back(Term{sg * a[e].val, a[e].col});
        return std::vector<Term>(f.rbegin(), f.rend());
    }
    bool is_bin(int c) const { return col[c].is_int && col[c].lb == 0.0 && col[c].ub == 1.0; }
    // 0 / 1 (already packing) / 2 (hidden packing; f and b rewritten)
    int hidden_packing(std::vector<Term> &f, double &b) const
    {
        int neg = 0;
        size_t k = 0;
        for (; k < f.size(); k++) {
            if (f[k].aj == +1.0) {
            } else if (f[k].aj == -1.0)
                neg++;
            else
                break;
        }
        if (k == f.size() && b == (double)(1 - neg)) return 1;
        double bb = b;
        for (const Term &e : f)
            if (e.aj < 0) bb -= e.aj;
        for (const Term &e : f)
            if (std::fabs(e.aj) > bb) return 0;
        int ej = -1, ek = -1;
        for (int t = 0; t < (int)f.size(); t++)
            if (ej < 0 || std::fabs(f[ej].aj) > std::fabs(f[t].aj)) ej = t;
        for (int t = 0; t < (int)f.size(); t++)
            if (t != ej && (ek < 0 || std::fabs(f[ek].aj) > std::fabs(f[t].aj))) ek = t;
        if (ej < 0 || ek < 0) throw NppFail("hidden_packing: fewer than two terms");
        const double eps = 1e-3 + 1e-6 * std::fabs(bb);
        if (std::fabs(f[ej].aj) + std::fabs(f[ek].aj) <= bb + eps) return 0;
        double nb = 1.0;
        for (Term &e : f) {
            if (e.aj > 0.0) e.aj = +1.0;
            else {
                e.aj = -1.0;
                nb -= 1.0;
            }
        }
        b = nb;
        return 2;
    }
    int hidden_covering(std::vector<Term> &f, double &b) const
    {
        int neg = 0;
        size_t k = 0;
        for (; k < f.size(); k++) {
            if (f[k].aj == +1.0) {
            } else if (f[k].aj == -1.0)
                neg++;
            else
                break;
        }
        if (k == f.size() && b == (double)(1 - neg)) return 1;
        double bb = b;
        for (const Term &e : f)
            if (e.aj < 0) bb -= e.aj;
        if (bb < 1e-3) return 0;
        const double eps = 1e-9 + 1e-12 * std::fabs(bb);
        for (const Term &e : f)
            if (std::fabs(e.aj) < bb - eps) return 0;
        double nb = 1.0;
        for (Term &e : f) {
            if (e.aj > 0.0) e.aj = +1.0;
            else {
                e.aj = -1.0;
                nb -= 1.0;
            }
        }
        b = nb;
        return 2;
    }
    int reduce_coef(std::vector<Term> &f, double &b) const
    {
        int count = 0;
        double h = 0.0;
        for (const Term &e : f) {
            if (e.aj > 0.0) {
                if (col[e.xj].lb == -BIG) return count;
                h += e.aj * col[e.xj].lb;
            } else {
                if (col[e.xj].ub == +BIG) return count;
                h += e.aj * col[e.xj].ub;
            }
        }
        for (Term &e : f) {
            if (!is_bin(e.xj)) continue;
            if (e.aj > 0.0) {
                const double inf_t = h;
                if (b - e.aj < inf_t && inf_t < b) {
                    const double new_a = b - inf_t;
                    if (new_a >= +1e-3 && e.aj - new_a >= 0.01 * (1.0 + e.aj)) {
                        e.aj = new_a;
                        count++;
                    }
                }
            } else {
                const double inf_t = h - e.aj;
                if (b < inf_t && inf_t < b - e.aj) {
                    const double new_a = e.aj + (inf_t - b);
                    if (new_a <= -1e-3 && new_a - e.aj >= 0.01 * (1.0 - e.aj)) {
                        e.aj = new_a;
                        h += (inf_t - b);
                        b = inf_t;
                        count++;
                    }
                }
            }
        }
        return count;
    }
    void erase_row(int r)
    {
        while (row[r].ptr >= 0) {
            const Aij &e = a[row[r].ptr];
            row[r].ptr = e.r_next;
            if (e.c_prev < 0) col[e.col].ptr = e.c_next; else a[e.c_prev].c_next = e.c_next;
            if (e.c_next >= 0) a[e.c_next].c_prev = e.c_prev;
        }
    }
    // the replacement step shared by npp_hidden_packing / _covering /
    // npp_reduce_ineq_coef: a copy of the row for its other bound (a
    // double-sided row), then the row rewritten from the form; returns the
    // row that carries on (the copy, if made)
    int replace_row(int r, const std::vector<Term> &f, double lb, double ub, bool copy_keeps_lb)
    {
        int cp = -1;
        if (!(row[r].lb == -BIG || row[r].ub == +BIG)) {
            cp = add_row();
            if (copy_keeps_lb) {
                row[cp].lb = row[r].lb;
                row[cp].ub = +BIG;
            } else {
                row[cp].lb = -BIG;
                row[cp].ub = row[r].ub;
            }
            for (int e = row[r].ptr; e >= 0; e = a[e].r_next) add_aij(cp, a[e].col, a[e].val);
        }
        erase_row(r);
        row[r].lb = lb;
        row[r].ub = ub;
        for (const Term &e : f) add_aij(r, e.xj, e.aj);
        return cp >= 0 ? cp : r;
    }
    int npp_hidden_packing(int r)
    {
        int count = 0;
        for (int kase = 0; kase <= 1; kase++) {
            std::vector<Term> f;
            double b;
            if (kase == 0) {
                if (row[r].ub == +BIG) continue;
                f = copy_form(r, +1.0);
                b = +row[r].ub;
            } else {
                if (row[r].lb == -BIG) continue;
                f = copy_form(r, -1.0);
                b = -row[r].lb;
            }
            const int ret = hidden_packing(f, b);
            if ((kase == 1 && ret == 1) || ret == 2) {
                count++;
                r = replace_row(r, f, -BIG, b, kase == 0);
            }
        }
        return count;
    }
    int npp_hidden_covering(int r)
    {
        int count = 0;
        for (int kase = 0; kase <= 1; kase++) {
            std::vector<Term> f;
            double b;
            if (kase == 0) {
                if (row[r].lb == -BIG) continue;
                f = copy_form(r, +1.0);
                b = +row[r].lb;
            } else {
                if (row[r].ub == +BIG) continue;
                f = copy_form(r, -1.0);
                b = -row[r].ub;
            }
            const int ret = hidden_covering(f, b);
            if ((kase == 1 && ret == 1) || ret == 2) {
                count++;
                r = replace_row(r, f, b, +BIG, kase == 1);
            }
        }
        return count;
    }
    int npp_reduce_ineq_coef(int r)
    {
        int count[2] = {0, 0};
        for (int kase = 0; kase <= 1; kase++) {
            std::vector<Term> f;
            double b;
            if (kase == 0) {
                if (row[r].lb == -BIG) continue;
                f = copy_form(r, +1.0);
                b = +row[r].lb;
            } else {
                if (row[r].ub == +BIG) continue;
                f = copy_form(r, -1.0);
                b = -row[r].ub;
            }
            count[kase] = reduce_coef(f, b);
            if (count[kase] > 0) r = replace_row(r, f, b, +BIG, kase == 1);
        }
        return count[0] + count[1];
    }
    // npp_integer (glpnpp05.js:437); msg[0..6]: binarize counts (nvars,
    // nbins, nrows, nfails), hidden packing, hidden covering, reduced
    int integer(int bin, int msg[7])
    {
        for (int k = 0; k < 7; k++) msg[k] = 0;
        int ret = process_prob(1);
        if (ret != 0) return ret;
        if (bin) binarize(msg);
        auto all_binary = [&](int r) {
            for (int e = row[r].ptr; e >= 0; e = a[e].r_next)
                if (!is_bin(a[e].col)) return false;
            return true;
        };
        int count = 0;
        for (int r = r_tail, pv; r >= 0; r = pv) {
            pv = row[r].prev;
            if (row[r].lb == -BIG && row[r].ub == +BIG) continue;
            if (row[r].lb == row[r].ub) continue;
            if (row[r].ptr < 0 || a[row[r].ptr].r_next < 0) continue;
            if (!all_binary(r)) continue;
            count += npp_hidden_packing(r);
        }
        msg[4] = count;
        count = 0;
        for (int r = r_tail, pv; r >= 0; r = pv) {
            pv = row[r].prev;
            if (row[r].lb == -BIG && row[r].ub == +BIG) continue;
            if (row[r].lb == row[r].ub) continue;
            if (row[r].ptr < 0 || a[row[r].ptr].r_next < 0 || a[a[row[r].ptr].r_next].r_next < 0) continue;
            if (!all_binary(r)) continue;
            count += npp_hidden_covering(r);
        }
        msg[5] = count;
        count = 0;
        for (int r = r_tail, pv; r >= 0; r = pv) {
            pv = row[r].prev;
            if (row[r].lb == row[r].ub) continue;
            count += npp_reduce_ineq_coef(r);
        }
        msg[6] = count;
        return 0;
    }

    // ---- glpnpp05.js ----------------------------------------------------
    void clean_prob()
    {
        for (int r = r_head, nx; r >= 0; r = nx) {
            nx = row[r].next;
            if (row[r].lb == -BIG && row[r].ub == +BIG) free_row(r);
        }
        for (int r = r_head, nx; r >= 0; r = nx) {
            nx = row[r].next;
            if (row[r].lb != -BIG && row[r].ub != +BIG && row[r].lb < row[r].ub) make_equality(r);
        }
        for (int c = c_head, nx; c >= 0; c = nx) {
            nx = col[c].next;
            if (col[c].lb == col[c].ub) fixed_col(c);
        }
        for (int c = c_head, nx; c >= 0; c = nx) {
            nx = col[c].next;
            if (col[c].lb != -BIG && col[c].ub != +BIG && col[c].lb < col[c].ub)
                if (make_fixed(c) == 1) fixed_col(c);
        }
    }
    void activate_rows_of(int c)
    {
        for (int e = col[c].ptr; e >= 0; e = a[e].c_next) activate_row(a[e].row);
    }
    int process_row(int p, int hard)
    {
        if (row[p].ptr < 0) return empty_row(p) == 0 ? 0 : ENOPFS;
        const int e0 = row[p].ptr;
        if (a[e0].r_next < 0) {
            const int q = a[e0].col;
            if (row[p].lb == row[p].ub) {
                const int ret = eq_singlet(p);
                if (ret != 0) return ENOPFS;
                activate_rows_of(q);
                fixed_col(q);
                return 0;
            }
            const int ret = ineq_singlet(p);
            if (ret == 4) return ENOPFS;
            activate_col(q);
            if (ret >= 2) activate_rows_of(q);
            if (ret == 3) fixed_col(q);
            return 0;
        }
        const int ret = analyze_row(p);
        if (ret == 0x33) return ENOPFS;
        // columns fixed by a forcing row, then the (now empty) free row
        auto fixup = [&] {
            for (int e = row[p].ptr, nx; e >= 0; e = nx) {
                const int c = a[e].col;
                nx = a[e].r_next;
                activate_rows_of(c);
                fixed_col(c);
            }
            free_row(p);
            return 0;
        };
        if ((ret & 0x0F) == 0x00) {
            if (row[p].lb != -BIG) inactive_bound(p, 0);
        } else if ((ret & 0x0F) == 0x02) {
            if (forcing_row(p, 0) == 0) return fixup();
        }
        if ((ret & 0xF0) == 0x00) {
            if (row[p].ub != +BIG) inactive_bound(p, 1);
        } else if ((ret & 0xF0) == 0x20) {
            if (forcing_row(p, 1) == 0) return fixup();
        }
        if (row[p].lb == -BIG && row[p].ub == +BIG) {
            for (int e = row[p].ptr; e >= 0; e = a[e].r_next) activate_col(a[e].col);
            free_row(p);
            return 0;
        }
        if (sol == MIP && hard)
            if (improve_bounds(p, 1) < 0) return ENOPFS;
        return 0;
    }
    int improve_bounds(int p, int flag)
    {
        implied_bounds(p);
        int count = 0;
        for (int e = row[p].ptr, nx; e >= 0; e = nx) {
            const int c = a[e].col;
            nx = a[e].r_next;
            for (int kase = 0; kase <= 1; kase++) {
                const double lb = col[c].lb, ub = col[c].ub;
                int ret;
                if (kase == 0) {
                    if (col[c].ll == -BIG) continue;
                    ret = implied_lower(c, col[c].ll);
                } else {
                    if (col[c].uu == +BIG) continue;
                    ret = implied_upper(c, col[c].uu);
                }
                if (ret == 0 || ret == 1) {
                    col[c].lb = lb;
                    col[c].ub = ub;
                } else if (ret == 2 || ret == 3) {
                    count++;
                    if (flag)
                        for (int f = col[c].ptr; f >= 0; f = a[f].c_next)
                            if (a[f].row != p) activate_row(a[f].row);
                    if (ret == 3) {
                        fixed_col(c);
                        break;
                    }
                } else
                    return -1;
            }
        }
        return count;
    }
    int process_col(int q)
    {
        if (col[q].ptr < 0) return empty_col(q) == 0 ? 0 : ENODFS;
        const int e0 = col[q].ptr;
        if (a[e0].c_next >= 0) return 0;
        const int p = a[e0].row;
        auto slack = [&] {
            implied_slack(q);
            if (row[p].lb == -BIG && row[p].ub == +BIG) {
                for (int e = row[p].ptr; e >= 0; e = a[e].r_next) activate_col(a[e].col);
                free_row(p);
            } else
                activate_row(p);
            return 0;
        };
        if (row[p].lb == row[p].ub) {
            if (!col[q].is_int) return slack();
        } else if (!col[q].is_int) {
            const int ret = implied_free(q);
            if (ret == 0) return slack();
            if (ret == 2) return ENODFS;
        }
        return 0;
    }
    int process_prob(int hard)
    {
        clean_prob();
        for (int r = r_head; r >= 0; r = row[r].next) row[r].temp = 1;
        for (int c = c_head; c >= 0; c = col[c].next) col[c].temp = 1;
        for (bool again = true; again;) {
            again = false;
            while (r_head >= 0 && row[r_head].temp) {
                const int r = r_head;
                deactivate_row(r);
                const int ret = process_row(r, hard);
                if (ret != 0) return ret;
                again = true;
            }
            while (c_head >= 0 && col[c_head].temp) {
                const int c = c_head;
                deactivate_col(c);
                const int ret = process_col(c);
                if (ret != 0) return ret;
                again = true;
            }
        }
        if (sol == MIP && !hard)
            for (int r = r_head; r >= 0; r = row[r].next)
                if (improve_bounds(r, 0) < 0) return ENOPFS;
        return 0;
    }

    // ---- recovery (the stack entries' routines) ---------------------------
    [[noreturn]] static void fail(const Tse &t)
    {
        throw NppFail("npp_postprocess: recovery of stack entry kind " + std::to_string(t.kind) + " failed");
    }
    void recover(const Tse &t)
    {
        auto rs = [&](int p) -> signed char & { return r_stat[p]; };
        auto cs = [&](int q) -> signed char & { return c_stat[q]; };
        switch (t.kind) {
        case T_FREE_ROW:
            if (sol == SOL) rs(t.p) = BS;
            if (sol != MIP) r_pi[t.p] = 0.0;
            return;
        case T_FIXED_COL:
            if (sol == SOL) cs(t.q) = NS;
            c_value[t.q] = t.s;
            return;
        case T_MAKE_EQ:
            if (sol == SOL) {
                if (rs(t.p) == BS) {
                } else if (rs(t.p) == NS)
                    rs(t.p) = r_pi[t.p] >= 0.0 ? NL : NU;
                else
                    fail(t);
            }
            return;
        case T_MAKE_FIXED:
            if (sol == SOL) {
                if (cs(t.q) == BS) {
                } else if (cs(t.q) == NS) {
                    double lambda = t.c;
                    for (int k = t.le_ - 1; k >= t.lb_; k--) lambda -= lfe[k].val * r_pi[lfe[k].ref];
                    cs(t.q) = lambda >= 0.0 ? NL : NU;
                } else
                    fail(t);
            }
            return;
        case T_EMPTY_COL:
            if (sol == SOL) cs(t.q) = (signed char)t.stat;
            return;
        case T_EQ_SINGLET:
            if (sol == SOL) {
                if (cs(t.q) != NS) fail(t);
                rs(t.p) = NS;
                cs(t.q) = BS;
            }
            if (sol != MIP) {
                double temp = t.c;
                for (int k = t.le_ - 1; k >= t.lb_; k--) temp -= lfe[k].val * r_pi[lfe[k].ref];
                r_pi[t.p] = temp / t.apq;
            }
            return;
        case T_INEQ_SINGLET: {
            if (sol == MIP) return;
            double lambda = t.c;
            for (int k = t.le_ - 1; k >= t.lb_; k--) lambda -= lfe[k].val * r_pi[lfe[k].ref];
            if (sol == SOL) {
                auto nl = [&] {
                    if (t.lb_changed) {
                        rs(t.p) = t.apq > 0.0 ? NL : NU;
                        cs(t.q) = BS;
                        r_pi[t.p] = lambda / t.apq;
                    } else {
                        rs(t.p) = BS;
                        r_pi[t.p] = 0.0;
                    }
                };
                auto nu = [&] {
                    if (t.ub_changed) {
                        rs(t.p) = t.apq > 0.0 ? NU : NL;
                        cs(t.q) = BS;
                        r_pi[t.p] = lambda / t.apq;
                    } else {
                        rs(t.p) = BS;
                        r_pi[t.p] = 0.0;
                    }
                };
                const int st = cs(t.q);
                if (st == BS) {
                    rs(t.p) = BS;
                    r_pi[t.p] = 0.0;
                } else if (st == NL)
                    nl();
                else if (st == NU)
                    nu();
                else if (st == NS) {
                    if (lambda > +1e-7 &&
                        ((t.apq > 0.0 && t.lb != -BIG) || (t.apq < 0.0 && t.ub != +BIG) || !t.lb_changed)) {
                        cs(t.q) = NL;
                        nl();
                        return;
                    }
                    if (lambda < -1e-7 &&
                        ((t.apq > 0.0 && t.ub != +BIG) || (t.apq < 0.0 && t.lb != -BIG) || !t.ub_changed)) {
                        cs(t.q) = NU;
                        nu();
                        return;
                    }
                    if (t.lb != -BIG && t.ub == +BIG) rs(t.p) = NL;
                    else if (t.lb == -BIG && t.ub != +BIG) rs(t.p) = NU;
                    else if (t.lb != -BIG && t.ub != +BIG)
                        rs(t.p) = t.apq * c_value[t.q] <= 0.5 * (t.lb + t.ub) ? NL : NU;
                    else
                        fail(t);
                    cs(t.q) = BS;
                    r_pi[t.p] = lambda / t.apq;
                } else
                    fail(t);
            }
            if (sol == IPT) {
                if ((lambda > +DBL_EPSILON && t.lb_changed) || (lambda < -DBL_EPSILON && t.ub_changed))
                    r_pi[t.p] = lambda / t.apq;
                else
                    r_pi[t.p] = 0.0;
            }
            return;
        }
        case T_IMPL_SLACK: {
            if (sol == SOL) {
                const int st = rs(t.p);
                if (st == BS || st == NF) cs(t.q) = (signed char)st;
                else if (st == NL) cs(t.q) = t.apq > 0.0 ? NU : NL;
                else if (st == NU) cs(t.q) = t.apq > 0.0 ? NL : NU;
                else fail(t);
                rs(t.p) = NS;
            }
            if (sol != MIP) r_pi[t.p] += t.c / t.apq;
            double temp = t.b;
            for (int k = t.le_ - 1; k >= t.lb_; k--) temp -= lfe[k].val * c_value[lfe[k].ref];
            c_value[t.q] = temp / t.apq;
            return;
        }
        case T_IMPL_FREE:
            if (sol == SOL) {
                if (rs(t.p) == BS) {
                } else if (rs(t.p) == NS) {
                    if (!(t.stat == NL || t.stat == NU)) fail(t);
                    rs(t.p) = (signed char)t.stat;
                } else
                    fail(t);
            }
            return;
        case T_FORCING: {
            if (sol == MIP) return;
            if (sol == SOL) {
                if (rs(t.p) != BS) fail(t);
                for (int k = t.fe - 1; k >= t.fb; k--) {
                    if (cs(fcol[k].j) != NS) fail(t);
                    cs(fcol[k].j) = (signed char)fcol[k].stat;
                }
            }
            // reduced costs d[j] (glpnpp03.js:904-909), kept in a copy: the
            // stack is replayed only once, as the reference's is
            for (int k = t.fe - 1; k >= t.fb; k--) {
                double d = fcol[k].c;
                for (int l = fcol[k].le - 1; l >= fcol[k].lb; l--) d -= lfe[l].val * r_pi[lfe[l].ref];
                fcol[k].c = d;
            }
            int piv = -1;
            double big = 0.0;
            for (int k = t.fe - 1; k >= t.fb; k--) {
                const double d = fcol[k].c, temp = std::fabs(d / fcol[k].a);
                if (fcol[k].stat == NL) {
                    if (d < 0.0 && big < temp) { piv = k; big = temp; }
                } else if (fcol[k].stat == NU) {
                    if (d > 0.0 && big < temp) { piv = k; big = temp; }
                } else
                    fail(t);
            }
            if (piv >= 0) {
                if (sol == SOL) {
                    rs(t.p) = (signed char)t.stat;
                    cs(fcol[piv].j) = BS;
                }
                r_pi[t.p] = fcol[piv].c / fcol[piv].a;
            }
            return;
        }
        case T_LBND_COL:
            if (sol == SOL) {
                const int st = cs(t.q);
                if (!(st == BS || st == NL || st == NU)) fail(t);
            }
            c_value[t.q] = t.s + c_value[t.q];
            return;
        case T_BINARIZE: {
            double sum = c_value[t.q], w = 2.0;
            for (int k = 1; k < t.nb; k++, w += w) sum += w * c_value[t.j0 + (k - 1)];
            c_value[t.q] = sum;
            return;
        }
        case T_INACTIVE:
            if (sol != SOL) fail(t);
            if (rs(t.p) != BS) rs(t.p) = (signed char)t.stat;
            return;
        }
        fail(t);
    }
};

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
struct gk_npp : Npp {
};

namespace {
int guard_impl(const char *what, const std::function<int()> &f)
{
    try {
        return f();
    } catch (const NppFail &e) {
        gk::set_err("%s: %s", what, e.what());
    } catch (const std::exception &e) {
        gk::set_err("%s: %s", what, e.what());
    }
    return GK_EABI;
}
}  // namespace

extern "C" gk_npp *gk_npp_create(void)
{
    try {
        return new gk_npp();
    } catch (...) {
        gk::set_err("gk_npp_create: out of memory");
        return nullptr;
    }
}

extern "C" void gk_npp_destroy(gk_npp *npp) { delete npp; }

// npp_load_prob (glpnpp01.js:262) with names = GLP_OFF and scaling = GLP_OFF
// (the glp_simplex / glp_intopt presolve calls); col_kind NULL for sol = SOL
extern "C" int gk_npp_load(gk_npp *npp, const gk_lp *P, const signed char *col_kind, int sol)
{
    return guard_impl("gk_npp_load", [&]() -> int {
        if (!npp || !P || P->m < 0 || P->n < 0) throw NppFail("invalid arguments");
        if (!(sol == SOL || sol == MIP)) throw NppFail("sol = " + std::to_string(sol) + "; invalid");
        if (sol == MIP && !col_kind) throw NppFail("col_kind required for GLP_MIP");
        if (!npp->row.empty() || !npp->tse.empty()) throw NppFail("workspace already loaded");
        if (P->dir != 1 && P->dir != 2) throw NppFail("dir = " + std::to_string(P->dir) + "; invalid");
        const double dir = P->dir == 1 ? +1.0 : -1.0;
        const int m = P->m, n = P->n;
        npp->orig_dir = P->dir;
        npp->orig_m = m;
        npp->orig_n = n;
        npp->orig_nnz = P->nnz;
        npp->c0 = dir * P->c0;
        npp->row.reserve(m);
        npp->col.reserve(n);
        auto bounds = [](int type, double lb, double ub, double &l, double &u) {
            switch (type) {
            case FR: l = -BIG; u = +BIG; break;
            case LO: l = lb; u = +BIG; break;
            case UP: l = -BIG; u = ub; break;
            case DB: l = lb; u = ub; break;
            case FX: l = u = lb; break;
            default: throw NppFail("invalid bound type " + std::to_string(type));
            }
        };
        for (int i = 1; i <= m; i++) {
            const int r = npp->add_row();
            bounds(P->row_type[i], P->row_lb[i], P->row_ub[i], npp->row[r].lb, npp->row[r].ub);
        }
        npp->a.reserve((size_t)P->nnz);
        for (int j = 1; j <= n; j++) {
            const int c = npp->add_col();
            Col &C = npp->col[c];
            if (sol == MIP) C.is_int = col_kind[j] == 2 || col_kind[j] == 3;   // GLP_IV (GLP_BV)
            bounds(P->col_type[j], P->col_lb[j], P->col_ub[j], C.lb, C.ub);
            C.coef = dir * P->col_coef[j];
            for (int k = P->A_ptr[j]; k < P->A_ptr[j + 1]; k++) {
                const int i = P->A_ind[k];
                if (i < 1 || i > m) throw NppFail("row index out of range");
                npp->add_aij(i - 1, c, P->A_val[k]);
            }
        }
        npp->sol = sol;
        return 0;
    });
}

// npp_simplex (glpnpp05.js:430): 0 | GLP_ENOPFS | GLP_ENODFS
extern "C" int gk_npp_simplex(gk_npp *npp)
{
    return guard_impl("gk_npp_simplex", [&]() -> int {
        if (!npp || npp->sol != SOL) throw NppFail("workspace not loaded for GLP_SOL");
        return npp->process_prob(0);
    });
}

// npp_integer (glpnpp05.js:437): 0 | GLP_ENOPFS | GLP_ENODFS; msg (7 ints,
// may be NULL) receives the counts the reference prints: integer variables
// binarized, binary variables made, rows added, binarization failures,
// hidden packing and covering inequalities, reduced coefficients
extern "C" int gk_npp_integer(gk_npp *npp, int binarize, int *msg)
{
    return guard_impl("gk_npp_integer", [&]() -> int {
        if (!npp || npp->sol != MIP) throw NppFail("workspace not loaded for GLP_MIP");
        int tmp[7];
        return npp->integer(binarize, msg ? msg : tmp);
    });
}

// the reduced problem's size (npp_build_prob, glpnpp01.js:396)
extern "C" int gk_npp_build_size(gk_npp *npp, int *m, int *n, int *nnz)
{
    return guard_impl("gk_npp_build_size", [&]() -> int {
        if (!npp) throw NppFail("null workspace");
        int mm = 0, nn = 0, zz = 0;
        for (int r = npp->r_head; r >= 0; r = npp->row[r].next) mm++;
        for (int c = npp->c_head; c >= 0; c = npp->col[c].next) {
            nn++;
            for (int e = npp->col[c].ptr; e >= 0; e = npp->a[e].c_next) zz++;
        }
        *m = mm;
        *n = nn;
        *nnz = zz;
        return 0;
    });
}

// npp_build_prob: rows and columns in list order; each column's elements in
// the order the reference's glp_set_mat_col leaves them in the new problem's
// column list (the reverse of the workspace list, glpapi01.js:415-440);
// arrays 1-based as gk_lp's (A_ptr[1] = 1).  row_ref / col_ref: the original
// row / column of each reduced one.
extern "C" int gk_npp_build(gk_npp *npp, signed char *row_type, double *row_lb, double *row_ub,
                            signed char *col_type, double *col_lb, double *col_ub, double *col_coef,
                            signed char *col_kind, int *A_ptr, int *A_ind, double *A_val, int *row_ref,
                            int *col_ref, double *c0)
{
    return guard_impl("gk_npp_build", [&]() -> int {
        if (!npp || npp->built) throw NppFail("workspace not loaded or already built");
        const double dir = npp->orig_dir == 1 ? +1.0 : -1.0;
        auto type_of = [](double lb, double ub) -> signed char {
            if (lb == -BIG && ub == +BIG) return FR;
            if (ub == +BIG) return LO;
            if (lb == -BIG) return UP;
            if (lb != ub) return DB;
            return FX;
        };
        int i = 0;
        for (int r = npp->r_head; r >= 0; r = npp->row[r].next) {
            Row &R = npp->row[r];
            R.temp = ++i;
            row_type[i] = type_of(R.lb, R.ub);
            // glp_set_row_bnds keeps only the bounds its type uses
            row_lb[i] = (row_type[i] == LO || row_type[i] == DB || row_type[i] == FX) ? R.lb : 0.0;
            row_ub[i] = (row_type[i] == UP || row_type[i] == DB) ? R.ub : (row_type[i] == FX ? R.lb : 0.0);
            npp->row_ref.push_back(r + 1);
        }
        int j = 0, k = 1;
        std::vector<int> tmp;
        for (int c = npp->c_head; c >= 0; c = npp->col[c].next) {
            const Col &C = npp->col[c];
            ++j;
            col_kind[j] = C.is_int ? 2 : 1;
            col_type[j] = type_of(C.lb, C.ub);
            col_lb[j] = (col_type[j] == LO || col_type[j] == DB || col_type[j] == FX) ? C.lb : 0.0;
            col_ub[j] = (col_type[j] == UP || col_type[j] == DB) ? C.ub : (col_type[j] == FX ? C.lb : 0.0);
            col_coef[j] = dir * C.coef;
            A_ptr[j] = k;
            tmp.clear();
            for (int e = C.ptr; e >= 0; e = npp->a[e].c_next) tmp.push_back(e);
            for (int t = (int)tmp.size() - 1; t >= 0; t--) {
                A_ind[k] = npp->row[npp->a[tmp[t]].row].temp;
                A_val[k] = npp->a[tmp[t]].val;
                k++;
            }
            npp->col_ref.push_back(c + 1);
        }
        A_ptr[j + 1] = k;
        npp->m = i;
        npp->n = j;
        npp->nnz = k - 1;
        for (int t = 0; t < i; t++) row_ref[t + 1] = npp->row_ref[t];
        for (int t = 0; t < j; t++) col_ref[t + 1] = npp->col_ref[t];
        *c0 = dir * npp->c0;
        npp->built = true;
        return 0;
    });
}

// npp_postprocess (glpnpp01.js:474) for a basic solution (sol = GLP_SOL) or a
// MIP solution (col_prim = mipx, the rest NULL): the reduced problem's
// solution in, the transformation stack replayed from its top
extern "C" int gk_npp_postprocess(gk_npp *npp, int stat1, int stat2, const signed char *row_stat,
                                  const double *row_dual, const signed char *col_stat, const double *col_prim)
{
    return guard_impl("gk_npp_postprocess", [&]() -> int {
        if (!npp || !npp->built) throw NppFail("reduced problem not built");
        const double dir = npp->orig_dir == 1 ? +1.0 : -1.0;
        const int nr = (int)npp->row.size(), nc = (int)npp->col.size();
        if (npp->sol == SOL) {
            npp->p_stat = stat1;
            npp->d_stat = stat2;
            npp->r_stat.assign(nr + 1, 0);
            npp->c_stat.assign(nc + 1, 0);
        } else
            npp->i_stat = stat1;
        npp->c_value.assign(nc + 1, BIG);
        if (npp->sol != MIP) npp->r_pi.assign(nr + 1, BIG);
        if (npp->sol == SOL) {
            for (int i = 1; i <= npp->m; i++) {
                const int k = npp->row_ref[i - 1];
                npp->r_stat[k] = row_stat[i];
                npp->r_pi[k] = dir * row_dual[i];
            }
            for (int j = 1; j <= npp->n; j++) {
                const int k = npp->col_ref[j - 1];
                npp->c_stat[k] = col_stat[j];
                npp->c_value[k] = col_prim[j];
            }
        } else
            for (int j = 1; j <= npp->n; j++) npp->c_value[npp->col_ref[j - 1]] = col_prim[j];
        for (int t = (int)npp->tse.size() - 1; t >= 0; t--) npp->recover(npp->tse[t]);
        npp->post = true;
        return 0;
    });
}

// npp_unload_sol (glpnpp01.js:572), basic solution: statuses, primal and dual
// values of the original problem written to P (P's problem arrays as loaded);
// the primal values of basic rows are summed over each row in descending
// column order (the row lists glp_load_matrix / glp_set_mat_col build), the
// reduced costs of non-basic columns over each column in list order
extern "C" int gk_npp_unload_sol(gk_npp *npp, gk_lp *P)
{
    return guard_impl("gk_npp_unload_sol", [&]() -> int {
        if (!npp || !npp->post || npp->sol != SOL) throw NppFail("no postprocessed basic solution");
        if (P->m != npp->orig_m || P->n != npp->orig_n || P->dir != npp->orig_dir)
            throw NppFail("problem differs from the loaded one");
        const double dir = npp->orig_dir == 1 ? +1.0 : -1.0;
        const int m = P->m, n = P->n;
        P->valid = 0;
        P->pbs_stat = npp->p_stat;
        P->dbs_stat = npp->d_stat;
        P->some = 0;
        double obj = P->c0;
        for (int i = 1; i <= m; i++) {
            const int st = npp->r_stat[i];
            P->row_stat[i] = (signed char)st;
            P->row_dual[i] = dir * npp->r_pi[i];
            const int t = P->row_type[i];
            switch (st) {
            case BS: P->row_dual[i] = 0.0; break;
            case NL: if (!(t == LO || t == DB)) throw NppFail("row status NL on a row without lower bound");
                     P->row_prim[i] = P->row_lb[i]; break;
            case NU: if (!(t == UP || t == DB)) throw NppFail("row status NU on a row without upper bound");
                     P->row_prim[i] = P->row_ub[i]; break;
            case NF: if (t != FR) throw NppFail("row status NF on a bounded row");
                     P->row_prim[i] = 0.0; break;
            case NS: if (t != FX) throw NppFail("row status NS on a non-fixed row");
                     P->row_prim[i] = P->row_lb[i]; break;
            default: throw NppFail("invalid row status");
            }
        }
        for (int j = 1; j <= n; j++) {
            const int st = npp->c_stat[j];
            P->col_stat[j] = (signed char)st;
            P->col_prim[j] = npp->c_value[j];
            const int t = P->col_type[j];
            switch (st) {
            case BS: P->col_dual[j] = 0.0; break;
            case NL: if (!(t == LO || t == DB)) throw NppFail("column status NL without lower bound");
                     P->col_prim[j] = P->col_lb[j]; break;
            case NU: if (!(t == UP || t == DB)) throw NppFail("column status NU without upper bound");
                     P->col_prim[j] = P->col_ub[j]; break;
            case NF: if (t != FR) throw NppFail("column status NF on a bounded column");
                     P->col_prim[j] = 0.0; break;
            case NS: if (t != FX) throw NppFail("column status NS on a non-fixed column");
                     P->col_prim[j] = P->col_lb[j]; break;
            default: throw NppFail("invalid column status");
            }
            obj += P->col_coef[j] * P->col_prim[j];
        }
        P->obj_val = obj;
        // rows by descending column
        std::vector<double> act(m + 1, 0.0);
        std::vector<char> bas(m + 1, 0);
        for (int i = 1; i <= m; i++) bas[i] = P->row_stat[i] == BS;
        for (int j = n; j >= 1; j--)
            for (int k = P->A_ptr[j]; k < P->A_ptr[j + 1]; k++)
                if (bas[P->A_ind[k]]) act[P->A_ind[k]] += P->A_val[k] * P->col_prim[j];
        for (int i = 1; i <= m; i++)
            if (bas[i]) P->row_prim[i] = act[i];
        for (int j = 1; j <= n; j++)
            if (P->col_stat[j] != BS) {
                double d = P->col_coef[j];
                for (int k = P->A_ptr[j]; k < P->A_ptr[j + 1]; k++) d -= P->A_val[k] * P->row_dual[P->A_ind[k]];
                P->col_dual[j] = d;
            }
        return 0;
    });
}

// npp_unload_sol for a MIP solution (glpnpp01.js:732-754): column values
// (integral for integer columns), the objective and the row activities (each
// row summed in descending column order, as gk_npp_unload_sol)
extern "C" int gk_npp_unload_mip(gk_npp *npp, const gk_lp *P, const signed char *col_kind, double *row_mipx,
                                 double *col_mipx, int *mip_stat, double *mip_obj)
{
    return guard_impl("gk_npp_unload_mip", [&]() -> int {
        if (!npp || !npp->post || npp->sol != MIP) throw NppFail("no postprocessed MIP solution");
        if (P->m != npp->orig_m || P->n != npp->orig_n || P->dir != npp->orig_dir)
            throw NppFail("problem differs from the loaded one");
        const int m = P->m, n = P->n;
        *mip_stat = npp->i_stat;
        double obj = P->c0;
        for (int j = 1; j <= n; j++) {
            col_mipx[j] = npp->c_value[j];
            if ((col_kind[j] == 2 || col_kind[j] == 3) && col_mipx[j] != std::floor(col_mipx[j]))
                throw NppFail("integer column with a fractional value");
            obj += P->col_coef[j] * col_mipx[j];
        }
        *mip_obj = obj;
        for (int i = 1; i <= m; i++) row_mipx[i] = 0.0;
        for (int j = n; j >= 1; j--)
            for (int k = P->A_ptr[j]; k < P->A_ptr[j + 1]; k++) row_mipx[P->A_ind[k]] += P->A_val[k] * col_mipx[j];
        return 0;
    });
}
