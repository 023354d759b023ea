// elp_lu_factor.cpp -- Markowitz factorization of the basis and the level
// schedules of the GPU's triangular solves (see elp_lu_factor.h).  The pivot
// rule and every floating-point operation follow oracle/elp_oracle_lu.c
// lu_factor (the CPU restatement the GPU engine is tested against); the data
// structures are this file's own.
#include "elp_lu_factor.h"

#include <math.h>

#include <algorithm>
#include <climits>

namespace elp {

namespace {
constexpr double LU_THRESH = 0.1;  // threshold partial pivoting: |a| >= 0.1 max|column|
constexpr int LU_SEARCH = 4;       // Markowitz: columns examined per step

// min segment tree over (count << 32 | index); INT64_MAX = inactive
struct MinTree {
    int64_t size = 1;
    std::vector<int64_t> t;
    explicit MinTree(int64_t n) {
        while (size < (n > 0 ? n : 1)) size <<= 1;
        t.assign((size_t)(2 * size), INT64_MAX);
    }
    void set(int64_t i, int64_t key) {
        int64_t p = size + i;
        t[(size_t)p] = key;
        for (p >>= 1; p >= 1; p >>= 1) t[(size_t)p] = std::min(t[(size_t)(2 * p)], t[(size_t)(2 * p + 1)]);
    }
    int64_t min() const { return t[1]; }
};
inline int64_t key_of(int64_t count, int64_t idx) { return (count << 32) | idx; }

struct ARow {  // active row: (column, value)
    std::vector<int64_t> c;
    std::vector<double> v;
    int64_t find(int64_t col) const {
        for (size_t t = 0; t < c.size(); ++t)
            if (c[t] == col) return (int64_t)t;
        return -1;
    }
};

void col_remove(std::vector<int64_t>& col, int64_t r) {
    for (size_t t = 0; t < col.size(); ++t)
        if (col[t] == r) {
            col[t] = col.back();
            col.pop_back();
            return;
        }
}

// transpose of step-space rows
void transpose_rows(int64_t nr, const std::vector<int64_t>& p, const std::vector<int32_t>& j,
                    const std::vector<double>& v, std::vector<int64_t>& op, std::vector<int32_t>& oj,
                    std::vector<double>& ov) {
    op.assign((size_t)nr + 1, 0);
    oj.assign(j.size(), 0);
    ov.assign(v.size(), 0.0);
    for (size_t t = 0; t < j.size(); ++t) op[(size_t)j[t] + 1]++;
    for (int64_t s = 0; s < nr; ++s) op[(size_t)s + 1] += op[(size_t)s];
    std::vector<int64_t> nx(op.begin(), op.end());
    for (int64_t s = 0; s < nr; ++s)
        for (int64_t t = p[(size_t)s]; t < p[(size_t)s + 1]; ++t) {
            const int64_t at = nx[(size_t)j[(size_t)t]]++;
            oj[(size_t)at] = (int32_t)s;
            ov[(size_t)at] = v[(size_t)t];
        }
}

// rows whose entries all point to earlier steps (forward) or later steps
// (backward): level = 1 + max level of the entries; rows grouped by level,
// ascending step within a level
void build_sched(int64_t m, const std::vector<int64_t>& p, const std::vector<int32_t>& j,
                 const std::vector<double>& v, bool forward, LuSched& sc) {
    std::vector<int32_t> lev((size_t)m, 0);
    int32_t nlev = 0;
    for (int64_t k = 0; k < m; ++k) {
        const int64_t s = forward ? k : m - 1 - k;
        int32_t l = 0;
        for (int64_t t = p[(size_t)s]; t < p[(size_t)s + 1]; ++t) l = std::max(l, lev[(size_t)j[(size_t)t]] + 1);
        lev[(size_t)s] = l;
        nlev = std::max(nlev, l + 1);
    }
    if (m == 0) nlev = 0;
    sc.lvptr.assign((size_t)nlev + 1, 0);
    for (int64_t s = 0; s < m; ++s) sc.lvptr[(size_t)lev[(size_t)s] + 1]++;
    for (int32_t l = 0; l < nlev; ++l) sc.lvptr[(size_t)l + 1] += sc.lvptr[(size_t)l];
    std::vector<int32_t> nx(sc.lvptr.begin(), sc.lvptr.end());
    sc.row.assign((size_t)m, 0);
    for (int64_t s = 0; s < m; ++s) sc.row[(size_t)nx[(size_t)lev[(size_t)s]]++] = (int32_t)s;
    sc.ptr.assign((size_t)m + 1, 0);
    for (int64_t i = 0; i < m; ++i) {
        const int32_t s = sc.row[(size_t)i];
        sc.ptr[(size_t)i + 1] = sc.ptr[(size_t)i] + (int32_t)(p[(size_t)s + 1] - p[(size_t)s]);
    }
    sc.j.resize(j.size());
    sc.v.resize(v.size());
    for (int64_t i = 0; i < m; ++i) {
        const int32_t s = sc.row[(size_t)i];
        int64_t at = sc.ptr[(size_t)i];
        for (int64_t t = p[(size_t)s]; t < p[(size_t)s + 1]; ++t, ++at) {
            sc.j[(size_t)at] = j[(size_t)t];
            sc.v[(size_t)at] = v[(size_t)t];
        }
    }
}
}  // namespace

int lu_factor(LuFactors& f, const LuColumns& a, const int32_t* head, double tol_singular) {
    const int64_t m = a.m;
    f = LuFactors{};
    f.m = m;
    f.prow.assign((size_t)m, 0);
    f.pcol.assign((size_t)m, 0);
    f.rstep.assign((size_t)m, 0);
    f.ud.assign((size_t)m, 0.0);
    std::vector<ARow> R((size_t)m);
    std::vector<std::vector<int64_t>> C((size_t)m);
    std::vector<ARow> Lr((size_t)m);  // per row: (step, l)
    std::vector<ARow> Ur((size_t)m);  // per step: (column, u)
    std::vector<int64_t> mark((size_t)m + 1, 0), cstep((size_t)m, 0);
    for (int64_t p = 0; p < m; ++p) {
        const int64_t var = head[p];
        if (var < a.n) {
            for (int64_t t = a.cp[var]; t < a.cp[var + 1]; ++t) {
                R[(size_t)a.ri[t]].c.push_back(p);
                R[(size_t)a.ri[t]].v.push_back(a.cv[t]);
                C[(size_t)p].push_back(a.ri[t]);
            }
        } else {
            const bool slack = var < a.n + a.m;
            const int64_t i = slack ? var - a.n : var - a.n - a.m;
            R[(size_t)i].c.push_back(p);
            R[(size_t)i].v.push_back(slack ? 1.0 : a.asgn[i]);
            C[(size_t)p].push_back(i);
        }
    }
    MinTree gc(m), gr(m);
    for (int64_t p = 0; p < m; ++p) {
        gc.set(p, key_of((int64_t)C[(size_t)p].size(), p));
        gr.set(p, key_of((int64_t)R[(size_t)p].c.size(), p));
    }
    int rc = 0;
    int64_t pop[LU_SEARCH], popk[LU_SEARCH];
    for (int64_t s = 0; s < m && !rc; ++s) {
        int64_t pr = -1, pc = -1;
        const int64_t kc = gc.min(), kr = gr.min();
        if (kc == INT64_MAX || (kc >> 32) == 0) {
            rc = -1;
            break;
        }
        if ((kc >> 32) == 1) {
            pc = kc & 0xffffffffll;
            pr = C[(size_t)pc][0];
            const int64_t t = R[(size_t)pr].find(pc);
            if (!(fabs(R[(size_t)pr].v[(size_t)t]) > tol_singular)) {
                rc = -1;
                break;
            }
        } else if (kr != INT64_MAX && (kr >> 32) == 1) {
            pr = kr & 0xffffffffll;
            pc = R[(size_t)pr].c[0];
            if (!(fabs(R[(size_t)pr].v[0]) > tol_singular)) pr = pc = -1;
        }
        if (pr < 0) {
            int64_t np = 0, best_cost = INT64_MAX;
            for (; np < LU_SEARCH && gc.min() != INT64_MAX; ++np) {
                popk[np] = gc.min();
                pop[np] = popk[np] & 0xffffffffll;
                gc.set(pop[np], INT64_MAX);
            }
            for (int64_t q = 0; q < np; ++q) {
                const int64_t c = pop[q];
                const std::vector<int64_t>& col = C[(size_t)c];
                double cmax = 0.0;
                for (int64_t i : col) {
                    const ARow& ri = R[(size_t)i];
                    const double v = fabs(ri.v[(size_t)ri.find(c)]);
                    if (v > cmax) cmax = v;
                }
                int64_t brow = -1, bcost = INT64_MAX;
                for (int64_t i : col) {
                    const ARow& ri = R[(size_t)i];
                    const double v = fabs(ri.v[(size_t)ri.find(c)]);
                    if (!(v >= LU_THRESH * cmax) || !(v > tol_singular)) continue;
                    const int64_t cost = ((int64_t)ri.c.size() - 1) * ((int64_t)col.size() - 1);
                    if (cost < bcost || (cost == bcost && i < brow)) {
                        bcost = cost;
                        brow = i;
                    }
                }
                if (brow >= 0 && bcost < best_cost) {
                    best_cost = bcost;
                    pr = brow;
                    pc = c;
                }
            }
            for (int64_t q = 0; q < np; ++q) gc.set(pop[q], popk[q]);
            if (pr < 0) {
                rc = -1;
                break;
            }
        }
        ARow& rp = R[(size_t)pr];
        const int64_t tp = rp.find(pc);
        const double piv = rp.v[(size_t)tp];
        f.prow[(size_t)s] = (int32_t)pr;
        f.pcol[(size_t)s] = (int32_t)pc;
        f.ud[(size_t)s] = piv;
        f.rstep[(size_t)pr] = (int32_t)s;
        cstep[(size_t)pc] = s;
        ARow& us = Ur[(size_t)s];
        for (size_t t = 0; t < rp.c.size(); ++t)
            if (rp.c[t] != pc) {
                us.c.push_back(rp.c[t]);
                us.v.push_back(rp.v[t]);
            }
        for (size_t t = 0; t < rp.c.size(); ++t) {
            const int64_t c = rp.c[t];
            col_remove(C[(size_t)c], pr);
            if (c != pc) gc.set(c, key_of((int64_t)C[(size_t)c].size(), c));
        }
        gc.set(pc, INT64_MAX);
        gr.set(pr, INT64_MAX);
        std::vector<int64_t>& pcol = C[(size_t)pc];
        for (size_t t = 0; t < pcol.size(); ++t) {
            const int64_t i = pcol[t];
            ARow& ri = R[(size_t)i];
            const int64_t ti = ri.find(pc);
            const double l = ri.v[(size_t)ti] / piv;
            Lr[(size_t)i].c.push_back(s);
            Lr[(size_t)i].v.push_back(l);
            ri.c[(size_t)ti] = ri.c.back();
            ri.v[(size_t)ti] = ri.v.back();
            ri.c.pop_back();
            ri.v.pop_back();
            for (size_t u = 0; u < ri.c.size(); ++u) mark[(size_t)ri.c[u]] = (int64_t)u + 1;
            for (size_t u = 0; u < us.c.size(); ++u) {
                const int64_t c = us.c[u];
                const double uv = us.v[u];
                if (mark[(size_t)c]) {
                    double& x = ri.v[(size_t)(mark[(size_t)c] - 1)];
                    x = fma(-l, uv, x);
                } else {
                    ri.c.push_back(c);
                    ri.v.push_back(fma(-l, uv, 0.0));
                    mark[(size_t)c] = (int64_t)ri.c.size();
                    C[(size_t)c].push_back(i);
                    gc.set(c, key_of((int64_t)C[(size_t)c].size(), c));
                }
            }
            for (size_t u = 0; u < ri.c.size(); ++u) mark[(size_t)ri.c[u]] = 0;
            gr.set(i, key_of((int64_t)ri.c.size(), i));
        }
        pcol.clear();
        rp.c.clear();
        rp.v.clear();
    }
    if (rc) return rc;
    f.Lp.assign((size_t)m + 1, 0);
    f.Up.assign((size_t)m + 1, 0);
    for (int64_t s = 0; s < m; ++s) {
        f.Lp[(size_t)s + 1] = f.Lp[(size_t)s] + (int64_t)Lr[(size_t)f.prow[(size_t)s]].c.size();
        f.Up[(size_t)s + 1] = f.Up[(size_t)s] + (int64_t)Ur[(size_t)s].c.size();
    }
    f.Lj.assign((size_t)f.Lp[(size_t)m], 0);
    f.Lv.assign((size_t)f.Lp[(size_t)m], 0.0);
    f.Uj.assign((size_t)f.Up[(size_t)m], 0);
    f.Uv.assign((size_t)f.Up[(size_t)m], 0.0);
    for (int64_t s = 0; s < m; ++s) {
        const ARow& l = Lr[(size_t)f.prow[(size_t)s]];
        for (size_t t = 0; t < l.c.size(); ++t) {
            f.Lj[(size_t)f.Lp[(size_t)s] + t] = (int32_t)l.c[t];
            f.Lv[(size_t)f.Lp[(size_t)s] + t] = l.v[t];
        }
        const int64_t b = f.Up[(size_t)s];
        const ARow& u = Ur[(size_t)s];
        for (size_t t = 0; t < u.c.size(); ++t) {  // columns -> steps, insertion sort
            const int32_t st = (int32_t)cstep[(size_t)u.c[t]];
            const double v = u.v[t];
            int64_t at = b + (int64_t)t;
            while (at > b && f.Uj[(size_t)at - 1] > st) {
                f.Uj[(size_t)at] = f.Uj[(size_t)at - 1];
                f.Uv[(size_t)at] = f.Uv[(size_t)at - 1];
                at--;
            }
            f.Uj[(size_t)at] = st;
            f.Uv[(size_t)at] = v;
        }
    }
    transpose_rows(m, f.Lp, f.Lj, f.Lv, f.LTp, f.LTj, f.LTv);
    transpose_rows(m, f.Up, f.Uj, f.Uv, f.UTp, f.UTj, f.UTv);
    return 0;
}

void lu_schedules(LuFactors& f) {
    build_sched(f.m, f.Lp, f.Lj, f.Lv, true, f.sL);
    build_sched(f.m, f.Up, f.Uj, f.Uv, false, f.sU);
    build_sched(f.m, f.UTp, f.UTj, f.UTv, true, f.sUT);
    build_sched(f.m, f.LTp, f.LTj, f.LTv, false, f.sLT);
}

}  // namespace elp

// CPU test hook (tests/test_lu_factor.py builds this file alone with g++ and
// compares against oracle/elp_oracle_lu.c orc_lu_factor): same arguments and
// outputs as orc_lu_factor.
extern "C" int elp_lu_factor_host(int64_t m, int64_t n, const int64_t* colptr, const int32_t* rowind,
                                  const double* val, const int64_t* head, double tol_singular, int64_t* prow,
                                  int64_t* pcol, double* ud, int64_t* nnz_lu, double* lsum, double* usum,
                                  int32_t* nlev) {
    std::vector<double> asgn((size_t)(m > 0 ? m : 1), 1.0);
    std::vector<int32_t> h((size_t)(m > 0 ? m : 1));
    for (int64_t p = 0; p < m; ++p) h[(size_t)p] = (int32_t)head[p];
    elp::LuColumns a{m, n, colptr, rowind, val, asgn.data()};
    elp::LuFactors f;
    const int rc = elp::lu_factor(f, a, h.data(), tol_singular);
    if (rc) return rc;
    elp::lu_schedules(f);
    for (int64_t s = 0; s < m; ++s) {
        prow[s] = f.prow[(size_t)s];
        pcol[s] = f.pcol[(size_t)s];
        ud[s] = f.ud[(size_t)s];
    }
    nnz_lu[0] = (int64_t)f.Lj.size();
    nnz_lu[1] = (int64_t)f.Uj.size();
    double a1 = 0.0, a2 = 0.0;
    for (size_t t = 0; t < f.Lj.size(); ++t) a1 = fma(a1, 1.0000001, f.Lv[t] * (double)(f.Lj[t] + 1));
    for (size_t t = 0; t < f.Uj.size(); ++t) a2 = fma(a2, 1.0000001, f.Uv[t] * (double)(f.Uj[t] + 1));
    *lsum = a1;
    *usum = a2;
    nlev[0] = f.sL.nlev();
    nlev[1] = f.sU.nlev();
    nlev[2] = f.sUT.nlev();
    nlev[3] = f.sLT.nlev();
    return 0;
}
