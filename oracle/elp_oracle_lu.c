/*
 * elp_oracle_lu.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the sparse-LU
 * engine of the CSC path (elp_control.basis = ELP_BASIS_LU; the HIP side is
 * easylp_amd/csrc/elp_lu.hip + the host factorization in elp_lu_host.cpp).
 *
 * What it restates: the solve R/class.R:276 hands to lp_solve, whose basis
 * factorization is LUSOL (a Markowitz LU with product-form / Forrest-Tomlin
 * updates).  Neither lp_solve nor LUSOL is in the reference or this image
 * (SURVEY.md 8c), so the arithmetic below is this repo's own contract -- the
 * GPU engine reproduces it bit for bit -- and its answers are pinned by the
 * HiGHS fixtures (tests/golden/sparse_lps.json, make_sparse.py) and by the
 * constructed-optimum LPs of tests/golden/make_sparse_lu.py.
 *
 * The engine:
 *   basis B (m x m): position p holds basic variable head[p]; its column is
 *   A[:, j] (structural j, scaled), e_i (slack n+i) or asgn_i e_i (artificial
 *   n+m+i);
 *   refactor: Markowitz LU  P B Q = L U  with threshold partial pivoting
 *   (lu_factor below), then a product-form eta file, one eta per pivot;
 *   FTRAN  x = B^-1 a :  t = P a; L solve (rows ascending); U solve (rows
 *     descending); x[pcol[s]] = t[s]; etas in order;
 *   BTRAN  y = B^-T c :  etas in reverse (lane_dot256 sums); U^T solve
 *     (ascending); L^T solve (descending); y[prow[s]] = t[s];
 *   every row / column sum is one fma chain in ascending step order, so any
 *   schedule that respects the dependencies (the GPU's level sets) computes
 *   the same bits;
 *   every iteration recomputes y = B^-T c_B exactly (no dual update), prices
 *   (column chains, Devex / Dantzig, Bland), runs FTRAN, the Harris two-pass
 *   ratio test over the m positions, and appends the eta -- the rules of
 *   elp_oracle.c run_phase (bound flips, degeneracy, Devex restarts, phase 1
 *   artificials, the optimality re-check after a refactor).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "elp_oracle.h"

#define VS_BASIC 0
#define VS_LOWER 1
#define VS_UPPER 2
#define VS_FREE 3
#define WAVE 64
#define LANES 256          /* lane_dot256: the GPU's 256-thread reduction */
#define DEVEX_WMAX 1e20
#define DEVEX_RESET 1e6
#define LU_THRESH 0.1      /* threshold partial pivoting: |a| >= 0.1 max|column| */
#define LU_SEARCH 4        /* Markowitz: columns examined per step */

/* ------------------------------------------------------------------ */
/* small helpers                                                       */
static double* dz(size_t n) { return (double*)calloc(n ? n : 1, sizeof(double)); }
static int64_t* iz(size_t n) { return (int64_t*)calloc(n ? n : 1, sizeof(int64_t)); }

/* a min segment tree over keys (count << 32 | index); INT64_MAX = inactive */
typedef struct {
    int64_t size; /* leaves (power of 2) */
    int64_t* t;
} segt;
static void seg_init(segt* g, int64_t n) {
    g->size = 1;
    while (g->size < (n > 0 ? n : 1)) g->size <<= 1;
    g->t = (int64_t*)malloc(sizeof(int64_t) * (size_t)(2 * g->size));
    for (int64_t i = 0; i < 2 * g->size; ++i) g->t[i] = INT64_MAX;
}
static void seg_set(segt* g, int64_t i, int64_t key) {
    int64_t p = g->size + i;
    g->t[p] = key;
    for (p >>= 1; p >= 1; p >>= 1) {
        const int64_t a = g->t[2 * p], b = g->t[2 * p + 1];
        g->t[p] = a < b ? a : b;
    }
}
static int64_t seg_min(const segt* g) { return g->t[1]; }
static void seg_free(segt* g) { free(g->t); }
static int64_t key_of(int64_t count, int64_t idx) { return (count << 32) | idx; }

/* dynamic row of the active submatrix: (column, value) */
typedef struct {
    int64_t n, cap;
    int64_t* c;
    double* v;
} lrow;
static void row_push(lrow* r, int64_t c, double v) {
    if (r->n == r->cap) {
        r->cap = r->cap ? 2 * r->cap : 8;
        r->c = (int64_t*)realloc(r->c, sizeof(int64_t) * (size_t)r->cap);
        r->v = (double*)realloc(r->v, sizeof(double) * (size_t)r->cap);
    }
    r->c[r->n] = c;
    r->v[r->n] = v;
    r->n++;
}
/* dynamic column pattern: rows */
typedef struct {
    int64_t n, cap;
    int64_t* r;
} lcol;
static void col_push(lcol* c, int64_t r) {
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 8;
        c->r = (int64_t*)realloc(c->r, sizeof(int64_t) * (size_t)c->cap);
    }
    c->r[c->n++] = r;
}
static void col_remove(lcol* c, int64_t r) {
    for (int64_t t = 0; t < c->n; ++t)
        if (c->r[t] == r) {
            c->r[t] = c->r[c->n - 1];
            c->n--;
            return;
        }
}
static int64_t row_find(const lrow* r, int64_t c) {
    for (int64_t t = 0; t < r->n; ++t)
        if (r->c[t] == c) return t;
    return -1;
}

/* compressed rows in step space: entries of row s in [p[s], p[s+1]) */
typedef struct {
    int64_t* p;
    int64_t* j;
    double* v;
    int64_t nnz;
} crows;
static void crows_free(crows* c) {
    free(c->p);
    free(c->j);
    free(c->v);
    memset(c, 0, sizeof *c);
}

typedef struct {
    int64_t m;
    int64_t *prow, *pcol;   /* step -> pivot row / basis position */
    double* ud;              /* U diagonal per step */
    crows L, U, LT, UT;      /* L rows (s' < s), U rows (s' > s), transposes */
    /* eta file (product form): eta e = pivot position epiv[e], value epv[e],
       entries [ep[e], ep[e+1]) of (position, alpha) without the pivot */
    int64_t ne, ecap, enz, enzcap;
    int64_t *ep, *epiv, *ei;
    double *epv, *ev;
} lu_t;

static void lu_free(lu_t* f) {
    free(f->prow);
    free(f->pcol);
    free(f->ud);
    crows_free(&f->L);
    crows_free(&f->U);
    crows_free(&f->LT);
    crows_free(&f->UT);
    free(f->ep);
    free(f->epiv);
    free(f->ei);
    free(f->epv);
    free(f->ev);
    memset(f, 0, sizeof *f);
}

/* transpose of step-space rows (nr rows): entries (s, v) of row s' land in row
   s' of the result as (s, v)... i.e. out row j holds (s, v) for every entry
   (j, v) of in row s, ascending s */
static void transpose_rows(int64_t nr, const crows* in, crows* out) {
    out->p = iz((size_t)nr + 1);
    out->j = iz((size_t)in->nnz);
    out->v = dz((size_t)in->nnz);
    out->nnz = in->nnz;
    for (int64_t t = 0; t < in->nnz; ++t) out->p[in->j[t] + 1]++;
    for (int64_t s = 0; s < nr; ++s) out->p[s + 1] += out->p[s];
    int64_t* nx = iz((size_t)nr + 1);
    memcpy(nx, out->p, sizeof(int64_t) * (size_t)(nr + 1));
    for (int64_t s = 0; s < nr; ++s)
        for (int64_t t = in->p[s]; t < in->p[s + 1]; ++t) {
            const int64_t at = nx[in->j[t]]++;
            out->j[at] = s;
            out->v[at] = in->v[t];
        }
    free(nx);
}

/* basis column of position p: (row, value) pairs, rows ascending */
typedef struct {
    int64_t m, n;
    const int64_t* cp;
    const int32_t* ri;
    const double* cv; /* scaled values */
    const double* asgn;
} colsrc;
static int64_t bcol(const colsrc* a, int64_t var, int64_t* rows, double* vals) {
    if (var < a->n) {
        int64_t c = 0;
        for (int64_t t = a->cp[var]; t < a->cp[var + 1]; ++t) {
            rows[c] = a->ri[t];
            vals[c++] = a->cv[t];
        }
        return c;
    }
    if (var < a->n + a->m) {
        rows[0] = var - a->n;
        vals[0] = 1.0;
        return 1;
    }
    rows[0] = var - a->n - a->m;
    vals[0] = a->asgn[var - a->n - a->m];
    return 1;
}

/* Markowitz LU of B = [column of head[p]]_p (see the file header).  Pivot
 * choice, a total order so any list order gives the same factors:
 *   1. a column singleton: the lowest (count, column) with count 1;
 *   2. else a row singleton: the lowest (count, row) with count 1 (its one
 *      entry, |a| > tol_singular);
 *   3. else Markowitz: the first LU_SEARCH columns in (count, column) order;
 *      in each, the entries with |a| >= LU_THRESH max|column| and |a| >
 *      tol_singular; cost (rowcount - 1)(colcount - 1); lowest cost wins, ties
 *      the earlier column, then the lower row.
 * Elimination of row i by the pivot row: a_ic' = fma(-l, u_c', a_ic'), fill
 * fma(-l, u_c', 0.0), l = a_ic / pivot.  Returns -1 on a singular basis. */
static int lu_factor(lu_t* f, const colsrc* a, const int64_t* head, double tol_singular) {
    const int64_t m = a->m;
    lu_free(f);
    f->m = m;
    f->prow = iz((size_t)m);
    f->pcol = iz((size_t)m);
    f->ud = dz((size_t)m);
    lrow* R = (lrow*)calloc((size_t)(m > 0 ? m : 1), sizeof(lrow));
    lcol* C = (lcol*)calloc((size_t)(m > 0 ? m : 1), sizeof(lcol));
    lrow* Lr = (lrow*)calloc((size_t)(m > 0 ? m : 1), sizeof(lrow)); /* per row: (step, l) */
    lrow* Ur = (lrow*)calloc((size_t)(m > 0 ? m : 1), sizeof(lrow)); /* per step: (column, u) */
    int64_t* rows = iz((size_t)m + 1);
    double* vals = dz((size_t)m + 1);
    int64_t* mark = iz((size_t)m + 1); /* column -> entry index + 1 in the row being updated */
    int64_t* rstep = iz((size_t)m);
    int64_t* cstep = iz((size_t)m);
    for (int64_t p = 0; p < m; ++p) {
        const int64_t c = bcol(a, head[p], rows, vals);
        for (int64_t t = 0; t < c; ++t) {
            row_push(&R[rows[t]], p, vals[t]);
            col_push(&C[p], rows[t]);
        }
    }
    segt gc, gr;
    seg_init(&gc, m);
    seg_init(&gr, m);
    for (int64_t p = 0; p < m; ++p) {
        seg_set(&gc, p, key_of(C[p].n, p));
        seg_set(&gr, p, key_of(R[p].n, p));
    }
    int rc = 0;
    int64_t pop[LU_SEARCH], popk[LU_SEARCH];
    for (int64_t s = 0; s < m && !rc; ++s) {
        int64_t pr = -1, pc = -1;
        const int64_t kc = seg_min(&gc), kr = seg_min(&gr);
        if (kc == INT64_MAX) {
            rc = -1;
            break;
        }
        if ((kc >> 32) == 0) { /* an empty column: singular */
            rc = -1;
            break;
        }
        if ((kc >> 32) == 1) {
            pc = kc & 0xffffffffll;
            pr = C[pc].r[0];
            const int64_t t = row_find(&R[pr], pc);
            if (!(fabs(R[pr].v[t]) > tol_singular)) {
                rc = -1;
                break;
            }
        } else if (kr != INT64_MAX && (kr >> 32) == 1) {
            pr = kr & 0xffffffffll;
            pc = R[pr].c[0];
            if (!(fabs(R[pr].v[0]) > tol_singular)) pr = pc = -1; /* fall through to the search */
        }
        if (pr < 0) {
            int64_t np = 0;
            int64_t best_cost = INT64_MAX;
            for (; np < LU_SEARCH && seg_min(&gc) != INT64_MAX; ++np) {
                popk[np] = seg_min(&gc);
                pop[np] = popk[np] & 0xffffffffll;
                seg_set(&gc, pop[np], INT64_MAX);
            }
            for (int64_t q = 0; q < np; ++q) {
                const int64_t c = pop[q];
                double cmax = 0.0;
                for (int64_t t = 0; t < C[c].n; ++t) {
                    const int64_t i = C[c].r[t];
                    const double v = fabs(R[i].v[row_find(&R[i], c)]);
                    if (v > cmax) cmax = v;
                }
                int64_t brow = -1, bcost = INT64_MAX;
                for (int64_t t = 0; t < C[c].n; ++t) {
                    const int64_t i = C[c].r[t];
                    const double v = fabs(R[i].v[row_find(&R[i], c)]);
                    if (!(v >= LU_THRESH * cmax) || !(v > tol_singular)) continue;
                    const int64_t cost = (R[i].n - 1) * (C[c].n - 1);
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
            for (int64_t q = 0; q < np; ++q) seg_set(&gc, pop[q], popk[q]);
            if (pr < 0) {
                rc = -1;
                break;
            }
        }
        /* pivot (pr, pc) at step s */
        const int64_t tp = row_find(&R[pr], pc);
        const double piv = R[pr].v[tp];
        f->prow[s] = pr;
        f->pcol[s] = pc;
        f->ud[s] = piv;
        rstep[pr] = s;
        cstep[pc] = s;
        for (int64_t t = 0; t < R[pr].n; ++t)
            if (R[pr].c[t] != pc) row_push(&Ur[s], R[pr].c[t], R[pr].v[t]);
        /* the pivot row leaves the active columns */
        for (int64_t t = 0; t < R[pr].n; ++t) {
            const int64_t c = R[pr].c[t];
            col_remove(&C[c], pr);
            if (c != pc) seg_set(&gc, c, key_of(C[c].n, c));
        }
        seg_set(&gc, pc, INT64_MAX);
        seg_set(&gr, pr, INT64_MAX);
        /* eliminate the other rows of the pivot column */
        for (int64_t t = 0; t < C[pc].n; ++t) {
            const int64_t i = C[pc].r[t];
            lrow* ri = &R[i];
            const int64_t ti = row_find(ri, pc);
            const double l = ri->v[ti] / piv;
            row_push(&Lr[i], s, l);
            /* drop the pivot-column entry (swap with last) */
            ri->c[ti] = ri->c[ri->n - 1];
            ri->v[ti] = ri->v[ri->n - 1];
            ri->n--;
            for (int64_t u = 0; u < ri->n; ++u) mark[ri->c[u]] = u + 1;
            for (int64_t u = 0; u < Ur[s].n; ++u) {
                const int64_t c = Ur[s].c[u];
                const double uv = Ur[s].v[u];
                if (mark[c]) {
                    ri->v[mark[c] - 1] = fma(-l, uv, ri->v[mark[c] - 1]);
                } else {
                    row_push(ri, c, fma(-l, uv, 0.0));
                    mark[c] = ri->n;
                    col_push(&C[c], i);
                    seg_set(&gc, c, key_of(C[c].n, c));
                }
            }
            for (int64_t u = 0; u < ri->n; ++u) mark[ri->c[u]] = 0;
            seg_set(&gr, i, key_of(ri->n, i));
        }
        C[pc].n = 0;
        R[pr].n = 0;
    }
    if (!rc) {
        /* step-space rows: L row s = row prow[s]'s multipliers (ascending
           step), U row s = the pivot row's other columns as steps (sorted) */
        f->L.p = iz((size_t)m + 1);
        f->U.p = iz((size_t)m + 1);
        for (int64_t s = 0; s < m; ++s) {
            f->L.p[s + 1] = f->L.p[s] + Lr[f->prow[s]].n;
            f->U.p[s + 1] = f->U.p[s] + Ur[s].n;
        }
        f->L.nnz = f->L.p[m];
        f->U.nnz = f->U.p[m];
        f->L.j = iz((size_t)f->L.nnz);
        f->L.v = dz((size_t)f->L.nnz);
        f->U.j = iz((size_t)f->U.nnz);
        f->U.v = dz((size_t)f->U.nnz);
        for (int64_t s = 0; s < m; ++s) {
            const lrow* l = &Lr[f->prow[s]];
            for (int64_t t = 0; t < l->n; ++t) { /* appended in step order */
                f->L.j[f->L.p[s] + t] = l->c[t];
                f->L.v[f->L.p[s] + t] = l->v[t];
            }
            /* U row: columns -> steps, insertion sort by step */
            const int64_t b = f->U.p[s];
            const lrow* u = &Ur[s];
            for (int64_t t = 0; t < u->n; ++t) {
                const int64_t st = cstep[u->c[t]];
                const double v = u->v[t];
                int64_t at = b + t;
                while (at > b && f->U.j[at - 1] > st) {
                    f->U.j[at] = f->U.j[at - 1];
                    f->U.v[at] = f->U.v[at - 1];
                    at--;
                }
                f->U.j[at] = st;
                f->U.v[at] = v;
            }
        }
        transpose_rows(m, &f->L, &f->LT);
        transpose_rows(m, &f->U, &f->UT);
    }
    for (int64_t i = 0; i < m; ++i) {
        free(R[i].c);
        free(R[i].v);
        free(C[i].r);
        free(Lr[i].c);
        free(Lr[i].v);
        free(Ur[i].c);
        free(Ur[i].v);
    }
    free(R);
    free(C);
    free(Lr);
    free(Ur);
    free(rows);
    free(vals);
    free(mark);
    free(rstep);
    free(cstep);
    seg_free(&gc);
    seg_free(&gr);
    f->ne = f->enz = 0;
    return rc;
}

/* the GPU's 256-thread sum: lane-strided fma chains, then a pairwise tree */
static double lane_dot256(int64_t len, const int64_t* idx, const double* a, const double* x) {
    double lane[LANES];
    for (int l = 0; l < LANES; ++l) {
        double acc = 0.0;
        for (int64_t e = l; e < len; e += LANES) acc = fma(a[e], x[idx[e]], acc);
        lane[l] = acc;
    }
    for (int off = 1; off < LANES; off <<= 1)
        for (int l = 0; l + off < LANES; l += 2 * off) lane[l] = lane[l] + lane[l + off];
    return lane[0];
}

/* x (positions) = B^-1 a (rows); t: work (m) */
static void lu_ftran(const lu_t* f, const double* a, double* x, double* t) {
    const int64_t m = f->m;
    for (int64_t s = 0; s < m; ++s) t[s] = a[f->prow[s]];
    for (int64_t s = 0; s < m; ++s) {
        double acc = t[s];
        for (int64_t e = f->L.p[s]; e < f->L.p[s + 1]; ++e) acc = fma(-f->L.v[e], t[f->L.j[e]], acc);
        t[s] = acc;
    }
    for (int64_t s = m - 1; s >= 0; --s) {
        double acc = t[s];
        for (int64_t e = f->U.p[s]; e < f->U.p[s + 1]; ++e) acc = fma(-f->U.v[e], t[f->U.j[e]], acc);
        t[s] = acc / f->ud[s];
    }
    for (int64_t s = 0; s < m; ++s) x[f->pcol[s]] = t[s];
    for (int64_t e = 0; e < f->ne; ++e) {
        const int64_t p = f->epiv[e];
        const double xp = x[p] / f->epv[e];
        x[p] = xp;
        for (int64_t t2 = f->ep[e]; t2 < f->ep[e + 1]; ++t2) x[f->ei[t2]] = fma(-f->ev[t2], xp, x[f->ei[t2]]);
    }
}

/* y (rows) = B^-T c (positions); c is overwritten; t: work (m) */
static void lu_btran(const lu_t* f, double* c, double* y, double* t) {
    const int64_t m = f->m;
    for (int64_t e = f->ne - 1; e >= 0; --e) {
        const int64_t p = f->epiv[e];
        const int64_t b = f->ep[e];
        const double dot = lane_dot256(f->ep[e + 1] - b, f->ei + b, f->ev + b, c);
        c[p] = (c[p] - dot) / f->epv[e];
    }
    for (int64_t s = 0; s < m; ++s) t[s] = c[f->pcol[s]];
    for (int64_t s = 0; s < m; ++s) {
        double acc = t[s];
        for (int64_t e = f->UT.p[s]; e < f->UT.p[s + 1]; ++e) acc = fma(-f->UT.v[e], t[f->UT.j[e]], acc);
        t[s] = acc / f->ud[s];
    }
    for (int64_t s = m - 1; s >= 0; --s) {
        double acc = t[s];
        for (int64_t e = f->LT.p[s]; e < f->LT.p[s + 1]; ++e) acc = fma(-f->LT.v[e], t[f->LT.j[e]], acc);
        t[s] = acc;
    }
    for (int64_t s = 0; s < m; ++s) y[f->prow[s]] = t[s];
}

static void eta_append(lu_t* f, int64_t r, const double* alpha) {
    const int64_t m = f->m;
    if (f->ne + 1 >= f->ecap) {
        f->ecap = f->ecap ? 2 * f->ecap : 64;
        f->ep = (int64_t*)realloc(f->ep, sizeof(int64_t) * (size_t)(f->ecap + 1));
        f->epiv = (int64_t*)realloc(f->epiv, sizeof(int64_t) * (size_t)f->ecap);
        f->epv = (double*)realloc(f->epv, sizeof(double) * (size_t)f->ecap);
    }
    if (f->ne == 0) f->ep[0] = 0;
    if (f->enz + m > f->enzcap) {
        f->enzcap = (f->enz + m) * 2;
        f->ei = (int64_t*)realloc(f->ei, sizeof(int64_t) * (size_t)f->enzcap);
        f->ev = (double*)realloc(f->ev, sizeof(double) * (size_t)f->enzcap);
    }
    for (int64_t i = 0; i < m; ++i)
        if (i != r && alpha[i] != 0.0) {
            f->ei[f->enz] = i;
            f->ev[f->enz++] = alpha[i];
        }
    f->epiv[f->ne] = r;
    f->epv[f->ne] = alpha[r];
    f->ne++;
    f->ep[f->ne] = f->enz;
}

/* ------------------------------------------------------------------ */
/* solver state                                                        */
typedef struct {
    int64_t m, n, nv;
    colsrc a;
    int64_t *rp, *ci; /* CSR of the scaled A (row activities) */
    double* rv;
    double *b, *lb, *ub, *cost, *xval, *asgn;
    int8_t* vstat;
    int64_t *head, *bpos;
    double* xB;
    lu_t f;
    double *y, *cB, *acol, *alpha, *t, *d, *dw, *dprev;
    double tol_inf, tol_singular;
    int64_t lu_nnz_max, eta_nnz_max;
} lus_t;

/* phase-1 infeasibility: artificial values in wave order over positions */
static double art_sum_lu(const lus_t* s) {
    double lane[WAVE];
    for (int l = 0; l < WAVE; ++l) {
        double acc = 0.0;
        for (int64_t p = l; p < s->m; p += WAVE)
            if (s->head[p] >= s->n + s->m) acc = acc + s->xB[p];
        lane[l] = acc;
    }
    for (int off = 1; off < WAVE; off <<= 1)
        for (int l = 0; l + off < WAVE; l += 2 * off) lane[l] = lane[l] + lane[l + off];
    return lane[0];
}

/* refactor: LU of the current basis, empty eta file, x_B = B^-1 (b - N x_N)
   with the row activities as one fma chain per row over its CSR entries
   (ascending column; nonbasic structurals with x_j != 0) */
static int refactor_lu(lus_t* s) {
    const int64_t m = s->m, n = s->n;
    if (lu_factor(&s->f, &s->a, s->head, s->tol_singular)) return -1;
    const int64_t nz = s->f.L.nnz + s->f.U.nnz + m;
    if (nz > s->lu_nnz_max) s->lu_nnz_max = nz;
    for (int64_t i = 0; i < m; ++i) {
        double acc = 0.0;
        for (int64_t t = s->rp[i]; t < s->rp[i + 1]; ++t) {
            const int64_t j = s->ci[t];
            const double xj = s->xval[j];
            if (s->vstat[j] != VS_BASIC && xj != 0.0) acc = fma(s->rv[t], xj, acc);
        }
        double r = s->b[i] - acc;
        if (s->vstat[n + i] != VS_BASIC) r = r - s->xval[n + i];
        s->acol[i] = r;
    }
    lu_ftran(&s->f, s->acol, s->xB, s->t);
    return 0;
}

enum { PH_OPTIMAL = 0, PH_UNBOUNDED = 3, PH_NUMFAIL = 5, PH_ITERCAP = 1, PH_P1DONE = 10 };

static int run_phase_lu(lus_t* s, int phase, const orc_control* ctl, int64_t* iter, int64_t max_iter,
                        int64_t* trace, int64_t trace_cap, orc_stats* st, int64_t* unb_var, double* unb_sigma,
                        int64_t* since_refactor) {
    const int64_t m = s->m, n = s->n;
    int64_t ndegen = 0;
    int bland = 0, recheck = 0;
    const int devex = ctl->price_rule == 1;
    int dv_valid = 0;
    int64_t dv_lv = -1;
    double dv_dq = 1.0, dv_wq = 1.0;
    if (devex)
        for (int64_t j = 0; j < n + m; ++j) s->dw[j] = 1.0;
    for (;;) {
        if (!recheck) {
            if (phase == 1 && art_sum_lu(s) <= s->tol_inf) return PH_P1DONE;
            if (*iter >= max_iter) return PH_ITERCAP;
            if (*since_refactor >= ctl->refactor_period) {
                if (refactor_lu(s)) return PH_NUMFAIL;
                st->refactors++;
                *since_refactor = 0;
            }
        }
        recheck = 0;
        /* ---- BTRAN: y = B^-T c_B, every iteration ---- */
        for (int64_t p = 0; p < m; ++p) s->cB[p] = s->cost[s->head[p]];
        lu_btran(&s->f, s->cB, s->y, s->t);
        /* ---- pricing: structural column chains, slacks d = c - y_i ---- */
        int64_t q = -1;
        double qscore = 0.0, dq = 0.0, qw = 1.0;
        const double dtol = ctl->tol_dual;
        for (int64_t j = 0; j < n + m; ++j) {
            const int8_t vs = s->vstat[j];
            if (vs == VS_BASIC || s->lb[j] == s->ub[j]) continue;
            double d;
            if (j < n) {
                double acc = 0.0;
                for (int64_t t = s->a.cp[j]; t < s->a.cp[j + 1]; ++t) acc = fma(s->a.cv[t], s->y[s->a.ri[t]], acc);
                d = s->cost[j] - acc;
            } else {
                d = s->cost[j] - s->y[j - n];
            }
            double wj = 1.0;
            if (devex) {
                wj = s->dw[j];
                if (dv_valid && j != dv_lv) {
                    const double r = (s->dprev[j] - d) / dv_dq;
                    double wn = (r * r) * dv_wq;
                    if (wn > DEVEX_WMAX) wn = DEVEX_WMAX;
                    if (wn > wj) {
                        wj = wn;
                        s->dw[j] = wj;
                    }
                }
                s->dprev[j] = d;
            }
            double score = 0.0;
            if ((vs == VS_LOWER || vs == VS_FREE) && d < -dtol) score = devex ? (d * d) / wj : -d;
            else if ((vs == VS_UPPER || vs == VS_FREE) && d > dtol) score = devex ? (d * d) / wj : d;
            else continue;
            if (bland) {
                if (q < 0) {
                    q = j;
                    dq = d;
                    qw = wj;
                }
                if (!devex) break;
                continue;
            }
            if (score > qscore) {
                qscore = score;
                q = j;
                dq = d;
                qw = wj;
            }
        }
        st->price_bytes += 12.0 * (double)s->a.cp[n] + 17.0 * (double)n + 8.0 * (double)m;
        if (q < 0) {
            if (phase == 2 && *since_refactor > 0) { /* after eta updates: confirm on a fresh LU */
                if (refactor_lu(s)) return PH_NUMFAIL;
                st->refactors++;
                *since_refactor = 0;
                recheck = 1;
                continue;
            }
            return PH_OPTIMAL;
        }
        const double sig = dq < 0.0 ? 1.0 : -1.0;
        /* ---- FTRAN ---- */
        for (int64_t i = 0; i < m; ++i) s->acol[i] = 0.0;
        if (q < n) {
            for (int64_t t = s->a.cp[q]; t < s->a.cp[q + 1]; ++t) s->acol[s->a.ri[t]] = s->a.cv[t];
        } else {
            s->acol[q - n] = 1.0;
        }
        lu_ftran(&s->f, s->acol, s->alpha, s->t);
        /* ---- ratio test (Harris two-pass; textbook under Bland) ---- */
        const double ptol = ctl->tol_primal, pivtol = ctl->tol_pivot, INF = HUGE_VAL;
        double theta_max = INF;
        for (int64_t p = 0; p < m; ++p) {
            const int64_t var = s->head[p];
            const double g = sig * s->alpha[p], x = s->xB[p];
            const double l = s->lb[var], u = s->ub[var];
            double r;
            if (g > pivtol && l > -INF) r = bland ? (x - l) / g : (x - l + ptol) / g;
            else if (g < -pivtol && u < INF) r = bland ? (u - x) / (-g) : (u - x + ptol) / (-g);
            else continue;
            if (r < theta_max) theta_max = r;
        }
        int64_t lv = -1, lpos = -1;
        double lg = 0.0, lratio = 0.0;
        for (int64_t p = 0; p < m; ++p) {
            const int64_t var = s->head[p];
            const double g = sig * s->alpha[p], x = s->xB[p];
            const double l = s->lb[var], u = s->ub[var];
            double r;
            if (g > pivtol && l > -INF) r = (x - l) / g;
            else if (g < -pivtol && u < INF) r = (u - x) / (-g);
            else continue;
            if (!(r <= theta_max)) continue;
            int take;
            if (lv < 0) take = 1;
            else if (bland) take = (r < lratio) || (r == lratio && var < lv);
            else take = (fabs(g) > fabs(lg)) || (fabs(g) == fabs(lg) && var < lv);
            if (take) {
                lv = var;
                lpos = p;
                lg = g;
                lratio = r;
            }
        }
        const double theta = lv >= 0 ? (lratio > 0.0 ? lratio : 0.0) : INF;
        const double flip = (s->lb[q] > -INF && s->ub[q] < INF) ? s->ub[q] - s->lb[q] : INF;
        (*iter)++;
        if (phase == 1) st->phase1_iterations++;
        if (flip < INF && flip <= theta) {
            for (int64_t p = 0; p < m; ++p) s->xB[p] = fma(-flip, sig * s->alpha[p], s->xB[p]);
            if (s->vstat[q] == VS_LOWER) {
                s->vstat[q] = VS_UPPER;
                s->xval[q] = s->ub[q];
            } else {
                s->vstat[q] = VS_LOWER;
                s->xval[q] = s->lb[q];
            }
            st->bound_flips++;
            if (trace && *iter - 1 < trace_cap) {
                trace[2 * (*iter - 1)] = q;
                trace[2 * (*iter - 1) + 1] = -1;
            }
            dv_valid = 0;
            ndegen = 0;
            bland = 0;
            continue;
        }
        if (theta == INF) {
            if (trace && *iter - 1 < trace_cap) {
                trace[2 * (*iter - 1)] = q;
                trace[2 * (*iter - 1) + 1] = -2;
            }
            *unb_var = q;
            *unb_sigma = sig;
            return PH_UNBOUNDED;
        }
        if (trace && *iter - 1 < trace_cap) {
            trace[2 * (*iter - 1)] = q;
            trace[2 * (*iter - 1) + 1] = lv;
        }
        if (devex && qw > DEVEX_RESET) {
            for (int64_t j = 0; j < n + m; ++j) s->dw[j] = 1.0;
            dv_valid = 0;
            st->devex_resets++;
        } else if (devex) {
            double wl = qw / (lg * lg);
            if (wl < 1.0) wl = 1.0;
            if (wl > DEVEX_WMAX) wl = DEVEX_WMAX;
            if (lv < n + m) s->dw[lv] = wl;
            dv_valid = 1;
            dv_lv = lv;
            dv_dq = dq;
            dv_wq = qw;
        }
        if (theta == 0.0) {
            st->degenerate++;
            if (++ndegen >= ctl->degen_switch) bland = 1;
        } else {
            ndegen = 0;
            bland = 0;
        }
        /* ---- primal update, basis change, eta ---- */
        for (int64_t p = 0; p < m; ++p) s->xB[p] = fma(-theta, sig * s->alpha[p], s->xB[p]);
        const double xq = s->xval[q] + sig * theta;
        const int at_lower = lg > 0.0;
        if (lv >= n + m) {
            s->lb[lv] = 0.0;
            s->ub[lv] = 0.0;
            s->vstat[lv] = VS_LOWER;
            s->xval[lv] = 0.0;
        } else {
            s->vstat[lv] = at_lower ? VS_LOWER : VS_UPPER;
            s->xval[lv] = at_lower ? s->lb[lv] : s->ub[lv];
        }
        s->vstat[q] = VS_BASIC;
        s->bpos[lv] = -1;
        s->bpos[q] = lpos;
        s->head[lpos] = q;
        s->xB[lpos] = xq;
        eta_append(&s->f, lpos, s->alpha);
        if (s->f.enz > s->eta_nnz_max) s->eta_nnz_max = s->f.enz;
        (*since_refactor)++;
    }
}

static int cmp_i64(const void* a, const void* b) {
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

/* CSC scaling factors (nonzeros only; the product's scale_csc): geometric
   row / column passes, then equilibrate */
static int floor_half(int v) { return v >= 0 ? v / 2 : -((1 - v) / 2); }
static void scale_csc(int64_t m, int64_t n, const int64_t* cp, const int32_t* ri, const double* val, int mode,
                      int32_t* rho, int32_t* gam) {
    const int EMN = 0x3fffffff, EMX = -0x3fffffff;
    for (int64_t i = 0; i < m; ++i) rho[i] = 0;
    for (int64_t j = 0; j < n; ++j) gam[j] = 0;
    int* mn = (int*)malloc(sizeof(int) * (size_t)(m > 0 ? m : 1));
    int* mx = (int*)malloc(sizeof(int) * (size_t)(m > 0 ? m : 1));
    for (int pass = 0; (mode & 4) && pass < 20; ++pass) {
        for (int64_t i = 0; i < m; ++i) {
            mn[i] = EMN;
            mx[i] = EMX;
        }
        for (int64_t j = 0; j < n; ++j)
            for (int64_t t = cp[j]; t < cp[j + 1]; ++t) {
                if (val[t] == 0.0) continue;
                const int e = ilogb(val[t]) + gam[j];
                if (e < mn[ri[t]]) mn[ri[t]] = e;
                if (e > mx[ri[t]]) mx[ri[t]] = e;
            }
        int ch = 0;
        for (int64_t i = 0; i < m; ++i) {
            const int r = mx[i] == EMX ? 0 : -floor_half(mn[i] + mx[i]);
            if (r != rho[i]) {
                rho[i] = r;
                ch = 1;
            }
        }
        int chc = 0;
        for (int64_t j = 0; j < n; ++j) {
            int a = EMN, b = EMX;
            for (int64_t t = cp[j]; t < cp[j + 1]; ++t) {
                if (val[t] == 0.0) continue;
                const int e = ilogb(val[t]) + rho[ri[t]];
                if (e < a) a = e;
                if (e > b) b = e;
            }
            const int g = b == EMX ? 0 : -floor_half(a + b);
            if (g != gam[j]) {
                gam[j] = g;
                chc = 1;
            }
        }
        if (!(ch | chc)) break;
    }
    if (mode & 64)
        for (int64_t j = 0; j < n; ++j) {
            int b = EMX;
            for (int64_t t = cp[j]; t < cp[j + 1]; ++t) {
                if (val[t] == 0.0) continue;
                const int e = ilogb(val[t]) + rho[ri[t]];
                if (e > b) b = e;
            }
            gam[j] = b == EMX ? 0 : -(b + 1);
        }
    free(mn);
    free(mx);
}

int orc_solve_lu(int64_t m, int64_t n, const int64_t* colptr, const int32_t* rowind, const double* val,
                 const int32_t* dir, const double* rhs, const double* obj, const double* lo, const double* up,
                 int32_t maximize, const orc_control* ctl_in, double* objval, double* xout, double* yout,
                 int64_t* basis, int64_t* trace, int64_t trace_cap, orc_stats* st_out) {
    if (m < 0 || n <= 0 || !colptr || !obj || (m > 0 && (!dir || !rhs))) return -1;
    for (int64_t i = 0; i < m; ++i)
        if (dir[i] < 1 || dir[i] > 3) return -2;
    orc_control ctl;
    if (ctl_in) ctl = *ctl_in;
    else orc_default_control(&ctl);
    if (ctl.refactor_period <= 0) ctl.refactor_period = 250;
    if (ctl.degen_switch <= 0) ctl.degen_switch = 50;
    const int64_t max_iter = ctl.max_iter > 0 ? ctl.max_iter : 100 * (m + n) + 10000;
    const double INF = HUGE_VAL, BIG = ctl.infinity;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    orc_stats st;
    memset(&st, 0, sizeof st);
    lus_t S;
    memset(&S, 0, sizeof S);
    lus_t* s = &S;
    const int64_t nnz = colptr[n], mm = m > 0 ? m : 1, nv = n + 2 * m;
    s->m = m;
    s->n = n;
    s->nv = nv;
    s->tol_singular = ctl.tol_singular;
    int32_t* rho = (int32_t*)calloc((size_t)mm, sizeof(int32_t));
    int32_t* gam = (int32_t*)calloc((size_t)n, sizeof(int32_t));
    const int scaled = (ctl.scaling & (4 | 64)) != 0;
    if (scaled) scale_csc(m, n, colptr, rowind, val, ctl.scaling, rho, gam);
    double* cv = dz((size_t)nnz);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t t = colptr[j]; t < colptr[j + 1]; ++t) cv[t] = scaled ? ldexp(val[t], rho[rowind[t]] + gam[j]) : val[t];
    s->asgn = dz((size_t)mm);
    s->a.m = m;
    s->a.n = n;
    s->a.cp = colptr;
    s->a.ri = rowind;
    s->a.cv = cv;
    s->a.asgn = s->asgn;
    /* CSR (counting sort by row: columns ascending within a row) */
    s->rp = iz((size_t)m + 1);
    s->ci = iz((size_t)nnz);
    s->rv = dz((size_t)nnz);
    for (int64_t t = 0; t < nnz; ++t) s->rp[rowind[t] + 1]++;
    for (int64_t i = 0; i < m; ++i) s->rp[i + 1] += s->rp[i];
    {
        int64_t* nx = iz((size_t)m + 1);
        memcpy(nx, s->rp, sizeof(int64_t) * (size_t)(m + 1));
        for (int64_t j = 0; j < n; ++j)
            for (int64_t t = colptr[j]; t < colptr[j + 1]; ++t) {
                const int64_t at = nx[rowind[t]]++;
                s->ci[at] = j;
                s->rv[at] = cv[t];
            }
        free(nx);
    }
    s->b = dz((size_t)mm);
    s->lb = dz((size_t)nv);
    s->ub = dz((size_t)nv);
    s->cost = dz((size_t)nv);
    s->xval = dz((size_t)nv);
    s->vstat = (int8_t*)calloc((size_t)nv, 1);
    s->head = iz((size_t)mm);
    s->bpos = iz((size_t)nv);
    s->xB = dz((size_t)mm);
    s->y = dz((size_t)mm);
    s->cB = dz((size_t)mm);
    s->acol = dz((size_t)mm);
    s->alpha = dz((size_t)mm);
    s->t = dz((size_t)mm);
    s->dw = dz((size_t)(n + m));
    s->dprev = dz((size_t)(n + m));
    for (int64_t v = 0; v < nv; ++v) s->bpos[v] = -1;
#define SCOL(v, j, sg) (scaled ? ldexp((v), (sg) * gam[j]) : (v))
#define SROW(v, i, sg) (scaled ? ldexp((v), (sg) * rho[i]) : (v))
    int status = 0;
    int64_t unb_var = -1;
    double unb_sigma = 0.0, bmax = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        double l = lo ? lo[j] : 0.0, u = up ? up[j] : INF;
        if (l <= -BIG) l = -INF;
        if (u >= BIG) u = INF;
        l = SCOL(l, j, -1);
        u = SCOL(u, j, -1);
        s->lb[j] = l;
        s->ub[j] = u;
        if (l > u) status = 2;
        if (l > -INF) {
            s->vstat[j] = VS_LOWER;
            s->xval[j] = l;
        } else if (u < INF) {
            s->vstat[j] = VS_UPPER;
            s->xval[j] = u;
        } else {
            s->vstat[j] = VS_FREE;
            s->xval[j] = 0.0;
        }
    }
    int64_t iter = 0, since = 0;
    if (status == 0) {
        int any_art = 0;
        for (int64_t i = 0; i < m; ++i) {
            double bi = rhs[i];
            if (bi <= -BIG) bi = -INF;
            if (bi >= BIG) bi = INF;
            bi = SROW(bi, i, 1);
            s->b[i] = bi;
            if (fabs(bi) < INF && fabs(bi) > bmax) bmax = fabs(bi);
            const int64_t sv = n + i, av = n + m + i;
            s->lb[sv] = dir[i] == 2 ? -INF : 0.0;
            s->ub[sv] = dir[i] == 1 ? INF : 0.0;
            s->lb[av] = 0.0;
            s->ub[av] = 0.0;
            s->vstat[av] = VS_LOWER;
            s->asgn[i] = 1.0;
            double acc = 0.0;
            for (int64_t t = s->rp[i]; t < s->rp[i + 1]; ++t) {
                const int64_t j = s->ci[t];
                if (s->xval[j] != 0.0) acc = fma(s->rv[t], s->xval[j], acc);
            }
            const double r = s->b[i] - acc;
            if (r >= s->lb[sv] && r <= s->ub[sv]) {
                s->vstat[sv] = VS_BASIC;
                s->head[i] = sv;
                s->bpos[sv] = i;
                s->xB[i] = r;
            } else {
                const double sl = r < s->lb[sv] ? s->lb[sv] : s->ub[sv];
                s->vstat[sv] = (sl == s->lb[sv]) ? VS_LOWER : VS_UPPER;
                s->xval[sv] = sl;
                const double res = r - sl;
                s->asgn[i] = res > 0.0 ? 1.0 : -1.0;
                s->ub[av] = INF;
                s->cost[av] = 1.0;
                s->vstat[av] = VS_BASIC;
                s->head[i] = av;
                s->bpos[av] = i;
                s->xB[i] = fabs(res);
                any_art = 1;
            }
        }
        s->tol_inf = 1e-9 * (1.0 + bmax);
        /* the slack / artificial basis: its LU (diagonal), no eta */
        if (lu_factor(&s->f, &s->a, s->head, s->tol_singular)) status = 5;
        if (status == 0 && any_art) {
            const int ph = run_phase_lu(s, 1, &ctl, &iter, max_iter, trace, trace_cap, &st, &unb_var, &unb_sigma,
                                        &since);
            if (ph == PH_NUMFAIL) status = 5;
            else if (ph == PH_ITERCAP) status = 1;
            else if (art_sum_lu(s) > s->tol_inf) status = 2;
        }
        if (status == 0) {
            for (int64_t i = 0; i < m; ++i) {
                const int64_t av = n + m + i;
                s->cost[av] = 0.0;
                s->lb[av] = 0.0;
                s->ub[av] = 0.0;
            }
            for (int64_t j = 0; j < n; ++j) s->cost[j] = SCOL(maximize ? -obj[j] : obj[j], j, 1);
            if (any_art) {
                if (refactor_lu(s)) status = 5;
                st.refactors++;
                since = 0;
            }
        }
        if (status == 0) {
            const int ph = run_phase_lu(s, 2, &ctl, &iter, max_iter, trace, trace_cap, &st, &unb_var, &unb_sigma,
                                        &since);
            if (ph == PH_NUMFAIL) status = 5;
            else if (ph == PH_ITERCAP) status = 1;
            else if (ph == PH_UNBOUNDED) status = 3;
            else status = 0;
        }
    }
    /* outputs, unscaled (exact) */
    int64_t kstruct = 0;
    for (int64_t j = 0; j < n; ++j) {
        const double v = SCOL(s->vstat[j] == VS_BASIC ? s->xB[s->bpos[j]] : s->xval[j], j, 1);
        if (s->vstat[j] == VS_BASIC) kstruct++;
        if (xout) xout[j] = (status == 3 && j == unb_var) ? (unb_sigma > 0 ? BIG : -BIG) : v;
    }
    if (objval) {
        if (status == 3) *objval = maximize ? BIG : -BIG;
        else {
            double acc = 0.0;
            for (int64_t j = 0; j < n; ++j)
                acc = fma(obj[j], SCOL(s->vstat[j] == VS_BASIC ? s->xB[s->bpos[j]] : s->xval[j], j, 1), acc);
            *objval = acc;
        }
    }
    if (yout)
        for (int64_t i = 0; i < m; ++i) yout[i] = SROW(maximize ? -s->y[i] : s->y[i], i, 1);
    if (basis && m) {
        for (int64_t p = 0; p < m; ++p) basis[p] = s->head[p];
        qsort(basis, (size_t)m, sizeof(int64_t), cmp_i64);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    st.iterations = iter;
    st.bump_dim = kstruct;
    st.lu_nnz = s->lu_nnz_max;
    st.eta_nnz = s->eta_nnz_max;
    st.seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (st_out) *st_out = st;
#undef SCOL
#undef SROW
    lu_free(&s->f);
    free(rho); free(gam); free(cv); free(s->asgn); free(s->rp); free(s->ci); free(s->rv);
    free(s->b); free(s->lb); free(s->ub); free(s->cost); free(s->xval); free(s->vstat);
    free(s->head); free(s->bpos); free(s->xB); free(s->y); free(s->cB); free(s->acol);
    free(s->alpha); free(s->t); free(s->dw); free(s->dprev);
    return status;
}

/* The factorization alone (tests: the product's host factorization must give
   the same factors): B = the columns head[0..m) of the CSC A (values as given)
   with slack / artificial ids as above (asgn = +1).  Writes the pivot
   sequences and the factor sizes; returns 0, or -1 if singular. */
int orc_lu_factor(int64_t m, int64_t n, const int64_t* colptr, const int32_t* rowind, const double* val,
                  const int64_t* head, double tol_singular, int64_t* prow, int64_t* pcol, double* ud,
                  int64_t* nnz_lu, double* lsum, double* usum) {
    double* asgn = dz((size_t)(m > 0 ? m : 1));
    for (int64_t i = 0; i < m; ++i) asgn[i] = 1.0;
    colsrc a = {m, n, colptr, rowind, val, asgn};
    lu_t f;
    memset(&f, 0, sizeof f);
    const int rc = lu_factor(&f, &a, head, tol_singular);
    if (!rc) {
        memcpy(prow, f.prow, sizeof(int64_t) * (size_t)m);
        memcpy(pcol, f.pcol, sizeof(int64_t) * (size_t)m);
        memcpy(ud, f.ud, sizeof(double) * (size_t)m);
        nnz_lu[0] = f.L.nnz;
        nnz_lu[1] = f.U.nnz;
        /* order-sensitive checksums of the factor values */
        double a1 = 0.0, a2 = 0.0;
        for (int64_t t = 0; t < f.L.nnz; ++t) a1 = fma(a1, 1.0000001, f.L.v[t] * (double)(f.L.j[t] + 1));
        for (int64_t t = 0; t < f.U.nnz; ++t) a2 = fma(a2, 1.0000001, f.U.v[t] * (double)(f.U.j[t] + 1));
        *lsum = a1;
        *usum = a2;
    }
    lu_free(&f);
    free(asgn);
    return rc;
}
