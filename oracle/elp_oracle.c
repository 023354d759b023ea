/*
 * elp_oracle.c -- CPU restatement of the dense revised-simplex hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see elp_oracle.h).  Compiled with
 * -ffp-contract=off; every fused multiply-add below is an explicit fma()
 * so that the HIP kernels (also -ffp-contract=off, explicit fma) produce
 * the same bits.  Reduction orders follow DESIGN.md "Reduction order
 * contract":
 *   price  : PRICE_SPLIT (4) slot classes p = w (mod PRICE_SPLIT), an fma chain per
 *            class in slot order, then the partials added in class order starting
 *            from 0.0 (PRICE_SPLIT)
 *   wave   : 64 lane-strided fma chains + pairwise tree, offsets 1,2,..,32 (wave_dot):
 *            FTRAN / BTRAN / B^-1 rows, phase-1 c_S correction, phase-1 sum
 *   zchunk : chunks of 32 bump positions, fma chain, sequential sum
 *   seq    : one fma chain in index order (row activities)
 *   column : price_mode 1 (the CSC path, elp_load_csc): d_j = c_j - one fma
 *            chain over column j's nonzero rows in ascending row order, with
 *            the full dual vector y (zero on slack-covered rows)
 *
 * Algorithm (bounded primal revised simplex, minimisation form):
 *   - rows a_i'x + s_i = b_i; slack bounds encode dir (R/class.R:271-274,
 *     "==" -> "=" at :272): '<=' [0,inf), '>=' (-inf,0], '==' [0,0];
 *   - the basis B is kept as unit columns (slacks / artificials) covering
 *     m-k rows plus a k x k "bump" M = A[R,S] (R: uncovered rows,
 *     S: basic structurals) whose inverse Minv is stored explicitly and
 *     updated by rank-one / bordered formulas (cases A-E below);
 *   - dual y is zero on slack-covered rows, so pricing sweeps only the
 *     rows Y = {i : slack i nonbasic}, kept as a row-major copy AR;
 *   - Devex pricing (price_rule 1, the default: largest d_j^2 / w_j with
 *     reference weights w updated from consecutive passes' reduced costs,
 *     run_phase) or Dantzig (price_rule 0: largest |d_j|); lowest index on
 *     ties.  lp_solve's default pricer is DEVEX (lp_solve 5.5 set_pivoting,
 *     PRICER_DEVEX + PRICE_ADAPTIVE); its exact weight recurrences are not in
 *     the reference, so this restatement defines the arithmetic.  Harris
 *     two-pass ratio test (largest |alpha|, lowest variable id on ties),
 *     bound flips, Bland fallback after a run of degenerate pivots,
 *     Gauss-Jordan refactor of M every refactor_period pivots;
 *   - phase 1 minimises the sum of artificials, phase 2 the real costs.
 */
#include "elp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define VS_BASIC 0
#define VS_LOWER 1
#define VS_UPPER 2
#define VS_FREE 3

#ifndef PRICE_SPLIT
#define PRICE_SPLIT 4 /* = the HIP side's ELP_PRICE_SPLIT */
#endif
#define ZCHUNK 32
#define WAVE 64
#define DEVEX_WMAX 1e20   /* Devex weight cap (both sides of the parity contract) */
#define DEVEX_RESET 1e6   /* entering weight above this: new reference framework */

/* ------------------------------------------------------------------ */
/* synthetic generator (bit-identical in HIP and numpy)                */
/* ------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline double gen_u01(uint64_t seed, uint64_t stream, uint64_t idx) {
    uint64_t key = mix64(seed * 0x9E3779B97F4A7C15ULL + stream * 0xD1B54A32D192ED03ULL +
                         0x632BE59BD9B4E019ULL);
    uint64_t z = mix64(key + (idx + 1) * 0x9E3779B97F4A7C15ULL);
    return (double)(z >> 11) * 0x1.0p-53;
}

void orc_generate_dense(uint64_t seed, int64_t m, int64_t n, int64_t col0, int64_t ncols,
                        double* A, double* b, double* c) {
    if (A)
        for (int64_t jj = 0; jj < ncols; ++jj) {
            const uint64_t j = (uint64_t)(col0 + jj);
            for (int64_t i = 0; i < m; ++i)
                A[(size_t)jj * (size_t)m + (size_t)i] =
                    gen_u01(seed, 0, (uint64_t)i + j * (uint64_t)m);
        }
    if (c)
        for (int64_t jj = 0; jj < ncols; ++jj) c[jj] = gen_u01(seed, 1, (uint64_t)(col0 + jj));
    if (b) {
        const double e = (double)n / 8.0, q = (double)n / 4.0;
        for (int64_t i = 0; i < m; ++i) b[i] = e + gen_u01(seed, 2, (uint64_t)i) * q;
    }
}

/* scaling exponents of a dense column-major A (test access to scale_factors) */
static void scale_factors_dense(int64_t m, int64_t n, const double* A, int mode, int32_t* rho, int32_t* gam);
void orc_scale_factors(int64_t m, int64_t n, const double* A, int32_t mode, int32_t* rho, int32_t* gam) {
    scale_factors_dense(m, n, A, mode, rho, gam);
}

void orc_generate_rows(uint64_t seed, int64_t m, int64_t n, const int64_t* rows, int64_t nrows,
                       double* out) {
    (void)n;
    for (int64_t r = 0; r < nrows; ++r)
        for (int64_t j = 0; j < n; ++j)
            out[(size_t)r * (size_t)n + (size_t)j] =
                gen_u01(seed, 0, (uint64_t)rows[r] + (uint64_t)j * (uint64_t)m);
}

/* ------------------------------------------------------------------ */
/* solver state                                                        */
/* ------------------------------------------------------------------ */
typedef struct {
    int64_t m, n, nv;
    const double* A; /* column-major m x n; NULL: generated on the fly (gen_seed) */
    uint64_t gen_seed;
    int32_t *srow, *scol; /* scaling exponents (NULL: unscaled): the solver sees
                             a_ij * 2^(srow_i + scol_j) */
    int a_scaled;         /* A (a scaled copy) already holds those values   */
    double* A_copy;       /* that copy (freed at the end)                   */
    double* b;
    double *lb, *ub, *cost, *xval;
    int8_t* vstat;
    double* asgn;     /* m: sign of artificial column n+m+i            */
    int64_t k;        /* bump dimension                                 */
    int64_t *cover;   /* m: covering unit variable or -1               */
    int64_t *rpos;    /* m: position in Rl or -1                       */
    int64_t *Rl, *Sl; /* m each                                         */
    int64_t* spos;    /* n: position in Sl or -1                       */
    double *xr, *xs;  /* values: covered rows, bump positions           */
    double* Minv;     /* m x m capacity, row-major, ld = ldm           */
    int64_t ldm;
    int64_t ny, ycap; /* Y slots                                        */
    int64_t *Yl, *ypos;
    double* AR; /* ycap x n row-major                                   */
    /* work */
    double *y, *t, *yR, *yy, *acol, *aR, *alS, *alU, *z, *v, *tmp, *part;
    int8_t* used;
    int64_t* perm;
    double tol_inf;
    int64_t nnz;      /* nonzeros of A (price_mode 1 byte count)          */
    int64_t *cp, *ri; /* price_mode 1: nonzero pattern of A by column      */
    int64_t gj_count; /* refactors that needed a fresh Gauss-Jordan */
    double emax_max;  /* largest Newton-Schulz residual max|E| seen  */
    int refactor_mode;
    double tol_singular;
    double *dw, *dprev; /* price_rule 1: Devex weight and last reduced cost
                           of each structural and slack (n + m)            */
    int64_t* nzl;       /* n: nz_nonbasic list                              */
    double* colbuf;     /* m: a generated column (Acol)                     */
    /* dual simplex (run_dual): the pivot row's class partials, rho_r dense
     * (m) and on the Y slots, the pass's reduced costs / pivot row (n + m) */
    double *apart, *rho, *rhoY, *dvec, *avec;
    /* its bound-flipping ratio test: candidate id, exact ratio, Harris bound,
     * |alpha|, u - l (inf: not boxed), alive; the flipped ids; a_F, B^-1 a_F */
    int64_t *cj, *flips;
    double *ct, *cb, *ca, *cr, *aF, *fS;
    int8_t* calive;
} orc_t;

/* v * 2^(sgn * exponent) of column j / row i (scaling; exact, inf stays inf) */
#define SC_COL(v, j, sgn) (s->scol ? ldexp((v), (sgn) * s->scol[j]) : (v))
#define SC_ROW(v, i, sgn) (s->srow ? ldexp((v), (sgn) * s->srow[i]) : (v))

static double* dalloc(size_t n) { return (double*)calloc(n ? n : 1, sizeof(double)); }
static int64_t* ialloc(size_t n) { return (int64_t*)calloc(n ? n : 1, sizeof(int64_t)); }

static inline double Araw(const orc_t* s, int64_t i, int64_t j) {
    if (!s->A) return gen_u01(s->gen_seed, 0, (uint64_t)i + (uint64_t)j * (uint64_t)s->m);
    return s->A[(size_t)j * (size_t)s->m + (size_t)i];
}
/* the matrix the simplex works on: A scaled (exactly: powers of 2) */
static inline double Aat(const orc_t* s, int64_t i, int64_t j) {
    const double a = Araw(s, i, j);
    return s->srow && !s->a_scaled ? ldexp(a, s->srow[i] + s->scol[j]) : a;
}
/* column j of the scaled A (in place when materialised, else built in buf) */
static inline const double* Acol(const orc_t* s, int64_t j, double* buf) {
    if (s->A && (!s->srow || s->a_scaled)) return &s->A[(size_t)j * (size_t)s->m];
    for (int64_t i = 0; i < s->m; ++i) buf[i] = Aat(s, i, j);
    return buf;
}

/* ------------------------------------------------------------------ */
/* scaling (the HIP side's k_scale_*): on the integer exponents            */
/* e_ij = ilogb|a_ij| of the nonzeros, geometric passes (at most 20, row    */
/* pass then column pass, until no factor moves) set each exponent to       */
/* -floor((min + max) / 2) of the currently scaled entries (lp_solve's      */
/* SCALE_GEOMETRIC, sqrt(min * max), in the log domain); equilibrate sets    */
/* each column's to -(max + 1) so its largest |a| lies in [1/2, 1)          */
/* (SCALE_EQUILIBRATE).  lp_solve's own scaling loop is not in the          */
/* reference: this arithmetic is the contract both sides implement.         */
#define SCALE_PASSES 20
#define SC_EMPTY_MIN 0x3fffffff
#define SC_EMPTY_MAX (-0x3fffffff)
static int floor_half(int v) { return v >= 0 ? v / 2 : -((1 - v) / 2); }
static int col_pass(const orc_t* s, int32_t* rho, int32_t* gam, int equilibrate) {
    int changed = 0;
    for (int64_t j = 0; j < s->n; ++j) {
        int mn = SC_EMPTY_MIN, mx = SC_EMPTY_MAX;
        for (int64_t i = 0; i < s->m; ++i) {
            const double a = Araw(s, i, j);
            if (a == 0.0 || !isfinite(a)) continue; /* (non-finite: no exponent) */
            const int e = ilogb(a) + rho[i];
            if (e < mn) mn = e;
            if (e > mx) mx = e;
        }
        const int g = mx == SC_EMPTY_MAX ? 0 : equilibrate ? -(mx + 1) : -floor_half(mn + mx);
        if (g != gam[j]) {
            gam[j] = g;
            changed = 1;
        }
    }
    return changed;
}
static int row_pass(const orc_t* s, int32_t* rho, const int32_t* gam) {
    const int64_t m = s->m, n = s->n;
    int* mn = (int*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int));
    int* mx = (int*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int));
    for (int64_t i = 0; i < m; ++i) {
        mn[i] = SC_EMPTY_MIN;
        mx[i] = SC_EMPTY_MAX;
    }
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i) {
            const double a = Araw(s, i, j);
            if (a == 0.0 || !isfinite(a)) continue;
            const int e = ilogb(a) + gam[j];
            if (e < mn[i]) mn[i] = e;
            if (e > mx[i]) mx[i] = e;
        }
    int changed = 0;
    for (int64_t i = 0; i < m; ++i) {
        const int r = mx[i] == SC_EMPTY_MAX ? 0 : -floor_half(mn[i] + mx[i]);
        if (r != rho[i]) {
            rho[i] = r;
            changed = 1;
        }
    }
    free(mn);
    free(mx);
    return changed;
}
static void scale_factors(const orc_t* s, int mode, int32_t* rho, int32_t* gam) {
    for (int64_t i = 0; i < s->m; ++i) rho[i] = 0;
    for (int64_t j = 0; j < s->n; ++j) gam[j] = 0;
    if (mode & 4)
        for (int pass = 0; pass < SCALE_PASSES; ++pass) {
            const int ch = row_pass(s, rho, gam);
            if (!(col_pass(s, rho, gam, 0) | ch)) break;
        }
    if (mode & 64) col_pass(s, rho, gam, 1);
}
static void scale_factors_dense(int64_t m, int64_t n, const double* A, int mode, int32_t* rho, int32_t* gam) {
    orc_t t;
    memset(&t, 0, sizeof t);
    t.m = m;
    t.n = n;
    t.A = A;
    scale_factors(&t, mode, rho, gam);
}
/* ascending list of nonbasic structurals with x_j != 0 (row activities) */
static int64_t nz_nonbasic(const orc_t* s, int64_t* list) {
    int64_t c = 0;
    for (int64_t j = 0; j < s->n; ++j)
        if (s->vstat[j] != VS_BASIC && s->xval[j] != 0.0) list[c++] = j;
    return c;
}
static inline double unit_sign(const orc_t* s, int64_t var) {
    return var >= s->n + s->m ? s->asgn[var - s->n - s->m] : 1.0;
}
static inline double* MI(orc_t* s, int64_t r, int64_t c) {
    return &s->Minv[(size_t)r * (size_t)s->ldm + (size_t)c];
}

/* the GPU's wave sum (elp_kernels.hip wave_tree): pairs of lanes, then pairs
   of pairs, ... -- offsets 1, 2, 4, ..., 32 ascending; lane 0's value */
static double wave_tree(double* lane) {
    for (int off = 1; off < WAVE; off <<= 1)
        for (int l = 0; l + off < WAVE; l += 2 * off) lane[l] = lane[l] + lane[l + off];
    return lane[0];
}

/* wave order: 64 lane-strided fma chains, then the wave tree */
static double wave_dot(int64_t len, const double* a, const double* b) {
    double lane[WAVE];
    for (int l = 0; l < WAVE; ++l) {
        double acc = 0.0;
        for (int64_t i = l; i < len; i += WAVE) acc = fma(a[i], b[i], acc);
        lane[l] = acc;
    }
    return wave_tree(lane);
}

/* z_i = sum_p A[i, S_p] * w_p in ZCHUNK order */
static double zchunk_row(const orc_t* s, int64_t i, const double* w) {
    double tot = 0.0;
    for (int64_t c0 = 0; c0 < s->k; c0 += ZCHUNK) {
        double acc = 0.0;
        const int64_t c1 = c0 + ZCHUNK < s->k ? c0 + ZCHUNK : s->k;
        for (int64_t p = c0; p < c1; ++p) acc = fma(Aat(s, i, s->Sl[p]), w[p], acc);
        tot = tot + acc;
    }
    return tot;
}

/* v_c = sum_q A[i, S_q] * Minv[q][c]  (wave order over q: one wave per c,
 * reading row c of Minv^T) */
static void row_times_minv(orc_t* s, int64_t i, double* out) {
    const int64_t k = s->k;
    for (int64_t q = 0; q < k; ++q) s->aR[q] = Aat(s, i, s->Sl[q]);
    for (int64_t c = 0; c < k; ++c) {
        for (int64_t q = 0; q < k; ++q) s->tmp[q] = *MI(s, q, c);
        out[c] = wave_dot(k, s->tmp, s->aR);
    }
}

static int y_grow(orc_t* s) {
    int64_t nc = s->ycap ? s->ycap * 2 : 16;
    if (nc > s->m) nc = s->m;
    double* p = (double*)realloc(s->AR, (size_t)nc * (size_t)s->n * sizeof(double) + 8);
    if (!p) return -1;
    s->AR = p;
    s->ycap = nc;
    return 0;
}
static int y_append(orc_t* s, int64_t i) {
    if (s->ny == s->ycap && y_grow(s)) return -1;
    const int64_t p = s->ny++;
    s->Yl[p] = i;
    s->ypos[i] = p;
    double* row = s->AR + (size_t)p * (size_t)s->n;
    for (int64_t j = 0; j < s->n; ++j) row[j] = Aat(s, i, j);
    return 0;
}
static void y_remove(orc_t* s, int64_t i) {
    const int64_t p = s->ypos[i], last = s->ny - 1;
    if (p != last) {
        s->Yl[p] = s->Yl[last];
        s->ypos[s->Yl[p]] = p;
        memcpy(s->AR + (size_t)p * (size_t)s->n, s->AR + (size_t)last * (size_t)s->n,
               (size_t)s->n * sizeof(double));
    }
    s->ypos[i] = -1;
    s->ny--;
}

/* ------------------------------------------------------------------ */
/* refactor: one Newton-Schulz correction of the maintained inverse    */
/* (E = I - M Minv; Minv += Minv E) when max|E| <= NS_TOL; from         */
/* NS_TOL up to NS_TOL2 a correction and, if the new residual is within */
/* NS_TOL, a second one (the residual squares: 1e-3 -> ~1e-6 -> ~1e-12, */
/* two k^3 products instead of a k-step Gauss-Jordan -- r06: 64 ms of   */
/* the CSC feasible-start LP's 0.53 s went into one at k = 3 452);      */
/* otherwise a fresh Gauss-Jordan inversion with partial pivoting; then */
/* x_B from b.                                                          */
/* ------------------------------------------------------------------ */
#define NS_TOL 1e-6
#define NS_TOL2 1e-2

static int gauss_jordan(orc_t* s) {
    const int64_t k = s->k;
    double *W = s->tmp, *W2 = s->tmp + (size_t)k * (size_t)k;
    for (int64_t a = 0; a < k; ++a)
        for (int64_t c = 0; c < k; ++c) W[a * k + c] = Aat(s, s->Rl[a], s->Sl[c]);
    memset(s->used, 0, (size_t)k);
    for (int64_t c = 0; c < k; ++c) {
        int64_t p = -1;
        double best = -1.0;
        for (int64_t r = 0; r < k; ++r)
            if (!s->used[r] && fabs(W[r * k + c]) > best) {
                best = fabs(W[r * k + c]);
                p = r;
            }
        const double piv = W[p * k + c];
        if (!(fabs(piv) > s->tol_singular)) return -1;
        s->perm[c] = p;
        for (int64_t r = 0; r < k; ++r) {
            if (r == p) {
                for (int64_t j = 0; j < k; ++j)
                    W2[r * k + j] = (j == c) ? 1.0 / piv : W[p * k + j] / piv;
            } else { /* (the zero rule, as basis_change's: a zero factor or quotient leaves the entry) */
                const double f = W[r * k + c];
                for (int64_t j = 0; j < k; ++j) {
                    if (j == c) {
                        W2[r * k + j] = -(f / piv);
                        continue;
                    }
                    const double q = W[p * k + j] / piv;
                    W2[r * k + j] = (f == 0.0 || q == 0.0) ? W[r * k + j] : fma(-f, q, W[r * k + j]);
                }
            }
        }
        s->used[p] = 1;
        double* sw = W;
        W = W2;
        W2 = sw;
    }
    for (int64_t a = 0; a < k; ++a)
        for (int64_t c = 0; c < k; ++c) *MI(s, a, s->perm[c]) = W[s->perm[a] * k + c];
    return 0;
}

/* one Newton-Schulz step; returns 1 if applied, 0 if the residual is   */
/* above tol (nothing changed)                                          */
static int newton_schulz(orc_t* s, double tol) {
    const int64_t k = s->k;
    double *E = s->tmp, *Mk = s->tmp + (size_t)k * (size_t)k;
    for (int64_t a = 0; a < k; ++a)
        for (int64_t c = 0; c < k; ++c) Mk[a * k + c] = Aat(s, s->Rl[a], s->Sl[c]);
    double emax = 0.0;
    for (int64_t i = 0; i < k; ++i)
        for (int64_t j = 0; j < k; ++j) {
            double acc = 0.0; /* (M Minv)_ij, seq order over l */
            for (int64_t l = 0; l < k; ++l) acc = fma(Mk[i * k + l], *MI(s, l, j), acc);
            const double e = (i == j ? 1.0 : 0.0) - acc;
            E[i * k + j] = e;
            if (fabs(e) > emax) emax = fabs(e);
        }
    if (emax > s->emax_max) s->emax_max = emax;
    if (!(emax <= tol)) return 0;
    /* Minv_new[i][j] = Minv[i][j] + sum_l Minv[i][l] E[l][j]  (seq, from Minv[i][j]) */
    double* Nw = Mk;
    for (int64_t i = 0; i < k; ++i)
        for (int64_t j = 0; j < k; ++j) {
            double acc = *MI(s, i, j);
            for (int64_t l = 0; l < k; ++l) acc = fma(*MI(s, i, l), E[l * k + j], acc);
            Nw[i * k + j] = acc;
        }
    for (int64_t i = 0; i < k; ++i)
        for (int64_t j = 0; j < k; ++j) *MI(s, i, j) = Nw[i * k + j];
    return 1;
}

static int refactor(orc_t* s) {
    const int64_t k = s->k, m = s->m, n = s->n;
    int ok = 0;
    if (k > 0 && s->refactor_mode == 0) {
        ok = newton_schulz(s, NS_TOL);
        if (!ok && newton_schulz(s, NS_TOL2)) ok = newton_schulz(s, NS_TOL);
    }
    if (k > 0 && !ok) {
        s->gj_count++;
        if (gauss_jordan(s)) return -1;
    }
    /* primal values: rhs_i = (b_i - sum_{j nonbasic struct, x_j != 0} a_ij x_j) - s_i */
    const int64_t nz = nz_nonbasic(s, s->nzl);
    (void)n;
    for (int64_t i = 0; i < m; ++i) {
        double acc = 0.0;
        for (int64_t t = 0; t < nz; ++t) acc = fma(Aat(s, i, s->nzl[t]), s->xval[s->nzl[t]], acc);
        double r = s->b[i] - acc;
        if (s->vstat[n + i] != VS_BASIC) r = r - s->xval[n + i];
        s->acol[i] = r;
    }
    for (int64_t p = 0; p < k; ++p) s->aR[p] = s->acol[s->Rl[p]];
    for (int64_t p = 0; p < k; ++p) s->xs[p] = wave_dot(k, MI(s, p, 0), s->aR);
    for (int64_t i = 0; i < m; ++i)
        if (s->cover[i] >= 0) s->xr[i] = unit_sign(s, s->cover[i]) * (s->acol[i] - zchunk_row(s, i, s->xs));
    return 0;
}

/* ------------------------------------------------------------------ */
/* one phase of the simplex                                           */
/* ------------------------------------------------------------------ */
enum { PH_OPTIMAL = 0, PH_UNBOUNDED = 3, PH_NUMFAIL = 5, PH_ITERCAP = 1, PH_P1DONE = 10, PH_INFEAS = 2 };

/* phase-1 infeasibility sum, in wave order (one 64-lane wave on the GPU) */
static double art_sum(const orc_t* s) {
    double lane[WAVE];
    for (int l = 0; l < WAVE; ++l) {
        double acc = 0.0;
        for (int64_t i = l; i < s->m; i += WAVE)
            if (s->cover[i] >= s->n + s->m) acc = acc + s->xr[i];
        lane[l] = acc;
    }
    return wave_tree(lane);
}

/* basic entry e: covered row e (< m) or bump position e - m */
static inline int basic_entry(const orc_t* s, int64_t e, double sig, int64_t* var, double* g,
                              double* x) {
    if (e < s->m) {
        if (s->cover[e] < 0) return 0;
        *var = s->cover[e];
        *g = sig * s->alU[e];
        *x = s->xr[e];
    } else {
        const int64_t p = e - s->m;
        *var = s->Sl[p];
        *g = sig * s->alS[p];
        *x = s->xs[p];
    }
    return 1;
}

/* y = B^-T c_B: covered rows take their unit variable's cost, the R rows
 * y_R = Minv' t with t_p = c_{S_p} - A[:,S_p]' y_cov (phase 1; y_cov = 0 in
 * phase 2 and in the dual, whose unit variables are the zero-cost slacks) */
static void btran(orc_t* s, int phase) {
    const int64_t m = s->m, k = s->k;
    for (int64_t i = 0; i < m; ++i) {
        const int64_t u = s->cover[i];
        s->y[i] = u >= 0 ? unit_sign(s, u) * s->cost[u] : 0.0;
    }
    /* wave order over all m rows with y = 0 on uncovered rows */
    if (phase == 1) {
        for (int64_t p = 0; p < k; ++p)
            s->t[p] = s->cost[s->Sl[p]] - wave_dot(m, Acol(s, s->Sl[p], s->colbuf), s->y);
    } else {
        for (int64_t p = 0; p < k; ++p) s->t[p] = s->cost[s->Sl[p]];
    }
    /* y_R = Minv' t: one wave per p over row p of Minv^T */
    for (int64_t p = 0; p < k; ++p) {
        for (int64_t q = 0; q < k; ++q) s->tmp[q] = *MI(s, q, p);
        s->yR[p] = wave_dot(k, s->tmp, s->t);
    }
    for (int64_t p = 0; p < k; ++p) s->y[s->Rl[p]] = s->yR[p];
}

/* Basis change after a pivot: entering q (now basic, value xq), leaving lv
 * (covered row lrow or bump position lpos); cases A-E of the header, the
 * bump inverse update, and -- phase 2 -- the dual update y += theta_d rho_r
 * with theta_d = dq / alpha_rq (run_phase and run_dual share it).  Returns
 * -1 on a numerical failure (case E off its row, AR growth).
 * The zero rule (r05): a rank-one term whose multiplier (the row's factor or
 * the pivot-row entry) is zero leaves the entry as it is -- fma(-w, v, m)
 * would return m then too, except m = -0 with a +0 product (+0) -- so the
 * HIP update can skip the rows and entries it does not change
 * (apply_minv_sru) and still match these bits. */
static int basis_change(orc_t* s, int phase, int64_t q, int64_t lv, int64_t lrow, int64_t lpos, double dq,
                        double xq) {
    const int64_t m = s->m, n = s->n, k = s->k;
    const int leave_art = lv >= n + m;
    /* ---- basis change ---- */
    if (q < n) {
        if (lpos >= 0) {
            /* case A: structural replaces structural at bump position lpos */
            const int64_t p = lpos;
            const double piv = s->alS[p];
            for (int64_t j = 0; j < k; ++j) s->v[j] = *MI(s, p, j) / piv;
            if (phase == 2) /* dual update: rho_r = Minv row p, theta_d = dq / piv */
                for (int64_t j = 0; j < k; ++j) s->y[s->Rl[j]] = fma(dq, s->v[j], s->y[s->Rl[j]]);
            for (int64_t i = 0; i < k; ++i) {
                if (i == p) continue;
                const double wi = s->alS[i];
                if (wi == 0.0) continue; /* (the zero rule) */
                for (int64_t j = 0; j < k; ++j)
                    if (s->v[j] != 0.0) *MI(s, i, j) = fma(-wi, s->v[j], *MI(s, i, j));
            }
            for (int64_t j = 0; j < k; ++j) *MI(s, p, j) = s->v[j];
            s->spos[lv] = -1;
            s->Sl[p] = q;
            s->spos[q] = p;
            s->xs[p] = xq;
        } else {
            /* case B: structural enters, unit var of row lrow leaves; bump grows */
            const int64_t i = lrow;
            const double delta = s->acol[i] - s->z[i];
            row_times_minv(s, i, s->v);
            for (int64_t c = 0; c < k; ++c) s->v[c] = s->v[c] / delta;
            if (phase == 2) { /* dual update: row i joins R with y_i = dq / delta */
                for (int64_t c = 0; c < k; ++c) s->y[s->Rl[c]] = fma(-dq, s->v[c], s->y[s->Rl[c]]);
                s->y[i] = dq / delta;
            }
            for (int64_t a = 0; a < k; ++a) {
                const double wa = s->alS[a];
                if (wa == 0.0) continue;
                for (int64_t c = 0; c < k; ++c)
                    if (s->v[c] != 0.0) *MI(s, a, c) = fma(wa, s->v[c], *MI(s, a, c));
            }
            for (int64_t a = 0; a < k; ++a) *MI(s, a, k) = -(s->alS[a] / delta);
            for (int64_t c = 0; c < k; ++c) *MI(s, k, c) = -s->v[c];
            *MI(s, k, k) = 1.0 / delta;
            s->Rl[k] = i;
            s->rpos[i] = k;
            s->Sl[k] = q;
            s->spos[q] = k;
            s->xs[k] = xq;
            s->cover[i] = -1;
            s->k = k + 1;
            if (!leave_art && y_append(s, i)) return -1;
        }
    } else {
        const int64_t i0 = q - n;
        const int64_t a = s->rpos[i0];
        if (a < 0) {
            /* case E: slack replaces the artificial covering the same row */
            if (lrow != i0) return -1;
            s->cover[i0] = q;
            s->xr[i0] = xq;
        } else if (lpos >= 0) {
            /* case C: slack of row i0 (in R) enters, structural at lpos leaves */
            const int64_t b = lpos, last = k - 1;
            const double piv = *MI(s, b, a);
            for (int64_t c = 0; c < k; ++c) s->v[c] = *MI(s, b, c) / piv;
            if (phase == 2) { /* dual update; row i0 leaves R (y = 0) */
                for (int64_t c = 0; c < k; ++c)
                    if (c != a) s->y[s->Rl[c]] = fma(dq, s->v[c], s->y[s->Rl[c]]);
                s->y[i0] = 0.0;
            }
            for (int64_t r = 0; r < k; ++r) {
                if (r == b) continue;
                const double f = *MI(s, r, a);
                if (f == 0.0) continue;
                for (int64_t c = 0; c < k; ++c)
                    if (c != a && s->v[c] != 0.0) *MI(s, r, c) = fma(-f, s->v[c], *MI(s, r, c));
            }
            if (b != last) {
                for (int64_t c = 0; c < k; ++c) *MI(s, b, c) = *MI(s, last, c);
                s->Sl[b] = s->Sl[last];
                s->spos[s->Sl[b]] = b;
                s->xs[b] = s->xs[last];
            }
            if (a != last) {
                for (int64_t r = 0; r < k; ++r) *MI(s, r, a) = *MI(s, r, last);
                s->Rl[a] = s->Rl[last];
                s->rpos[s->Rl[a]] = a;
            }
            s->spos[lv] = -1;
            s->rpos[i0] = -1;
            s->cover[i0] = q;
            s->xr[i0] = xq;
            s->k = k - 1;
        } else {
            /* case D: slack of row i0 (in R) enters, unit var of row i1 leaves */
            const int64_t i1 = lrow;
            row_times_minv(s, i1, s->v);
            const double piv = s->v[a];
            if (phase == 2) { /* dual update; row i1 takes position a */
                const double w = dq / piv;
                for (int64_t c = 0; c < k; ++c)
                    if (c != a) s->y[s->Rl[c]] = fma(w, s->v[c], s->y[s->Rl[c]]);
                s->y[i0] = 0.0;
                s->y[i1] = -w;
            }
            for (int64_t r = 0; r < k; ++r) s->t[r] = *MI(s, r, a) / piv;
            for (int64_t r = 0; r < k; ++r) {
                const double f = s->t[r];
                if (f != 0.0)
                    for (int64_t c = 0; c < k; ++c)
                        if (c != a && s->v[c] != 0.0) *MI(s, r, c) = fma(-f, s->v[c], *MI(s, r, c));
                *MI(s, r, a) = f;
            }
            s->Rl[a] = i1;
            s->rpos[i1] = a;
            s->rpos[i0] = -1;
            s->cover[i1] = -1;
            s->cover[i0] = q;
            s->xr[i0] = xq;
        }
        y_remove(s, i0);
        if (a >= 0 && lpos < 0 && !leave_art) {
            if (y_append(s, lrow)) return -1;
        }
    }
    return 0;
}

static int run_phase(orc_t* s, int phase, const orc_control* ctl, int64_t* iter, int64_t max_iter,
                     int64_t* trace, int64_t trace_cap, orc_stats* st, int64_t* unb_var,
                     double* unb_sigma) {
    const int64_t m = s->m, n = s->n;
    int64_t since_refactor = 0, ndegen = 0;
    int bland = 0;
    /* phase 2 keeps y by the dual update y += theta_d rho_r after each pivot
     * (the cases below); BTRAN recomputes it only when y_valid == 0: at the
     * phase start and after every refactor.  Optimality found with updated
     * duals is re-checked after a refactor (recheck: no loop-top checks). */
    int y_valid = 0, recheck = 0;
    /* Devex (price_rule 1): reference framework = the nonbasic set at the
     * phase start (all weights 1).  After a pivot with entering q (reduced
     * cost d_q, weight w_q) the next pricing pass has d_j' = d_j - (d_q /
     * alpha_rq) alpha_rj, so the pivot-row ratio alpha_rj / alpha_rq is
     * (d_j - d_j') / d_q -- read off the two passes' reduced costs without
     * forming the pivot row -- and w_j = max(w_j, (alpha_rj / alpha_rq)^2 w_q);
     * the leaving variable takes max(w_q / alpha_rq^2, 1).  Bound flips change
     * no d (dv_valid = 0).  Weights are capped at DEVEX_WMAX; a pivot whose
     * entering weight exceeds DEVEX_RESET restarts the framework (all 1). */
    const int devex = ctl->price_rule == 1;
    int dv_valid = 0;
    int64_t dv_lv = -1;
    double dv_dq = 1.0, dv_wq = 1.0;
    if (devex)
        for (int64_t j = 0; j < n + m; ++j) s->dw[j] = 1.0;
    for (;;) {
        if (*iter == ctl->t_mark_iter && st->seconds_at_mark == 0.0) {
            struct timespec tm;
            clock_gettime(CLOCK_MONOTONIC, &tm);
            st->seconds_at_mark = (double)tm.tv_sec + 1e-9 * (double)tm.tv_nsec;
        }
        if (!recheck) {
            if (phase == 1 && art_sum(s) <= s->tol_inf) return PH_P1DONE;
            if (*iter >= max_iter) return PH_ITERCAP;
            if (since_refactor >= ctl->refactor_period) {
                if (refactor(s)) return PH_NUMFAIL;
                st->refactors++;
                since_refactor = 0;
                y_valid = 0;
            }
        }
        recheck = 0;
        const int64_t k = s->k;
        /* ---- BTRAN (phase 1: every iteration) ---- */
        if (phase == 1 || !y_valid) {
            y_valid = 1;
            btran(s, phase);
        }
        /* ---- pricing over structurals (AR sweep) and slacks ---- */
        const int64_t ny = s->ny;
        for (int64_t p = 0; p < ny; ++p) s->yy[p] = s->y[s->Yl[p]];
        if (ctl->price_mode == 1) {
            /* column chains (CSC): the sum lands in part[0], part[1..] stay 0
             * and add exactly */
            for (int w = 1; w < PRICE_SPLIT; ++w)
                for (int64_t j = 0; j < n; ++j) s->part[(size_t)w * (size_t)n + (size_t)j] = 0.0;
            for (int64_t j = 0; j < n; ++j) {
                const double* col = Acol(s, j, s->colbuf);
                double acc = 0.0;
                for (int64_t t = s->cp[j]; t < s->cp[j + 1]; ++t)  /* ascending rows */
                    acc = fma(col[s->ri[t]], s->y[s->ri[t]], acc);
                s->part[j] = acc;
            }
            st->price_bytes += 12.0 * (double)s->nnz + 17.0 * (double)n;
        } else {
        for (int w = 0; w < PRICE_SPLIT; ++w) {
            double* pw = s->part + (size_t)w * (size_t)n;
            for (int64_t j = 0; j < n; ++j) pw[j] = 0.0;
            /* chunk w = the slots p = w (mod PRICE_SPLIT), in slot order */
            for (int64_t p = w; p < ny; p += PRICE_SPLIT) {
                const double yp = s->yy[p];
                const double* row = s->AR + (size_t)p * (size_t)n;
                for (int64_t j = 0; j < n; ++j) pw[j] = fma(row[j], yp, pw[j]);
            }
        }
        st->price_bytes += 8.0 * ((double)ny * (double)n + (double)n + (double)ny);
        }
        int64_t q = -1;
        double qscore = 0.0, dq = 0.0, qw = 1.0;
        const double dtol = ctl->tol_dual;
        for (int64_t j = 0; j < n + m; ++j) {
            const int8_t vs = s->vstat[j];
            if (vs == VS_BASIC || s->lb[j] == s->ub[j]) continue;
            double d;
            if (j < n) {
                double tot = 0.0;
                for (int w = 0; w < PRICE_SPLIT; ++w) tot = tot + s->part[(size_t)w * (size_t)n + (size_t)j];
                d = s->cost[j] - tot;
            } else {
                d = s->cost[j] - s->y[j - n];
            }
            double wj = 1.0;
            if (devex) { /* every priced column, eligible or not */
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
            if (bland) { /* lowest eligible index (Devex keeps updating weights) */
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
        if (q < 0) {
            if (phase == 2 && since_refactor > 0) {  /* updated duals: confirm */
                if (refactor(s)) return PH_NUMFAIL;
                st->refactors++;
                since_refactor = 0;
                y_valid = 0;
                recheck = 1;
                continue;
            }
            return PH_OPTIMAL;
        }
        const double sig = dq < 0.0 ? 1.0 : -1.0;
        /* ---- FTRAN ---- */
        for (int64_t i = 0; i < m; ++i) s->acol[i] = (q < n) ? Aat(s, i, q) : (i == q - n ? 1.0 : 0.0);
        for (int64_t p = 0; p < k; ++p) s->aR[p] = s->acol[s->Rl[p]];
        for (int64_t p = 0; p < k; ++p) s->alS[p] = wave_dot(k, MI(s, p, 0), s->aR);
        for (int64_t i = 0; i < m; ++i) {
            if (s->cover[i] < 0) continue;
            s->z[i] = zchunk_row(s, i, s->alS);
            s->alU[i] = unit_sign(s, s->cover[i]) * (s->acol[i] - s->z[i]);
        }
        /* ---- ratio test (Harris two-pass, or textbook under Bland) ----
         * basic entries e < m are covered rows, e >= m bump positions. */
        const double ptol = ctl->tol_primal, pivtol = ctl->tol_pivot, INF = HUGE_VAL;
        double theta_max = INF;
        for (int64_t e = 0; e < m + k; ++e) {
            int64_t var;
            double g, x;
            if (!basic_entry(s, e, sig, &var, &g, &x)) continue;
            const double l = s->lb[var], u = s->ub[var];
            double r;
            if (g > pivtol && l > -INF) r = bland ? (x - l) / g : (x - l + ptol) / g;
            else if (g < -pivtol && u < INF) r = bland ? (u - x) / (-g) : (u - x + ptol) / (-g);
            else continue;
            if (r < theta_max) theta_max = r;
        }
        int64_t lv = -1, lrow = -1, lpos = -1;
        double lg = 0.0, lratio = 0.0;
        for (int64_t e = 0; e < m + k; ++e) {
            int64_t var;
            double g, x;
            if (!basic_entry(s, e, sig, &var, &g, &x)) continue;
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
                lrow = e < m ? e : -1;
                lpos = e < m ? -1 : e - m;
                lg = g;
                lratio = r;
            }
        }
        double theta = lv >= 0 ? (lratio > 0.0 ? lratio : 0.0) : INF;
        const double flip = (s->lb[q] > -INF && s->ub[q] < INF) ? s->ub[q] - s->lb[q] : INF;
        (*iter)++;
        if (phase == 1) st->phase1_iterations++;
        if (flip < INF && flip <= theta) {
            /* bound flip */
            for (int64_t i = 0; i < m; ++i)
                if (s->cover[i] >= 0) s->xr[i] = fma(-flip, sig * s->alU[i], s->xr[i]);
            for (int64_t p = 0; p < k; ++p) s->xs[p] = fma(-flip, sig * s->alS[p], s->xs[p]);
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
            if (trace && *iter - 1 < trace_cap) { /* unbounded ray: leaving -2 */
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
            /* the weights have outgrown the framework: restart it from the
             * current nonbasic set (all weights 1, no update next pass) */
            for (int64_t j = 0; j < n + m; ++j) s->dw[j] = 1.0;
            dv_valid = 0;
            st->devex_resets++;
        } else if (devex) { /* the leaving variable's weight; this pivot for the next pass */
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
        /* ---- primal update ---- */
        for (int64_t i = 0; i < m; ++i)
            if (s->cover[i] >= 0) s->xr[i] = fma(-theta, sig * s->alU[i], s->xr[i]);
        for (int64_t p = 0; p < k; ++p) s->xs[p] = fma(-theta, sig * s->alS[p], s->xs[p]);
        const double xq = s->xval[q] + sig * theta;
        /* leaving variable goes to the bound it hit */
        const int at_lower = lg > 0.0;
        const int leave_art = lv >= n + m;
        if (leave_art) {
            s->lb[lv] = 0.0;
            s->ub[lv] = 0.0;
            s->vstat[lv] = VS_LOWER;
            s->xval[lv] = 0.0;
        } else {
            s->vstat[lv] = at_lower ? VS_LOWER : VS_UPPER;
            s->xval[lv] = at_lower ? s->lb[lv] : s->ub[lv];
        }
        s->vstat[q] = VS_BASIC;
        if (basis_change(s, phase, q, lv, lrow, lpos, dq, xq)) return PH_NUMFAIL;
        since_refactor++;
    }
}

/* The dual's pricing pass (run_dual, warm_core): ONE sweep of the Y rows
 * (PRICE_SPLIT slot classes, the pricing order) for d_j = c_j - y'a_j and the
 * pivot row alpha_j = rho'a_j, the covered leaving row xrow's own entry added
 * last; CSC (price_mode 1): column chains over the dense y and rho.  Slacks:
 * d = c - y_i, alpha = rho_i.  Results in dvec / avec (n + m). */
static void dual_sweep(orc_t* s, const orc_control* ctl, orc_stats* st, int64_t xrow, double xsig) {
    const int64_t m = s->m, n = s->n;
    const int64_t ny = s->ny;
    for (int64_t p = 0; p < ny; ++p) {
        s->yy[p] = s->y[s->Yl[p]];
        s->rhoY[p] = s->rho[s->Yl[p]];
    }
    if (ctl->price_mode == 1) {
        for (int64_t j = 0; j < n; ++j) {
            const double* col = Acol(s, j, s->colbuf);
            double ad = 0.0, aa = 0.0;
            for (int64_t t = s->cp[j]; t < s->cp[j + 1]; ++t) { /* ascending rows */
                ad = fma(col[s->ri[t]], s->y[s->ri[t]], ad);
                aa = fma(col[s->ri[t]], s->rho[s->ri[t]], aa);
            }
            s->dvec[j] = s->cost[j] - ad;
            s->avec[j] = aa;
        }
        st->price_bytes += 12.0 * (double)s->nnz + 17.0 * (double)n;
    } else {
        for (int w = 0; w < PRICE_SPLIT; ++w) {
            double* pw = s->part + (size_t)w * (size_t)n;
            double* qw = s->apart + (size_t)w * (size_t)n;
            for (int64_t j = 0; j < n; ++j) pw[j] = qw[j] = 0.0;
            for (int64_t p = w; p < ny; p += PRICE_SPLIT) {
                const double yp = s->yy[p], rp = s->rhoY[p];
                const double* row = s->AR + (size_t)p * (size_t)n;
                for (int64_t j = 0; j < n; ++j) {
                    pw[j] = fma(row[j], yp, pw[j]);
                    qw[j] = fma(row[j], rp, qw[j]);
                }
            }
        }
        for (int64_t j = 0; j < n; ++j) {
            double td = 0.0, ta = 0.0;
            for (int w = 0; w < PRICE_SPLIT; ++w) {
                td = td + s->part[(size_t)w * (size_t)n + (size_t)j];
                ta = ta + s->apart[(size_t)w * (size_t)n + (size_t)j];
            }
            s->dvec[j] = s->cost[j] - td;
            s->avec[j] = xrow >= 0 ? fma(xsig, Aat(s, xrow, j), ta) : ta;
        }
        st->price_bytes += 8.0 * ((double)ny * (double)n + (double)n + (double)ny);
    }
    for (int64_t i = 0; i < m; ++i) {
        s->dvec[n + i] = s->cost[n + i] - s->y[i];
        s->avec[n + i] = s->rho[i];
    }
}

/* ------------------------------------------------------------------ */
/* dual simplex phase 1 (lp_solve's default SIMPLEX_DUAL_PRIMAL: the dual */
/* simplex while the basis is primal infeasible, then the primal; reached */
/* through R/class.R:262 lp.control and :276 solve).  lp_solve's own dual */
/* loop is not in the reference (third-party, absent): this restatement   */
/* defines the arithmetic and the HIP side reproduces it bit for bit.     */
/*   start: the slack basis with every boxed column at the bound its cost */
/*     sign makes dual feasible; a column that no bound makes dual        */
/*     feasible (one-sided or free with the wrong-signed cost) has its    */
/*     cost zeroed for the phase (solve_core);                            */
/*   CHUZR: the basic variable most out of its bounds by delta^2 / w      */
/*     (dual Devex reference weights w per basic variable, all 1 at the   */
/*     start) or by delta (price_rule 0), lowest variable id on ties;     */
/*   rho_r = row r of B^-1: Minv row p for bump position p; for the slack */
/*     covering row i: sigma (e_i - (A[i,S] Minv) on R);                  */
/*   pivot row alpha_j = rho_r' a_j and d_j = c_j - y' a_j in ONE sweep of */
/*     the Y rows (the pricing order: PRICE_SPLIT slot classes), the       */
/*     covered leaving row's own entry added last (fma(sigma, a_ij, .)); */
/*     CSC (price_mode 1): one column chain each over the dense rho / y;  */
/*   Harris dual ratio test: with s = +1 (x_r below its lower bound) or   */
/*     -1 and ah = s alpha_j, columns at lower (or free with ah < 0) need */
/*     ah < -tol_pivot and bound (d_j + tol_dual) / -ah, at upper (or     */
/*     free with ah > 0) ah > tol_pivot and (tol_dual - d_j) / ah; pass 2 */
/*     takes the largest |alpha_j| among exact ratios <= the minimum      */
/*     bound, lowest id on ties (after degen_switch dual-degenerate       */
/*     pivots: Bland -- the lowest infeasible variable, the smallest      */
/*     exact ratio); no candidate: primal infeasible;                     */
/*   FTRAN of a_q, primal step |x_r - beta_r| / |alpha_rq| (column value) */
/*     in the entering direction, leaving variable to beta_r, then the    */
/*     primal simplex's basis change and dual update y += (d_q/a_rq) rho; */
/*   dual Devex: w_e = max(w_e, (alpha_eq / alpha_rq)^2 w_r) for the other */
/*     basic entries, w_q = max(w_r / alpha_rq^2, 1); restart (all 1)     */
/*     when w_q > DEVEX_RESET.                                            */
/* Returns PH_P1DONE (primal feasible), PH_INFEAS, PH_ITERCAP, PH_NUMFAIL. */
static int run_dual(orc_t* s, const orc_control* ctl, int64_t* iter, int64_t max_iter, int64_t* trace,
                    int64_t trace_cap, orc_stats* st) {
    const int64_t m = s->m, n = s->n;
    const double ptol = ctl->tol_primal, dtol = ctl->tol_dual, pivtol = ctl->tol_pivot, INF = HUGE_VAL;
    const int devex = ctl->price_rule == 1;
    int64_t since_refactor = 0, ndegen = 0;
    int bland = 0, recheck = 0;
    for (int64_t j = 0; j < n + m; ++j) s->dw[j] = 1.0;
    btran(s, 2);
    for (;;) {
        if (!recheck) {
            if (*iter >= max_iter) return PH_ITERCAP;
            if (since_refactor >= ctl->refactor_period) {
                if (refactor(s)) return PH_NUMFAIL;
                st->refactors++;
                since_refactor = 0;
                btran(s, 2);
            }
        }
        recheck = 0;
        const int64_t k = s->k;
        /* ---- CHUZR ---- */
        int64_t rv = -1, re = -1;
        double rscore = 0.0, rx = 0.0, rbeta = 0.0;
        int rs = 0;
        for (int64_t e = 0; e < m + k; ++e) {
            int64_t var;
            double x;
            if (e < m) {
                if (s->cover[e] < 0) continue;
                var = s->cover[e];
                x = s->xr[e];
            } else {
                var = s->Sl[e - m];
                x = s->xs[e - m];
            }
            const double l = s->lb[var], u = s->ub[var];
            double delta, beta;
            int sd;
            if (x < l - ptol) {
                delta = l - x;
                beta = l;
                sd = 1;
            } else if (x > u + ptol) {
                delta = x - u;
                beta = u;
                sd = -1;
            } else {
                continue;
            }
            const double score = devex ? (delta * delta) / s->dw[var] : delta;
            int take;
            if (rv < 0) take = 1;
            else if (bland) take = var < rv;
            else take = score > rscore || (score == rscore && var < rv);
            if (take) {
                rv = var;
                re = e;
                rscore = score;
                rx = x;
                rbeta = beta;
                rs = sd;
            }
        }
        if (rv < 0) {
            if (since_refactor > 0) { /* updated values: confirm on a fresh x_B */
                if (refactor(s)) return PH_NUMFAIL;
                st->refactors++;
                since_refactor = 0;
                btran(s, 2);
                recheck = 1;
                continue;
            }
            return PH_P1DONE;
        }
        /* ---- rho_r on the R rows (position order) and the covered row ---- */
        int64_t xrow = -1;
        double xsig = 0.0;
        if (re >= m) {
            for (int64_t c = 0; c < k; ++c) s->v[c] = *MI(s, re - m, c);
        } else {
            xrow = re;
            xsig = unit_sign(s, s->cover[re]);
            row_times_minv(s, re, s->v);
            for (int64_t c = 0; c < k; ++c) s->v[c] = -(xsig * s->v[c]);
        }
        for (int64_t i = 0; i < m; ++i) s->rho[i] = 0.0;
        for (int64_t c = 0; c < k; ++c) s->rho[s->Rl[c]] = s->v[c];
        if (xrow >= 0) s->rho[xrow] = xsig;
        /* ---- one sweep: d_j (y) and alpha_j (rho) ---- */
        dual_sweep(s, ctl, st, xrow, xsig);
        /* ---- bound-flipping Harris ratio test ---- */
        int64_t nc = 0;
        for (int64_t j = 0; j < n + m; ++j) { /* candidates, ascending id */
            const int8_t vs = s->vstat[j];
            if (vs == VS_BASIC || s->lb[j] == s->ub[j]) continue;
            const double a = s->avec[j], ah = rs * a, dj = s->dvec[j];
            int side = 0;
            if (vs == VS_LOWER || (vs == VS_FREE && ah < 0.0)) side = ah < -pivtol ? 1 : 0;
            else if (vs == VS_UPPER || (vs == VS_FREE && ah > 0.0)) side = ah > pivtol ? -1 : 0;
            if (!side) continue;
            s->cj[nc] = j;
            s->ct[nc] = side > 0 ? dj / (-ah) : (-dj) / ah;
            s->cb[nc] = bland ? s->ct[nc] : side > 0 ? (dj + dtol) / (-ah) : (dtol - dj) / ah;
            s->ca[nc] = fabs(a);
            s->cr[nc] = (s->lb[j] > -INF && s->ub[j] < INF) ? s->ub[j] - s->lb[j] : INF;
            s->calive[nc] = 1;
            nc++;
        }
        /* bunches: the candidates whose exact ratio is within the Harris bound
         * of the ones left are flipped together while every one of them is
         * boxed and the slope (the primal infeasibility of x_r) stays above
         * tol_primal past them (their |alpha| (u - l) summed in ascending id);
         * otherwise the largest |alpha| of the bunch enters */
        double slope = fabs(rx - rbeta);
        int64_t q = -1, nflip = 0;
        double qt = 0.0, qa = 0.0;
        for (;;) {
            double thmax = INF;
            int any = 0;
            for (int64_t c = 0; c < nc; ++c)
                if (s->calive[c]) {
                    any = 1;
                    if (s->cb[c] < thmax) thmax = s->cb[c];
                }
            if (!any) break;
            double sum = 0.0;
            int allbox = 1, nq = 0;
            for (int64_t c = 0; c < nc; ++c)
                if (s->calive[c] && s->ct[c] <= thmax) {
                    nq++;
                    if (s->cr[c] == INF) allbox = 0;
                    else sum = fma(s->ca[c], s->cr[c], sum);
                }
            if (nq == 0) break; /* (NaN ratios only: no candidate qualifies -- the ray) */
            if (allbox && sum < slope - ptol) { /* (x_r still out by more than tol_primal past them) */
                slope = slope - sum;
                for (int64_t c = 0; c < nc; ++c)
                    if (s->calive[c] && s->ct[c] <= thmax) {
                        s->calive[c] = 0;
                        s->flips[nflip++] = s->cj[c];
                    }
                continue;
            }
            int64_t qc = -1;
            for (int64_t c = 0; c < nc; ++c) {
                if (!s->calive[c] || !(s->ct[c] <= thmax)) continue;
                int take;
                if (qc < 0) take = 1;
                else if (bland) take = s->ct[c] < s->ct[qc] || (s->ct[c] == s->ct[qc] && s->cj[c] < s->cj[qc]);
                else take = s->ca[c] > s->ca[qc] || (s->ca[c] == s->ca[qc] && s->cj[c] < s->cj[qc]);
                if (take) qc = c;
            }
            q = s->cj[qc];
            qt = s->ct[qc];
            qa = s->avec[q];
            break;
        }
        (*iter)++;
        st->phase1_iterations++;
        st->dual_iterations++;
        if (q < 0) { /* dual unbounded: every move of the nonbasics leaves x_r infeasible */
            if (trace && *iter - 1 < trace_cap) {
                trace[2 * (*iter - 1)] = -2;
                trace[2 * (*iter - 1) + 1] = rv;
            }
            return PH_INFEAS;
        }
        /* ---- the flips: a_F = sum_j a_j dx_j (ascending j), x_B -= B^-1 a_F ---- */
        if (nflip > 0) {
            for (int64_t i = 0; i < m; ++i) s->aF[i] = 0.0;
            for (int64_t f = 0; f < nflip; ++f) {
                const int64_t j = s->flips[f];
                const double dx = s->vstat[j] == VS_LOWER ? s->ub[j] - s->lb[j] : s->lb[j] - s->ub[j];
                for (int64_t i = 0; i < m; ++i) s->aF[i] = fma(Aat(s, i, j), dx, s->aF[i]);
                s->vstat[j] = s->vstat[j] == VS_LOWER ? VS_UPPER : VS_LOWER;
                s->xval[j] = s->vstat[j] == VS_LOWER ? s->lb[j] : s->ub[j];
            }
            for (int64_t p = 0; p < k; ++p) s->aR[p] = s->aF[s->Rl[p]];
            for (int64_t p = 0; p < k; ++p) s->fS[p] = wave_dot(k, MI(s, p, 0), s->aR);
            for (int64_t i = 0; i < m; ++i)
                if (s->cover[i] >= 0)
                    s->xr[i] = s->xr[i] - unit_sign(s, s->cover[i]) * (s->aF[i] - zchunk_row(s, i, s->fS));
            for (int64_t p = 0; p < k; ++p) s->xs[p] = s->xs[p] - s->fS[p];
            st->bound_flips += nflip;
            rx = re < m ? s->xr[re] : s->xs[re - m];
        }
        {
            const double dq = s->dvec[q];
            const double sig = (s->vstat[q] == VS_LOWER || (s->vstat[q] == VS_FREE && rs * qa < 0.0)) ? 1.0 : -1.0;
            /* ---- FTRAN ---- */
            for (int64_t i = 0; i < m; ++i) s->acol[i] = (q < n) ? Aat(s, i, q) : (i == q - n ? 1.0 : 0.0);
            for (int64_t p = 0; p < k; ++p) s->aR[p] = s->acol[s->Rl[p]];
            for (int64_t p = 0; p < k; ++p) s->alS[p] = wave_dot(k, MI(s, p, 0), s->aR);
            for (int64_t i = 0; i < m; ++i) {
                if (s->cover[i] < 0) continue;
                s->z[i] = zchunk_row(s, i, s->alS);
                s->alU[i] = unit_sign(s, s->cover[i]) * (s->acol[i] - s->z[i]);
            }
            const double arq = re < m ? s->alU[re] : s->alS[re - m];
            const double step = fabs((rx - rbeta) / arq);
            if (trace && *iter - 1 < trace_cap) {
                trace[2 * (*iter - 1)] = q;
                trace[2 * (*iter - 1) + 1] = rv;
            }
            /* ---- dual Devex weights of the basic entries (old basis) ---- */
            if (devex) {
                const double wr = s->dw[rv];
                for (int64_t e = 0; e < m + k; ++e) {
                    if (e == re) continue;
                    int64_t var;
                    double ae;
                    if (e < m) {
                        if (s->cover[e] < 0) continue;
                        var = s->cover[e];
                        ae = s->alU[e];
                    } else {
                        var = s->Sl[e - m];
                        ae = s->alS[e - m];
                    }
                    const double r = ae / arq;
                    double wn = (r * r) * wr;
                    if (wn > DEVEX_WMAX) wn = DEVEX_WMAX;
                    if (wn > s->dw[var]) s->dw[var] = wn;
                }
                double wq = wr / (arq * arq);
                if (wq < 1.0) wq = 1.0;
                if (wq > DEVEX_WMAX) wq = DEVEX_WMAX;
                if (wq > DEVEX_RESET) {
                    for (int64_t j = 0; j < n + m; ++j) s->dw[j] = 1.0;
                    st->devex_resets++;
                } else {
                    s->dw[q] = wq;
                }
            }
            if (!(qt > 0.0)) {
                st->degenerate++;
                if (++ndegen >= ctl->degen_switch) bland = 1;
            } else {
                ndegen = 0;
                bland = 0;
            }
            /* ---- primal update: x_B -= step sig alpha, x_r to its bound ---- */
            for (int64_t i = 0; i < m; ++i)
                if (s->cover[i] >= 0) s->xr[i] = fma(-step, sig * s->alU[i], s->xr[i]);
            for (int64_t p = 0; p < k; ++p) s->xs[p] = fma(-step, sig * s->alS[p], s->xs[p]);
            const double xq = s->xval[q] + sig * step;
            const int at_lower = rs > 0;
            s->vstat[rv] = at_lower ? VS_LOWER : VS_UPPER;
            s->xval[rv] = rbeta;
            s->vstat[q] = VS_BASIC;
            if (basis_change(s, 2, q, rv, re < m ? re : -1, re < m ? -1 : re - m, dq, xq)) return PH_NUMFAIL;
            since_refactor++;
        }
    }
}

/* ------------------------------------------------------------------ */
/* sensitivity from the final (optimal) basis: what get.sensitivity.obj and
 * get.sensitivity.rhs return to R/class.R:613-646.  Textbook ranging on the
 * basis the solve ended with (lp_solve's own routine is absent from this image:
 * parity with it is unpinned; DESIGN.md documents the conventions):
 *   reduced cost d_j = c_j - a_j'y (dense: wave order over all m rows;
 *   price_mode 1: the column chain), slack d = -y_i;
 *   objective ranging: nonbasic at lower [c - d, inf), at upper (-inf, c - d],
 *   free nonbasic [c, c], fixed (-inf, inf); basic S_p: c + [dlo, dhi] with
 *   alpha_pk = rho_p' a_k, rho_p = row p of Minv on the R rows, and
 *   dhi = min d_k/alpha_pk over s_k alpha_pk > tol, dlo = max over < -tol
 *   (s_k = +1 at lower, -1 at upper, both for free);
 *   rhs ranging: basic slack: [activity, inf) for <=, (-inf, activity] for >=,
 *   [b, b] for ==; artificial-covered row [b, b]; row R_c: b + [lo, hi] from
 *   the primal ratio test along g = B^-1 e_i (g_S = Minv[:,c],
 *   g_u = -sigma_u A[i',S] Minv[:,c] on covered rows);
 *   variable entries of dualsfrom / dualstill: -inf / inf.
 * Output (user sense, +-infinity as +-BIG): objfrom[n] objtill[n]
 * duals[m+n] dualsfrom[m+n] dualstill[m+n]. */
static void sensitivity(orc_t* s, const orc_control* ctl, const int32_t* dir, int maximize,
                        double BIG, double* out) {
    const int64_t m = s->m, n = s->n, k = s->k;
    const double INF = HUGE_VAL, tol = ctl->tol_pivot;
    double *objfrom = out, *objtill = out + n, *duals = out + 2 * n;
    double *dfrom = duals + (m + n), *dtill = dfrom + (m + n);
    double* d = dalloc((size_t)(n + m));
    for (int64_t j = 0; j < n; ++j) {
        const double* col = Acol(s, j, s->colbuf);
        double dot = 0.0;
        if (ctl->price_mode == 1) {
            for (int64_t i = 0; i < m; ++i)
                if (col[i] != 0.0) dot = fma(col[i], s->y[i], dot);
        } else {
            dot = wave_dot(m, col, s->y);
        }
        d[j] = s->vstat[j] == VS_BASIC ? 0.0 : s->cost[j] - dot;
    }
    for (int64_t i = 0; i < m; ++i) d[n + i] = s->vstat[n + i] == VS_BASIC ? 0.0 : -s->y[i];
    const double sg = maximize ? -1.0 : 1.0;
    /* (everything below is in the scaled problem; outputs are unscaled) */
    for (int64_t i = 0; i < m; ++i) duals[i] = SC_ROW(sg * s->y[i], i, 1);
    for (int64_t j = 0; j < n; ++j) duals[m + j] = SC_COL(sg * d[j], j, -1);
    /* ---- objective ranging (internal min-form costs) */
    for (int64_t j = 0; j < n; ++j) {
        double lo = -INF, hi = INF;
        const double c = s->cost[j];
        if (s->vstat[j] == VS_BASIC) {
            const int64_t p = s->spos[j];
            double dlo = -INF, dhi = INF;
            for (int64_t kk = 0; kk < n + m; ++kk) {
                if (s->vstat[kk] == VS_BASIC || s->lb[kk] == s->ub[kk]) continue;
                double a = 0.0;
                if (kk < n) {
                    for (int64_t cc = 0; cc < k; ++cc)
                        a = fma(*MI(s, p, cc), Aat(s, s->Rl[cc], kk), a);
                } else {
                    const int64_t cc = s->rpos[kk - n];
                    if (cc < 0) continue;
                    a = *MI(s, p, cc);
                }
                const int8_t vs = s->vstat[kk];
                const double r = d[kk] / a;
                if (vs == VS_FREE) {
                    if (fabs(a) > tol) {
                        if (r < dhi) dhi = r;
                        if (r > dlo) dlo = r;
                    }
                    continue;
                }
                const double sa = vs == VS_LOWER ? a : -a;
                if (sa > tol && r < dhi) dhi = r;
                if (sa < -tol && r > dlo) dlo = r;
            }
            lo = c + dlo;
            hi = c + dhi;
        } else if (s->lb[j] == s->ub[j]) {
            lo = -INF;
            hi = INF;
        } else if (s->vstat[j] == VS_LOWER) {
            lo = c - d[j];
        } else if (s->vstat[j] == VS_UPPER) {
            hi = c - d[j];
        } else {
            lo = hi = c;
        }
        /* user sense: max negated the costs */
        const double ulo = SC_COL(maximize ? -hi : lo, j, -1), uhi = SC_COL(maximize ? -lo : hi, j, -1);
        objfrom[j] = ulo <= -INF ? -BIG : ulo >= INF ? BIG : ulo;
        objtill[j] = uhi <= -INF ? -BIG : uhi >= INF ? BIG : uhi;
    }
    /* ---- rhs ranging */
    for (int64_t i = 0; i < m; ++i) {
        double lo = -INF, hi = INF;
        const double b = s->b[i];
        const int64_t u = s->cover[i];
        if (u == n + i) {  /* basic slack: a_i x = b - s */
            const double act = b - s->xr[i];
            if (dir[i] == 1) lo = act;
            else if (dir[i] == 2) hi = act;
            else lo = hi = b;
        } else if (u >= n + m) {
            lo = hi = b;
        } else {
            const int64_t c = s->rpos[i];
            double glo = -INF, ghi = INF;
            for (int64_t p = 0; p < k; ++p) {  /* basic structurals */
                const double gv = *MI(s, p, c);
                const int64_t v = s->Sl[p];
                const double x = s->xs[p], l = s->lb[v], h = s->ub[v];
                if (gv > tol) {
                    if ((h - x) / gv < ghi) ghi = (h - x) / gv;
                    if ((l - x) / gv > glo) glo = (l - x) / gv;
                } else if (gv < -tol) {
                    if ((l - x) / gv < ghi) ghi = (l - x) / gv;
                    if ((h - x) / gv > glo) glo = (h - x) / gv;
                }
            }
            for (int64_t i2 = 0; i2 < m; ++i2) {  /* covering unit variables */
                const int64_t u2 = s->cover[i2];
                if (u2 < 0) continue;
                double z = 0.0;
                for (int64_t p = 0; p < k; ++p) z = fma(Aat(s, i2, s->Sl[p]), *MI(s, p, c), z);
                const double gv = -unit_sign(s, u2) * z;
                const double x = s->xr[i2], l = s->lb[u2], h = s->ub[u2];
                if (gv > tol) {
                    if ((h - x) / gv < ghi) ghi = (h - x) / gv;
                    if ((l - x) / gv > glo) glo = (l - x) / gv;
                } else if (gv < -tol) {
                    if ((l - x) / gv < ghi) ghi = (l - x) / gv;
                    if ((h - x) / gv > glo) glo = (h - x) / gv;
                }
            }
            lo = b + glo;
            hi = b + ghi;
        }
        lo = SC_ROW(lo, i, -1);
        hi = SC_ROW(hi, i, -1);
        dfrom[i] = lo <= -INF ? -BIG : lo >= INF ? BIG : lo;
        dtill[i] = hi <= -INF ? -BIG : hi >= INF ? BIG : hi;
    }
    for (int64_t j = 0; j < n; ++j) {
        dfrom[m + j] = -BIG;
        dtill[m + j] = BIG;
    }
    free(d);
}

/* elp_control.simplex's default (include/easylp_hip.h): 0 means it --
 * SIMPLEX_DUAL_PRIMAL, lp_solve's default (set_simplextype) */
#define ORC_SIMPLEX_DEFAULT 6
static int simplex_type(const orc_control* c) { return c->simplex == 0 ? ORC_SIMPLEX_DEFAULT : c->simplex; }

void orc_default_control(orc_control* c) {
    c->tol_primal = 1e-9;
    c->tol_dual = 1e-9;
    c->tol_pivot = 1e-9;
    c->infinity = 1e30;
    c->max_iter = 0;
    c->refactor_period = 250;  // lp_solve's default set_maxpivot
    c->degen_switch = 50;
    c->t_mark_iter = -1;
    c->refactor_mode = 0;
    c->price_mode = 0;
    c->price_rule = 1;
    c->scaling = 4 | 64; /* = elp_default_control: geometric + equilibrate */
    c->tol_singular = 1e-13;
    c->simplex = 0;
    c->pad0 = 0;
}

static int cmp_i64(const void* a, const void* b) {
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

int orc_solve_dense(int64_t m, int64_t n, const double* A, const int32_t* dir, const double* rhs,
                    const double* obj, const double* lo, const double* up, int32_t maximize,
                    const orc_control* ctl_in, double* objval, double* xout, double* yout,
                    int64_t* basis, int64_t* trace, int64_t trace_cap, orc_stats* st_out) {
    return orc_solve_dense_sens(m, n, A, dir, rhs, obj, lo, up, maximize, ctl_in, objval, xout,
                                yout, basis, trace, trace_cap, st_out, NULL);
}

static int solve_core(int64_t m, int64_t n, const double* A, uint64_t gen_seed, const int32_t* dir,
                      const double* rhs, const double* obj, const double* lo, const double* up,
                      int32_t maximize, const orc_control* ctl_in, double* objval, double* xout,
                      double* yout, int64_t* basis, int64_t* trace, int64_t trace_cap,
                      orc_stats* st_out, double* sens, orc_t* keep);

int orc_solve_dense_sens(int64_t m, int64_t n, const double* A, const int32_t* dir,
                         const double* rhs, const double* obj, const double* lo,
                         const double* up, int32_t maximize, const orc_control* ctl_in,
                         double* objval, double* xout, double* yout, int64_t* basis,
                         int64_t* trace, int64_t trace_cap, orc_stats* st_out, double* sens) {
    if (m > 0 && !A) return -1;
    return solve_core(m, n, A, 0, dir, rhs, obj, lo, up, maximize, ctl_in, objval, xout, yout, basis,
                      trace, trace_cap, st_out, sens, NULL);
}

int orc_solve_generated(uint64_t seed, int64_t m, int64_t n, const orc_control* ctl, double* objval,
                        double* x, double* y, int64_t* basis, int64_t* trace, int64_t trace_cap,
                        orc_stats* st) {
    if (m < 0 || n <= 0 || (ctl && ctl->price_mode != 0)) return -1;
    double* b = dalloc((size_t)(m > 0 ? m : 1));
    double* c = dalloc((size_t)n);
    int32_t* dir = (int32_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int32_t));
    orc_generate_dense(seed, m, n, 0, n, NULL, b, c);
    for (int64_t i = 0; i < m; ++i) dir[i] = 1;
    const int r = solve_core(m, n, NULL, seed, dir, b, c, NULL, NULL, 1, ctl, objval, x, y, basis, trace,
                             trace_cap, st, NULL, NULL);
    free(b);
    free(c);
    free(dir);
    return r;
}

static void free_state(orc_t* s) {
    free(s->b); free(s->lb); free(s->ub); free(s->cost); free(s->xval); free(s->vstat);
    free(s->asgn); free(s->cover); free(s->rpos); free(s->Rl); free(s->Sl); free(s->spos);
    free(s->xr); free(s->xs); free(s->Minv); free(s->Yl); free(s->ypos); free(s->AR);
    free(s->y); free(s->t); free(s->yR); free(s->yy); free(s->acol); free(s->aR);
    free(s->alS); free(s->alU); free(s->z); free(s->v); free(s->tmp); free(s->part);
    free(s->dw); free(s->dprev);
    free(s->apart); free(s->rho); free(s->rhoY); free(s->dvec); free(s->avec);
    free(s->cj); free(s->flips); free(s->ct); free(s->cb); free(s->ca); free(s->cr); free(s->aF); free(s->fS);
    free(s->calive);
    free(s->used); free(s->perm); free(s->cp); free(s->ri); free(s->nzl); free(s->colbuf);
    free(s->srow); free(s->scol); free(s->A_copy);
}

/* get.objective / get.variables (R/class.R:277-278), unscaled exactly
 * (x_j = 2^scol_j x~_j); unbounded: the ray's variable and the objective +-BIG */
static void emit_outputs(const orc_t* s, int status, int64_t unb_var, double unb_sigma, int32_t maximize,
                         const double* obj, double BIG, double* objval, double* xout) {
    const int64_t n = s->n;
    if (xout)
        for (int64_t j = 0; j < n; ++j) {
            double v = SC_COL(s->vstat[j] == VS_BASIC ? s->xs[s->spos[j]] : s->xval[j], j, 1);
            if (status == 3 && j == unb_var) v = unb_sigma > 0 ? BIG : -BIG;
            xout[j] = v;
        }
    if (objval) {
        if (status == 3) *objval = maximize ? BIG : -BIG;
        else {
            double acc = 0.0;
            for (int64_t j = 0; j < n; ++j) {
                const double v = SC_COL(s->vstat[j] == VS_BASIC ? s->xs[s->spos[j]] : s->xval[j], j, 1);
                acc = fma(obj[j], v, acc);
            }
            *objval = acc;
        }
    }
}

static int solve_core(int64_t m, int64_t n, const double* A, uint64_t gen_seed, const int32_t* dir,
                      const double* rhs, const double* obj, const double* lo, const double* up,
                      int32_t maximize, const orc_control* ctl_in, double* objval, double* xout,
                      double* yout, int64_t* basis, int64_t* trace, int64_t trace_cap,
                      orc_stats* st_out, double* sens, orc_t* keep) {
    if (m < 0 || n <= 0 || (m > 0 && (!dir || !rhs)) || !obj) return -1;
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

    orc_t S;
    memset(&S, 0, sizeof S);
    orc_t* s = &S;
    s->m = m;
    s->n = n;
    s->nv = n + 2 * m;
    s->A = A;
    s->gen_seed = gen_seed;
    s->nnz = 0;
    s->cp = ialloc((size_t)n + 1);
    if (ctl.price_mode == 1) { /* the column pattern (CSC order) */
        for (size_t t = 0; t < (size_t)m * (size_t)n; ++t) s->nnz += A[t] != 0.0;
        s->ri = ialloc((size_t)s->nnz);
        for (int64_t j = 0, t = 0; j < n; ++j) {
            for (int64_t i = 0; i < m; ++i)
                if (A[(size_t)j * (size_t)m + (size_t)i] != 0.0) s->ri[t++] = i;
            s->cp[j + 1] = t;
        }
    } else {
        s->ri = ialloc(1);
    }
    s->nzl = ialloc((size_t)n);
    s->colbuf = dalloc((size_t)(m > 0 ? m : 1));
    s->srow = s->scol = NULL;
    if (ctl.scaling & (4 | 64)) {
        s->srow = (int32_t*)calloc((size_t)(m > 0 ? m : 1), sizeof(int32_t));
        s->scol = (int32_t*)calloc((size_t)n, sizeof(int32_t));
        scale_factors(s, ctl.scaling, s->srow, s->scol);
        if (A) { /* a materialised input: scale a copy once (exact) */
            s->A_copy = (double*)malloc((size_t)m * (size_t)n * sizeof(double) + 8);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < m; ++i)
                    s->A_copy[(size_t)j * (size_t)m + (size_t)i] =
                        ldexp(A[(size_t)j * (size_t)m + (size_t)i], s->srow[i] + s->scol[j]);
            s->A = s->A_copy;
            s->a_scaled = 1;
        }
    }
    /* scaled vectors: infinite values stay infinite (|v| >= infinity first) */
    s->refactor_mode = ctl.refactor_mode;
    s->tol_singular = ctl.tol_singular;
    const int64_t nv = s->nv, mm = m > 0 ? m : 1;
    s->b = dalloc((size_t)mm);
    s->lb = dalloc((size_t)nv);
    s->ub = dalloc((size_t)nv);
    s->cost = dalloc((size_t)nv);
    s->xval = dalloc((size_t)nv);
    s->vstat = (int8_t*)calloc((size_t)nv, 1);
    s->asgn = dalloc((size_t)mm);
    s->cover = ialloc((size_t)mm);
    s->rpos = ialloc((size_t)mm);
    s->Rl = ialloc((size_t)mm);
    s->Sl = ialloc((size_t)mm);
    s->spos = ialloc((size_t)n);
    s->xr = dalloc((size_t)mm);
    s->xs = dalloc((size_t)mm);
    s->ldm = mm;
    s->Minv = dalloc((size_t)mm * (size_t)mm);
    s->Yl = ialloc((size_t)mm);
    s->ypos = ialloc((size_t)mm);
    s->y = dalloc((size_t)mm);
    s->t = dalloc((size_t)mm);
    s->yR = dalloc((size_t)mm);
    s->yy = dalloc((size_t)mm);
    s->acol = dalloc((size_t)mm);
    s->aR = dalloc((size_t)mm);
    s->alS = dalloc((size_t)mm);
    s->alU = dalloc((size_t)mm);
    s->z = dalloc((size_t)mm);
    s->v = dalloc((size_t)mm);
    s->tmp = dalloc(2 * (size_t)mm * (size_t)mm);
    s->part = dalloc((size_t)PRICE_SPLIT * (size_t)n);
    s->used = (int8_t*)calloc((size_t)mm, 1);
    s->perm = ialloc((size_t)mm);
    s->dw = dalloc((size_t)(n + m));
    s->dprev = dalloc((size_t)(n + m));
    s->apart = dalloc((size_t)PRICE_SPLIT * (size_t)n);
    s->rho = dalloc((size_t)mm);
    s->rhoY = dalloc((size_t)mm);
    s->dvec = dalloc((size_t)(n + m));
    s->avec = dalloc((size_t)(n + m));
    s->cj = ialloc((size_t)(n + m));
    s->flips = ialloc((size_t)(n + m));
    s->ct = dalloc((size_t)(n + m));
    s->cb = dalloc((size_t)(n + m));
    s->ca = dalloc((size_t)(n + m));
    s->cr = dalloc((size_t)(n + m));
    s->aF = dalloc((size_t)mm);
    s->fS = dalloc((size_t)mm);
    s->calive = (int8_t*)calloc((size_t)(n + m), 1);

    int status = 0;
    int64_t unb_var = -1;
    double unb_sigma = 0.0;
    double bmax = 0.0;
    /* bounds and costs (R/class.R:261-269); |v| >= infinity means infinite */
    for (int64_t j = 0; j < n; ++j) {
        double l = lo ? lo[j] : 0.0, u = up ? up[j] : INF;
        if (l <= -BIG) l = -INF;
        if (u >= BIG) u = INF;
        l = SC_COL(l, j, -1);
        u = SC_COL(u, j, -1);
        s->lb[j] = l;
        s->ub[j] = u;
        s->cost[j] = 0.0;
        s->spos[j] = -1;
        if (l > u) status = 2; /* R/class.R:297-298 */
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
    int64_t iter = 0;
    if (status == 0) {
        int any_art = 0, dual = 0;
        int64_t nzc = nz_nonbasic(s, s->nzl); /* (no basic structural yet) */
        for (int64_t i = 0; i < m; ++i) {
            double bi = rhs[i];
            if (bi <= -BIG) bi = -INF;
            if (bi >= BIG) bi = INF;
            bi = SC_ROW(bi, i, 1);
            s->b[i] = bi;
            if (fabs(bi) < INF && fabs(bi) > bmax) bmax = fabs(bi);
            const int64_t sv = n + i, av = n + m + i;
            s->lb[sv] = dir[i] == 2 ? -INF : 0.0;
            s->ub[sv] = dir[i] == 1 ? INF : 0.0;
            s->lb[av] = 0.0;
            s->ub[av] = 0.0;
            s->vstat[av] = VS_LOWER;
            s->rpos[i] = -1;
            s->ypos[i] = -1;
        }
        /* SIMPLEX_DUAL_PRIMAL: is the slack basis primal infeasible? */
        if (simplex_type(&ctl) == 6)
            for (int64_t i = 0; i < m && !dual; ++i) {
                double acc = 0.0;
                for (int64_t t = 0; t < nzc; ++t) acc = fma(Aat(s, i, s->nzl[t]), s->xval[s->nzl[t]], acc);
                const double r = s->b[i] - acc;
                dual = !(r >= s->lb[n + i] && r <= s->ub[n + i]);
            }
        if (dual) {
            /* dual-feasible start: boxed columns at the bound their cost sign
             * asks for; columns no bound makes dual feasible lose their cost
             * for the phase (run_dual) */
            for (int64_t j = 0; j < n; ++j) {
                const double cj = SC_COL(maximize ? -obj[j] : obj[j], j, 1);
                s->cost[j] = cj;
                const double l = s->lb[j], u = s->ub[j];
                if (l > -INF && u < INF && l != u) {
                    s->vstat[j] = cj < 0.0 ? VS_UPPER : VS_LOWER;
                    s->xval[j] = cj < 0.0 ? u : l;
                }
                const int8_t vs = s->vstat[j];
                if (l != u && ((vs == VS_LOWER && cj < 0.0) || (vs == VS_UPPER && cj > 0.0) ||
                               (vs == VS_FREE && cj != 0.0))) {
                    s->cost[j] = 0.0;
                    st.flattened++;
                }
            }
            nzc = nz_nonbasic(s, s->nzl);
        }
        for (int64_t i = 0; i < m; ++i) {
            const int64_t sv = n + i, av = n + m + i;
            double acc = 0.0;
            for (int64_t t = 0; t < nzc; ++t) acc = fma(Aat(s, i, s->nzl[t]), s->xval[s->nzl[t]], acc);
            const double r = s->b[i] - acc;
            if (dual || (r >= s->lb[sv] && r <= s->ub[sv])) {  /* (dual: the slack, feasible or not) */
                s->vstat[sv] = VS_BASIC;
                s->cover[i] = sv;
                s->xr[i] = r;
            } else {
                const double sl = r < s->lb[sv] ? s->lb[sv] : s->ub[sv];
                s->vstat[sv] = (sl == s->lb[sv]) ? VS_LOWER : VS_UPPER;
                s->xval[sv] = sl;
                const double res = r - sl;
                s->asgn[i] = res > 0.0 ? 1.0 : -1.0;
                s->ub[av] = INF;
                s->cost[av] = 1.0;
                s->vstat[av] = VS_BASIC;
                s->cover[i] = av;
                s->xr[i] = fabs(res);
                any_art = 1;
                if (y_append(s, i)) status = -3;
            }
        }
        s->tol_inf = 1e-9 * (1.0 + bmax);
        if (dual) {
            int ph = run_dual(s, &ctl, &iter, max_iter, trace, trace_cap, &st);
            if (ph == PH_NUMFAIL) status = 5;
            else if (ph == PH_ITERCAP) status = 1;
            else if (ph == PH_INFEAS) status = 2;
        } else if (any_art && status == 0) {
            int ph = run_phase(s, 1, &ctl, &iter, max_iter, trace, trace_cap, &st, &unb_var, &unb_sigma);
            if (ph == PH_NUMFAIL) status = 5;
            else if (ph == PH_ITERCAP) status = 1;
            else if (art_sum(s) > s->tol_inf) status = 2;
        }
        if (status == 0) {
            for (int64_t i = 0; i < m; ++i) {
                const int64_t av = n + m + i;
                s->cost[av] = 0.0;
                s->lb[av] = 0.0;
                s->ub[av] = 0.0;
            }
            for (int64_t j = 0; j < n; ++j) s->cost[j] = SC_COL(maximize ? -obj[j] : obj[j], j, 1);
            if ((any_art || dual) && refactor(s)) status = 5;
        }
        if (status == 0) {
            int ph = run_phase(s, 2, &ctl, &iter, max_iter, trace, trace_cap, &st, &unb_var, &unb_sigma);
            if (ph == PH_NUMFAIL) status = 5;
            else if (ph == PH_ITERCAP) status = 1;
            else if (ph == PH_UNBOUNDED) status = 3;
            else status = 0;
        }
    }

    /* ---- outputs (get.objective / get.variables, R/class.R:277-278) ---- */
    emit_outputs(s, status, unb_var, unb_sigma, maximize, obj, BIG, objval, xout);
    if (yout)
        for (int64_t i = 0; i < m; ++i) yout[i] = SC_ROW(maximize ? -s->y[i] : s->y[i], i, 1);
    if (basis) {
        int64_t c = 0;
        for (int64_t i = 0; i < m; ++i)
            if (s->cover[i] >= 0) basis[c++] = s->cover[i];
        for (int64_t p = 0; p < s->k; ++p) basis[c++] = s->Sl[p];
        qsort(basis, (size_t)c, sizeof(int64_t), cmp_i64);
    }
    if (sens && status == 0) sensitivity(s, &ctl, dir, maximize, BIG, sens);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    st.iterations = iter;
    st.gj_refactors = s->gj_count;
    st.max_inv_resid = s->emax_max;
    st.bump_dim = s->k;
    st.y_rows = s->ny;
    st.seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (st.seconds_at_mark != 0.0) /* -> seconds from the mark to the end */
        st.seconds_at_mark = ((double)t1.tv_sec + 1e-9 * (double)t1.tv_nsec) - st.seconds_at_mark;
    if (st_out) *st_out = st;
    if (keep) *keep = S; /* the caller's warm_core continues from this state */
    else free_state(s);
    return status;
}

/* Re-solve after a change of the column bounds, from the basis the state's
 * last solve ended on (MIP node warm start, SIMPLEX_DUAL_PRIMAL; the HIP side's
 * warm reload in elp_api.hip run_bnb).  The basis stays; costs are the real
 * ones again; y = B^-T c_B; each nonbasic structural takes the new value of
 * its bound (a status whose bound is gone moves to the finite one: lower,
 * else upper, else free; a fixed column sits at lower), boxed columns whose
 * reduced cost has the wrong sign for their bound move to the other one, and
 * any other nonbasic column or slack that stays dual infeasible (beyond
 * tol_dual) has its cost shifted by -d_j for the dual phase; then x_B from b,
 * the dual phase (which returns at once when x_B is feasible), the real costs,
 * and the primal phase 2 -- solve_core's sequence after its start. */
static int warm_core(orc_t* s, const double* lo, const double* up, int32_t maximize, const double* obj,
                     const orc_control* ctl_in, double* objval, double* xout, orc_stats* st_out) {
    orc_control ctl = *ctl_in;
    if (ctl.refactor_period <= 0) ctl.refactor_period = 250;
    if (ctl.degen_switch <= 0) ctl.degen_switch = 50;
    const int64_t m = s->m, n = s->n;
    const int64_t max_iter = ctl.max_iter > 0 ? ctl.max_iter : 100 * (m + n) + 10000;
    const double INF = HUGE_VAL, BIG = ctl.infinity, dtol = ctl.tol_dual;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    orc_stats st;
    memset(&st, 0, sizeof st);
    int status = 0;
    int64_t iter = 0, unb_var = -1;
    double unb_sigma = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        double l = lo ? lo[j] : 0.0, u = up ? up[j] : INF;
        if (l <= -BIG) l = -INF;
        if (u >= BIG) u = INF;
        s->lb[j] = SC_COL(l, j, -1);
        s->ub[j] = SC_COL(u, j, -1);
        if (s->lb[j] > s->ub[j]) status = 2; /* R/class.R:297-298 */
        s->cost[j] = SC_COL(maximize ? -obj[j] : obj[j], j, 1);
    }
    for (int64_t i = 0; i < m; ++i) s->cost[n + i] = 0.0;
    if (status == 0) {
        btran(s, 2);
        for (int64_t i = 0; i < m; ++i) s->rho[i] = 0.0;
        dual_sweep(s, &ctl, &st, -1, 0.0);
        for (int64_t j = 0; j < n + m; ++j) {
            int8_t vs = s->vstat[j];
            if (vs == VS_BASIC) continue;
            const double l = s->lb[j], u = s->ub[j], d = s->dvec[j];
            if (j < n) {
                const int lo_ok = l > -INF, up_ok = u < INF;
                if (l == u) {
                    s->vstat[j] = VS_LOWER;
                    s->xval[j] = l;
                    continue;
                }
                if (vs == VS_LOWER && !lo_ok) vs = up_ok ? VS_UPPER : VS_FREE;
                else if (vs == VS_UPPER && !up_ok) vs = lo_ok ? VS_LOWER : VS_FREE;
                else if (vs == VS_FREE && (lo_ok || up_ok)) vs = lo_ok ? VS_LOWER : VS_UPPER;
                if (vs == VS_LOWER && d < -dtol && up_ok) vs = VS_UPPER;
                else if (vs == VS_UPPER && d > dtol && lo_ok) vs = VS_LOWER;
                s->vstat[j] = vs;
                s->xval[j] = vs == VS_LOWER ? l : vs == VS_UPPER ? u : 0.0;
            } else if (l == u) {
                continue;
            }
            if ((vs == VS_LOWER && d < -dtol) || (vs == VS_UPPER && d > dtol) || (vs == VS_FREE && fabs(d) > dtol)) {
                s->cost[j] = s->cost[j] - d;
                st.flattened++;
            }
        }
        if (refactor(s)) status = 5;
    }
    if (status == 0) {
        int ph = run_dual(s, &ctl, &iter, max_iter, NULL, 0, &st);
        if (ph == PH_NUMFAIL) status = 5;
        else if (ph == PH_ITERCAP) status = 1;
        else if (ph == PH_INFEAS) status = 2;
    }
    if (status == 0) {
        for (int64_t j = 0; j < n; ++j) s->cost[j] = SC_COL(maximize ? -obj[j] : obj[j], j, 1);
        for (int64_t i = 0; i < m; ++i) s->cost[n + i] = 0.0;
        if (refactor(s)) status = 5;
    }
    if (status == 0) {
        int ph = run_phase(s, 2, &ctl, &iter, max_iter, NULL, 0, &st, &unb_var, &unb_sigma);
        if (ph == PH_NUMFAIL) status = 5;
        else if (ph == PH_ITERCAP) status = 1;
        else if (ph == PH_UNBOUNDED) status = 3;
    }
    emit_outputs(s, status, unb_var, unb_sigma, maximize, obj, BIG, objval, xout);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    st.iterations = iter;
    st.bump_dim = s->k;
    st.y_rows = s->ny;
    st.seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (st_out) *st_out = st;
    return status;
}

/* ------------------------------------------------------------------ */
/* MIP: depth-first branch and bound over LP relaxations (the integer /   */
/* binary columns of R/class.R:123-128, set.type at :265).  Rules (shared  */
/* with the HIP host driver, easylp_amd/csrc/elp_api.hip run_bnb):         */
/*   integer bounds tightened to ceil(lo - 1e-9) / floor(up + 1e-9);       */
/*   node LP solved cold (SIMPLEX_PRIMAL_PRIMAL) or warm from the last    */
/*   node's basis (SIMPLEX_DUAL_PRIMAL, warm_core); LP unbounded -> MIP    */
/*   status 3; infeasible or      */
/*   numerical failure -> prune; bound test zmin >= best - max(1e-11,      */
/*   1e-9 |best|) -> prune (zmin: objective in minimisation form);         */
/*   branch on the lowest-index integer column with |x - round(x)| > 1e-7  */
/*   (lp_solve's epsint); ceiling branch explored first (lp_solve's        */
/*   default floor_first = CEILING); LIFO stack.  ctl->max_iter > 0 bounds  */
/*   the LP iterations of the whole tree: a node that hits it ends the      */
/*   search; a node that fails numerically is skipped.  Either makes the    */
/*   tree incomplete: incumbent -> 1 (sub-optimal), none -> that node's     */
/*   status.                                                               */
typedef struct { double* lo; double* up; } bnb_node;

int orc_solve_mip(int64_t m, int64_t n, const double* A, const int32_t* dir, const double* rhs,
                  const double* obj, const double* lo, const double* up, int32_t maximize,
                  const int32_t* is_int, const orc_control* ctl, int64_t max_nodes,
                  double* objval, double* xout, int64_t* nodes_out, int64_t* lp_iters_out) {
    const double INF = HUGE_VAL;
    const double BIG = ctl ? ctl->infinity : 1e30;
    int64_t cap = 64, top = 0, nodes = 0, iters = 0;
    bnb_node* stack = (bnb_node*)malloc((size_t)cap * sizeof(bnb_node));
    double* l0 = dalloc((size_t)n);
    double* u0 = dalloc((size_t)n);
    for (int64_t j = 0; j < n; ++j) {
        double l = lo ? lo[j] : 0.0, u = up ? up[j] : INF;
        if (l <= -BIG) l = -INF;
        if (u >= BIG) u = INF;
        if (is_int[j]) {
            if (l > -INF) l = ceil(l - 1e-9);
            if (u < INF) u = floor(u + 1e-9);
        }
        l0[j] = l;
        u0[j] = u;
    }
    stack[top].lo = l0;
    stack[top].up = u0;
    top++;
    double best = INF;
    double* xbest = dalloc((size_t)n);
    double* x = dalloc((size_t)n);
    int have = 0, status = -1, failed = -1;
    orc_stats st;
    orc_control nctl;
    if (ctl) nctl = *ctl;
    else orc_default_control(&nctl);
    /* SIMPLEX_DUAL_PRIMAL: node LPs after the first continue from the basis of
     * the node solved last (warm_core: the dual simplex repairs the bounds the
     * branch changed), as lp_solve re-solves B&B nodes from a kept basis */
    const int warm = simplex_type(&nctl) == 6 && m > 0;
    orc_t state;
    int have_state = 0;
    while (top > 0) {
        bnb_node nd = stack[--top];
        if (max_nodes > 0 && nodes >= max_nodes) {
            free(nd.lo);
            free(nd.up);
            status = 1;
            continue;
        }
        nodes++;
        double z = 0.0;
        if (ctl && ctl->max_iter > 0) nctl.max_iter = ctl->max_iter - iters > 0 ? ctl->max_iter - iters : 0;
        /* (max_iter 0 would mean "default": a spent budget runs no iteration) */
        int s;
        if (ctl && ctl->max_iter > 0 && nctl.max_iter == 0) {
            s = 1;
            memset(&st, 0, sizeof st);
        } else if (warm && have_state) {
            s = warm_core(&state, nd.lo, nd.up, maximize, obj, &nctl, &z, x, &st);
        } else {
            s = solve_core(m, n, A, 0, dir, rhs, obj, nd.lo, nd.up, maximize, &nctl, &z, x, NULL, NULL, NULL, 0,
                           &st, NULL, warm ? &state : NULL);
            have_state = warm;
        }
        if (have_state && s != 0 && s != 2 && s != 3) { /* (a failed node: the next one starts cold) */
            free_state(&state);
            have_state = 0;
        }
        iters += st.iterations;
        int branched = 0;
        if (s != 0 && s != 2 && s != 3) { /* iteration budget or numerical failure */
            if (failed < 0) failed = s;
            free(nd.lo);
            free(nd.up);
            if (s == 1) break;
            continue;
        }
        if (s == 3) {
            status = 3;
            free(nd.lo);
            free(nd.up);
            while (top > 0) {
                --top;
                free(stack[top].lo);
                free(stack[top].up);
            }
            break;
        }
        if (s == 0) {
            const double zmin = maximize ? -z : z;
            const double tol = fabs(best) < INF ? fmax(1e-11, 1e-9 * fabs(best)) : 0.0;
            if (!(fabs(best) < INF && zmin >= best - tol)) {
                int64_t jb = -1;
                for (int64_t j = 0; j < n; ++j)
                    if (is_int[j] && fabs(x[j] - nearbyint(x[j])) > 1e-7) {
                        jb = j;
                        break;
                    }
                if (jb < 0) {
                    best = zmin;
                    memcpy(xbest, x, (size_t)n * sizeof(double));
                    have = 1;
                } else {
                    if (top + 2 > cap) {
                        cap *= 2;
                        stack = (bnb_node*)realloc(stack, (size_t)cap * sizeof(bnb_node));
                    }
                    /* floor child pushed first so the ceiling child is explored first */
                    double* fl = dalloc((size_t)n);
                    double* fu = dalloc((size_t)n);
                    memcpy(fl, nd.lo, (size_t)n * sizeof(double));
                    memcpy(fu, nd.up, (size_t)n * sizeof(double));
                    fu[jb] = floor(x[jb]);
                    stack[top].lo = fl;
                    stack[top].up = fu;
                    top++;
                    nd.lo[jb] = ceil(x[jb]);
                    stack[top].lo = nd.lo;
                    stack[top].up = nd.up;
                    top++;
                    branched = 1;
                }
            }
        }
        if (!branched) {
            free(nd.lo);
            free(nd.up);
        }
    }
    while (top > 0) { /* a limit ended the search */
        --top;
        free(stack[top].lo);
        free(stack[top].up);
    }
    if (status != 3) {
        const int limit = status == 1;
        if (have) status = (limit || failed >= 0) ? 1 : 0;
        else if (failed >= 0) status = failed;
        else status = limit ? 1 : 2;
    }
    if (have && status != 3) {
        if (xout) memcpy(xout, xbest, (size_t)n * sizeof(double));
        if (objval) {
            double acc = 0.0;
            for (int64_t j = 0; j < n; ++j) acc = fma(obj[j], xbest[j], acc);
            *objval = acc;
        }
    }
    if (have_state) free_state(&state);
    if (nodes_out) *nodes_out = nodes;
    if (lp_iters_out) *lp_iters_out = iters;
    free(xbest);
    free(x);
    free(stack);
    return status;
}
