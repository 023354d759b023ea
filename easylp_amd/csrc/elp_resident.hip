// elp_resident.hip -- the resident small-LP solver: the whole simplex loop of
// an LP with at most 64 rows whose state fits in one CU's LDS, run by ONE
// wave in ONE launch.
//
// Why: the multi-workgroup pipeline (elp_kernels.hip) pays 4-7 dependent
// launches per pivot, a ~20 us floor per pivot that no amount of bandwidth
// hides.  The models EasyLP's R front-end actually builds (README, test-DOP.R,
// the vignettes, the MIP tests' nodes; BASELINE configs[4]'s Klee-Minty cube)
// are a few dozen rows and columns: their whole state fits beside one wave,
// which does a pivot's pricing, FTRAN, ratio test and update with no kernel
// boundary and no global round trip.
//
// Layout: lane r holds row r's values (x_B of a covered row, its cover, rpos,
// Y slot, y_r, a_q's entry, alpha_U, ...), lane p bump position p's (S_p,
// R_p, x_S, alpha_S) and Y slot p's row, all in registers; a value of another
// lane is a v_readlane (uniform index) or a ds_bpermute (per-lane index, in
// uniform control flow).  LDS holds what is indexed by column or variable: A
// (column-major), the bump inverse, bounds / costs / values / statuses, Devex
// weights, the dual ratio test's candidates.  One wave's LDS operations
// complete in issue order, so a store and another lane's later load need only
// the compiler's ordering (R_FENCE).
//
// Arithmetic: identical to oracle/elp_oracle.c (run_phase, run_dual,
// basis_change, refactor, btran) and therefore to the pipeline -- the same
// reduction shapes, evaluated per output lane: a wave_dot (64 lane-strided
// fma chains + the pairwise tree, offsets 1, 2, ..., 32) becomes one lane's
// terms in order folded by the same tree (wdot: the fixed 64-leaf tree in
// blocks of eight), zchunk, the price
// slot classes and the column chains are per-output fma chains already.  The
// orchestration is elp_api.hip run_loop's: loop-top checks (phase-1 sum,
// iteration cap, budget stop, time limit, refactor period), the recheck
// refactor after updated values reach optimality, and the phase changes
// (primal phase 1 or the dual phase -> real costs, refactor, primal phase 2).
//
// State is read from the device buffers the load left (elp_api.hip
// load_common / reload_bounds_warm) and written back at exit in the
// pipeline's own layout -- lists, bump inverse (and MinvT), AS, AR, the
// per-position / per-row / per-slot caches -- so elp_get_solution,
// elp_sensitivity, elp_iterate and a MIP node's warm start read it as if the
// pipeline had run.
#include "elp_internal.h"

#include <math.h>

namespace elp {
namespace {

#define RDEV __device__ __forceinline__
constexpr int RW = 64;
constexpr double R_WMAX = 1e20;   // DEVEX_WMAX (oracle, elp_kernels.hip)
constexpr double R_RESET = 1e6;   // DEVEX_RESET
constexpr double R_INF = HUGE_VAL;
#define R_FENCE() asm volatile("" ::: "memory")
// diagnostic build (tools/build_variant.sh resprof "-DELP_RES_PROF=1"): shader
// cycles (s_memtime) per loop stage, summed in ResOut::stage
#ifndef ELP_RES_PROF
#define ELP_RES_PROF 0
#endif
__shared__ unsigned long long r_prof[25];  // [24]: the last stamp
#define R_STAMP(i)                                                        \
    do {                                                                  \
        if (ELP_RES_PROF && threadIdx.x == 0) {                           \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
            r_prof[i] += t_ - r_prof[24];                                 \
            r_prof[24] = t_;                                              \
        }                                                                 \
    } while (0)

// ------------------------------------------------------------ wave helpers
template <int CTRL>
RDEV double r_dpp(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
RDEV double r_swz16(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_swizzle((int)b, 0x401F);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x401F);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// lane l's value (l uniform)
RDEV double rl(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
RDEV int rli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// lane src's value, src per lane (0..63); every lane active
RDEV double shf(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)b);
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
RDEV double r_wmax(double v) {
    v = fmax(v, r_dpp<0xB1>(v));
    v = fmax(v, r_dpp<0x4E>(v));
    v = fmax(v, r_dpp<0x141>(v));
    v = fmax(v, r_dpp<0x140>(v));
    v = fmax(v, r_swz16(v));
    return fmax(rl(v, 0), rl(v, 32));
}
RDEV double r_wmin(double v) {
    v = fmin(v, r_dpp<0xB1>(v));
    v = fmin(v, r_dpp<0x4E>(v));
    v = fmin(v, r_dpp<0x141>(v));
    v = fmin(v, r_dpp<0x140>(v));
    v = fmin(v, r_swz16(v));
    return fmin(rl(v, 0), rl(v, 32));
}
RDEV int r_wmini(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_ds_swizzle(v, 0x401F));
    return min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 32));
}
// the lane holding the best record: largest key (smallest with MIN), then the
// smallest id; -1 when no lane is valid (uniform)
template <bool MIN>
RDEV int r_argbest(bool valid, double key, int id) {
    const unsigned long long vm = __ballot(valid);
    if (vm == 0ull) return -1;
    const double b = MIN ? r_wmin(valid ? key : R_INF) : r_wmax(valid ? key : -R_INF);
    bool in = valid && key == b;
    if (__ballot(in) == 0ull) in = valid;  // (NaN keys only)
    const unsigned long long im = __ballot(in);
    if (__popcll(im) == 1) return __builtin_amdgcn_readfirstlane(__ffsll((long long)im) - 1);
    const int mn = r_wmini(in ? id : 0x7fffffff);
    return __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(in && id == mn)) - 1);
}
RDEV int r_argminid(bool valid, int id) {
    if (__ballot(valid) == 0ull) return -1;
    const int mn = r_wmini(valid ? id : 0x7fffffff);
    return __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(valid && id == mn)) - 1);
}
// the GPU wave_tree of one value per lane (uniform result)
RDEV double r_wtree(double acc) {
    acc = acc + r_dpp<0xB1>(acc);
    acc = acc + r_dpp<0x4E>(acc);
    acc = acc + r_dpp<0x141>(acc);
    acc = acc + r_dpp<0x140>(acc);
    acc = acc + r_swz16(acc);
    return rl(acc, 0) + rl(acc, 32);
}

// wave_dot's bits in one lane, for len <= 64: lane l's chain is one fma
// from 0.0, the idle lanes (l >= len) hold +0.0, and the tree pairs lanes
// (l, l + off) for off = 1, 2, ..., 32 -- so the sum is the fixed 64-leaf
// tree: eight blocks ((t0+t1)+(t2+t3))+((t4+t5)+(t6+t7)), then the blocks'
// tree.  Blocks past len are +0.0 (their adds change nothing but a zero's
// sign, which the top level reproduces by adding the +0.0 as the oracle
// does).  X(l): x_l (a per-lane load), Y(l): y_l (a readlane at a constant
// lane); a block's 8 loads go out together.
template <class FX, class FY>
RDEV double wdot(FX X, FY Y, int len) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, tot = 0.0;  // the blocks' tree: pending block, pair, quad
    // len <= 16: blocks 2..7 are +0.0 and fold to ((B0 + B1) + 0) + 0 = (B0 + B1) + 0
    const int nb = len <= 16 ? 2 : 8;
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        double B = 0.0;
        if (8 * b < len) {
            double x[8], t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = X(8 * b + u < len ? 8 * b + u : len - 1);
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = 8 * b + u < len ? fma(x[u], Y(8 * b + u), 0.0) : 0.0;
            B = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
        }
        if ((b & 1) == 0) {
            s0 = B;
        } else {
            const double pr = s0 + B;
            if ((b & 2) == 0) {
                s1 = pr;
            } else {
                const double qd = s1 + pr;
                if ((b & 4) == 0) s2 = qd;
                else tot = s2 + qd;
            }
        }
    }
    return nb == 2 ? s1 + 0.0 : tot;
}

// ------------------------------------------------------------ LDS state
struct RS {
    int m, n, nv, lda, kc, ldm;
    double* A;      // m x n, column-major, ld lda (scaled values)
    double* Mi;     // bump inverse kc x kc, row-major, ld ldm
    double* W;      // refactor work: 2 * kc * kc
    double *lb, *ub, *cost, *xval;  // nv
    double *dw, *dprev;             // n + m
    double *dvec, *avec, *ct, *cb, *ca, *cr;  // n + m
    int* spos;                      // n
    int *cj, *flips;                // n + m
    int8_t *vst, *calive;           // nv, n + m
};
__host__ __device__ inline size_t r_carve(RS& s, char* base, int m, int n) {
    s.m = m;
    s.n = n;
    s.nv = n + 2 * m;
    s.lda = m | 1;  // (odd: lanes reading one row of different columns hit distinct banks)
    s.kc = m < n ? m : n;
    if (s.kc < 1) s.kc = 1;
    s.ldm = s.kc | 1;
    size_t off = 0;
    auto dd = [&](double*& p, size_t cnt) {
        p = (double*)(base + off);
        off += cnt * sizeof(double);
    };
    auto ii = [&](int*& p, size_t cnt) {
        p = (int*)(base + off);
        off += cnt * sizeof(int);
        off = (off + 7) & ~7;
    };
    auto bb = [&](int8_t*& p, size_t cnt) {
        p = (int8_t*)(base + off);
        off += cnt;
        off = (off + 7) & ~7;
    };
    const size_t nm = n + m, kc = s.kc;
    dd(s.A, s.lda * n);
    dd(s.Mi, s.ldm * kc);
    dd(s.W, 2 * kc * kc);
    dd(s.lb, s.nv);
    dd(s.ub, s.nv);
    dd(s.cost, s.nv);
    dd(s.xval, s.nv);
    dd(s.dw, nm);
    dd(s.dprev, nm);
    dd(s.dvec, nm);
    dd(s.avec, nm);
    dd(s.ct, nm);
    dd(s.cb, nm);
    dd(s.ca, nm);
    dd(s.cr, nm);
    ii(s.spos, n);
    ii(s.cj, nm);
    ii(s.flips, nm);
    bb(s.vst, s.nv);
    bb(s.calive, nm);
    return off;
}

// the lane-resident vectors (lane r: row r; lane p: bump position / Y slot p)
struct RV {
    double b, xr, asgn, y;      // row
    int cover, rpos, ypos;      // row
    int Sl, Rl, Yl;             // position / slot
    double xs;                  // position
    double acol, z, alU;        // FTRAN of the entering column (row)
    double alS;                 // (position)
};
// run statistics, in LDS (lane 0 updates them: no registers held across the loop)
struct RStat {
    int64_t phase1_iters, flips, degenerate, dual_iters, refactors, gj, resets;
    double price_bytes, iter_bytes, emax_max, unb_sig;
    int32_t unb_var, pad;
};
// the uniform scalars of the loop
struct RC {
    int phase;  // 1 primal phase 1, 2 primal phase 2, 3 dual phase 1 (h->phase)
    int k, ny;
    int64_t iter, iter_limit, iter_stop;
    int since, period, ndegen, bland, degen_switch;
    int devex, ddevex, dv_valid, dv_lv;
    double dv_dq, dv_wq;
    double tol_primal, tol_dual, tol_pivot, tol_inf, tol_singular;
    double art_sum;
    int status;
    RStat* st;
    int y_valid;
    int64_t trace_cap;
};

RDEV double r_usign(const RS& s, const RV& v, int var) { return var >= s.n + s.m ? v.asgn : 1.0; }  // (row lane)
RDEV double r_colA(const RS& s, int i, int j) {
    return j < s.n ? s.A[i + j * s.lda] : (i == j - s.n ? 1.0 : 0.0);
}
// lane r: z_r = sum_p A[r, S_p] w_p in zchunk order (w: per-position register)
RDEV double r_zchunk(const RS& s, const RV& v, int r, double w, int k) {
    double tot = 0.0;
    for (int c0 = 0; c0 < k; c0 += ZCHUNK) {
        const int c1 = c0 + ZCHUNK < k ? c0 + ZCHUNK : k;
        double acc = 0.0;
        for (int p0 = c0; p0 < c1; p0 += 8) {
            double a[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int p = p0 + u < c1 ? p0 + u : c1 - 1;
                a[u] = s.A[r + rli(v.Sl, p) * s.lda];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (p0 + u < c1) acc = fma(a[u], rl(w, p0 + u), acc);
        }
        tot = tot + acc;
    }
    return tot;
}
// lane p: row p of Minv . w (wave order over the k positions; w per position)
RDEV double r_minv_row(const RS& s, int p, double w, int k) {
    const double* row = s.Mi + (p < k ? p : 0) * s.ldm;
    return wdot([&](int l) { return row[l]; }, [&](int l) { return rl(w, l); }, k);
}
// lane c: column c of Minv . w (BTRAN / row_times_minv: wave order over rows)
RDEV double r_minv_col(const RS& s, int c, double w, int k) {
    const double* col = s.Mi + (c < k ? c : 0);
    const int ld = s.ldm;
    return wdot([&](int l) { return col[l * ld]; }, [&](int l) { return rl(w, l); }, k);
}

// ------------------------------------------------------------ refactor
// M = A[R, S] into W (k x k) -- lane c: column c
RDEV void r_load_M(const RS& s, const RV& v, int k, double* W) {
    const int lane = threadIdx.x;
    const double* col = s.A + (lane < k ? v.Sl : 0) * s.lda;
    for (int a = 0; a < k; ++a) {
        const int ra = rli(v.Rl, a);
        if (lane < k) W[a * k + lane] = col[ra];
    }
    R_FENCE();
}
RDEV bool r_gauss_jordan(RS& s, const RV& v, RC& c) {
    const int k = c.k, lane = threadIdx.x;
    double* W = s.W;  // k x k, row-major (ld k), in place
    r_load_M(s, v, k, W);
    bool used = false;  // (lane r: row r used)
    int perm = 0;       // (lane c: the pivot row of column c)
    for (int col = 0; col < k; ++col) {
        const double wv = lane < k ? W[lane * k + col] : 0.0;
        const bool cand = lane < k && !used;
        const int pl = r_argbest<false>(cand, fabs(wv), lane);  // largest |W[r][c]|, lowest row
        const int p = pl >= 0 ? pl : 0;
        const double piv = rl(wv, p);
        if (!(fabs(piv) > c.tol_singular)) return false;
        if (lane == col) perm = p;
        if (lane == p) used = true;
        const double q = lane < k ? W[p * k + lane] / piv : 0.0;  // row p's quotient of column lane
        const double f = wv;                                                // row lane's factor
        R_FENCE();
        for (int r0 = 0; r0 < k; r0 += 8) {  // rows r0.., every column j = lane: 8 loads, then 8 stores
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = lane < k ? W[(r0 + u < k ? r0 + u : k - 1) * k + lane] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int r = r0 + u;
                if (r >= k) break;
                const double fr = rl(f, r);
                if (r == p) x[u] = lane == col ? 1.0 / piv : q;
                else if (lane == col) x[u] = -(fr / piv);
                else if (fr != 0.0 && q != 0.0) x[u] = fma(-fr, q, x[u]);
                if (lane < k) W[r * k + lane] = x[u];
            }
        }
        R_FENCE();
    }
    // Minv[a][perm[c]] = W[perm[a]][c]: lane c writes column perm[c]
    for (int a = 0; a < k; ++a) {
        const int pa = rli(perm, a);
        if (lane < k) s.Mi[a * s.ldm + perm] = W[pa * k + lane];
    }
    R_FENCE();
    return true;
}
// one Newton-Schulz correction; false: the residual is above tol (nothing changed)
RDEV bool r_newton_schulz(RS& s, const RV& v, RC& c, double tol) {
    const int k = c.k, lane = threadIdx.x;
    double* M = s.W;
    double* E = s.W + k * k;
    r_load_M(s, v, k, M);
    double emax = 0.0;
    for (int i = 0; i < k; ++i) {  // E[i][j], lane j: (M Minv)_ij seq over l (8 terms' loads at a time)
        double acc = 0.0;
        if (lane < k)
            for (int l0 = 0; l0 < k; l0 += 8) {
                double mv[8], iv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int l = l0 + u < k ? l0 + u : k - 1;
                    mv[u] = M[i * k + l];
                    iv[u] = s.Mi[l * s.ldm + lane];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (l0 + u < k) acc = fma(mv[u], iv[u], acc);
            }
        const double ev = (i == lane ? 1.0 : 0.0) - acc;
        if (lane < k) {
            E[i * k + lane] = ev;
            emax = fmax(emax, fabs(ev));
        }
    }
    emax = r_wmax(emax);
    if (threadIdx.x == 0 && emax > c.st->emax_max) c.st->emax_max = emax;
    if (!(emax <= tol)) return false;
    R_FENCE();
    for (int i = 0; i < k; ++i) {  // Minv_new[i][j] = Minv[i][j] + sum_l Minv[i][l] E[l][j], row by row in place
        double acc = 0.0;
        if (lane < k) {
            acc = s.Mi[i * s.ldm + lane];
            for (int l0 = 0; l0 < k; l0 += 8) {
                double mv[8], ev[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int l = l0 + u < k ? l0 + u : k - 1;
                    mv[u] = s.Mi[i * s.ldm + l];
                    ev[u] = E[l * k + lane];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (l0 + u < k) acc = fma(mv[u], ev[u], acc);
            }
        }
        R_FENCE();
        if (lane < k) s.Mi[i * s.ldm + lane] = acc;
        R_FENCE();
    }
    return true;
}
// oracle refactor(): the inverse corrected or rebuilt, then x_B from b
RDEV bool r_refactor(RS& s, RV& v, RC& c, int refactor_mode) {
    const int k = c.k, m = s.m, n = s.n, lane = threadIdx.x;
    if (k > 0) {
        // oracle refactor(): a correction within NS_TOL; else one within NS_TOL2
        // and, if the new residual is within NS_TOL, a second; else Gauss-Jordan
        // (one call site: the loop keeps the code in the instruction cache)
        bool ok = false;
        for (int t = 0; refactor_mode == 0 && t < 3; ++t) {
            const bool applied = r_newton_schulz(s, v, c, t == 1 ? NS_TOL2 : NS_TOL);
            if (t == 0 && applied) {
                ok = true;
                break;
            }
            if (t == 1 && !applied) break;
            if (t == 2) ok = applied;
        }
        if (!ok) {
            if (threadIdx.x == 0) c.st->gj++;
            if (!r_gauss_jordan(s, v, c)) return false;
        }
    }
    double acc = 0.0;  // lane r: nonzero nonbasic structurals, ascending j
    for (int j0 = 0; j0 < n; j0 += 8) {
        double a[8], x[8];
        bool on[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u < n ? j0 + u : n - 1;
            a[u] = lane < m ? s.A[lane + j * s.lda] : 0.0;
            x[u] = s.xval[j];
            on[u] = j0 + u < n && s.vst[j] != VS_BASIC;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (on[u] && x[u] != 0.0) acc = fma(a[u], x[u], acc);
    }
    double r = v.b - acc;
    if (lane < m && s.vst[n + lane] != VS_BASIC) r = r - s.xval[n + lane];
    v.acol = r;
    const double aR = shf(v.acol, v.Rl & 63);  // (position lane)
    v.xs = lane < k ? r_minv_row(s, lane, aR, k) : v.xs;
    if (lane < m && v.cover >= 0) v.xr = r_usign(s, v, v.cover) * (v.acol - r_zchunk(s, v, lane, v.xs, k));
    if (threadIdx.x == 0) c.st->refactors++;
    R_FENCE();
    return true;
}

// y = B^-T c_B (oracle btran): covered rows sigma_u c_u, R rows Minv^T t
RDEV void r_btran(RS& s, RV& v, RC& c, int phase) {
    const int k = c.k, m = s.m, lane = threadIdx.x;
    v.y = (lane < m && v.cover >= 0) ? r_usign(s, v, v.cover) * s.cost[v.cover] : 0.0;
    double t = 0.0;  // lane p
    if (lane < k) {
        t = s.cost[v.Sl];
        if (phase == 1) {
            const double* col = s.A + v.Sl * s.lda;
            const double yv = v.y;
            t = t - wdot([&](int i) { return col[i]; }, [&](int i) { return rl(yv, i); }, m);
        }
    }
    const double yR = r_minv_col(s, lane, t, k);  // lane p
    const double g = shf(yR, v.rpos & 63);
    if (lane < m && v.rpos >= 0) v.y = g;
}

// phase-1 infeasibility sum (oracle art_sum: wave order, one row per lane)
RDEV double r_art_sum(const RS& s, const RV& v) {
    const int lane = threadIdx.x;
    double acc = 0.0;
    if (lane < s.m && v.cover >= s.n + s.m) acc = acc + v.xr;
    return r_wtree(acc);
}

// FTRAN of column q: alpha_S (positions), alpha_U on covered rows
RDEV void r_ftran(const RS& s, RV& v, const RC& c, int q) {
    const int k = c.k, m = s.m, lane = threadIdx.x;
    v.acol = lane < m ? r_colA(s, lane, q) : 0.0;
    const double aR = shf(v.acol, v.Rl & 63);
    R_STAMP(8);
    v.alS = lane < k ? r_minv_row(s, lane, aR, k) : 0.0;
    R_STAMP(9);
    v.z = 0.0;
    v.alU = 0.0;
    if (lane < m && v.cover >= 0) {
        v.z = r_zchunk(s, v, lane, v.alS, k);
        v.alU = r_usign(s, v, v.cover) * (v.acol - v.z);
    }
    R_STAMP(10);
}
// lane c: A[i, S] Minv (oracle row_times_minv)
RDEV double r_row_times_minv(const RS& s, const RV& v, int k, int i) {
    const int lane = threadIdx.x;
    const double aR = lane < k ? s.A[i + v.Sl * s.lda] : 0.0;
    return r_minv_col(s, lane, aR, k);
}

RDEV void r_y_append(RV& v, RC& c, int i) {
    const int lane = threadIdx.x;
    if (lane == c.ny) v.Yl = i;
    if (lane == i) v.ypos = c.ny;
    c.ny++;
}
RDEV void r_y_remove(RV& v, RC& c, int i) {
    const int lane = threadIdx.x;
    const int p = rli(v.ypos, i), last = c.ny - 1;
    if (p != last) {
        const int moved = rli(v.Yl, last);
        if (lane == p) v.Yl = moved;
        if (lane == moved) v.ypos = p;
    }
    if (lane == i) v.ypos = -1;
    c.ny--;
}
// y_r = fma(f, u(rpos_r), y_r) on the rows of R (u: per position), position skip excepted
RDEV void r_dual_upd(const RS& s, RV& v, double f, double u, int skip) {
    const int lane = threadIdx.x;
    const double g = shf(u, v.rpos & 63);
    if (lane < s.m && v.rpos >= 0 && v.rpos != skip) v.y = fma(f, g, v.y);
}

// oracle basis_change (cases A-E, the zero rule, phase 2: the dual update)
// the rank-one update of the bump inverse (oracle basis_change, zero rule):
// Mi[r][lane] = fma(-f_r, vv, Mi[r][lane]) for rows r != skip with f_r != 0,
// on lanes < k other than `keep` whose vv != 0; eight rows' entries (and
// factors) loaded before any is stored -- each entry's arithmetic unchanged
template <class F>
RDEV void r_rank1(double* Mi, int ld, int k, int skip, int keep, double vv, F fac) {
    const int lane = threadIdx.x;
    const bool lw = lane < k && lane != keep && vv != 0.0;
    for (int r0 = 0; r0 < k; r0 += 8) {
        double x[8], f[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = r0 + u < k ? r0 + u : k - 1;
            f[u] = fac(r);
            x[u] = lw ? Mi[r * ld + lane] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = r0 + u;
            if (r >= k) break;
            if (r != skip && f[u] != 0.0 && lw) Mi[r * ld + lane] = fma(-f[u], vv, x[u]);
        }
    }
}

RDEV bool r_basis_change(RS& s, RV& v, RC& c, int phase, int q, int lv, int lrow, int lpos, double dq,
                         double xq) {
    const int m = s.m, n = s.n, k = c.k, lane = threadIdx.x;
    const int ld = s.ldm;
    const bool leave_art = lv >= n + m;
    double* Mi = s.Mi;
    if (q < n) {
        if (lpos >= 0) {  // case A: structural replaces structural at position p
            const int p = lpos;
            const double piv = rl(v.alS, p);
            const double vv = lane < k ? Mi[p * ld + lane] / piv : 0.0;
            if (phase == 2) r_dual_upd(s, v, dq, vv, -1);
            R_FENCE();
            r_rank1(Mi, ld, k, p, -1, vv, [&](int i) { return rl(v.alS, i); });
            if (lane < k) Mi[p * ld + lane] = vv;
            if (lane == p) {
                v.Sl = q;
                v.xs = xq;
            }
            if (lane == 0) {
                s.spos[lv] = -1;
                s.spos[q] = p;
            }
        } else {  // case B: structural enters, the unit variable of row i leaves
            const int i = lrow;
            const double delta = rl(v.acol, i) - rl(v.z, i);
            const double vv = r_row_times_minv(s, v, k, i) / delta;
            if (phase == 2) {
                r_dual_upd(s, v, -dq, vv, -1);
                if (lane == i) v.y = dq / delta;
            }
            R_FENCE();
            r_rank1(Mi, ld, k, -1, -1, vv, [&](int a) { return -rl(v.alS, a); });  // (fma(-(-w), vv, .) = fma(w, vv, .))
            if (lane < k) {
                Mi[lane * ld + k] = -(v.alS / delta);
                Mi[k * ld + lane] = -vv;
            }
            if (lane == 0) {
                Mi[k * ld + k] = 1.0 / delta;
                s.spos[q] = k;
            }
            if (lane == k) {
                v.Rl = i;
                v.Sl = q;
                v.xs = xq;
            }
            if (lane == i) {
                v.rpos = k;
                v.cover = -1;
            }
            c.k = k + 1;
            if (!leave_art) r_y_append(v, c, i);
        }
    } else {
        const int i0 = q - n;
        const int a = rli(v.rpos, i0);
        if (a < 0) {  // case E: the slack replaces the artificial of its own row
            if (lrow != i0) return false;
            if (lane == i0) {
                v.cover = q;
                v.xr = xq;
            }
        } else if (lpos >= 0) {  // case C: slack of row i0 (in R) enters, structural at b leaves
            const int b = lpos, last = k - 1;
            const double piv = Mi[b * ld + a];
            const double vv = lane < k ? Mi[b * ld + lane] / piv : 0.0;
            if (phase == 2) r_dual_upd(s, v, dq, vv, a);
            R_FENCE();
            r_rank1(Mi, ld, k, b, a, vv, [&](int r) { return Mi[r * ld + a]; });  // (column a is not written)
            R_FENCE();
            if (phase == 2 && lane == i0) v.y = 0.0;
            const int sl_last = rli(v.Sl, last), rl_last = rli(v.Rl, last);
            const double xs_last = rl(v.xs, last);
            if (b != last) {
                if (lane < k) Mi[b * ld + lane] = Mi[last * ld + lane];
                if (lane == b) {
                    v.Sl = sl_last;
                    v.xs = xs_last;
                }
                if (lane == 0) s.spos[sl_last] = b;
            }
            R_FENCE();
            if (a != last) {
                if (lane < k) Mi[lane * ld + a] = Mi[lane * ld + last];
                if (lane == a) v.Rl = rl_last;
                if (lane == rl_last) v.rpos = a;
            }
            if (lane == 0) s.spos[lv] = -1;
            if (lane == i0) {
                v.rpos = -1;
                v.cover = q;
                v.xr = xq;
            }
            c.k = k - 1;
        } else {  // case D: slack of row i0 (in R) enters, unit variable of row i1 leaves
            const int i1 = lrow;
            const double vv = r_row_times_minv(s, v, k, i1);
            const double piv = rl(vv, a);
            if (phase == 2) {
                const double w = dq / piv;
                r_dual_upd(s, v, w, vv, a);
                if (lane == i0) v.y = 0.0;
                if (lane == i1) v.y = -w;
            }
            const double tr = lane < k ? Mi[lane * ld + a] / piv : 0.0;  // (lane r)
            R_FENCE();
            r_rank1(Mi, ld, k, -1, a, vv, [&](int r) { return rl(tr, r); });
            if (lane < k) Mi[lane * ld + a] = tr;
            if (lane == a) v.Rl = i1;
            if (lane == i1) {
                v.rpos = a;
                v.cover = -1;
            }
            if (lane == i0) {
                v.rpos = -1;
                v.cover = q;
                v.xr = xq;
            }
        }
        r_y_remove(v, c, i0);
        if (a >= 0 && lpos < 0 && !leave_art) r_y_append(v, c, lrow);
    }
    R_FENCE();
    return true;
}

RDEV void r_trace(const Dev& d, const RC& c, int a, int b) {
    if (threadIdx.x == 0 && c.iter - 1 < c.trace_cap) {
        d.trace[2 * (c.iter - 1)] = a;
        d.trace[2 * (c.iter - 1) + 1] = b;
    }
}
RDEV void r_dw_reset(RS& s) {
    for (int j = threadIdx.x; j < s.n + s.m; j += RW) s.dw[j] = 1.0;
    R_FENCE();
}

// pricing sums of structural j: the price slot classes over the Y rows (yY:
// y on the slot of this lane) or CSC's column chain over the nonzero rows
RDEV double r_price_sum(const RS& s, const RV& v, const RC& c, int j, bool mode1, double yY) {
    const double* col = s.A + j * s.lda;
    if (mode1) {
        double acc = 0.0;
        for (int i0 = 0; i0 < s.m; i0 += 8) {
            double a[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] = col[i0 + u < s.m ? i0 + u : s.m - 1];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (i0 + u < s.m && a[u] != 0.0) acc = fma(a[u], rl(v.y, i0 + u), acc);
        }
        return acc;
    }
    double pw[PRICE_SPLIT] = {0.0, 0.0, 0.0, 0.0};
    const int ny = c.ny;
    for (int p0 = 0; p0 < ny; p0 += 2 * PRICE_SPLIT) {
        double a[2 * PRICE_SPLIT];
#pragma unroll
        for (int w = 0; w < 2 * PRICE_SPLIT; ++w) a[w] = col[rli(v.Yl, p0 + w < ny ? p0 + w : ny - 1)];
#pragma unroll
        for (int w = 0; w < 2 * PRICE_SPLIT; ++w)
            if (p0 + w < ny) pw[w % PRICE_SPLIT] = fma(a[w], rl(yY, p0 + w), pw[w % PRICE_SPLIT]);
    }
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < PRICE_SPLIT; ++w) tot = tot + pw[w];
    return tot;
}

// a warm-started node's nonbasic column j re-placed for the node's bounds and
// its reduced cost dj (elp_kernels.hip warm_fix, oracle warm_core); 1 when its
// cost was flattened to make it dual feasible
RDEV int r_warm_fix(RS& s, int j, bool structural, double dj, double dtol) {
    int8_t vs = s.vst[j];
    if (vs == VS_BASIC) return 0;
    const double l = s.lb[j], u = s.ub[j];
    if (l == u) {
        if (structural) {
            s.vst[j] = VS_FIXED;
            s.xval[j] = l;
        }
        return 0;
    }
    if (structural) {
        const bool lo_ok = l > -R_INF, up_ok = u < R_INF;
        if (vs == VS_FIXED) vs = VS_LOWER;
        if (vs == VS_LOWER && !lo_ok) vs = up_ok ? VS_UPPER : VS_FREE;
        else if (vs == VS_UPPER && !up_ok) vs = lo_ok ? VS_LOWER : VS_FREE;
        else if (vs == VS_FREE && (lo_ok || up_ok)) vs = lo_ok ? VS_LOWER : VS_UPPER;
        if (vs == VS_LOWER && dj < -dtol && up_ok) vs = VS_UPPER;
        else if (vs == VS_UPPER && dj > dtol && lo_ok) vs = VS_LOWER;
        s.vst[j] = vs;
        s.xval[j] = vs == VS_LOWER ? l : vs == VS_UPPER ? u : 0.0;
    }
    if ((vs == VS_LOWER && dj < -dtol) || (vs == VS_UPPER && dj > dtol) || (vs == VS_FREE && fabs(dj) > dtol)) {
        s.cost[j] = s.cost[j] - dj;
        return 1;
    }
    return 0;
}

enum { R_CONT = 0, R_EXIT = 1, R_RECHECK = 2, R_TO_P2 = 3, R_PIVOT = 4 };

// the pivot an iteration chose: entering q (reduced cost dq, its Devex
// weight qw, direction sig), the leaving variable and entry, the new value of
// q; the dual's leaving row (CHUZR) rides along
struct Piv {
    int q, lv, lrow, lpos;
    double dq, qw, sig, xq;
    int rv, re, rs;
    double rx, rbeta, qt, qa;
};

// primal pricing (oracle run_phase, after the loop top and BTRAN): the
// entering column, or the phase's end
RDEV int r_primal_select(const Dev& d, RS& s, RV& v, RC& c, bool mode1, Piv& P) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    const int ph = c.phase;
    const double yY = mode1 ? 0.0 : shf(v.y, v.Yl & 63);  // (slot lane: y on its Y row)
    const double dtol = c.tol_dual;
    const bool devex = c.devex != 0;
    int bq = 0x7fffffff;
    double bscore = 0.0, bd = 0.0, bw = 1.0;
    for (int j0 = 0; j0 < n + m; j0 += RW) {
        const int j = j0 + lane;
        const double sum = j0 < n ? r_price_sum(s, v, c, j < n ? j : n - 1, mode1, yY) : 0.0;
        const double yslack = shf(v.y, (j - n) & 63);
        if (j >= n + m) continue;
        const int8_t vs = s.vst[j];
        if (vs == VS_BASIC || s.lb[j] == s.ub[j]) continue;
        const double dj = j < n ? s.cost[j] - sum : s.cost[j] - yslack;
        double wj = 1.0;
        if (devex) {
            wj = s.dw[j];
            if (c.dv_valid && j != c.dv_lv) {
                const double r = (s.dprev[j] - dj) / c.dv_dq;
                double wn = (r * r) * c.dv_wq;
                if (wn > R_WMAX) wn = R_WMAX;
                if (wn > wj) {
                    wj = wn;
                    s.dw[j] = wj;
                }
            }
            s.dprev[j] = dj;
        }
        double score;
        if ((vs == VS_LOWER || vs == VS_FREE) && dj < -dtol) score = devex ? (dj * dj) / wj : -dj;
        else if ((vs == VS_UPPER || vs == VS_FREE) && dj > dtol) score = devex ? (dj * dj) / wj : dj;
        else continue;
        const bool take = c.bland ? bq == 0x7fffffff : (bq == 0x7fffffff || score > bscore);
        if (take) {
            bq = j;
            bscore = score;
            bd = dj;
            bw = wj;
        }
    }
    R_FENCE();
    R_STAMP(11);
    if (lane == 0) c.st->price_bytes += mode1 ? 12.0 * (double)d.nnz + 17.0 * n : 8.0 * ((double)c.ny * n + n + c.ny);
    const bool have = bq != 0x7fffffff;
    const int wl = c.bland ? r_argminid(have, bq) : r_argbest<false>(have, bscore, bq);
    R_STAMP(12);
    if (wl < 0) {
        if (ph == 2 && c.since > 0) return R_RECHECK;  // optimal under updated duals: confirm
        if (ph == 1) {
            if (c.art_sum > c.tol_inf) {
                c.status = ST_PHASE_OPT;  // (the host: infeasible)
                return R_EXIT;
            }
            return R_TO_P2;
        }
        c.status = ST_PHASE_OPT;
        return R_EXIT;
    }
    P.q = rli(bq, wl);
    P.dq = rl(bd, wl);
    P.qw = rl(bw, wl);
    P.sig = P.dq < 0.0 ? 1.0 : -1.0;
    return R_PIVOT;
}

// primal ratio test and update (after the FTRAN of P.q)
RDEV int r_primal_finish(const Dev& d, RS& s, RV& v, RC& c, Piv& P) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    const int ph = c.phase, k = c.k, q = P.q;
    const double dq = P.dq, qw = P.qw, sig = P.sig;
    const bool devex = c.devex != 0;
    // Harris two-pass ratio test (textbook under Bland) over each lane's two
    // basic entries: its covered row (e = lane), its bump position (e = m + lane)
    const double ptol = c.tol_primal, pivtol = c.tol_pivot;
    int evar[2], ee[2];
    double eg[2], rr[2];
    bool ok[2];
    evar[0] = lane < m ? v.cover : -1;
    ee[0] = lane;
    eg[0] = sig * v.alU;
    evar[1] = lane < k ? v.Sl : -1;
    ee[1] = m + lane;
    eg[1] = sig * v.alS;
    const double ex[2] = {v.xr, v.xs};
    double tmax = R_INF;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        ok[h] = false;
        rr[h] = 0.0;
        if (evar[h] < 0) continue;
        const double l = s.lb[evar[h]], u = s.ub[evar[h]], g = eg[h], x = ex[h];
        double r1;
        if (g > pivtol && l > -R_INF) {
            r1 = c.bland ? (x - l) / g : (x - l + ptol) / g;
            rr[h] = (x - l) / g;
        } else if (g < -pivtol && u < R_INF) {
            r1 = c.bland ? (u - x) / (-g) : (u - x + ptol) / (-g);
            rr[h] = (u - x) / (-g);
        } else {
            continue;
        }
        ok[h] = true;
        if (r1 < tmax) tmax = r1;
    }
    tmax = r_wmin(tmax);
    R_STAMP(13);
    int lv = -1, le = 0;
    double lg = 0.0, lr = 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (!ok[h] || !(rr[h] <= tmax)) continue;
        const int var = evar[h];
        const double g = eg[h], r = rr[h];
        bool take;
        if (lv < 0) take = true;
        else if (c.bland) take = (r < lr) || (r == lr && var < lv);
        else take = (fabs(g) > fabs(lg)) || (fabs(g) == fabs(lg) && var < lv);
        if (take) {
            lv = var;
            le = ee[h];
            lg = g;
            lr = r;
        }
    }
    const bool lhave = lv >= 0;
    const int ll = c.bland ? r_argbest<true>(lhave, lr, lv) : r_argbest<false>(lhave, fabs(lg), lv);
    if (ll >= 0) {
        lv = rli(lv, ll);
        le = rli(le, ll);
        lg = rl(lg, ll);
        lr = rl(lr, ll);
    } else {
        lv = -1;
    }
    R_STAMP(14);
    const double theta = lv >= 0 ? (lr > 0.0 ? lr : 0.0) : R_INF;
    const double flip = (s.lb[q] > -R_INF && s.ub[q] < R_INF) ? s.ub[q] - s.lb[q] : R_INF;
    c.iter++;
    if (lane == 0) {
        if (ph == 1) c.st->phase1_iters++;
        c.st->iter_bytes += 8.0 * (6.0 * k * k + (double)m * k + 2.0 * n + 2.0 * m);
    }
    if (flip < R_INF && flip <= theta) {  // bound flip
        if (lane < m && v.cover >= 0) v.xr = fma(-flip, sig * v.alU, v.xr);
        if (lane < k) v.xs = fma(-flip, sig * v.alS, v.xs);
        if (lane == 0) {
            if (s.vst[q] == VS_LOWER) {
                s.vst[q] = VS_UPPER;
                s.xval[q] = s.ub[q];
            } else {
                s.vst[q] = VS_LOWER;
                s.xval[q] = s.lb[q];
            }
        }
        if (lane == 0) c.st->flips++;
        r_trace(d, c, q, -1);
        c.dv_valid = 0;
        c.ndegen = 0;
        c.bland = 0;
        R_FENCE();
        return R_CONT;
    }
    if (theta == R_INF) {
        r_trace(d, c, q, -2);
        if (lane == 0) {
            c.st->unb_var = q;
            c.st->unb_sig = sig;
        }
        c.status = ST_UNBOUNDED;
        return R_EXIT;
    }
    r_trace(d, c, q, lv);
    if (devex && qw > R_RESET) {
        r_dw_reset(s);
        c.dv_valid = 0;
        if (lane == 0) c.st->resets++;
    } else if (devex) {
        double wl2 = qw / (lg * lg);
        if (wl2 < 1.0) wl2 = 1.0;
        if (wl2 > R_WMAX) wl2 = R_WMAX;
        if (lane == 0 && lv < n + m) s.dw[lv] = wl2;
        c.dv_valid = 1;
        c.dv_lv = lv;
        c.dv_dq = dq;
        c.dv_wq = qw;
    }
    if (theta == 0.0) {
        if (lane == 0) c.st->degenerate++;
        if (++c.ndegen >= c.degen_switch) c.bland = 1;
    } else {
        c.ndegen = 0;
        c.bland = 0;
    }
    if (lane < m && v.cover >= 0) v.xr = fma(-theta, sig * v.alU, v.xr);
    if (lane < k) v.xs = fma(-theta, sig * v.alS, v.xs);
    const double xq = s.xval[q] + sig * theta;
    const bool at_lower = lg > 0.0;
    R_FENCE();
    if (lane == 0) {
        if (lv >= n + m) {
            s.lb[lv] = 0.0;
            s.ub[lv] = 0.0;
            s.vst[lv] = VS_FIXED;
            s.xval[lv] = 0.0;
        } else {
            const double l = s.lb[lv], u = s.ub[lv];
            s.vst[lv] = l == u ? VS_FIXED : at_lower ? VS_LOWER : VS_UPPER;
            s.xval[lv] = at_lower ? l : u;
        }
        s.vst[q] = VS_BASIC;
    }
    R_FENCE();
    P.lv = lv;
    P.lrow = le < m ? le : -1;
    P.lpos = le < m ? -1 : le - m;
    P.xq = xq;
    return R_PIVOT;
}

// dual CHUZR, pivot row, bound-flipping ratio test and the flips (oracle
// run_dual, after the loop top): the entering column, or the phase's end
RDEV int r_dual_select(const Dev& d, RS& s, RV& v, RC& c, bool mode1, Piv& P) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    const double ptol = c.tol_primal, dtol = c.tol_dual, pivtol = c.tol_pivot;
    const bool devex = c.ddevex != 0;
    const int k = c.k;
    // ---- CHUZR over this lane's covered row and bump position
    int rv = -1, re = 0, rs = 0;
    double rscore = 0.0, rx = 0.0, rbeta = 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int var = h == 0 ? (lane < m ? v.cover : -1) : (lane < k ? v.Sl : -1);
        if (var < 0) continue;
        const double x = h == 0 ? v.xr : v.xs;
        const double l = s.lb[var], u = s.ub[var];
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
        const double score = devex ? (delta * delta) / (var < n + m ? s.dw[var] : 1.0) : delta;
        bool take;
        if (rv < 0) take = true;
        else if (c.bland) take = var < rv;
        else take = score > rscore || (score == rscore && var < rv);
        if (take) {
            rv = var;
            re = h == 0 ? lane : m + lane;
            rscore = score;
            rx = x;
            rbeta = beta;
            rs = sd;
        }
    }
    const bool rh = rv >= 0;
    const int wl = c.bland ? r_argminid(rh, rv) : r_argbest<false>(rh, rscore, rv);
    if (wl < 0) return c.since > 0 ? R_RECHECK : R_TO_P2;  // (recheck: confirm on a fresh x_B)
    R_STAMP(16);
    rv = rli(rv, wl);
    re = rli(re, wl);
    rs = rli(rs, wl);
    rx = rl(rx, wl);
    rbeta = rl(rbeta, wl);
    // ---- rho_r (per position), then on the rows
    int xrow = -1;
    double xsig = 0.0, vv;
    if (re >= m) {
        vv = lane < k ? s.Mi[(re - m) * s.ldm + lane] : 0.0;
    } else {
        xrow = re;
        xsig = rli(v.cover, re) >= n + m ? rl(v.asgn, re) : 1.0;
        vv = -(xsig * r_row_times_minv(s, v, k, re));
    }
    double rho = shf(vv, v.rpos & 63);
    if (!(lane < m && v.rpos >= 0)) rho = 0.0;
    if (lane == xrow) rho = xsig;
    R_STAMP(17);
    // ---- one sweep: d_j (y) and alpha_j (rho)
    const double yY = mode1 ? 0.0 : shf(v.y, v.Yl & 63), rY = mode1 ? 0.0 : shf(rho, v.Yl & 63);
    for (int j0 = 0; j0 < n; j0 += RW) {
        const int j = j0 + lane < n ? j0 + lane : n - 1;
        const double* col = s.A + j * s.lda;
        double td = 0.0, ta = 0.0;
        if (mode1) {
            for (int i0 = 0; i0 < m; i0 += 8) {
                double a[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) a[u] = col[i0 + u < m ? i0 + u : m - 1];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (i0 + u < m && a[u] != 0.0) {
                        td = fma(a[u], rl(v.y, i0 + u), td);
                        ta = fma(a[u], rl(rho, i0 + u), ta);
                    }
            }
        } else {
            double pd[PRICE_SPLIT] = {0.0, 0.0, 0.0, 0.0}, pa[PRICE_SPLIT] = {0.0, 0.0, 0.0, 0.0};
            const int ny = c.ny;
            for (int p0 = 0; p0 < ny; p0 += 2 * PRICE_SPLIT) {
                double a[2 * PRICE_SPLIT];
#pragma unroll
                for (int w = 0; w < 2 * PRICE_SPLIT; ++w) a[w] = col[rli(v.Yl, p0 + w < ny ? p0 + w : ny - 1)];
#pragma unroll
                for (int w = 0; w < 2 * PRICE_SPLIT; ++w)
                    if (p0 + w < ny) {
                        pd[w % PRICE_SPLIT] = fma(a[w], rl(yY, p0 + w), pd[w % PRICE_SPLIT]);
                        pa[w % PRICE_SPLIT] = fma(a[w], rl(rY, p0 + w), pa[w % PRICE_SPLIT]);
                    }
            }
            double sd2 = 0.0, sa = 0.0;
#pragma unroll
            for (int w = 0; w < PRICE_SPLIT; ++w) {
                sd2 = sd2 + pd[w];
                sa = sa + pa[w];
            }
            td = sd2;
            ta = xrow >= 0 ? fma(xsig, col[xrow], sa) : sa;
        }
        if (j0 + lane < n) {
            s.dvec[j] = s.cost[j] - td;
            s.avec[j] = ta;
        }
    }
    if (lane < m) {
        s.dvec[n + lane] = s.cost[n + lane] - v.y;
        s.avec[n + lane] = rho;
    }
    if (lane == 0) c.st->price_bytes += mode1 ? 12.0 * (double)d.nnz + 17.0 * n : 8.0 * ((double)c.ny * n + n + c.ny);
    R_FENCE();
    R_STAMP(18);
    // ---- candidates, ascending id (ballot compaction)
    int nc = 0;
    for (int j0 = 0; j0 < n + m; j0 += RW) {
        const int j = j0 + lane;
        bool f = false;
        double t = 0.0, bnd = 0.0, aab = 0.0, rr = 0.0;
        if (j < n + m) {
            const int8_t vs = s.vst[j];
            if (vs != VS_BASIC && s.lb[j] != s.ub[j]) {
                const double a = s.avec[j], ah = rs * a, dj = s.dvec[j];
                int side = 0;
                if (vs == VS_LOWER || (vs == VS_FREE && ah < 0.0)) side = ah < -pivtol ? 1 : 0;
                else if (vs == VS_UPPER || (vs == VS_FREE && ah > 0.0)) side = ah > pivtol ? -1 : 0;
                if (side) {
                    f = true;
                    t = side > 0 ? dj / (-ah) : (-dj) / ah;
                    bnd = c.bland ? t : side > 0 ? (dj + dtol) / (-ah) : (dtol - dj) / ah;
                    aab = fabs(a);
                    rr = (s.lb[j] > -R_INF && s.ub[j] < R_INF) ? s.ub[j] - s.lb[j] : R_INF;
                }
            }
        }
        const unsigned long long bm = __ballot(f);
        if (f) {
            const int o = nc + __popcll(bm & ((1ull << lane) - 1ull));
            s.cj[o] = j;
            s.ct[o] = t;
            s.cb[o] = bnd;
            s.ca[o] = aab;
            s.cr[o] = rr;
            s.calive[o] = 1;
        }
        nc += __popcll(bm);
    }
    R_FENCE();
    R_STAMP(19);
    // ---- bound-flipping Harris ratio test
    double slope = fabs(rx - rbeta);
    int q = -1, nflip = 0;
    double qt = 0.0, qa = 0.0;
    for (;;) {
        double thmax = R_INF;
        bool any = false;
        for (int cc = lane; cc < nc; cc += RW)
            if (s.calive[cc]) {
                any = true;
                if (s.cb[cc] < thmax) thmax = s.cb[cc];
            }
        if (__ballot(any) == 0ull) break;
        thmax = r_wmin(thmax);
        int nq = 0;
        bool allbox = true;
        double sum = 0.0;
        for (int c0 = 0; c0 < nc; c0 += RW) {
            const int cc = c0 + lane;
            const int ccc = cc < nc ? cc : 0;
            const bool in = cc < nc && s.calive[ccc] && s.ct[ccc] <= thmax;
            const double cav = s.ca[ccc], crv = s.cr[ccc];
            unsigned long long bm = __ballot(in);
            nq += __popcll(bm);
            if (__ballot(in && crv == R_INF)) allbox = false;
            while (bm) {  // (uniform: the bunch in ascending order)
                const int t = __ffsll((long long)bm) - 1;
                bm &= bm - 1ull;
                const double crt = rl(crv, t);
                if (crt != R_INF) sum = fma(rl(cav, t), crt, sum);
            }
        }
        if (nq == 0) break;  // (NaN ratios only)
        if (allbox && sum < slope - ptol) {
            slope = slope - sum;
            for (int c0 = 0; c0 < nc; c0 += RW) {
                const int cc = c0 + lane;
                const bool in = cc < nc && s.calive[cc] && s.ct[cc] <= thmax;
                const unsigned long long bm = __ballot(in);
                if (in) {
                    s.calive[cc] = 0;
                    s.flips[nflip + __popcll(bm & ((1ull << lane) - 1ull))] = s.cj[cc];
                }
                nflip += __popcll(bm);
            }
            R_FENCE();
            continue;
        }
        bool h = false;
        int bc = 0x7fffffff, bj = 0x7fffffff;
        double bt = 0.0, ba = 0.0;
        for (int cc = lane; cc < nc; cc += RW) {
            if (!s.calive[cc] || !(s.ct[cc] <= thmax)) continue;
            const int j = s.cj[cc];
            const double t = s.ct[cc], a = s.ca[cc];
            bool take;
            if (!h) take = true;
            else if (c.bland) take = t < bt || (t == bt && j < bj);
            else take = a > ba || (a == ba && j < bj);
            if (take) {
                h = true;
                bc = cc;
                bj = j;
                bt = t;
                ba = a;
            }
        }
        const int w2 = c.bland ? r_argbest<true>(h, bt, bj) : r_argbest<false>(h, ba, bj);
        bc = rli(bc, w2);
        q = s.cj[bc];
        qt = s.ct[bc];
        qa = s.avec[q];
        break;
    }
    R_STAMP(20);
    c.iter++;
    if (lane == 0) {
        c.st->phase1_iters++;
        c.st->dual_iters++;
        c.st->iter_bytes += 8.0 * (6.0 * k * k + (double)m * k + 2.0 * n + 2.0 * m);
    }
    if (q < 0) {  // the dual ray: primal infeasible
        r_trace(d, c, -2, rv);
        c.status = ST_DUALINF;
        return R_EXIT;
    }
    // ---- the flips: a_F = sum_j a_j dx_j (flip order), x_B -= B^-1 a_F
    if (nflip > 0) {
        double* dx = s.cb;  // (the ratio test is done with it)
        for (int f = lane; f < nflip; f += RW) {
            const int j = s.flips[f];
            dx[f] = s.vst[j] == VS_LOWER ? s.ub[j] - s.lb[j] : s.lb[j] - s.ub[j];
        }
        R_FENCE();
        double aF = 0.0;  // (row lane)
        for (int f = 0; f < nflip; ++f) {
            const int j = s.flips[f];
            aF = fma(lane < m ? r_colA(s, lane, j) : 0.0, dx[f], aF);
        }
        R_FENCE();
        for (int f = lane; f < nflip; f += RW) {
            const int j = s.flips[f];
            const int8_t nvs = s.vst[j] == VS_LOWER ? VS_UPPER : VS_LOWER;
            s.vst[j] = nvs;
            s.xval[j] = nvs == VS_LOWER ? s.lb[j] : s.ub[j];
        }
        const double aR = shf(aF, v.Rl & 63);
        const double fS = lane < k ? r_minv_row(s, lane, aR, k) : 0.0;
        if (lane < m && v.cover >= 0) v.xr = v.xr - r_usign(s, v, v.cover) * (aF - r_zchunk(s, v, lane, fS, k));
        if (lane < k) v.xs = v.xs - fS;
        if (lane == 0) c.st->flips += nflip;
        R_FENCE();
        rx = re < m ? rl(v.xr, re) : rl(v.xs, re - m);
    }
    R_STAMP(21);
    const int8_t vq = s.vst[q];
    P.q = q;
    P.dq = s.dvec[q];
    P.sig = (vq == VS_LOWER || (vq == VS_FREE && rs * qa < 0.0)) ? 1.0 : -1.0;
    P.rv = rv;
    P.re = re;
    P.rs = rs;
    P.rx = rx;
    P.rbeta = rbeta;
    P.qt = qt;
    return R_PIVOT;
}

// the dual update (after the FTRAN of P.q)
RDEV int r_dual_finish(const Dev& d, RS& s, RV& v, RC& c, Piv& P) {
    const int m = s.m, n = s.n, lane = threadIdx.x, k = c.k, q = P.q, rv = P.rv, re = P.re, rs = P.rs;
    const bool devex = c.ddevex != 0;
    const double sig = P.sig, rx = P.rx, rbeta = P.rbeta, qt = P.qt;
    const double arq = re < m ? rl(v.alU, re) : rl(v.alS, re - m);
    const double step = fabs((rx - rbeta) / arq);
    r_trace(d, c, q, rv);
    if (devex) {  // dual Devex weights of the basic entries (old basis)
        const double wr = rv < n + m ? s.dw[rv] : 1.0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int e = h == 0 ? lane : m + lane;
            const int var = h == 0 ? (lane < m ? v.cover : -1) : (lane < k ? v.Sl : -1);
            if (var < 0 || e == re) continue;
            const double ae = h == 0 ? v.alU : v.alS;
            const double r = ae / arq;
            double wn = (r * r) * wr;
            if (wn > R_WMAX) wn = R_WMAX;
            if (var < n + m && wn > s.dw[var]) s.dw[var] = wn;
        }
        R_FENCE();
        double wq = wr / (arq * arq);
        if (wq < 1.0) wq = 1.0;
        if (wq > R_WMAX) wq = R_WMAX;
        if (wq > R_RESET) {
            r_dw_reset(s);
            if (lane == 0) c.st->resets++;
        } else if (lane == 0) {
            s.dw[q] = wq;
        }
    }
    if (!(qt > 0.0)) {
        if (lane == 0) c.st->degenerate++;
        if (++c.ndegen >= c.degen_switch) c.bland = 1;
    } else {
        c.ndegen = 0;
        c.bland = 0;
    }
    if (lane < m && v.cover >= 0) v.xr = fma(-step, sig * v.alU, v.xr);
    if (lane < k) v.xs = fma(-step, sig * v.alS, v.xs);
    const double xq = s.xval[q] + sig * step;
    R_FENCE();
    if (lane == 0) {
        const double l = s.lb[rv], u = s.ub[rv];
        s.vst[rv] = l == u ? VS_FIXED : rs > 0 ? VS_LOWER : VS_UPPER;
        s.xval[rv] = rbeta;
        s.vst[q] = VS_BASIC;
    }
    R_FENCE();
    P.lv = rv;
    P.lrow = re < m ? re : -1;
    P.lpos = re < m ? -1 : re - m;
    P.xq = xq;
    return R_PIVOT;
}

// the real costs and the primal phase 2 (launch_phase2; the refactor and BTRAN follow)
RDEV void r_to_phase2(const Dev& d, RS& s, RC& c, int price_rule) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    for (int j = lane; j < n; j += RW) s.cost[j] = d.maximize ? -d.obj[j] : d.obj[j];
    if (lane < m) {
        const int av = n + m + lane;
        s.cost[n + lane] = 0.0;
        s.cost[av] = 0.0;
        s.lb[av] = 0.0;
        s.ub[av] = 0.0;
    }
    r_dw_reset(s);
    c.dv_valid = 0;
    c.phase = 2;
    c.since = 0;
    c.ndegen = 0;
    c.bland = 0;
    c.devex = price_rule == 1;
    c.y_valid = 0;
}

// dst[e] = src(e) for e < cnt, 8 global loads in flight per lane
template <class T, class F>
RDEV void r_gather(T* dst, int64_t cnt, F src) {
    for (int64_t e0 = threadIdx.x; e0 < cnt; e0 += RW * 8) {
        T x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t e = e0 + (int64_t)u * RW;
            x[u] = src(e < cnt ? e : cnt - 1);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (e0 + (int64_t)u * RW < cnt) dst[e0 + (int64_t)u * RW] = x[u];
    }
}

__global__ void __launch_bounds__(RW) k_resident(Dev d, ResArgs a) {
    extern __shared__ __attribute__((aligned(16))) char r_smem[];
    RS s;
    r_carve(s, r_smem, d.m, d.n);
    const int m = s.m, n = s.n, nv = s.nv, lane = threadIdx.x;
    const bool mode1 = d.csc != 0;
    DevCtl* g = d.ctl;
    RC c;
    c.phase = a.phase;
    c.k = g->k;
    c.ny = g->ny;
    c.iter = g->iter;
    c.iter_limit = g->iter_limit;
    c.iter_stop = g->iter_stop;
    __shared__ RStat r_stat;
    c.st = &r_stat;
    if (lane == 0) {
        r_stat.phase1_iters = g->phase1_iters;
        r_stat.flips = g->flips;
        r_stat.degenerate = g->degenerate;
        r_stat.dual_iters = g->dual_iters;
        r_stat.unb_sig = g->unb_sig;
        r_stat.unb_var = g->unb_var;
        r_stat.price_bytes = g->price_bytes;
        r_stat.iter_bytes = g->iter_bytes;
        r_stat.refactors = r_stat.gj = r_stat.resets = 0;
        r_stat.emax_max = 0.0;
    }
    c.since = g->since_refactor;
    c.period = g->refactor_period;
    c.ndegen = g->ndegen;
    c.bland = g->bland;
    c.degen_switch = g->degen_switch;
    c.devex = g->devex;
    c.ddevex = g->ddevex;
    c.dv_valid = g->dv_valid;
    c.dv_lv = g->dv_lv;
    c.dv_dq = g->dv_dq;
    c.dv_wq = g->dv_wq;
    c.tol_primal = g->tol_primal;
    c.tol_dual = g->tol_dual;
    c.tol_pivot = g->tol_pivot;
    c.tol_inf = g->tol_inf;
    c.tol_singular = d.tol_singular;
    c.art_sum = g->art_sum;
    c.status = ST_RUN;
    c.trace_cap = d.trace ? g->trace_cap : 0;
    c.y_valid = 1;  // (the load's BTRAN, or the updated duals of the last exit)
    const int k0 = c.k, ny0 = c.ny;
    // ---- state into LDS and registers (global loads 8 in flight per lane)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (mode1) {
        for (int e = lane; e < s.lda * n; e += RW) s.A[e] = 0.0;
        R_FENCE();
        // lane j: column j's entries, 4 in flight
        for (int j0 = 0; j0 < n; j0 += RW) {
            const int j = j0 + lane < n ? j0 + lane : n - 1;
            const int64_t c0 = d.cptr[j], c1 = j0 + lane < n ? d.cptr[j + 1] : c0;
            for (int64_t t = c0; __ballot(t < c1); t += 4) {
                int ri[4];
                double vv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int64_t tt = t + u < c1 ? t + u : (c1 > c0 ? c1 - 1 : c0);
                    ri[u] = c1 > c0 ? d.rind[tt] : 0;
                    vv[u] = c1 > c0 ? d.cval[tt] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (t + u < c1) s.A[ri[u] + j * s.lda] = vv[u];
            }
        }
    } else {
        r_gather(s.A, (int64_t)s.lda * n, [&](int64_t e) {
            const int64_t j = e / s.lda, i = e - j * s.lda;
            if (i >= m) return 0.0;
            const double x = d.A[(size_t)j * m + i];
            return d.srow ? ldexp(x, d.srow[i] + d.scol[j]) : x;
        });
    }
    // the per-variable arrays together: one round trip for every 4 x 64 variables
    // (seven gathers one after another cost seven -- ~10 us of a MIP node's launch)
    for (int e0 = lane; e0 < nv; e0 += RW * 4) {
        double xl[4], xu[4], xc[4], xx[4], xw[4], xp[4];
        int8_t xs8[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * RW < nv ? e0 + u * RW : nv - 1;
            const int e2 = e < n + m ? e : n + m - 1;
            xl[u] = d.lb[e];
            xu[u] = d.ub[e];
            xc[u] = d.cost[e];
            xx[u] = d.xval[e];
            xs8[u] = d.vstat[e];
            xw[u] = d.dw[e2];
            xp[u] = d.dprev[e2];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * RW;
            if (e < nv) {
                s.lb[e] = xl[u];
                s.ub[e] = xu[u];
                s.cost[e] = xc[u];
                s.xval[e] = xx[u];
                s.vst[e] = xs8[u];
            }
            if (e < n + m) {
                s.dw[e] = xw[u];
                s.dprev[e] = xp[u];
            }
        }
    }
    for (int j = lane; j < n; j += RW) s.spos[j] = -1;
    RV v;
    const bool rowl = lane < m;
    const int rr = rowl ? lane : 0;
    v.b = d.b[rr];
    v.xr = d.xr[rr];
    v.asgn = d.asgn[rr];
    v.y = d.y[rr];
    v.cover = d.cover[rr];
    v.rpos = d.rpos[rr];
    v.ypos = d.ypos[rr];
    v.Yl = d.Yl[lane < ny0 ? lane : 0];
    v.Rl = d.Rl[lane < k0 ? lane : 0];
    v.Sl = d.Sl[lane < k0 ? lane : 0];
    v.xs = d.xs[lane < k0 ? lane : 0];
    if (!rowl) {
        v.b = v.xr = v.y = 0.0;
        v.asgn = 1.0;
        v.cover = v.rpos = v.ypos = -1;
    }
    if (lane >= ny0) v.Yl = 0;
    if (lane >= k0) {
        v.Rl = v.Sl = 0;
        v.xs = 0.0;
    }
    v.acol = v.z = v.alU = v.alS = 0.0;
    for (int i0 = 0; i0 < k0; i0 += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            x[u] = lane < k0 ? d.Minv[(size_t)(i0 + u < k0 ? i0 + u : k0 - 1) * d.ldm + lane] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u < k0 && lane < k0) s.Mi[(i0 + u) * s.ldm + lane] = x[u];
    }
    R_FENCE();
    if (lane < k0) s.spos[v.Sl] = lane;
    if (c.dv_valid == 2) {  // (the pipeline's deferred framework restart)
        r_dw_reset(s);
        c.dv_valid = 0;
    }
    R_FENCE();
    // The loop (elp_api.hip run_loop / oracle solve_core): one call site each
    // for the refactor, BTRAN, FTRAN and basis change keeps the code small
    // enough to stay in the instruction cache.
    enum { RF_NONE = 0, RF_TOP, RF_RECHECK, RF_TO_P2 };
    int recheck = 0, refac = RF_NONE;
    Piv P;
    int64_t flat = 0;
    if (a.warm) {
        // a branch-and-bound node from the last node's basis (reload_bounds_warm:
        // launch_warm_start, do_refactor, launch_devex_reset): the real costs, y
        // of them on the last inverse, each nonbasic column re-placed for the
        // node's bounds (the host wrote them) and its reduced cost, then the
        // refactor; the dual phase starts at its loop top
        for (int j = lane; j < n; j += RW) s.cost[j] = d.maximize ? -d.obj[j] : d.obj[j];
        if (lane < m) s.cost[n + lane] = 0.0;
        R_FENCE();
        r_btran(s, v, c, 2);
        const double yY = mode1 ? 0.0 : shf(v.y, v.Yl & 63);
        int nf = 0;
        for (int j0 = 0; j0 < n; j0 += RW) {
            const int j = j0 + lane < n ? j0 + lane : n - 1;
            const double td = r_price_sum(s, v, c, j, mode1, yY);
            if (j0 + lane < n) nf += r_warm_fix(s, j, true, s.cost[j] - td, c.tol_dual);
        }
        if (lane < m) nf += r_warm_fix(s, n + lane, false, s.cost[n + lane] - v.y, c.tol_dual);
        flat = (int64_t)r_wtree((double)nf);  // (exact: small integers)
        R_FENCE();
        r_dw_reset(s);
        c.dv_valid = 0;
        refac = RF_TO_P2;
    }
    if (ELP_RES_PROF && lane == 0) {
        for (int i = 0; i < 24; ++i) r_prof[i] = 0;
        r_prof[24] = __builtin_amdgcn_s_memtime();
    }
    for (;;) {
        R_STAMP(7);
        if (refac != RF_NONE) {
            const bool ok = r_refactor(s, v, c, a.refactor_mode);
            R_STAMP(5);
            if (!ok) {
                c.status = ST_NUMFAIL;
                break;
            }
            c.since = 0;
            c.y_valid = 0;
            // after the loop top's refactor the iteration runs; a recheck skips
            // the loop top; a new phase 2 starts at its loop top
            recheck = refac != RF_TO_P2;
            refac = RF_NONE;
            continue;
        }
        if (!recheck) {
            if (c.phase == 1) {
                c.art_sum = r_art_sum(s, v);
                if (c.art_sum <= c.tol_inf) {
                    r_to_phase2(d, s, c, a.price_rule);
                    refac = RF_TO_P2;
                    continue;
                }
            }
            if (c.iter >= c.iter_limit) {
                c.status = ST_ITERCAP;
                break;
            }
            if (c.iter >= c.iter_stop) {
                c.status = ST_STOP;
                break;
            }
            if (a.tick_budget > 0 && (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.tick_budget) {
                c.status = ST_TIMEOUT;
                break;
            }
            if (c.since >= c.period) {
                refac = RF_TOP;
                continue;
            }
        }
        recheck = 0;
        if (c.phase == 1 || !c.y_valid) {  // (phase 1: every iteration; else after a refactor)
            c.y_valid = 1;
            r_btran(s, v, c, c.phase == 1 ? 1 : 2);
        }
        R_STAMP(0);
        int r = c.phase == 3 ? r_dual_select(d, s, v, c, mode1, P) : r_primal_select(d, s, v, c, mode1, P);
        R_STAMP(1);
        if (r == R_EXIT) break;
        if (r == R_RECHECK) {
            refac = RF_RECHECK;
            continue;
        }
        if (r == R_TO_P2) {
            r_to_phase2(d, s, c, a.price_rule);
            refac = RF_TO_P2;
            continue;
        }
        r_ftran(s, v, c, P.q);
        R_STAMP(2);
        r = c.phase == 3 ? r_dual_finish(d, s, v, c, P) : r_primal_finish(d, s, v, c, P);
        R_STAMP(3);
        if (r == R_EXIT) break;
        if (r == R_CONT) continue;
        const bool ok = r_basis_change(s, v, c, c.phase == 1 ? 1 : 2, P.q, P.lv, P.lrow, P.lpos, P.dq, P.xq);
        R_STAMP(4);
        if (!ok) {
            c.status = ST_NUMFAIL;
            break;
        }
        c.since++;
    }
    R_FENCE();
    // ---- write back in the pipeline's layout
    const int k = c.k, ny = c.ny;
    for (int j = lane; j < nv; j += RW) {
        d.lb[j] = s.lb[j];
        d.ub[j] = s.ub[j];
        d.cost[j] = s.cost[j];
        d.xval[j] = s.xval[j];
        d.vstat[j] = s.vst[j];
    }
    for (int j = lane; j < n + m; j += RW) {
        d.dw[j] = s.dw[j];
        d.dprev[j] = s.dprev[j];
    }
    if (d.spos)
        for (int j = lane; j < n; j += RW) d.spos[j] = s.spos[j];
    if (rowl) {
        d.xr[lane] = v.xr;
        d.y[lane] = v.y;
        d.cover[lane] = v.cover;
        d.rpos[lane] = v.rpos;
        d.ypos[lane] = v.ypos;
        if (v.cover >= 0) {
            d.rlo[lane] = s.lb[v.cover];
            d.rhi[lane] = s.ub[v.cover];
        }
    }
    const double yYl = shf(v.y, v.Yl & 63);
    if (lane < ny) {
        d.Yl[lane] = v.Yl;
        d.yvs[lane] = d.rowvs[v.Yl];
        d.yy[lane] = yYl;
    }
    if (lane < k) {
        d.Rl[lane] = v.Rl;
        d.Sl[lane] = v.Sl;
        d.xs[lane] = v.xs;
        d.cS[lane] = s.cost[v.Sl];
        d.slo[lane] = s.lb[v.Sl];
        d.shi[lane] = s.ub[v.Sl];
    }
    for (int i = 0; i < k; ++i)
        if (lane < k) {
            const double x = s.Mi[i * s.ldm + lane];
            d.Minv[(size_t)i * d.ldm + lane] = x;
            if (!d.noT) d.MinvT[(size_t)lane * d.ldm + i] = x;
        }
    for (int p = 0; p < k; ++p) {
        const double* col = s.A + rli(v.Sl, p) * s.lda;
        if (rowl) d.AS[(size_t)p * m + lane] = col[lane];
    }
    if (a.xout)  // the structurals' values (k_extract + k_extract_basic)
        for (int j0 = 0; j0 < n; j0 += RW) {
            const int j = j0 + lane < n ? j0 + lane : n - 1;
            const int p = s.spos[j];
            const double xb = shf(v.xs, p & 63);
            if (j0 + lane < n) a.xout[j] = p >= 0 ? xb : s.xval[j];
        }
    if (!mode1 && d.AR) {
        const int64_t tw = d.tile_w;
        for (int p = 0; p < ny; ++p) {
            const int i = rli(v.Yl, p);
            for (int j = lane; j < n; j += RW)
                d.AR[((size_t)(j / tw) * (size_t)d.arcap + (size_t)p) * (size_t)tw + (size_t)(j % tw)] =
                    s.A[i + j * s.lda];
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        g->status = c.status;
        g->phase = c.phase;
        g->k = k;
        g->ny = ny;
        g->iter = c.iter;
        g->phase1_iters = r_stat.phase1_iters;
        g->flips = r_stat.flips;
        g->degenerate = r_stat.degenerate;
        g->dual_iters = r_stat.dual_iters;
        if (a.warm) g->dflat += flat;
        g->since_refactor = c.since;
        g->ndegen = c.ndegen;
        g->bland = c.bland;
        g->devex = c.devex;
        g->ddevex = c.ddevex;
        g->dv_valid = c.dv_valid;
        g->dv_lv = c.dv_lv;
        g->dv_dq = c.dv_dq;
        g->dv_wq = c.dv_wq;
        g->art_sum = c.art_sum;
        g->unb_var = r_stat.unb_var;
        g->unb_sig = r_stat.unb_sig;
        g->price_bytes = r_stat.price_bytes;
        g->iter_bytes = r_stat.iter_bytes;
        a.out->phase = c.phase;
        a.out->refactors = r_stat.refactors;
        a.out->gj_refactors = r_stat.gj;
        a.out->devex_resets = r_stat.resets;
        a.out->emax_max = r_stat.emax_max;
        a.out->ticks = (int64_t)(t1 - t0);
        for (int i = 0; i < 8; ++i) a.out->stage[i] = ELP_RES_PROF ? (int64_t)(r_prof[i] + (i == 0 ? 0 : 0)) : 0;
        for (int i = 8; i < 16; ++i) a.out->stage2[i - 8] = ELP_RES_PROF ? (int64_t)r_prof[i] : 0;
        for (int i = 16; i < 24; ++i) a.out->stage3[i - 16] = ELP_RES_PROF ? (int64_t)r_prof[i] : 0;
    }
}

}  // namespace

size_t resident_lds_bytes(int m, int n) {
    if (m > RW) return -1;  // (one row per lane)
    RS s;
    return r_carve(s, nullptr, m, n);
}

hipError_t launch_resident(const Dev& d, const ResArgs& a, size_t lds, hipStream_t st) {
    static size_t attr = 0;
    if (lds > 65536 && lds > attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)k_resident, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = lds;
    }
    hipLaunchKernelGGL(k_resident, dim3(1), dim3(RW), lds, st, d, a);
    return hipGetLastError();
}

}  // namespace elp
