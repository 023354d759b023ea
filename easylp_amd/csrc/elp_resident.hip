// elp_resident.hip -- the resident small-LP solver: the whole simplex loop of
// an LP that fits in one CU's LDS, run by ONE wave in ONE launch.
//
// Why: the multi-workgroup pipeline (elp_kernels.hip) pays 4-7 dependent
// launches per pivot, a ~25 us floor per pivot that no amount of bandwidth
// hides.  The models EasyLP's R front-end actually builds (README, test-DOP.R,
// the vignettes, the MIP tests' nodes; BASELINE configs[4]'s Klee-Minty cube)
// are a few dozen rows and columns: their whole state -- A, the bump inverse,
// every per-variable and per-row vector -- fits in the 160 KiB of LDS, and one
// wave of 64 lanes does a pivot's pricing, FTRAN, ratio test and update in a
// few hundred dependent LDS / DPP steps, no kernel boundary and no global
// round trip between them.
//
// Arithmetic: identical to oracle/elp_oracle.c (run_phase, run_dual,
// basis_change, refactor, btran) and therefore to the multi-workgroup kernels
// -- the same reduction shapes evaluated lane-serially: a wave_dot (64
// lane-strided fma chains + the pairwise tree, offsets 1, 2, ..., 32) becomes
// one lane's chains and the same tree (carry stack over the chains in lane
// order); zchunk, the price slot classes and the column chains are already
// per-output fma chains.  The orchestration is elp_api.hip run_loop's: loop-top
// checks (phase-1 sum, iteration cap, budget stop, refactor period), the
// recheck refactor after updated values reach optimality, the phase changes
// (primal phase 1 or dual phase -> real costs, refactor, primal phase 2).
//
// State: read from the device buffers the load left (elp_api.hip
// load_common / reload_bounds_warm), kept in LDS during the solve, written
// back at exit in the multi-workgroup path's own layout -- lists, bump inverse
// (and MinvT), AS, AR, the per-position / per-row / per-slot caches -- so
// elp_get_solution, elp_sensitivity and a MIP node's warm start read it as if
// the pipeline had run.
#include "elp_internal.h"

#include <math.h>

namespace elp {
namespace {

#define RDEV __device__ __forceinline__
constexpr int RW = 64;
constexpr double R_WMAX = 1e20;   // DEVEX_WMAX (oracle, elp_kernels.hip)
constexpr double R_RESET = 1e6;   // DEVEX_RESET
constexpr double R_INF = HUGE_VAL;

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
RDEV double r_rl(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
RDEV int r_rli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
RDEV double r_wmax(double v) {
    v = fmax(v, r_dpp<0xB1>(v));
    v = fmax(v, r_dpp<0x4E>(v));
    v = fmax(v, r_dpp<0x141>(v));
    v = fmax(v, r_dpp<0x140>(v));
    v = fmax(v, r_swz16(v));
    return fmax(r_rl(v, 0), r_rl(v, 32));
}
RDEV double r_wmin(double v) {
    v = fmin(v, r_dpp<0xB1>(v));
    v = fmin(v, r_dpp<0x4E>(v));
    v = fmin(v, r_dpp<0x141>(v));
    v = fmin(v, r_dpp<0x140>(v));
    v = fmin(v, r_swz16(v));
    return fmin(r_rl(v, 0), r_rl(v, 32));
}
RDEV int r_wmini(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_ds_swizzle(v, 0x401F));
    return min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 32));
}
// the lane holding the best record: largest key (or smallest with MIN), then
// the smallest id; -1 when no lane is valid (uniform)
template <bool MIN>
RDEV int r_argbest(bool valid, double key, int id) {
    const unsigned long long vm = __ballot(valid);
    if (vm == 0ull) return -1;
    const double b = MIN ? r_wmin(valid ? key : R_INF) : r_wmax(valid ? key : -R_INF);
    bool in = valid && key == b;
    if (__ballot(in) == 0ull) in = valid;  // (NaN keys only)
    const int im = r_wmini(in ? id : 0x7fffffff);
    return __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(in && id == im)) - 1);
}
RDEV int r_argminid(bool valid, int id) {
    if (__ballot(valid) == 0ull) return -1;
    const int im = r_wmini(valid ? id : 0x7fffffff);
    return __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(valid && id == im)) - 1);
}
#define RSYNC() __syncthreads()

// wave_dot's bits, one lane: chain l = fma over i = l, l + 64, ... < len of
// x(i) * y(i), then the pairwise tree over the chains in lane order, folded
// as a carry stack (a pair (l, l + off) exists only when l + off < min(len,
// 64); the chains past it are the +0.0 of an idle lane)
template <class F>
RDEV double lane_wave_dot(F xy, int len) {
    const int nl = len < RW ? len : RW;
    double st[7];
    int cnt = 0;
    for (int l = 0; l < nl; ++l) {
        double v = 0.0;
        for (int i = l; i < len; i += RW) v = xy(i, v);
#pragma unroll
        for (int L = 0; L < 7; ++L) {
            if (cnt & (1 << L)) {
                v = st[L] + v;
            } else {
                st[L] = v;
                break;
            }
        }
        ++cnt;
    }
    double t = 0.0;
    bool have = false;
#pragma unroll
    for (int L = 0; L < 7; ++L)
        if (cnt & (1 << L)) {
            t = have ? st[L] + t : st[L];
            have = true;
        }
    return t;
}

// ------------------------------------------------------------ LDS state
struct RS {
    int m, n, nv, lda, kc, ldm;
    double* A;      // m x n, column-major, ld lda (scaled values)
    double* Mi;     // bump inverse kc x kc, row-major, ld ldm
    double* W;      // refactor work: 2 * kc * kc
    double *lb, *ub, *cost, *xval;  // nv
    double *dw, *dprev;             // n + m
    double *b, *xr, *asgn, *y, *rho, *acol, *z, *alU, *aF, *yy, *rhoY;  // m
    double *xs, *alS, *aR, *v, *tv, *fS;  // kc
    double *dvec, *avec, *ct, *cb, *ca, *cr;  // n + m
    int *cover, *rpos, *Rl, *Yl, *ypos;  // m
    int *Sl, *perm;                      // kc
    int* spos;                           // n
    int *cj, *flips;                     // n + m
    int8_t *vst, *calive;                // nv, n + m
};
// carve dynamic LDS (base may be null: only the size is wanted)
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
        off = (off + 7) & ~(size_t)7;
    };
    auto bb = [&](int8_t*& p, size_t cnt) {
        p = (int8_t*)(base + off);
        off += cnt;
        off = (off + 7) & ~(size_t)7;
    };
    const size_t mm = m > 0 ? m : 1, nm = (size_t)n + m, kc = s.kc;
    dd(s.A, (size_t)s.lda * n);
    dd(s.Mi, (size_t)s.ldm * kc);
    dd(s.W, 2 * kc * kc);
    dd(s.lb, s.nv);
    dd(s.ub, s.nv);
    dd(s.cost, s.nv);
    dd(s.xval, s.nv);
    dd(s.dw, nm);
    dd(s.dprev, nm);
    dd(s.b, mm);
    dd(s.xr, mm);
    dd(s.asgn, mm);
    dd(s.y, mm);
    dd(s.rho, mm);
    dd(s.acol, mm);
    dd(s.z, mm);
    dd(s.alU, mm);
    dd(s.aF, mm);
    dd(s.yy, mm);
    dd(s.rhoY, mm);
    dd(s.xs, kc);
    dd(s.alS, kc);
    dd(s.aR, kc);
    dd(s.v, kc);
    dd(s.tv, kc);
    dd(s.fS, kc);
    dd(s.dvec, nm);
    dd(s.avec, nm);
    dd(s.ct, nm);
    dd(s.cb, nm);
    dd(s.ca, nm);
    dd(s.cr, nm);
    ii(s.cover, mm);
    ii(s.rpos, mm);
    ii(s.Rl, mm);
    ii(s.Yl, mm);
    ii(s.ypos, mm);
    ii(s.Sl, kc);
    ii(s.perm, kc);
    ii(s.spos, n);
    ii(s.cj, nm);
    ii(s.flips, nm);
    bb(s.vst, s.nv);
    bb(s.calive, nm);
    return off;
}

// the uniform scalars of the loop (every lane holds the same values)
struct RC {
    int phase;  // 1 primal phase 1, 2 primal phase 2, 3 dual phase 1 (h->phase)
    int k, ny;
    int64_t iter, iter_limit, iter_stop, phase1_iters, flips, degenerate, dual_iters;
    int since, period, ndegen, bland, degen_switch;
    int devex, ddevex, dv_valid, dv_lv;
    double dv_dq, dv_wq;
    double tol_primal, tol_dual, tol_pivot, tol_inf, tol_singular;
    double art_sum, unb_sig;
    int unb_var, status;
    double price_bytes, iter_bytes;
    int64_t refactors, gj, resets;
    double emax_max;
    int y_valid;
    int64_t trace_cap;
};

RDEV double r_usign(const RS& s, int var, int row) { return var >= s.n + s.m ? s.asgn[row] : 1.0; }
RDEV double r_colA(const RS& s, int i, int j) {
    return j < s.n ? s.A[i + (size_t)j * s.lda] : (i == j - s.n ? 1.0 : 0.0);
}
// zchunk_row: z_i = sum_p A[i, S_p] w_p, chunks of 32 positions
RDEV double r_zchunk(const RS& s, int i, const double* w, int k) {
    double tot = 0.0;
    for (int c0 = 0; c0 < k; c0 += ZCHUNK) {
        double acc = 0.0;
        const int c1 = c0 + ZCHUNK < k ? c0 + ZCHUNK : k;
        for (int p = c0; p < c1; ++p) acc = fma(s.A[i + (size_t)s.Sl[p] * s.lda], w[p], acc);
        tot = tot + acc;
    }
    return tot;
}
// row p of Minv . w (wave order over the k positions)
RDEV double r_minv_row_dot(const RS& s, int p, const double* w, int k) {
    const double* row = s.Mi + (size_t)p * s.ldm;
    return lane_wave_dot([&](int i, double acc) { return fma(row[i], w[i], acc); }, k);
}
// column c of Minv . w (row_times_minv / BTRAN: one wave per c over rows of Minv^T)
RDEV double r_minv_col_dot(const RS& s, int c, const double* w, int k) {
    const double* col = s.Mi + c;
    const int ld = s.ldm;
    return lane_wave_dot([&](int i, double acc) { return fma(col[(size_t)i * ld], w[i], acc); }, k);
}

// ------------------------------------------------------------ refactor
RDEV bool r_gauss_jordan(RS& s, RC& c) {
    const int k = c.k, lane = threadIdx.x;
    double* W = s.W;               // k x k, row-major (ld k)
    double* q = s.W + (size_t)k * k;  // row p's quotients (k), then the factors (k)
    double* f = q + k;
    for (int e = lane; e < k * k; e += RW) {
        const int a = e / k, cc = e - a * k;
        W[e] = s.A[s.Rl[a] + (size_t)s.Sl[cc] * s.lda];
    }
    for (int r = lane; r < k; r += RW) s.calive[r] = 0;  // (used rows)
    RSYNC();
    for (int col = 0; col < k; ++col) {
        double bv = -1.0;
        int br = 0x7fffffff;
        for (int r = lane; r < k; r += RW) {
            if (s.calive[r]) continue;
            const double a = fabs(W[(size_t)r * k + col]);
            if (a > bv) {  // (ascending r per lane: the lowest row on ties)
                bv = a;
                br = r;
            }
        }
        const int wl = r_argbest<false>(br != 0x7fffffff, bv, br);
        const int p = wl >= 0 ? r_rli(br, wl) : 0;
        const double piv = W[(size_t)p * k + col];
        if (!(fabs(piv) > c.tol_singular)) return false;
        for (int j = lane; j < k; j += RW) q[j] = W[(size_t)p * k + j] / piv;
        for (int r = lane; r < k; r += RW) f[r] = W[(size_t)r * k + col];
        if (lane == 0) {
            s.perm[col] = p;
            s.calive[p] = 1;
        }
        RSYNC();
        for (int e = lane; e < k * k; e += RW) {
            const int r = e / k, j = e - r * k;
            double& x = W[e];
            if (r == p) {
                x = j == col ? 1.0 / piv : q[j];
            } else if (j == col) {
                x = -(f[r] / piv);
            } else {
                const double fr = f[r], qj = q[j];
                if (fr != 0.0 && qj != 0.0) x = fma(-fr, qj, x);
            }
        }
        RSYNC();
    }
    for (int e = lane; e < k * k; e += RW) {
        const int a = e / k, cc = e - a * k;
        s.Mi[(size_t)a * s.ldm + s.perm[cc]] = W[(size_t)s.perm[a] * k + cc];
    }
    RSYNC();
    return true;
}
// one Newton-Schulz correction; false: the residual is too large
RDEV bool r_newton_schulz(RS& s, RC& c) {
    const int k = c.k, lane = threadIdx.x;
    double* E = s.W;
    double* N = s.W + (size_t)k * k;
    double emax = 0.0;
    for (int e = lane; e < k * k; e += RW) {
        const int i = e / k, j = e - i * k;
        const int ri = s.Rl[i];
        double acc = 0.0;  // (M Minv)_ij, seq over l
        for (int l = 0; l < k; ++l) acc = fma(s.A[ri + (size_t)s.Sl[l] * s.lda], s.Mi[(size_t)l * s.ldm + j], acc);
        const double ev = (i == j ? 1.0 : 0.0) - acc;
        E[e] = ev;
        emax = fmax(emax, fabs(ev));
    }
    emax = r_wmax(emax);
    if (emax > c.emax_max) c.emax_max = emax;
    if (!(emax <= NS_TOL)) return false;
    RSYNC();
    for (int e = lane; e < k * k; e += RW) {
        const int i = e / k, j = e - i * k;
        double acc = s.Mi[(size_t)i * s.ldm + j];
        for (int l = 0; l < k; ++l) acc = fma(s.Mi[(size_t)i * s.ldm + l], E[(size_t)l * k + j], acc);
        N[e] = acc;
    }
    RSYNC();
    for (int e = lane; e < k * k; e += RW) {
        const int i = e / k, j = e - i * k;
        s.Mi[(size_t)i * s.ldm + j] = N[e];
    }
    RSYNC();
    return true;
}
// oracle refactor(): the inverse corrected or rebuilt, then x_B from b
RDEV bool r_refactor(RS& s, RC& c, int refactor_mode) {
    const int k = c.k, m = s.m, n = s.n, lane = threadIdx.x;
    if (k > 0) {
        if (refactor_mode != 0 || !r_newton_schulz(s, c)) {
            c.gj++;
            if (!r_gauss_jordan(s, c)) return false;
        }
    }
    for (int i = lane; i < m; i += RW) {
        double acc = 0.0;  // nonzero nonbasic structurals, ascending j
        for (int j = 0; j < n; ++j) {
            const double xj = s.xval[j];
            if (s.vst[j] != VS_BASIC && xj != 0.0) acc = fma(s.A[i + (size_t)j * s.lda], xj, acc);
        }
        double r = s.b[i] - acc;
        if (s.vst[n + i] != VS_BASIC) r = r - s.xval[n + i];
        s.acol[i] = r;
    }
    RSYNC();
    for (int p = lane; p < k; p += RW) s.aR[p] = s.acol[s.Rl[p]];
    RSYNC();
    for (int p = lane; p < k; p += RW) s.xs[p] = r_minv_row_dot(s, p, s.aR, k);
    RSYNC();
    for (int i = lane; i < m; i += RW) {
        const int u = s.cover[i];
        if (u >= 0) s.xr[i] = r_usign(s, u, i) * (s.acol[i] - r_zchunk(s, i, s.xs, k));
    }
    c.refactors++;
    RSYNC();
    return true;
}

// y = B^-T c_B (oracle btran): covered rows sigma_u c_u, R rows Minv^T t
RDEV void r_btran(RS& s, RC& c, int phase) {
    const int k = c.k, m = s.m, lane = threadIdx.x;
    for (int i = lane; i < m; i += RW) {
        const int u = s.cover[i];
        s.y[i] = u >= 0 ? r_usign(s, u, i) * s.cost[u] : 0.0;
    }
    RSYNC();
    for (int p = lane; p < k; p += RW) {
        const int sp = s.Sl[p];
        if (phase == 1) {
            const double* col = s.A + (size_t)sp * s.lda;
            const double* y = s.y;
            s.tv[p] = s.cost[sp] - lane_wave_dot([&](int i, double acc) { return fma(col[i], y[i], acc); }, m);
        } else {
            s.tv[p] = s.cost[sp];
        }
    }
    RSYNC();
    for (int p = lane; p < k; p += RW) s.fS[p] = r_minv_col_dot(s, p, s.tv, k);  // (fS: scratch)
    RSYNC();
    for (int p = lane; p < k; p += RW) s.y[s.Rl[p]] = s.fS[p];
    RSYNC();
}

// phase-1 infeasibility sum (oracle art_sum: wave order)
RDEV double r_art_sum(const RS& s) {
    const int lane = threadIdx.x;
    double acc = 0.0;
    for (int i = lane; i < s.m; i += RW)
        if (s.cover[i] >= s.n + s.m) acc = acc + s.xr[i];
    acc = acc + r_dpp<0xB1>(acc);  // (the GPU wave tree: pairs, then pairs of pairs, ...)
    acc = acc + r_dpp<0x4E>(acc);
    acc = acc + r_dpp<0x141>(acc);
    acc = acc + r_dpp<0x140>(acc);
    acc = acc + r_swz16(acc);
    return r_rl(acc, 0) + r_rl(acc, 32);
}

// FTRAN of column q: alpha_S (bump), alpha_U on covered rows (oracle run_phase)
RDEV void r_ftran(RS& s, const RC& c, int q, const double* aq /* null: column q of A or the unit */) {
    const int k = c.k, m = s.m, n = s.n, lane = threadIdx.x;
    for (int i = lane; i < m; i += RW) s.acol[i] = aq ? aq[i] : r_colA(s, i, q);
    (void)n;
    RSYNC();
    for (int p = lane; p < k; p += RW) s.aR[p] = s.acol[s.Rl[p]];
    RSYNC();
    for (int p = lane; p < k; p += RW) s.alS[p] = r_minv_row_dot(s, p, s.aR, k);
    RSYNC();
    for (int i = lane; i < m; i += RW) {
        const int u = s.cover[i];
        if (u < 0) continue;
        const double z = r_zchunk(s, i, s.alS, k);
        s.z[i] = z;
        s.alU[i] = r_usign(s, u, i) * (s.acol[i] - z);
    }
    RSYNC();
}
// v = A[i, S] Minv (oracle row_times_minv)
RDEV void r_row_times_minv(RS& s, const RC& c, int i) {
    const int k = c.k, lane = threadIdx.x;
    for (int p = lane; p < k; p += RW) s.aR[p] = s.A[i + (size_t)s.Sl[p] * s.lda];
    RSYNC();
    for (int cc = lane; cc < k; cc += RW) s.v[cc] = r_minv_col_dot(s, cc, s.aR, k);
    RSYNC();
}

RDEV void r_y_append(RS& s, RC& c, int i) {
    if (threadIdx.x == 0) {
        s.Yl[c.ny] = i;
        s.ypos[i] = c.ny;
    }
    c.ny++;
}
RDEV void r_y_remove(RS& s, RC& c, int i) {
    if (threadIdx.x == 0) {
        const int p = s.ypos[i], last = c.ny - 1;
        if (p != last) {
            s.Yl[p] = s.Yl[last];
            s.ypos[s.Yl[p]] = p;
        }
        s.ypos[i] = -1;
    }
    c.ny--;
}

// oracle basis_change (cases A-E, the zero rule, phase 2: the dual update)
RDEV bool r_basis_change(RS& s, RC& c, int phase, int q, int lv, int lrow, int lpos, double dq, double xq) {
    const int m = s.m, n = s.n, k = c.k, lane = threadIdx.x;
    const size_t ld = s.ldm;
    const bool leave_art = lv >= n + m;
    double* Mi = s.Mi;
    if (q < n) {
        if (lpos >= 0) {  // case A: structural replaces structural at position p
            const int p = lpos;
            const double piv = s.alS[p];
            for (int j = lane; j < k; j += RW) s.v[j] = Mi[(size_t)p * ld + j] / piv;
            RSYNC();
            if (phase == 2)
                for (int j = lane; j < k; j += RW) s.y[s.Rl[j]] = fma(dq, s.v[j], s.y[s.Rl[j]]);
            for (int e = lane; e < k * k; e += RW) {
                const int i = e / k, j = e - i * k;
                if (i == p) continue;
                const double wi = s.alS[i], vj = s.v[j];
                if (wi != 0.0 && vj != 0.0) Mi[(size_t)i * ld + j] = fma(-wi, vj, Mi[(size_t)i * ld + j]);
            }
            RSYNC();
            for (int j = lane; j < k; j += RW) Mi[(size_t)p * ld + j] = s.v[j];
            if (lane == 0) {
                s.spos[lv] = -1;
                s.Sl[p] = q;
                s.spos[q] = p;
                s.xs[p] = xq;
            }
        } else {  // case B: structural enters, the unit variable of row i leaves
            const int i = lrow;
            const double delta = s.acol[i] - s.z[i];
            r_row_times_minv(s, c, i);
            for (int cc = lane; cc < k; cc += RW) s.v[cc] = s.v[cc] / delta;
            RSYNC();
            if (phase == 2) {
                for (int cc = lane; cc < k; cc += RW) s.y[s.Rl[cc]] = fma(-dq, s.v[cc], s.y[s.Rl[cc]]);
                if (lane == 0) s.y[i] = dq / delta;
            }
            for (int e = lane; e < k * k; e += RW) {
                const int a = e / k, cc = e - a * k;
                const double wa = s.alS[a], vc = s.v[cc];
                if (wa != 0.0 && vc != 0.0) Mi[(size_t)a * ld + cc] = fma(wa, vc, Mi[(size_t)a * ld + cc]);
            }
            RSYNC();
            for (int a = lane; a < k; a += RW) Mi[(size_t)a * ld + k] = -(s.alS[a] / delta);
            for (int cc = lane; cc < k; cc += RW) Mi[(size_t)k * ld + cc] = -s.v[cc];
            if (lane == 0) {
                Mi[(size_t)k * ld + k] = 1.0 / delta;
                s.Rl[k] = i;
                s.rpos[i] = k;
                s.Sl[k] = q;
                s.spos[q] = k;
                s.xs[k] = xq;
                s.cover[i] = -1;
            }
            c.k = k + 1;
            if (!leave_art) r_y_append(s, c, i);
        }
    } else {
        const int i0 = q - n;
        const int a = s.rpos[i0];
        if (a < 0) {  // case E: the slack replaces the artificial of its own row
            if (lrow != i0) return false;
            if (lane == 0) {
                s.cover[i0] = q;
                s.xr[i0] = xq;
            }
        } else if (lpos >= 0) {  // case C: slack of row i0 (in R) enters, structural at b leaves
            const int b = lpos, last = k - 1;
            const double piv = Mi[(size_t)b * ld + a];
            for (int cc = lane; cc < k; cc += RW) s.v[cc] = Mi[(size_t)b * ld + cc] / piv;
            RSYNC();
            if (phase == 2)
                for (int cc = lane; cc < k; cc += RW)
                    if (cc != a) s.y[s.Rl[cc]] = fma(dq, s.v[cc], s.y[s.Rl[cc]]);
            for (int e = lane; e < k * k; e += RW) {
                const int r = e / k, cc = e - r * k;
                if (r == b || cc == a) continue;
                const double f = Mi[(size_t)r * ld + a], vc = s.v[cc];
                if (f != 0.0 && vc != 0.0) Mi[(size_t)r * ld + cc] = fma(-f, vc, Mi[(size_t)r * ld + cc]);
            }
            RSYNC();
            if (phase == 2 && lane == 0) s.y[i0] = 0.0;
            if (b != last) {
                for (int cc = lane; cc < k; cc += RW) Mi[(size_t)b * ld + cc] = Mi[(size_t)last * ld + cc];
                if (lane == 0) {
                    s.Sl[b] = s.Sl[last];
                    s.spos[s.Sl[b]] = b;
                    s.xs[b] = s.xs[last];
                }
            }
            RSYNC();
            if (a != last) {
                for (int r = lane; r < k; r += RW) Mi[(size_t)r * ld + a] = Mi[(size_t)r * ld + last];
                if (lane == 0) {
                    s.Rl[a] = s.Rl[last];
                    s.rpos[s.Rl[a]] = a;
                }
            }
            if (lane == 0) {
                s.spos[lv] = -1;
                s.rpos[i0] = -1;
                s.cover[i0] = q;
                s.xr[i0] = xq;
            }
            c.k = k - 1;
        } else {  // case D: slack of row i0 (in R) enters, unit variable of row i1 leaves
            const int i1 = lrow;
            r_row_times_minv(s, c, i1);
            const double piv = s.v[a];
            if (phase == 2) {
                const double w = dq / piv;
                for (int cc = lane; cc < k; cc += RW)
                    if (cc != a) s.y[s.Rl[cc]] = fma(w, s.v[cc], s.y[s.Rl[cc]]);
                if (lane == 0) {
                    s.y[i0] = 0.0;
                    s.y[i1] = -w;
                }
            }
            for (int r = lane; r < k; r += RW) s.tv[r] = Mi[(size_t)r * ld + a] / piv;
            RSYNC();
            for (int e = lane; e < k * k; e += RW) {
                const int r = e / k, cc = e - r * k;
                if (cc == a) continue;
                const double f = s.tv[r], vc = s.v[cc];
                if (f != 0.0 && vc != 0.0) Mi[(size_t)r * ld + cc] = fma(-f, vc, Mi[(size_t)r * ld + cc]);
            }
            RSYNC();
            for (int r = lane; r < k; r += RW) Mi[(size_t)r * ld + a] = s.tv[r];
            if (lane == 0) {
                s.Rl[a] = i1;
                s.rpos[i1] = a;
                s.rpos[i0] = -1;
                s.cover[i1] = -1;
                s.cover[i0] = q;
                s.xr[i0] = xq;
            }
        }
        RSYNC();
        r_y_remove(s, c, i0);
        RSYNC();
        if (a >= 0 && lpos < 0 && !leave_art) r_y_append(s, c, lrow);
    }
    RSYNC();
    return true;
}

// pricing of structural j: d_j = c_j - y'a_j (price slot classes over the Y
// rows, or CSC's column chain over the nonzero rows)
RDEV double r_price_col(const RS& s, const RC& c, int j, bool mode1) {
    const double* col = s.A + (size_t)j * s.lda;
    if (mode1) {
        double acc = 0.0;
        for (int i = 0; i < s.m; ++i) {
            const double a = col[i];
            if (a != 0.0) acc = fma(a, s.y[i], acc);
        }
        return s.cost[j] - acc;
    }
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < PRICE_SPLIT; ++w) {
        double pw = 0.0;
        for (int p = w; p < c.ny; p += PRICE_SPLIT) pw = fma(col[s.Yl[p]], s.yy[p], pw);
        tot = tot + pw;
    }
    return s.cost[j] - tot;
}

RDEV void r_trace(const Dev& d, const RC& c, int a, int b) {
    if (threadIdx.x == 0 && c.iter - 1 < c.trace_cap) {
        d.trace[2 * (c.iter - 1)] = a;
        d.trace[2 * (c.iter - 1) + 1] = b;
    }
}
RDEV void r_dw_reset(RS& s) {
    for (int j = threadIdx.x; j < s.n + s.m; j += RW) s.dw[j] = 1.0;
}

enum { R_CONT = 0, R_EXIT = 1, R_RECHECK = 2, R_TO_P2 = 3 };

// one primal iteration (oracle run_phase body after the loop top)
RDEV int r_primal(const Dev& d, RS& s, RC& c, bool mode1, int refactor_mode) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    const int ph = c.phase;
    if (ph == 1 || !c.y_valid) {
        c.y_valid = 1;
        r_btran(s, c, ph);
    }
    if (!mode1) {
        for (int p = lane; p < c.ny; p += RW) s.yy[p] = s.y[s.Yl[p]];
        RSYNC();
    }
    const double dtol = c.tol_dual;
    const bool devex = c.devex != 0;
    int bq = 0x7fffffff;
    double bscore = 0.0, bd = 0.0, bw = 1.0;
    for (int j = lane; j < n + m; j += RW) {
        const int8_t vs = s.vst[j];
        if (vs == VS_BASIC || s.lb[j] == s.ub[j]) continue;
        const double dj = j < n ? r_price_col(s, c, j, mode1) : s.cost[j] - s.y[j - n];
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
    c.price_bytes += mode1 ? 12.0 * (double)d.nnz + 17.0 * n : 8.0 * ((double)c.ny * n + n + c.ny);
    const bool have = bq != 0x7fffffff;
    const int wl = c.bland ? r_argminid(have, bq) : r_argbest<false>(have, bscore, bq);
    RSYNC();  // (dw / dprev written; yy read)
    if (wl < 0) {
        if (ph == 2 && c.since > 0) {  // optimal under updated duals: confirm
            if (!r_refactor(s, c, refactor_mode)) {
                c.status = ST_NUMFAIL;
                return R_EXIT;
            }
            c.since = 0;
            c.y_valid = 0;
            return R_RECHECK;
        }
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
    const int q = r_rli(bq, wl);
    const double dq = r_rl(bd, wl), qw = r_rl(bw, wl);
    const double sig = dq < 0.0 ? 1.0 : -1.0;
    const int k = c.k;
    r_ftran(s, c, q, nullptr);
    // Harris two-pass ratio test (textbook under Bland)
    const double ptol = c.tol_primal, pivtol = c.tol_pivot;
    double tmax = R_INF;
    for (int e = lane; e < m + k; e += RW) {
        int var;
        double g, x;
        if (e < m) {
            var = s.cover[e];
            if (var < 0) continue;
            g = sig * s.alU[e];
            x = s.xr[e];
        } else {
            var = s.Sl[e - m];
            g = sig * s.alS[e - m];
            x = s.xs[e - m];
        }
        const double l = s.lb[var], u = s.ub[var];
        double r;
        if (g > pivtol && l > -R_INF) r = c.bland ? (x - l) / g : (x - l + ptol) / g;
        else if (g < -pivtol && u < R_INF) r = c.bland ? (u - x) / (-g) : (u - x + ptol) / (-g);
        else continue;
        if (r < tmax) tmax = r;
    }
    tmax = r_wmin(tmax);
    int lv = -1, le = 0;
    double lg = 0.0, lr = 0.0;
    for (int e = lane; e < m + k; e += RW) {
        int var;
        double g, x;
        if (e < m) {
            var = s.cover[e];
            if (var < 0) continue;
            g = sig * s.alU[e];
            x = s.xr[e];
        } else {
            var = s.Sl[e - m];
            g = sig * s.alS[e - m];
            x = s.xs[e - m];
        }
        const double l = s.lb[var], u = s.ub[var];
        double r;
        if (g > pivtol && l > -R_INF) r = (x - l) / g;
        else if (g < -pivtol && u < R_INF) r = (u - x) / (-g);
        else continue;
        if (!(r <= tmax)) continue;
        bool take;
        if (lv < 0) take = true;
        else if (c.bland) take = (r < lr) || (r == lr && var < lv);
        else take = (fabs(g) > fabs(lg)) || (fabs(g) == fabs(lg) && var < lv);
        if (take) {
            lv = var;
            le = e;
            lg = g;
            lr = r;
        }
    }
    const bool lhave = lv >= 0;
    const int ll = c.bland ? r_argbest<true>(lhave, lr, lv) : r_argbest<false>(lhave, fabs(lg), lv);
    if (ll >= 0) {
        lv = r_rli(lv, ll);
        le = r_rli(le, ll);
        lg = r_rl(lg, ll);
        lr = r_rl(lr, ll);
    } else {
        lv = -1;
    }
    const double theta = lv >= 0 ? (lr > 0.0 ? lr : 0.0) : R_INF;
    const double flip = (s.lb[q] > -R_INF && s.ub[q] < R_INF) ? s.ub[q] - s.lb[q] : R_INF;
    c.iter++;
    if (ph == 1) c.phase1_iters++;
    c.iter_bytes += 8.0 * (6.0 * k * k + (double)m * k + 2.0 * n + 2.0 * m);
    if (flip < R_INF && flip <= theta) {  // bound flip
        for (int i = lane; i < m; i += RW)
            if (s.cover[i] >= 0) s.xr[i] = fma(-flip, sig * s.alU[i], s.xr[i]);
        for (int p = lane; p < k; p += RW) s.xs[p] = fma(-flip, sig * s.alS[p], s.xs[p]);
        if (lane == 0) {
            if (s.vst[q] == VS_LOWER) {
                s.vst[q] = VS_UPPER;
                s.xval[q] = s.ub[q];
            } else {
                s.vst[q] = VS_LOWER;
                s.xval[q] = s.lb[q];
            }
        }
        c.flips++;
        r_trace(d, c, q, -1);
        c.dv_valid = 0;
        c.ndegen = 0;
        c.bland = 0;
        RSYNC();
        return R_CONT;
    }
    if (theta == R_INF) {
        r_trace(d, c, q, -2);
        c.unb_var = q;
        c.unb_sig = sig;
        c.status = ST_UNBOUNDED;
        return R_EXIT;
    }
    r_trace(d, c, q, lv);
    if (devex && qw > R_RESET) {
        r_dw_reset(s);
        c.dv_valid = 0;
        c.resets++;
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
        c.degenerate++;
        if (++c.ndegen >= c.degen_switch) c.bland = 1;
    } else {
        c.ndegen = 0;
        c.bland = 0;
    }
    for (int i = lane; i < m; i += RW)
        if (s.cover[i] >= 0) s.xr[i] = fma(-theta, sig * s.alU[i], s.xr[i]);
    for (int p = lane; p < k; p += RW) s.xs[p] = fma(-theta, sig * s.alS[p], s.xs[p]);
    const double xq = s.xval[q] + sig * theta;
    const bool at_lower = lg > 0.0;
    RSYNC();
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
    RSYNC();
    const int lrow = le < m ? le : -1, lpos = le < m ? -1 : le - m;
    if (!r_basis_change(s, c, ph, q, lv, lrow, lpos, dq, xq)) {
        c.status = ST_NUMFAIL;
        return R_EXIT;
    }
    c.since++;
    return R_CONT;
}

// one dual iteration (oracle run_dual body after the loop top)
RDEV int r_dual(const Dev& d, RS& s, RC& c, bool mode1, int refactor_mode) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    const double ptol = c.tol_primal, dtol = c.tol_dual, pivtol = c.tol_pivot;
    const bool devex = c.ddevex != 0;
    int k = c.k;
    // ---- CHUZR
    int rv = -1, re = 0, rs = 0;
    double rscore = 0.0, rx = 0.0, rbeta = 0.0;
    for (int e = lane; e < m + k; e += RW) {
        int var;
        double x;
        if (e < m) {
            var = s.cover[e];
            if (var < 0) continue;
            x = s.xr[e];
        } else {
            var = s.Sl[e - m];
            x = s.xs[e - m];
        }
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
            re = e;
            rscore = score;
            rx = x;
            rbeta = beta;
            rs = sd;
        }
    }
    const bool rh = rv >= 0;
    const int wl = c.bland ? r_argminid(rh, rv) : r_argbest<false>(rh, rscore, rv);
    if (wl < 0) {
        if (c.since > 0) {  // updated values: confirm on a fresh x_B
            if (!r_refactor(s, c, refactor_mode)) {
                c.status = ST_NUMFAIL;
                return R_EXIT;
            }
            c.since = 0;
            r_btran(s, c, 2);
            return R_RECHECK;
        }
        return R_TO_P2;
    }
    rv = r_rli(rv, wl);
    re = r_rli(re, wl);
    rs = r_rli(rs, wl);
    rx = r_rl(rx, wl);
    rbeta = r_rl(rbeta, wl);
    // ---- rho_r
    int xrow = -1;
    double xsig = 0.0;
    if (re >= m) {
        for (int cc = lane; cc < k; cc += RW) s.v[cc] = s.Mi[(size_t)(re - m) * s.ldm + cc];
    } else {
        xrow = re;
        xsig = r_usign(s, s.cover[re], re);
        r_row_times_minv(s, c, re);
        for (int cc = lane; cc < k; cc += RW) s.v[cc] = -(xsig * s.v[cc]);
    }
    for (int i = lane; i < m; i += RW) s.rho[i] = 0.0;
    RSYNC();
    for (int cc = lane; cc < k; cc += RW) s.rho[s.Rl[cc]] = s.v[cc];
    if (xrow >= 0 && lane == 0) s.rho[xrow] = xsig;
    RSYNC();
    // ---- one sweep: d_j (y) and alpha_j (rho)
    if (!mode1) {
        for (int p = lane; p < c.ny; p += RW) {
            s.yy[p] = s.y[s.Yl[p]];
            s.rhoY[p] = s.rho[s.Yl[p]];
        }
        RSYNC();
    }
    for (int j = lane; j < n; j += RW) {
        const double* col = s.A + (size_t)j * s.lda;
        if (mode1) {
            double ad = 0.0, aa = 0.0;
            for (int i = 0; i < m; ++i) {
                const double a = col[i];
                if (a == 0.0) continue;
                ad = fma(a, s.y[i], ad);
                aa = fma(a, s.rho[i], aa);
            }
            s.dvec[j] = s.cost[j] - ad;
            s.avec[j] = aa;
        } else {
            double td = 0.0, ta = 0.0;
#pragma unroll
            for (int w = 0; w < PRICE_SPLIT; ++w) {
                double pd = 0.0, pa = 0.0;
                for (int p = w; p < c.ny; p += PRICE_SPLIT) {
                    const double a = col[s.Yl[p]];
                    pd = fma(a, s.yy[p], pd);
                    pa = fma(a, s.rhoY[p], pa);
                }
                td = td + pd;
                ta = ta + pa;
            }
            s.dvec[j] = s.cost[j] - td;
            s.avec[j] = xrow >= 0 ? fma(xsig, col[xrow], ta) : ta;
        }
    }
    for (int i = lane; i < m; i += RW) {
        s.dvec[n + i] = s.cost[n + i] - s.y[i];
        s.avec[n + i] = s.rho[i];
    }
    c.price_bytes += mode1 ? 12.0 * (double)d.nnz + 17.0 * n : 8.0 * ((double)c.ny * n + n + c.ny);
    RSYNC();
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
    RSYNC();
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
        // the bunch: alive and exact ratio <= thmax; its boxed members' sum in ascending order
        int nq = 0;
        bool allbox = true;
        double sum = 0.0;
        for (int c0 = 0; c0 < nc; c0 += RW) {
            const int cc = c0 + lane;
            const bool in = cc < nc && s.calive[cc] && s.ct[cc] <= thmax;
            unsigned long long bm = __ballot(in);
            nq += __popcll(bm);
            if (__ballot(in && s.cr[cc < nc ? cc : 0] == R_INF)) allbox = false;
            while (bm) {  // (uniform: every lane walks the bunch in ascending order)
                const int t = __ffsll((long long)bm) - 1;
                bm &= bm - 1ull;
                const int ct = c0 + t;
                if (s.cr[ct] != R_INF) sum = fma(s.ca[ct], s.cr[ct], sum);
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
            RSYNC();
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
        bc = r_rli(bc, w2);
        q = s.cj[bc];
        qt = s.ct[bc];
        qa = s.avec[q];
        break;
    }
    c.iter++;
    c.phase1_iters++;
    c.dual_iters++;
    c.iter_bytes += 8.0 * (6.0 * k * k + (double)m * k + 2.0 * n + 2.0 * m);
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
        RSYNC();
        for (int i = lane; i < m; i += RW) {
            double acc = 0.0;
            for (int f = 0; f < nflip; ++f) acc = fma(r_colA(s, i, s.flips[f]), dx[f], acc);
            s.aF[i] = acc;
        }
        RSYNC();
        for (int f = lane; f < nflip; f += RW) {
            const int j = s.flips[f];
            const int8_t nv = s.vst[j] == VS_LOWER ? VS_UPPER : VS_LOWER;
            s.vst[j] = nv;
            s.xval[j] = nv == VS_LOWER ? s.lb[j] : s.ub[j];
        }
        for (int p = lane; p < k; p += RW) s.aR[p] = s.aF[s.Rl[p]];
        RSYNC();
        for (int p = lane; p < k; p += RW) s.fS[p] = r_minv_row_dot(s, p, s.aR, k);
        RSYNC();
        for (int i = lane; i < m; i += RW) {
            const int u = s.cover[i];
            if (u >= 0) s.xr[i] = s.xr[i] - r_usign(s, u, i) * (s.aF[i] - r_zchunk(s, i, s.fS, k));
        }
        for (int p = lane; p < k; p += RW) s.xs[p] = s.xs[p] - s.fS[p];
        c.flips += nflip;
        RSYNC();
        rx = re < m ? s.xr[re] : s.xs[re - m];
    }
    const double dq = s.dvec[q];
    const int8_t vq = s.vst[q];
    const double sig = (vq == VS_LOWER || (vq == VS_FREE && rs * qa < 0.0)) ? 1.0 : -1.0;
    r_ftran(s, c, q, nullptr);
    const double arq = re < m ? s.alU[re] : s.alS[re - m];
    const double step = fabs((rx - rbeta) / arq);
    r_trace(d, c, q, rv);
    if (devex) {  // dual Devex weights of the basic entries (old basis)
        const double wr = rv < n + m ? s.dw[rv] : 1.0;
        for (int e = lane; e < m + k; e += RW) {
            if (e == re) continue;
            int var;
            double ae;
            if (e < m) {
                var = s.cover[e];
                if (var < 0) continue;
                ae = s.alU[e];
            } else {
                var = s.Sl[e - m];
                ae = s.alS[e - m];
            }
            const double r = ae / arq;
            double wn = (r * r) * wr;
            if (wn > R_WMAX) wn = R_WMAX;
            if (var < n + m && wn > s.dw[var]) s.dw[var] = wn;
        }
        RSYNC();
        double wq = wr / (arq * arq);
        if (wq < 1.0) wq = 1.0;
        if (wq > R_WMAX) wq = R_WMAX;
        if (wq > R_RESET) {
            r_dw_reset(s);
            c.resets++;
        } else if (lane == 0) {
            s.dw[q] = wq;
        }
    }
    if (!(qt > 0.0)) {
        c.degenerate++;
        if (++c.ndegen >= c.degen_switch) c.bland = 1;
    } else {
        c.ndegen = 0;
        c.bland = 0;
    }
    for (int i = lane; i < m; i += RW)
        if (s.cover[i] >= 0) s.xr[i] = fma(-step, sig * s.alU[i], s.xr[i]);
    for (int p = lane; p < k; p += RW) s.xs[p] = fma(-step, sig * s.alS[p], s.xs[p]);
    const double xq = s.xval[q] + sig * step;
    RSYNC();
    if (lane == 0) {
        const double l = s.lb[rv], u = s.ub[rv];
        s.vst[rv] = l == u ? VS_FIXED : rs > 0 ? VS_LOWER : VS_UPPER;
        s.xval[rv] = rbeta;
        s.vst[q] = VS_BASIC;
    }
    RSYNC();
    if (!r_basis_change(s, c, 2, q, rv, re < m ? re : -1, re < m ? -1 : re - m, dq, xq)) {
        c.status = ST_NUMFAIL;
        return R_EXIT;
    }
    c.since++;
    return R_CONT;
}

// the real costs and the primal phase 2 (launch_phase2 + do_refactor + BTRAN)
RDEV bool r_to_phase2(const Dev& d, RS& s, RC& c, int price_rule, int refactor_mode) {
    const int m = s.m, n = s.n, lane = threadIdx.x;
    for (int j = lane; j < n; j += RW) s.cost[j] = d.maximize ? -d.obj[j] : d.obj[j];
    for (int i = lane; i < m; i += RW) {
        const int av = n + m + i;
        s.cost[n + i] = 0.0;
        s.cost[av] = 0.0;
        s.lb[av] = 0.0;
        s.ub[av] = 0.0;
    }
    r_dw_reset(s);
    RSYNC();
    c.dv_valid = 0;
    if (!r_refactor(s, c, refactor_mode)) return false;
    c.phase = 2;
    c.since = 0;
    c.ndegen = 0;
    c.bland = 0;
    c.devex = price_rule == 1;
    c.y_valid = 0;
    return true;
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
    c.phase1_iters = g->phase1_iters;
    c.flips = g->flips;
    c.degenerate = g->degenerate;
    c.dual_iters = g->dual_iters;
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
    c.unb_sig = g->unb_sig;
    c.unb_var = g->unb_var;
    c.status = ST_RUN;
    c.price_bytes = g->price_bytes;
    c.iter_bytes = g->iter_bytes;
    c.refactors = c.gj = c.resets = 0;
    c.emax_max = 0.0;
    c.trace_cap = d.trace ? g->trace_cap : 0;
    c.y_valid = 1;  // (the load's BTRAN, or the updated duals of the last exit)
    const int k0 = c.k, ny0 = c.ny;
    // ---- state into LDS
    if (mode1) {
        for (int e = lane; e < s.lda * n; e += RW) s.A[e] = 0.0;
        RSYNC();
        for (int j = 0; j < n; ++j)
            for (int64_t t = d.cptr[j] + lane; t < d.cptr[j + 1]; t += RW) s.A[d.rind[t] + (size_t)j * s.lda] = d.cval[t];
    } else {
        for (int j = 0; j < n; ++j)
            for (int i = lane; i < m; i += RW) {
                const double v = d.A[(size_t)j * m + i];
                s.A[i + (size_t)j * s.lda] = d.srow ? ldexp(v, d.srow[i] + d.scol[j]) : v;
            }
    }
    for (int j = lane; j < nv; j += RW) {
        s.lb[j] = d.lb[j];
        s.ub[j] = d.ub[j];
        s.cost[j] = d.cost[j];
        s.xval[j] = d.xval[j];
        s.vst[j] = d.vstat[j];
    }
    for (int j = lane; j < n + m; j += RW) {
        s.dw[j] = d.dw[j];
        s.dprev[j] = d.dprev[j];
    }
    for (int j = lane; j < n; j += RW) s.spos[j] = -1;
    for (int i = lane; i < m; i += RW) {
        s.b[i] = d.b[i];
        s.xr[i] = d.xr[i];
        s.asgn[i] = d.asgn[i];
        s.y[i] = d.y[i];
        s.cover[i] = d.cover[i];
        s.rpos[i] = d.rpos[i];
        s.ypos[i] = d.ypos[i];
    }
    for (int p = lane; p < ny0; p += RW) s.Yl[p] = d.Yl[p];
    for (int p = lane; p < k0; p += RW) {
        s.Rl[p] = d.Rl[p];
        s.Sl[p] = d.Sl[p];
        s.xs[p] = d.xs[p];
    }
    for (int e = lane; e < k0 * k0; e += RW) {
        const int i = e / k0, j = e - i * k0;
        s.Mi[(size_t)i * s.ldm + j] = d.Minv[(size_t)i * d.ldm + j];
    }
    RSYNC();
    for (int p = lane; p < k0; p += RW) s.spos[s.Sl[p]] = p;
    if (c.dv_valid == 2) {  // (the pipeline's deferred framework restart)
        r_dw_reset(s);
        c.dv_valid = 0;
    }
    RSYNC();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int recheck = 0;
    for (;;) {
        if (!recheck) {
            if (c.phase == 1) {
                c.art_sum = r_art_sum(s);
                if (c.art_sum <= c.tol_inf) {
                    if (!r_to_phase2(d, s, c, a.price_rule, a.refactor_mode)) {
                        c.status = ST_NUMFAIL;
                        break;
                    }
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
                if (!r_refactor(s, c, a.refactor_mode)) {
                    c.status = ST_NUMFAIL;
                    break;
                }
                c.since = 0;
                c.y_valid = 0;
                if (c.phase == 3) r_btran(s, c, 2);
            }
        }
        recheck = 0;
        const int r = c.phase == 3 ? r_dual(d, s, c, mode1, a.refactor_mode) : r_primal(d, s, c, mode1, a.refactor_mode);
        if (r == R_EXIT) break;
        if (r == R_RECHECK) {
            recheck = 1;
            continue;
        }
        if (r == R_TO_P2) {
            if (!r_to_phase2(d, s, c, a.price_rule, a.refactor_mode)) {
                c.status = ST_NUMFAIL;
                break;
            }
        }
    }
    RSYNC();
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
    for (int i = lane; i < m; i += RW) {
        d.xr[i] = s.xr[i];
        d.y[i] = s.y[i];
        const int u = s.cover[i];
        d.cover[i] = u;
        d.rpos[i] = s.rpos[i];
        d.ypos[i] = s.ypos[i];
        if (u >= 0) {
            d.rlo[i] = s.lb[u];
            d.rhi[i] = s.ub[u];
        }
    }
    for (int p = lane; p < ny; p += RW) {
        const int i = s.Yl[p];
        d.Yl[p] = i;
        d.yvs[p] = d.rowvs[i];
        d.yy[p] = s.y[i];
    }
    for (int p = lane; p < k; p += RW) {
        const int j = s.Sl[p];
        d.Rl[p] = s.Rl[p];
        d.Sl[p] = j;
        d.xs[p] = s.xs[p];
        d.cS[p] = s.cost[j];
        d.slo[p] = s.lb[j];
        d.shi[p] = s.ub[j];
    }
    for (int e = lane; e < k * k; e += RW) {
        const int i = e / k, j = e - i * k;
        const double v = s.Mi[(size_t)i * s.ldm + j];
        d.Minv[(size_t)i * d.ldm + j] = v;
        if (!d.noT) d.MinvT[(size_t)j * d.ldm + i] = v;
    }
    for (int p = 0; p < k; ++p) {
        const double* col = s.A + (size_t)s.Sl[p] * s.lda;
        for (int i = lane; i < m; i += RW) d.AS[(size_t)p * m + i] = col[i];
    }
    if (!mode1 && d.AR) {
        const int64_t tw = d.tile_w;
        for (int p = 0; p < ny; ++p) {
            const int i = s.Yl[p];
            for (int j = lane; j < n; j += RW)
                d.AR[((size_t)(j / tw) * (size_t)d.arcap + (size_t)p) * (size_t)tw + (size_t)(j % tw)] =
                    s.A[i + (size_t)j * s.lda];
        }
    }
    if (lane == 0) {
        g->status = c.status;
        g->phase = c.phase;
        g->k = k;
        g->ny = ny;
        g->iter = c.iter;
        g->phase1_iters = c.phase1_iters;
        g->flips = c.flips;
        g->degenerate = c.degenerate;
        g->dual_iters = c.dual_iters;
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
        g->unb_var = c.unb_var;
        g->unb_sig = c.unb_sig;
        g->price_bytes = c.price_bytes;
        g->iter_bytes = c.iter_bytes;
        a.out->phase = c.phase;
        a.out->refactors = c.refactors;
        a.out->gj_refactors = c.gj;
        a.out->devex_resets = c.resets;
        a.out->emax_max = c.emax_max;
        a.out->ticks = (int64_t)(__builtin_amdgcn_s_memrealtime() - t0);
    }
}

}  // namespace

size_t resident_lds_bytes(int m, int n) {
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
