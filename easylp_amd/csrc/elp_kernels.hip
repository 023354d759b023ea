// elp_kernels.hip -- gfx950 kernels of the dense revised simplex.
//
// One simplex iteration is six launches on one stream:
//   k_btran        loop-top checks; y_R = Minv^T c_S, one wave per row   O(k^2)
//   k_price        d_j = c_j - AR[:,j]^T y_Y + Dantzig argmin per tile    O(|Y| n)  <- the HBM sweep
//   k_select_ftran min-loc over tiles + slacks (every workgroup), then
//                  alpha_S = Minv a_R(q), one wave per bump row           O(k^2)
//   k_ftran_zr     alpha on covered rows (z = AS alpha_S, chunked) fused
//                  with Harris pass 1 and pass-2 candidate emission       O(m k)
//   k_ratio        Harris pass 2, pivot plan, row of B^-1 (cases B/D)     O(k^2)
//   k_update       Minv/MinvT update, x_B update, AS / AR copies          O(k^2 + n)
// Sharded runs split k_select_ftran into k_select_local / (all-gather) /
// k_select_global / (all-reduce) / k_select_finish + k_ftran_bump.
// Every fp reduction follows the order of oracle/elp_oracle.c (explicit fma,
// built with -ffp-contract=off), so the pivot sequence is the oracle's.
// Kernels read the device control block and return early unless the loop is
// running, so the host can enqueue several iterations between polls.
#include "elp_internal.h"

#include <hip/hip_ext.h>
#include <math.h>

#include <type_traits>

// The per-iteration kernels take Dev by value from the kernel arguments.  A
// pointer to a device copy (r03) measured slower -- 38.3-38.9 against
// 36.8-37.3 us per C3 iteration: pointers loaded from memory lose their global
// address space, so the control-block reads became flat loads that wait for
// every load in flight; kernel-argument pointers stay global -- and r06
// removed it.

namespace elp {

#define DEV __device__ __forceinline__

// ------------------------------------------------------------ generator
DEV uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
DEV uint64_t gen_key(uint64_t seed, uint64_t stream) {
    return mix64(seed * 0x9E3779B97F4A7C15ULL + stream * 0xD1B54A32D192ED03ULL +
                 0x632BE59BD9B4E019ULL);
}
DEV double gen_u01k(uint64_t key, uint64_t idx) {
    const uint64_t z = mix64(key + (idx + 1) * 0x9E3779B97F4A7C15ULL);
    return (double)(z >> 11) * 0x1.0p-53;
}

__global__ void k_gen_A(uint64_t seed, int m, int64_t ncols, int64_t col0, double* __restrict__ A) {
    const uint64_t key = gen_key(seed, 0);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int64_t jj = blockIdx.y; jj < ncols; jj += gridDim.y) {
        const uint64_t j = (uint64_t)(col0 + jj);
        A[(size_t)jj * (size_t)m + (size_t)i] = gen_u01k(key, (uint64_t)i + j * (uint64_t)m);
    }
}
__global__ void k_gen_bc(uint64_t seed, int m, int64_t ncols, int64_t col0, int64_t n_global,
                         double* __restrict__ b, double* __restrict__ c) {
    const uint64_t kb = gen_key(seed, 2), kc = gen_key(seed, 1);
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double e = (double)n_global / 8.0, qq = (double)n_global / 4.0;
    if (b && t < m) b[t] = e + gen_u01k(kb, (uint64_t)t) * qq;
    if (c && t < ncols) c[t] = gen_u01k(kc, (uint64_t)(col0 + t));
}

// ------------------------------------------------------------ helpers
// lane-strided fma chain over x[0:len) . y[0:len) (lane l: x[l] y[l], then +64,
// ... in order -- the oracle's wave_dot lanes), loads issued 8 at a time: a
// plain loop waited for each load before issuing the next (k > 512 bumps)
DEV double lane_chain(const double* __restrict__ x, const double* y, int len) {
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    for (int j0 = lane; j0 < len; j0 += 64 * 8) {
        double v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = x[min(j0 + 64 * t, len - 1)];
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (j0 + 64 * t < len) acc = fma(v[t], y[j0 + 64 * t], acc);
    }
    return acc;
}
// wave sum in the oracle's wave_dot tree (pairs of lanes, then pairs of pairs,
// ... : offsets 1, 2, 4, ..., 32 ascending): DPP inside 16-lane rows (after
// the quad sums every lane of a quad holds the same value, so the mirrors pair
// whole groups like xor 4 / xor 8 would), ds_swizzle for xor 16, the halves by
// readlane.  Uniform result.
template <int CTRL>
DEV double dpp_f64(double v);
DEV double swz16_f64(double v);
DEV double readlane_f64(double v, int l);
DEV double wave_tree(double v) {
    v = v + dpp_f64<0xB1>(v);
    v = v + dpp_f64<0x4E>(v);
    v = v + dpp_f64<0x141>(v);
    v = v + dpp_f64<0x140>(v);
    v = v + swz16_f64(v);
    return readlane_f64(v, 0) + readlane_f64(v, 32);
}
DEV double unit_sign(const Dev& d, int var, int row) {  // var: global id
    return var >= d.N + d.m ? d.asgn[row] : 1.0;
}
// global var id -> shard-local per-variable index (-1: another shard's column)
DEV int loc_of(const Dev& d, int g) {
    if (g < d.N) {
        const int64_t j = (int64_t)g - d.col0;
        return (j >= 0 && j < d.n) ? (int)j : -1;
    }
    return d.n + (g - d.N);
}
// an element of A as the solver sees it: scaled on the fly when A is the
// caller's unscaled matrix (Dev::srow / scol), as stored otherwise
DEV double sca(const Dev& d, double a, int64_t i, int64_t jg) {
    return d.srow ? ldexp(a, d.srow[i] + d.scol[jg]) : a;
}
// element i of the entering column q (a column pointer of qcolumn): the
// exchanged packet and the CSC scatter hold scaled values already
DEV double qcol_at(const Dev& d, const double* col, int q, int64_t i) {
    return col == d.pkt || d.csc ? col[i] : sca(d, col[i], i, q);
}
// the entering structural column q (global id): read in place on one GPU or
// from the replicated A, else from the exchanged packet
DEV const double* qcolumn(const Dev& d, int q) {
    if (d.csc) return d.qcol;
    if (!d.sharded) return d.A + (size_t)(q - d.col0) * (size_t)d.m;
    if (d.Afull) return d.Afull + (size_t)q * (size_t)d.m;
    return d.pkt;
}
// KEEP(x): an empty asm that reads x.  Placed on an early-exit path it keeps
// the compiler from sinking a prefetch load below the exit test (which would
// serialise the prefetch behind the control-block round trip); the wait for x
// lands on the exit path only.
#define KEEP(x) asm volatile("" ::"v"(x))
// Unconditional load of p[min(idx, lim - 1)] (p[0] when lim <= 0): a prefetch
// whose bound is only an upper bound stays straight-line code, so the compiler
// counts it in vmcnt instead of branching around it and draining the queue.
template <class T>
DEV T ld_clamp(const T* p, int idx, int lim) {
    const int i = idx < lim ? idx : (lim > 0 ? lim - 1 : 0);
    return p[i];
}
DEV bool cand_better(const Cand& a, const Cand& b, int bland) {
    if (a.j < 0) return false;
    if (b.j < 0) return true;
    if (bland) return a.j < b.j;
    return a.score > b.score || (a.score == b.score && a.j < b.j);
}
// field-wise select (a whole-struct conditional copy of Cand was observed to
// be miscompiled on gfx950: the d field kept its old value)
DEV void cand_take(Cand& c, const Cand& o, bool take) {
    c.score = take ? o.score : c.score;
    c.d = take ? o.d : c.d;
    c.w = take ? o.w : c.w;
    c.j = take ? o.j : c.j;
}
// Cross-lane moves without LDS: DPP inside a row of 16 lanes (xor 1, xor 2,
// half-row mirror, row mirror -- a butterfly over 16 lanes when each step
// follows a full reduction of the previous group), ds_swizzle for xor 16, then
// the two halves by readlane.
template <int CTRL>
DEV double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
DEV double swz16_f64(double v) {  // lane ^ 16 inside each half-wave
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_swizzle((int)b, 0x401F);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x401F);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
DEV double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
DEV long long readlane_i64(long long v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)v, l), hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return ((long long)hi << 32) | (long long)(unsigned)lo;
}
// wave-wide max (the result is uniform)
DEV double wave_max_f64(double v) {
    v = fmax(v, dpp_f64<0xB1>(v));   // quad_perm [1,0,3,2]: lane ^ 1
    v = fmax(v, dpp_f64<0x4E>(v));   // quad_perm [2,3,0,1]: lane ^ 2
    v = fmax(v, dpp_f64<0x141>(v));  // row_half_mirror: the other quad of the 8
    v = fmax(v, dpp_f64<0x140>(v));  // row_mirror: the other 8 of the 16
    v = fmax(v, swz16_f64(v));
    return fmax(readlane_f64(v, 0), readlane_f64(v, 32));
}
// The best candidate of a wave whose candidate indices increase with the lane
// (a pricing tile: lane l holds the better of its columns 2l, 2l+1).  The same
// total order as cand_better: the highest score, then the lowest index -- the
// lowest lane among the highest scores; Bland: the lowest valid lane.
DEV Cand wave_best_mono(const Cand& c, int bland) {
    const bool valid = c.j >= 0;
    const unsigned long long vm = __ballot(valid);
    Cand r;
    r.j = -1;
    r.score = 0.0;
    r.d = 0.0;
    r.w = 1.0;
    if (vm == 0ull) return r;
    int win;
    if (bland) {
        win = __ffsll((long long)vm) - 1;
    } else {
        const double smax = wave_max_f64(valid ? c.score : -1.0);
        const unsigned long long mm = __ballot(valid && c.score == smax);
        win = __ffsll((long long)(mm ? mm : vm)) - 1;  // (NaN scores only: the lowest valid lane)
    }
    win = __builtin_amdgcn_readfirstlane(win);
    r.score = readlane_f64(c.score, win);
    r.d = readlane_f64(c.d, win);
    r.w = readlane_f64(c.w, win);
    r.j = readlane_i64((long long)c.j, win);
    return r;
}
// wave-wide min (uniform result)
DEV double wave_min_f64(double v) {
    v = fmin(v, dpp_f64<0xB1>(v));
    v = fmin(v, dpp_f64<0x4E>(v));
    v = fmin(v, dpp_f64<0x141>(v));
    v = fmin(v, dpp_f64<0x140>(v));
    v = fmin(v, swz16_f64(v));
    return fmin(readlane_f64(v, 0), readlane_f64(v, 32));
}
DEV int wave_min_i32(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_ds_swizzle(v, 0x401F));
    return min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 32));
}
// The lane holding the lowest index among the lanes of `mask` (non-empty):
// usually one lane (no tie), else a min-reduction of the indices
DEV int lowest_index_lane(unsigned long long mask, bool in, int idx) {
    if (__popcll(mask) == 1) return __ffsll((long long)mask) - 1;
    const int im = wave_min_i32(in ? idx : 0x7fffffff);
    return __ffsll((long long)__ballot(in && idx == im)) - 1;
}
// the best candidate of a wave in cand_better's total order (highest score,
// then lowest index; Bland: lowest index), without LDS
DEV Cand wave_best(const Cand& c, int bland) {
    const bool valid = c.j >= 0;
    const unsigned long long vm = __ballot(valid);
    Cand r;
    r.j = -1;
    r.score = 0.0;
    r.d = 0.0;
    r.w = 1.0;
    if (vm == 0ull) return r;
    unsigned long long mask = vm;
    bool in = valid;
    if (!bland) {
        const double smax = wave_max_f64(valid ? c.score : -1.0);
        in = valid && c.score == smax;
        mask = __ballot(in);
        if (mask == 0ull) {  // (NaN scores only) the lowest index among the valid lanes
            in = valid;
            mask = vm;
        }
    }
    const int win = __builtin_amdgcn_readfirstlane(lowest_index_lane(mask, in, (int)c.j));
    r.score = readlane_f64(c.score, win);
    r.d = readlane_f64(c.d, win);
    r.w = readlane_f64(c.w, win);
    r.j = readlane_i64((long long)c.j, win);
    return r;
}
// block-wide argmax of candidates; result valid in every thread
template <int NT>
DEV Cand block_best(Cand c, int bland, Cand* lds) {
    c = wave_best(c, bland);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) lds[w] = c;
    __syncthreads();
    int win = 0;  // the winning wave, then one copy of its record
    for (int i = 1; i < NT / 64; ++i)
        if (cand_better(lds[i], lds[win], bland)) win = i;
    const Cand r = lds[win];
    __syncthreads();
    return r;
}
template <int NT>
DEV double block_min(double v, double* lds) {
    v = wave_min_f64(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) lds[w] = v;
    __syncthreads();
    double r = lds[0];
    for (int i = 1; i < NT / 64; ++i) r = fmin(r, lds[i]);
    __syncthreads();
    return r;
}
template <int NT>
DEV double block_max(double v, double* lds, int ltid = -1) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    if (ltid < 0) ltid = threadIdx.x;
    const int w = ltid >> 6, lane = ltid & 63;
    if (lane == 0) lds[w] = v;
    __syncthreads();
    double r = lds[0];
    for (int i = 1; i < NT / 64; ++i) r = fmax(r, lds[i]);
    __syncthreads();
    return r;
}

// exclusive block scan of one int per thread (NT threads); returns the total
template <int NT>
DEV int block_scan_excl(int v, int* excl, int* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off);
        if (lane >= off) incl += u;
    }
    if (lane == 63) lds[w] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) base += lds[i];
        tot += lds[i];
    }
    __syncthreads();
    *excl = base + incl - v;
    return tot;
}

// ---------------------------------------------------------- sparse operands
// Hypersparse products against the bump inverse (CSC input, large bumps): the
// operand of a wave_dot -- a_R, a_F[R] (FTRAN), A[i, S] (a row of B^-1) -- has
// a handful of nonzeros among k positions.  A list of them, lane-bucketed
// (sorted by (position mod 64, position); lsb[l] = first entry of lane l,
// lsb[64] = n), lets lane l run exactly its chain of the dense lane_chain
// (positions l, l + 64, ... ascending) over the nonzero terms only: every
// skipped term is fma(x, 0, acc) = acc, so the value is the dense one bit for
// bit, at O(n) loads per wave instead of O(k).
constexpr int SPL = 256;  // entries per list at most (more: the dense path)
// lane l's chain over its bucket, loads 4 at a time in flight
DEV double sparse_lane_chain(const double* __restrict__ x, const int* lpos, const double* lval, const int* lsb) {
    const int lane = threadIdx.x & 63;
    const int s = lsb[lane], e = lsb[lane + 1];
    double acc = 0.0;
    for (int t0 = s; t0 < e; t0 += 4) {
        double xv[4], vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = t0 + u < e ? t0 + u : e - 1;
            xv[u] = x[lpos[t]];
            vv[u] = lval[t];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (t0 + u < e) acc = fma(xv[u], vv[u], acc);
    }
    return acc;
}
// lane_chain / sparse_lane_chain over x(j) computed by a functor (the deferred
// update's new inverse, minv_new)
template <class F>
DEV double lane_chain_f(F x, const double* y, int len) {
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    for (int j0 = lane; j0 < len; j0 += 64 * 8) {
        double v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = x(min(j0 + 64 * t, len - 1));
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (j0 + 64 * t < len) acc = fma(v[t], y[j0 + 64 * t], acc);
    }
    return acc;
}
template <class F>
DEV double sparse_lane_chain_f(F x, const int* lpos, const double* lval, const int* lsb) {
    const int lane = threadIdx.x & 63;
    const int s = lsb[lane], e = lsb[lane + 1];
    double acc = 0.0;
    for (int t0 = s; t0 < e; t0 += 4) {
        double xv[4], vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = t0 + u < e ? t0 + u : e - 1;
            xv[u] = x(lpos[t]);
            vv[u] = lval[t];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (t0 + u < e) acc = fma(xv[u], vv[u], acc);
    }
    return acc;
}

// Lane-bucketed list from one candidate entry per thread (NT threads; valid
// entries carry distinct positions): compaction, rank by (p mod 64, p), bucket
// starts.  lkey: NT ints of scratch.  Returns n (uniform); ends with a barrier.
template <int NT>
DEV int spl_build(bool valid, int p, double v, int* lpos, double* lval, int* lsb, int* lkey, int* scan) {
    int excl;
    const int n = block_scan_excl<NT>(valid ? 1 : 0, &excl, scan);
    const int key = ((p & 63) << 25) | p;  // (positions < 2^25)
    if (valid) lkey[excl] = key;
    __syncthreads();
    if (valid) {
        int r = 0;
        for (int t = 0; t < n; ++t) r += lkey[t] < key ? 1 : 0;
        lpos[r] = p;
        lval[r] = v;
    }
    if ((int)threadIdx.x <= 64) {
        int b = 0;
        for (int t = 0; t < n; ++t) b += (lkey[t] >> 25) < (int)threadIdx.x ? 1 : 0;
        lsb[threadIdx.x] = b;
    }
    __syncthreads();
    return n;
}

// wave-order phase-1 sum (oracle art_sum): executed by ONE wave
DEV double wave_art_sum(const Dev& d) {
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    for (int i = lane; i < d.m; i += 64)
        if (d.cover[i] >= d.N + d.m) acc = acc + d.xr[i];
    return wave_tree(acc);
}

// ============================================================== init
__global__ void k_init_cols(Dev d, const double* __restrict__ lo, const double* __restrict__ up) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.n) return;
    // (the host mapped |v| >= elp_control.infinity to +-inf BEFORE scaling; a
    //  finite bound that crosses 1e30 once scaled stays finite, as in the oracle)
    const double l = lo ? lo[j] : 0.0, u = up ? up[j] : HUGE_VAL;
    if (d.spos) d.spos[j] = -1;  // (CSC: no basic structural at a fresh start)
    d.lb[j] = l;
    d.ub[j] = u;
    d.cost[j] = 0.0;
    if (l > u) atomicOr(&d.ctl->infeasible_bounds, 1);
    if (l == u) {
        d.vstat[j] = VS_FIXED;
        d.xval[j] = l;
    } else if (l > -HUGE_VAL) {
        d.vstat[j] = VS_LOWER;
        d.xval[j] = l;
    } else if (u < HUGE_VAL) {
        d.vstat[j] = VS_UPPER;
        d.xval[j] = u;
    } else {
        d.vstat[j] = VS_FREE;
        d.xval[j] = 0.0;
    }
}

// ordered compaction: nzlist = { j < n : vstat != BASIC && xval != 0 }, ascending.
// One workgroup per chunk of 1024 * NZ_RUN columns; thread t owns NZ_RUN
// consecutive columns (a bit mask of flags, loads all in flight).  Pass 1
// counts each chunk; pass 2 offsets the chunk by the counts before it (a wave
// scan + the waves' totals inside the chunk) and writes.
constexpr int NZ_RUN = 16, NZ_CHUNK = 1024 * NZ_RUN;
DEV unsigned nz_flags(const Dev& d, int64_t js) {
    unsigned mask = 0;
    if (js + NZ_RUN <= d.n) {  // whole run: one 16-byte status load, 8 value loads
        const int4 v4 = *reinterpret_cast<const int4*>(d.vstat + js);  // (hipMalloc base, js % 16 == 0)
        double2 xv[NZ_RUN / 2];
#pragma unroll
        for (int u = 0; u < NZ_RUN / 2; ++u) xv[u] = *reinterpret_cast<const double2*>(d.xval + js + 2 * u);
        const int8_t* vb = reinterpret_cast<const int8_t*>(&v4);
#pragma unroll
        for (int u = 0; u < NZ_RUN; ++u) {
            const double x = (u & 1) ? xv[u >> 1].y : xv[u >> 1].x;
            mask |= (unsigned)((vb[u] != VS_BASIC) & (x != 0.0)) << u;
        }
    } else {
        for (int u = 0; u < NZ_RUN; ++u) {
            const int64_t j = js + u;
            const bool f = j < d.n && d.vstat[j] != VS_BASIC && d.xval[j] != 0.0;
            mask |= (unsigned)f << u;
        }
    }
    return mask;
}
__global__ void __launch_bounds__(1024) k_nzlist_count(Dev d) {
    __shared__ int wsum[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t js = (int64_t)blockIdx.x * NZ_CHUNK + (int64_t)threadIdx.x * NZ_RUN;
    int cnt = __popc(nz_flags(d, js));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if (lane == 0) wsum[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < 16; ++i) t += wsum[i];
        d.nzchunk[blockIdx.x] = t;
    }
}
__global__ void __launch_bounds__(1024) k_nzlist(Dev d) {
    __shared__ int wsum[16];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t js = (int64_t)blockIdx.x * NZ_CHUNK + (int64_t)threadIdx.x * NZ_RUN;
    const unsigned mask = nz_flags(d, js);
    if (threadIdx.x < 64) {  // the counts of the chunks before this one
        int b = 0;
        for (int c = lane; c < (int)blockIdx.x; c += 64) b += d.nzchunk[c];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) b += __shfl_xor(b, off);
        if (lane == 0) s_base = b;
    }
    const int cnt = __popc(mask);
    int incl = cnt;  // inclusive scan over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int pos = s_base + incl - cnt, tot = s_base;
    for (int i = 0; i < 16; ++i) {
        if (i < w) pos += wsum[i];
        tot += wsum[i];
    }
    for (int u = 0; u < NZ_RUN; ++u)
        if (mask >> u & 1u) d.nzlist[pos++] = (int)(js + u);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *d.nzcount = tot;
}

// ract_i = chain(ract_i, a_ij x_j over this shard's nonzero nonbasic columns,
// ascending j): the oracle's seq order, continued shard after shard
__global__ void k_row_chain(Dev d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    const int nz = *d.nzcount;
    double acc = d.ract[i];
    for (int t = 0; t < nz; ++t) {
        const int j = d.nzlist[t];
        acc = fma(sca(d, d.A[(size_t)j * (size_t)d.m + (size_t)i], i, d.col0 + j), d.xval[j], acc);
    }
    d.ract[i] = acc;
}

// CSC input: the same chain over row i's CSR entries (ascending j), with the
// nonzero-list filter (nonbasic, x_j != 0) applied per entry; zero entries of
// the dense layout contribute fma(0, x, acc) = acc there, so both agree
__global__ void k_row_chain_csr(Dev d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    double acc = d.ract[i];
    for (int64_t t = d.rptr[i]; t < d.rptr[i + 1]; ++t) {
        const int j = d.cind[t];
        const double xj = d.xval[j];
        if (d.vstat[j] != VS_BASIC && xj != 0.0) acc = fma(d.rval[t], xj, acc);
    }
    d.ract[i] = acc;
}

__global__ void k_init_rows(Dev d, const double* __restrict__ rhs_in) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    const double bi = rhs_in[i];  // (infinite values mapped by the host before scaling)
    d.b[i] = bi;
    const int n = d.n, m = d.m, sv = n + i, av = n + m + i;  // local ids
    const int svg = d.N + i, avg = d.N + m + i;                 // global ids
    // d.lb/d.ub for slacks were written by the host (dir); artificials:
    d.lb[av] = 0.0;
    d.ub[av] = 0.0;
    d.cost[sv] = 0.0;
    d.cost[av] = 0.0;
    d.vstat[av] = VS_FIXED;
    d.xval[av] = 0.0;
    d.rpos[i] = -1;
    d.ypos[i] = -1;
    d.asgn[i] = 1.0;
    const double r = bi - d.ract[i];
    const double sl = d.lb[sv], su = d.ub[sv];
    d.rowvs[i] = sl == su ? VS_FIXED : sl > -HUGE_VAL ? VS_LOWER : VS_UPPER;
    if (r >= sl && r <= su) {
        d.vstat[sv] = VS_BASIC;
        d.cover[i] = svg;
        d.xr[i] = r;
        d.xval[sv] = 0.0;
        d.rlo[i] = sl;
        d.rhi[i] = su;
    } else {
        const double s = r < sl ? sl : su;
        d.vstat[sv] = (sl == su) ? VS_FIXED : (s == sl) ? VS_LOWER : VS_UPPER;
        d.xval[sv] = s;
        const double res = r - s;
        d.asgn[i] = res > 0.0 ? 1.0 : -1.0;
        d.ub[av] = HUGE_VAL;
        d.cost[av] = 1.0;
        d.vstat[av] = VS_BASIC;
        d.cover[i] = avg;
        d.xr[i] = fabs(res);
        d.rlo[i] = 0.0;
        d.rhi[i] = HUGE_VAL;
    }
}

// single block: Y = rows covered by an artificial, ascending; tol_inf from max|b|
__global__ void __launch_bounds__(1024) k_init_Y(Dev d) {
    __shared__ int wsum[16];
    __shared__ int base;
    __shared__ double red[16];
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double bmax = 0.0;
    for (int i0 = 0; i0 < d.m; i0 += 1024) {
        const int i = i0 + threadIdx.x;
        bool f = false;
        if (i < d.m) {
            f = d.cover[i] >= d.N + d.m;
            const double bi = fabs(d.b[i]);
            if (bi < HUGE_VAL && bi > bmax) bmax = bi;
        }
        const unsigned long long bal = __ballot(f);
        const int before = __popcll(bal & ((1ULL << lane) - 1ULL));
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int k = 0; k < w; ++k) off += wsum[k];
        if (f) {
            d.Yl[off + before] = i;
            d.ypos[i] = off + before;
            d.yvs[off + before] = d.rowvs[i];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int k = 0; k < 16; ++k) t += wsum[k];
            base += t;
        }
        __syncthreads();
    }
    bmax = block_max<1024>(bmax, red);
    if (threadIdx.x == 0) {
        d.ctl->ny = base;
        d.ctl->k = 0;
        d.ctl->tol_inf = 1e-9 * (1.0 + bmax);
    }
}

// a_ij of this shard, read along a row (AR row copies): the column-major A,
// one line per element (r01-r05's opt-in row-major copy measured no faster)
DEV double a_row(const Dev& d, int64_t i, int64_t j) {
    return sca(d, d.A[(size_t)j * (size_t)d.m + (size_t)i], i, d.col0 + j);
}

// ============================================================== scaling
// lp_solve-style scaling (elp_control.scaling; oracle scale_factors): every
// factor is a power of two, so the scaled problem is exact and unscaling is
// exact.  On the integer exponents e_ij = ilogb|a_ij| of the nonzeros,
// geometric passes set row then column exponents to -floor((min + max) / 2) of
// the currently scaled entries (lp_solve's sqrt(min * max) in the log domain);
// equilibrate sets each column's to -(max + 1), so its largest scaled |a| lies
// in [1/2, 1).  Integer min / max: identical on the GPU and the oracle.
DEV int floor_half(int s) { return s >= 0 ? s / 2 : -((1 - s) / 2); }
constexpr int SCALE_EMPTY_MIN = 0x3fffffff, SCALE_EMPTY_MAX = -0x3fffffff;

// column pass: one workgroup per column (grid-stride), rows strided by thread
__global__ void __launch_bounds__(256) k_scale_col(int m, int64_t ncols, const double* __restrict__ A,
                                                   const int32_t* __restrict__ rho, int32_t* __restrict__ gam,
                                                   int equilibrate, int32_t* changed) {
    __shared__ int smn[4], smx[4];
    for (int64_t j = blockIdx.x; j < ncols; j += gridDim.x) {
        const double* col = A + (size_t)j * (size_t)m;
        int mn = SCALE_EMPTY_MIN, mx = SCALE_EMPTY_MAX;
        for (int i0 = threadIdx.x; i0 < m; i0 += 256 * 8) {  // 8 loads in flight per thread
            double a[8];
            int r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int ii = min(i0 + 256 * u, m - 1);
                a[u] = col[ii];
                r[u] = rho[ii];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (i0 + 256 * u < m && a[u] != 0.0 && isfinite(a[u])) {  // (non-finite: no exponent)
                    const int e = ilogb(a[u]) + r[u];
                    mn = min(mn, e);
                    mx = max(mx, e);
                }
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            mn = min(mn, __shfl_xor(mn, off));
            mx = max(mx, __shfl_xor(mx, off));
        }
        if ((threadIdx.x & 63) == 0) {
            smn[threadIdx.x >> 6] = mn;
            smx[threadIdx.x >> 6] = mx;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < 4; ++w) {
                mn = min(mn, smn[w]);
                mx = max(mx, smx[w]);
            }
            int g = 0;
            if (mx != SCALE_EMPTY_MAX) g = equilibrate ? -(mx + 1) : -floor_half(mn + mx);
            if (g != gam[j]) {
                gam[j] = g;
                *changed = 1;
            }
        }
        __syncthreads();
    }
}

// row pass, part 1: thread = row, a chunk of SCALE_RCOLS columns per workgroup
// row; per-row max of -(e_ij + gamma_j) and of e_ij + gamma_j into rnm / rmx
// (integer atomics; both maxima, so shards combine with one all-reduce max)
constexpr int SCALE_RCOLS = 512;
__global__ void __launch_bounds__(256) k_scale_row_part(int m, int64_t ncols, const double* __restrict__ A,
                                                        const int32_t* __restrict__ gam, int32_t* rmn,
                                                        int32_t* rmx) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int64_t j0 = (int64_t)blockIdx.y * SCALE_RCOLS;
    const int64_t j1 = j0 + SCALE_RCOLS < ncols ? j0 + SCALE_RCOLS : ncols;
    int mn = SCALE_EMPTY_MIN, mx = SCALE_EMPTY_MAX;
    for (int64_t j = j0; j < j1; j += 8) {  // 8 loads in flight per thread
        double a[8];
        int g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t jj = j + u < j1 ? j + u : j1 - 1;
            a[u] = A[(size_t)jj * (size_t)m + i];
            g[u] = gam[jj];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (j + u < j1 && a[u] != 0.0 && isfinite(a[u])) {
                const int e = ilogb(a[u]) + g[u];
                mn = min(mn, e);
                mx = max(mx, e);
            }
        }
    }
    if (mx != SCALE_EMPTY_MAX) {
        atomicMax(&rmn[i], -mn);
        atomicMax(&rmx[i], mx);
    }
}

// row pass, part 2: rho_i from the row's min / max
__global__ void k_scale_row_final(int m, int32_t* rmn, int32_t* rmx, int32_t* rho, int32_t* changed) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int mn = -rmn[i], mx = rmx[i];
    const int r = mx == SCALE_EMPTY_MAX ? 0 : -floor_half(mn + mx);
    if (r != rho[i]) {
        rho[i] = r;
        *changed = 1;
    }
    rmn[i] = SCALE_EMPTY_MAX;  // ready for the next pass
    rmx[i] = SCALE_EMPTY_MAX;
}

__global__ void k_scale_init(int m, int64_t ncols, int32_t* rho, int32_t* gam, int32_t* rmn, int32_t* rmx) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < m) {
        rho[t] = 0;
        rmn[t] = SCALE_EMPTY_MAX;
        rmx[t] = SCALE_EMPTY_MAX;
    }
    if (t < ncols) gam[t] = 0;
}

// A_ij *= 2^(rho_i + gamma_j) (exact)
__global__ void k_scale_apply(int m, int64_t ncols, double* __restrict__ A, const int32_t* __restrict__ rho,
                              const int32_t* __restrict__ gam) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int r = rho[i];
    for (int64_t j = blockIdx.y; j < ncols; j += gridDim.y) {
        double* a = A + (size_t)j * (size_t)m + i;
        *a = ldexp(*a, r + gam[j]);
    }
}

// element (row p, column j) of the tile-major AR
DEV size_t ar_at(const Dev& d, int64_t p, int64_t j) {
    const int64_t tw = d.tile_w;  // columns per tile (<= TILE_COLS), also the row stride inside a tile
    return ((size_t)(j / tw) * (size_t)d.arcap + (size_t)p) * (size_t)tw + (size_t)(j % tw);
}

// AR[p][j] = A[Yl[p]][j] for p < ny (initial fill)
__global__ void k_fill_AR(Dev d) {
    const int ny = d.ctl->ny;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.n) return;
    for (int p = blockIdx.y; p < ny; p += gridDim.y)
        d.AR[ar_at(d, p, j)] = a_row(d, d.Yl[p], j);
}

// grow AR: rows [0, rows) of every tile into the new capacity
__global__ void k_ar_relayout(Dev d, const double* __restrict__ old_ar, int64_t old_cap, int rows) {
    const int64_t tw = d.tile_w, ntiles = d.ldr / tw;
    const int64_t total = ntiles * (int64_t)rows * tw;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = e / ((int64_t)rows * tw);
        const int64_t r = e % ((int64_t)rows * tw);
        d.AR[(size_t)t * (size_t)d.arcap * tw + (size_t)r] = old_ar[(size_t)t * (size_t)old_cap * tw + (size_t)r];
    }
}

// ============================================================== BTRAN
// phase 1: y on covered rows (sigma_u c_u), 0 on R rows
__global__ void k_ycov(Dev d) {
    if (d.ctl->status != ST_RUN) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    const int u = d.cover[i];
    const double yi = u >= 0 ? unit_sign(d, u, i) * d.cost[loc_of(d, u)] : 0.0;
    d.y[i] = yi;
    const int sl = d.ypos[i];
    if (u >= 0 && sl >= 0) d.yy[sl] = yi;
}
// phase 1: t_p = c_{S_p} - wave_dot(AS[:,p], y_cov)   (one wave per p)
__global__ void __launch_bounds__(256) k_btran_t(Dev d) {
    if (d.ctl->status != ST_RUN) return;
    const int k = d.ctl->k;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= k) return;
    const double* col = d.AS + (size_t)p * (size_t)d.m;
    double acc = 0.0;
    for (int i = lane; i < d.m; i += 64) acc = fma(col[i], d.y[i], acc);
    acc = wave_tree(acc);
    if (lane == 0) d.t[p] = d.cS[p] - acc;
}

// loop-top checks (block 0, wave 0) + y on covered rows (phase 2: sigma*0)
// + y_R[p] = wave_dot(MinvT[p, 0:k], tv) scattered to y[R_p]  (one wave per p)
DEV void btran_body(const Dev& d, int phase, const double* __restrict__ tv);

__global__ void __launch_bounds__(256) k_btran(Dev d, int phase, const double* __restrict__ tv) {
    DevCtl* c = d.ctl;
    if (c->status != ST_RUN) return;
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        // oracle run_phase loop top: phase-1 done, iteration cap, stop, refactor
        double s = 0.0;
        if (phase == 1) s = wave_art_sum(d);
        if (threadIdx.x == 0) {
            if (phase == 1) c->art_sum = s;
            if (phase == 1 && s <= c->tol_inf) c->status = ST_P1DONE;
            else if (c->iter >= c->iter_limit) c->status = ST_ITERCAP;
            else if (c->iter >= c->iter_stop) c->status = ST_STOP;
            else if (c->since_refactor >= c->refactor_period) c->status = ST_REFACTOR;
        }
    }
    btran_body(d, phase, tv);
}

// exact duals after a refactor / at the phase-2 start (phase 2 then keeps y by
// the dual update in k_ratio): no status test, no loop-top checks
__global__ void __launch_bounds__(256) k_btran_exact(Dev d) { btran_body(d, 2, d.cS); }

DEV void btran_body(const Dev& d, int phase, const double* __restrict__ tv) {
    const int k = d.ctl->k;
    if (phase == 2) {
        const int gid = blockIdx.x * blockDim.x + threadIdx.x;
        const int gsz = gridDim.x * blockDim.x;
        for (int i = gid; i < d.m; i += gsz) {
            const int u = d.cover[i];
            if (u < 0) continue;
            const double yi = unit_sign(d, u, i) * d.cost[loc_of(d, u)];
            d.y[i] = yi;
            const int sl = d.ypos[i];
            if (sl >= 0) d.yy[sl] = yi;
        }
    }
    const int lane = threadIdx.x & 63;
    // (row p of MinvT = column p of Minv: read with stride ldm when d.noT)
    const int64_t ts = d.noT ? d.ldm : 1;
    for (int p = blockIdx.x * 4 + (threadIdx.x >> 6); p < k; p += gridDim.x * 4) {
        const double* row = d.noT ? d.Minv + p : d.MinvT + (size_t)p * d.ldm;
        double acc = 0.0;
        for (int q = lane; q < k; q += 64) acc = fma(row[q * ts], tv[q], acc);
        acc = wave_tree(acc);
        if (lane == 0) {
            const int i = d.Rl[p];
            d.y[i] = acc;
            d.yy[d.ypos[i]] = acc;  // R rows always have a nonbasic slack
        }
    }
}

// deferred update (phase 2): defined with k_update below
struct Plan;
DEV void apply_plan(const Dev& d, const Plan& P, int blk, int nb, int nb_minv, bool do_ar, bool batch = true);
DEV void apply_minv(const Dev& d, const Plan& P, int64_t e0, int64_t estride, bool batch = true);
DEV void apply_copy(const Dev& d, const Plan& P, int64_t t0, int64_t tstride, bool do_ar);
template <int NT>
DEV void apply_minv_sru(const Dev& d, const Plan& P, int wg, int nwg);
DEV bool plan_pending(const DevCtl* c) { return c->plan_seq != c->applied_seq && c->plan.action != ACT_NONE; }
// the pricing launch's trailing `napply` workgroups apply the pending plan
// batch: the inverse update's loads grouped ahead of its stores (apply_minv);
// the dense pricing launch's trailing workgroups keep one element at a time
// (batched, its launch measured 0.6-1.5 us longer at 5000 x 50000, r04k A/B)
DEV bool apply_role(const Dev& d, int napply, int nb_minv, bool batch = true) {
    if ((int)blockIdx.x < (int)gridDim.x - napply) return false;
    const DevCtl* c = d.ctl;
    if (plan_pending(c) && c->status != ST_NUMFAIL) {
        const Plan P = c->plan;
        apply_plan(d, P, blockIdx.x - (gridDim.x - napply), napply, nb_minv, false, batch);
    }
    return true;
}

// ============================================================== pricing
// ELP_PDBG (diagnostic builds only, tools/build_variant.sh): six stamps per
// pricing workgroup -- start, control block in, wave 0's sweep done, every
// wave's sweep done, epilogue before the argmin, end -- so the host
// can dump one launch's timeline (ELP_PDBG_ITER); slot 1 holds the role of a
// non-tile workgroup (1 apply, 2 slacks)
#ifdef ELP_PDBG
constexpr int PSTRIDE = 6;
#define PDBG(slot, v) do { if (ELP_DIAG && d.ptimer && threadIdx.x == 0) d.pstamp[PSTRIDE * blockIdx.x + (slot)] = (v); } while (0)
#else
constexpr int PSTRIDE = 2;
#define PDBG(slot, v) do {} while (0)
#endif
// Devex reference weights (oracle run_phase, price_rule 1): the last pivot's
// ratio alpha_rj / alpha_rq = (d_j - d_j') / d_q from this pass's d_j' and the
// previous pass's d_j, w_j = max(w_j, (alpha_rj / alpha_rq)^2 w_q) (capped);
// the leaving variable's weight was set by k_ratio and is not updated here.
// DevCtl::dv_valid: 0 no update (phase start, bound flip), 1 update, 2 the
// framework restarts (every priced weight back to 1).
constexpr double DEVEX_WMAX = 1e20;
constexpr double DEVEX_RESET = 1e6;  // entering weight above this: new reference framework
struct DevexIn {
    int32_t valid, lv;
    double dq, wq;
};
DEV DevexIn devex_in(const DevCtl* c) {
    DevexIn x;
    x.valid = c->dv_valid;
    x.lv = c->dv_lv;
    x.dq = c->dv_dq;
    x.wq = c->dv_wq;
    return x;
}
// jl: local id (dw / dprev index), jg: global id; w0 / dp0: dw[jl], dprev[jl]
// as loaded by the caller (issued early, off the dependent tail)
DEV double devex_weight(const Dev& d, const DevexIn& x, int64_t jl, int64_t jg, double dj, double w0,
                        double dp0) {
    double wj = w0;
    if (x.valid == 2) {  // framework restart (k_ratio): weight 1, no update
        wj = 1.0;
        d.dw[jl] = 1.0;
    } else if (x.valid == 1 && jg != x.lv) {
        const double r = (dp0 - dj) / x.dq;
        double wn = (r * r) * x.wq;
        if (wn > DEVEX_WMAX) wn = DEVEX_WMAX;
        if (wn > wj) {
            wj = wn;
            d.dw[jl] = wj;
        }
    }
    d.dprev[jl] = dj;
    return wj;
}
// candidate of a priced column: Dantzig score |d|, Devex d^2 / w
DEV Cand price_cand(int8_t vs, double dj, double wj, int devex, double dtol, int64_t jg) {
    Cand o;
    o.j = -1;
    o.score = 0.0;
    o.d = dj;
    o.w = wj;
    if ((vs == VS_LOWER || vs == VS_FREE) && dj < -dtol) {
        o.j = jg;
        o.score = devex ? (dj * dj) / wj : -dj;
    } else if ((vs == VS_UPPER || vs == VS_FREE) && dj > dtol) {
        o.j = jg;
        o.score = devex ? (dj * dj) / wj : dj;
    }
    return o;
}
// The slack candidates (replicated on every rank; a slack's cost is 0, so
// d = -y on the Y slots, in slot order): nsw extra workgroups of the pricing
// launch (the host sizes them from its bound on |Y|: one slot per thread),
// workgroup s writing candidate [ntiles + s] next to the tiles'
template <int NT>
DEV void price_slacks(const Dev& d, int64_t ntiles, int s, int nsw, Cand* red) {
    const DevCtl* c = d.ctl;
    const int ny = c->ny, bland = c->bland, devex = c->devex;
    const double dtol = c->tol_dual;
    const DevexIn dx = devex_in(c);
    Cand best;
    best.j = -1;
    best.score = 0.0;
    best.d = 0.0;
    best.w = 1.0;
    for (int p = s * NT + threadIdx.x; p < ny; p += nsw * NT) {
        const int8_t v = d.yvs[p];
        if (v == VS_FIXED) continue;
        const int i = d.Yl[p];
        const double dj = 0.0 - d.yy[p];
        const double wj = devex ? devex_weight(d, dx, d.n + i, d.N + i, dj, d.dw[d.n + i], d.dprev[d.n + i]) : 1.0;
        const Cand o = price_cand(v, dj, wj, devex, dtol, d.N + i);
        cand_take(best, o, cand_better(o, best, bland));
    }
    best = block_best<NT>(best, bland, red);
    if (threadIdx.x == 0) d.cand[ntiles + s] = best;
}

// Pricing (k_price): see price_body.  The chunk partials are combined in LDS in
// chunk order, then the tile's argmin.
constexpr int PRICE_THREADS = 64 * PRICE_SPLIT;
typedef double dbl2 __attribute__((ext_vector_type(2)));
// plain (cached) loads: the live AR rows (~80 MB at 5000x50000) stay in the
// 256 MiB Infinity Cache between passes; non-temporal loads measured 10% slower
// there.  NTL (host's choice, sweep_nt): non-temporal loads once the sweep is
// larger than the Infinity Cache anyway (10 000 x 500 000), so it does not evict
// the bump (AS, Minv) the latency kernels re-read every iteration
#define AR_LOAD(ptr) (NTL ? __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(ptr)) \
                          : *reinterpret_cast<const dbl2*>(ptr))
#ifndef ELP_PRICE_UNR
#define ELP_PRICE_UNR 16
#endif
// lane l's double, read by every lane (v_readlane pair)
DEV double lane_bcast(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
// One tile workgroup = PRICE_SPLIT waves = 128 columns x all Y slots.  Wave w
// sweeps the slots p = w, w + PRICE_SPLIT, w + 2 PRICE_SPLIT, ... (an fma chain
// in slot order; the oracle's price order): its first UNR rows do not depend
// on |Y|, so they go out right behind the control-block loads, before the
// control block arrives (rows past |Y| are masked when it does), and the sweep
// overlaps the control-block round trip instead of following it.
// Grid: [d.ntiles column tiles of TILE_COLS columns][nsw slack workgroups]
// [napply trailing workgroups that apply the last pivot's deferred plan (phase
// 2; nothing the sweep reads)].  r03 applied the plan in waves 1..3 of every
// tile and put the slack workgroups first; r04's A/B measured both slower
// (k_price 17.94 us under rocprof against 18.83 with the slacks first; 25.4k
// against 24.7k iterations/s with the tiles applying the plan), and r06
// removed those variants.  TW: the tile width (TILE_COLS: every AR row offset
// a shift).
template <int NTL, int TW>
DEV void price_body(const Dev& d, int nsw, int napply, int nb_minv) {
    __shared__ double part[PRICE_SPLIT][TILE_COLS];
    __shared__ Cand red[PRICE_SPLIT];
    const int64_t ntiles = d.ntiles;
    if (napply > 0 && apply_role(d, napply, nb_minv, false)) return;
    const int sw = (int)blockIdx.x - (int)ntiles;  // slack workgroup index
    if (sw >= 0 && sw < nsw) {
        PDBG(1, 2ull);
        PDBG(2, 0ull);
        PDBG(3, 0ull);
        PDBG(4, 0ull);
        if (d.ctl->status != ST_RUN) return;
        price_slacks<PRICE_THREADS>(d, ntiles, sw, nsw, red);  // a slack workgroup
        return;
    }
    const int64_t tile = (int64_t)blockIdx.x;
    constexpr int tw = TW;
    // Software-pipelined sweep: the control block is loaded FIRST (vmcnt
    // retires in issue order, so the status test and the loop bound wait for
    // it alone, not for the rows issued behind it), then the first UNR rows
    // (independent of |Y|), then the epilogue operands; each loop step issues
    // the next UNR rows before it consumes the current ones, so a wave keeps
    // rows in flight through the whole sweep instead of draining them every
    // UNR rows.  Consumption order -- one fma chain per slot class in slot
    // order -- is the oracle's, unchanged.  With y read once per block (one
    // lane per row, v_readlane at the fma) instead of one uniform load per row,
    // r02m A/B at 5000x50000: launch 20.5 -> 19.6 us, 35.4 -> 34.6 us per
    // iteration (pipelining alone: no change; 8 / 12 rows per block: same);
    // at 10 000 x 500 000, HBM-bound, unchanged (338 vs 341 us, one run each).
    constexpr int S = PRICE_SPLIT;
    constexpr int UNR = ELP_PRICE_UNR;
    constexpr int SU = S * UNR;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const DevCtl* c = d.ctl;
    int32_t st0 = c->status;
    int ny = c->ny, bland = c->bland, devex = c->devex;
    DevexIn dx = devex_in(c);
    double dtol = c->tol_dual;
    __builtin_amdgcn_sched_barrier(0);
    // lanes past the tile's width read their last valid pair again (same line: no traffic)
    const int lcol = 2 * lane < tw ? 2 * lane : ((tw - 1) & ~1);
    const double* col = d.AR + (size_t)tile * (size_t)d.arcap * (size_t)tw + lcol;  // rows tw apart
    const double* __restrict__ yy = d.yy;
    const int cap = (int)d.arcap;
    dbl2 va[UNR], vb[UNR];
    // y of a block: lane l loads slot p + S (l mod UNR), the fma takes it by readlane
    double ya, yb;
    ya = yy[min(w + S * (lane % UNR), cap - 1)];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {  // slot w + S u, clamped into AR (masked by |Y| at use)
        const int pp = min(w + S * u, cap - 1);
        va[u] = AR_LOAD(col + (size_t)pp * (size_t)tw);
    }
    // the epilogue's per-column operands (status, cost, Devex weight, previous
    // d) of columns 2 lane, 2 lane + 1 -- wave 0's: the other waves load element
    // 0 (one line); clamped, no branch to drain
    const int64_t jA = tile * tw + 2 * lane;
    const bool inA = 2 * lane < tw, inB = 2 * lane + 1 < tw;  // (tile widths are even: both)
    const int64_t jc0 = (w == 0 && inA && jA < d.n) ? jA : 0, jc1 = (w == 0 && inB && jA + 1 < d.n) ? jA + 1 : 0;
    const int8_t pf_vs0 = d.vstat[jc0], pf_vs1 = d.vstat[jc1];
    const double pf_c0 = d.cost[jc0], pf_w0 = d.dw[jc0], pf_dp0 = d.dprev[jc0];
    const double pf_c1 = d.cost[jc1], pf_w1 = d.dw[jc1], pf_dp1 = d.dprev[jc1];
    __builtin_amdgcn_sched_barrier(0);  // all of the above issued before any use
    // (the control-block values stay vector values up to here -- their scalar
    //  copies would otherwise be made above the row loads, which would then
    //  wait for the control block; the wait here is for the control block only)
    asm volatile("" : "+v"(st0), "+v"(ny), "+v"(bland), "+v"(devex), "+v"(dx.valid), "+v"(dx.lv));
    asm volatile("" : "+v"(dx.dq), "+v"(dx.wq), "+v"(dtol));
    if (st0 != ST_RUN) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) KEEP(va[u].x);
        KEEP(ya);
        KEEP(pf_c0);
        KEEP(pf_c1);
        return;
    }
    PDBG(1, __builtin_amdgcn_s_memrealtime());
    const int nys = __builtin_amdgcn_readfirstlane(ny);
    double acc0 = 0.0, acc1 = 0.0;
    // rows of a block at or past |Y| re-read the block's first row (p < |Y|;
    // an L1/L2 hit) and are masked when consumed
#define PIPE_ISSUE(V, Y, P)                                                          \
    do {                                                                             \
        _Pragma("unroll") for (int u = 0; u < UNR; ++u) {                            \
            const int r_ = (P) + S * u < nys ? (P) + S * u : (P);                    \
            V[u] = AR_LOAD(col + (size_t)r_ * (size_t)tw);                           \
        }                                                                            \
        const int ry_ = (P) + S * (lane % UNR);                                      \
        Y = yy[ry_ < nys ? ry_ : (P)];                                               \
    } while (0)
#define PIPE_Y(Y, u) lane_bcast(Y, u)
#define PIPE_CONSUME(V, Y, P)                                                        \
    do {                                                                             \
        _Pragma("unroll") for (int u = 0; u < UNR; ++u) {                            \
            if ((P) + S * u < nys) {                                                 \
                const double y_ = PIPE_Y(Y, u);                                      \
                acc0 = fma(V[u].x, y_, acc0);                                        \
                acc1 = fma(V[u].y, y_, acc1);                                        \
            }                                                                        \
        }                                                                            \
    } while (0)
    int p = w;
    if (p < nys) {
        for (;;) {
            if (p + SU >= nys) {
                PIPE_CONSUME(va, ya, p);
                break;
            }
            PIPE_ISSUE(vb, yb, p + SU);
            __builtin_amdgcn_sched_barrier(0);
            PIPE_CONSUME(va, ya, p);
            p += SU;
            if (p + SU >= nys) {
                PIPE_CONSUME(vb, yb, p);
                break;
            }
            PIPE_ISSUE(va, ya, p + SU);
            __builtin_amdgcn_sched_barrier(0);
            PIPE_CONSUME(vb, yb, p);
            p += SU;
        }
    }
#undef PIPE_ISSUE
#undef PIPE_CONSUME
#undef PIPE_Y
    PDBG(2, __builtin_amdgcn_s_memrealtime());
    part[w][2 * lane] = acc0;
    part[w][2 * lane + 1] = acc1;
    __syncthreads();
    PDBG(3, __builtin_amdgcn_s_memrealtime());
    // the epilogue is wave 0's: lane l finishes columns 2l, 2l+1 (the classes
    // added in order), takes the better of the two, and the wave reduces
    // without LDS or a barrier
    if (w != 0) return;
    Cand cb[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        cb[h].j = -1;
        cb[h].score = 0.0;
        cb[h].d = 0.0;
        cb[h].w = 1.0;
        const int64_t j = jA + h;
        const int8_t vs = h ? pf_vs1 : pf_vs0;
        if ((h ? inB : inA) && j < d.n && vs != VS_BASIC && vs != VS_FIXED) {
            double tot = 0.0;
#pragma unroll
            for (int ww = 0; ww < PRICE_SPLIT; ++ww) tot = tot + part[ww][2 * lane + h];
            const double dj = (h ? pf_c1 : pf_c0) - tot;
            const double wj = devex ? devex_weight(d, dx, j, d.col0 + j, dj, h ? pf_w1 : pf_w0, h ? pf_dp1 : pf_dp0)
                                    : 1.0;
            cb[h] = price_cand(vs, dj, wj, devex, dtol, d.col0 + j);
        }
    }
    Cand best = cb[0];
    cand_take(best, cb[1], cand_better(cb[1], cb[0], bland));
    PDBG(4, __builtin_amdgcn_s_memrealtime());
    best = wave_best_mono(best, bland);
    if (lane == 0) d.cand[tile] = best;
}

// the pricing-launch timer (Dev::ptimer): every workgroup stamps its start and
// its end (after all its waves), so first start -> last end is the launch
template <int NT>
DEV void pstamp_begin(const Dev& d) {
    if (ELP_DIAG && d.ptimer && threadIdx.x == 0) {
        d.pstamp[PSTRIDE * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        if (blockIdx.x == 0) d.ctl->price_grid = (int32_t)gridDim.x;
    }
}
DEV void pstamp_end(const Dev& d) {
    if (!ELP_DIAG || !d.ptimer) return;
    __syncthreads();  // (every return path of the bodies is workgroup-uniform)
    if (threadIdx.x == 0) d.pstamp[PSTRIDE * blockIdx.x + PSTRIDE - 1] = __builtin_amdgcn_s_memrealtime();
}

// The release build's pricing timer: on the sampled chunks
// (ELP_PROFILE_SAMPLE / _EVENTS) the host launches the TIMED variant, whose
// workgroups stamp s_memrealtime (the 100 MHz constant clock) at entry and,
// after a barrier, at exit into slot tslot of Dev::ptst; k_ptimer_reduce then
// adds first start -> last end of each slot to DevCtl::price_ticks.  Only the
// sampled launches pay the end barrier and the two stores.
DEV void tstamp_begin(const Dev& d, int tslot) {
    if (threadIdx.x == 0 && (int)blockIdx.x < d.ptcap) {
        d.ptst[2 * ((size_t)tslot * d.ptcap + blockIdx.x)] = __builtin_amdgcn_s_memrealtime();
        if (blockIdx.x == 0) d.ptgrid[tslot] = (int32_t)gridDim.x;
    }
}
DEV void tstamp_end(const Dev& d, int tslot) {
    __syncthreads();  // (every return path of the bodies is workgroup-uniform)
    if (threadIdx.x == 0 && (int)blockIdx.x < d.ptcap)
        d.ptst[2 * ((size_t)tslot * d.ptcap + blockIdx.x) + 1] = __builtin_amdgcn_s_memrealtime();
}

template <int NTL, int TW, bool TIMED = false>
__global__ void __launch_bounds__(PRICE_THREADS) k_price(Dev d, int nsw, int napply, int nb_minv,
                                                         int tslot) {
    if (TIMED) tstamp_begin(d, tslot);
    pstamp_begin<PRICE_THREADS>(d);
    price_body<NTL, TW>(d, nsw, napply, nb_minv);
    pstamp_end(d);
    if (TIMED) tstamp_end(d, tslot);
}

// one workgroup per timed slot of the chunk: first start -> last end
__global__ void __launch_bounds__(256) k_ptimer_reduce(Dev d) {
    __shared__ unsigned long long slo[256], shi[256];
    const int s = blockIdx.x, t = threadIdx.x;
    const int g = min(d.ptgrid[s], d.ptcap);
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int w = t; w < g; w += 256) {
        const unsigned long long a = d.ptst[2 * ((size_t)s * d.ptcap + w)], b = d.ptst[2 * ((size_t)s * d.ptcap + w) + 1];
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    slo[t] = lo;
    shi[t] = hi;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
        if (t < h) {
            slo[t] = slo[t + h] < slo[t] ? slo[t + h] : slo[t];
            shi[t] = shi[t + h] > shi[t] ? shi[t + h] : shi[t];
        }
        __syncthreads();
    }
    if (t == 0 && shi[0] > slo[0]) {
        atomicAdd(&d.ctl->price_ticks, shi[0] - slo[0]);
        atomicAdd(reinterpret_cast<unsigned long long*>(&d.ctl->price_timed), 1ull);
    }
}

// algorithmic bytes of one pricing pass.  Dense: the AR sweep (8|Y|n), c and
// status (9n), y_Y and Yl (12|Y|).  CSC: row index + value per nonzero (12 nnz),
// column pointer, c, status (17n); the y gathers hit L2 (m doubles)
DEV double price_pass_bytes(const Dev& d, int ny, int devex) {
    // Devex adds w and the previous d per column: read both, write d (24n)
    const double dvx = devex ? 24.0 * (double)d.n : 0.0;
    if (d.csc) return 12.0 * (double)d.nnz + 17.0 * (double)d.n + 8.0 * (double)d.m + dvx;
    return 8.0 * (double)ny * (double)d.n + 9.0 * (double)d.n + 12.0 * (double)ny + dvx;
}

// CSC pricing: one workgroup = one tile of TILE_COLS columns, one thread per
// column.  The tile's nonzeros are contiguous in the CSC arrays: the workgroup
// stages them in LDS with coalesced loads (value, and y gathered at the row
// index), then each thread runs its column's fma chain from LDS in ascending
// row order (oracle price_mode 1).  Tiles with more than CSC_STAGE nonzeros
// read straight from global memory (same order).
// staged nonzeros per tile: 16 KiB of LDS (2048 / 32 KiB until r04: the LDS
// limited the launch -- its deferred-update workgroups too -- to 2 waves per
// SIMD; 1024 measured 5 % faster on the sparse LPs, r04q)
#ifndef ELP_CSC_STAGE
#define ELP_CSC_STAGE 1024
#endif
constexpr int CSC_STAGE = ELP_CSC_STAGE;
DEV void price_csc_body(const Dev& d, int napply, int nb_minv, int nsw);
template <bool TIMED = false>
__global__ void __launch_bounds__(TILE_COLS) k_price_csc(Dev d, int napply, int nb_minv, int nsw, int tslot) {
    if (TIMED) tstamp_begin(d, tslot);
    pstamp_begin<TILE_COLS>(d);
    price_csc_body(d, napply, nb_minv, nsw);
    pstamp_end(d);
    if (TIMED) tstamp_end(d, tslot);
}
DEV void price_csc_body(const Dev& d, int napply, int nb_minv, int nsw) {
    __shared__ double sv[CSC_STAGE], sy[CSC_STAGE];
    __shared__ Cand red[TILE_COLS / 64];
    if ((int)blockIdx.x >= (int)gridDim.x - napply) {  // (apply_role; the sparse update under Dev::sru_on)
        PDBG(1, 1ull);
        const DevCtl* cc = d.ctl;
        if (plan_pending(cc) && cc->status != ST_NUMFAIL) {
            const Plan P = cc->plan;
            const int blk = (int)blockIdx.x - ((int)gridDim.x - napply);
            if (d.sru_on && blk < nb_minv) apply_minv_sru<TILE_COLS>(d, P, blk, nb_minv);
            else apply_plan(d, P, blk, napply, nb_minv, false, true);
        }
        return;
    }
    const DevCtl* c = d.ctl;
    const int64_t ntiles = gridDim.x - napply - nsw;
    const bool tilewg = (int64_t)blockIdx.x < ntiles;
    // the tile's extent and this column's (start, end, status, cost) issued
    // with the control block's loads (straight-line: one round trip, not three)
    const int64_t j0 = tilewg ? (int64_t)blockIdx.x * TILE_COLS : 0;
    const int64_t j = j0 + threadIdx.x;
    const int64_t jend = j0 + TILE_COLS < d.n ? j0 + TILE_COLS : d.n;
    const int64_t jc = j < d.n ? j : (d.n > 0 ? d.n - 1 : 0);
    const int64_t s0 = d.cptr[j0], s1 = d.cptr[jend];
    const int64_t a = d.cptr[jc], b = d.cptr[jc + 1];
    const int8_t vsj = d.vstat[jc];
    const double cj = d.cost[jc];
    const double dwj = d.dw ? d.dw[jc] : 1.0, dpj = d.dprev ? d.dprev[jc] : 0.0;
    const int cdevex = c->devex;  // (the control fields the epilogue needs, with the status)
    const DevexIn cdx = devex_in(c);
    const double ctold = c->tol_dual;
    __builtin_amdgcn_sched_barrier(0);
    if (c->status != ST_RUN) {
        KEEP(s0);
        KEEP(a);
        KEEP(cj);
        KEEP(dwj);
        return;
    }
    if (!tilewg) {  // a slack workgroup
        PDBG(1, 2ull);
        price_slacks<TILE_COLS>(d, ntiles, (int)(blockIdx.x - ntiles), nsw, red);
        return;
    }
    PDBG(1, __builtin_amdgcn_s_memrealtime());
    const int bland = c->bland;
    const bool staged = s1 - s0 <= CSC_STAGE;
    if (staged && s1 > s0) {  // (<= CSC_STAGE / TILE_COLS entries per thread: every gather in flight at once)
        constexpr int SPT = CSC_STAGE / TILE_COLS;
        int ii[SPT];
        double vv[SPT], yv[SPT];
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const int64_t t = s0 + threadIdx.x + (int64_t)u * TILE_COLS;
            const int64_t tc = t < s1 ? t : s1 - 1;  // (s1 > s0: an entry of the tile)
            ii[u] = d.rind[tc];
            vv[u] = d.cval[tc];
        }
#pragma unroll
        for (int u = 0; u < SPT; ++u) yv[u] = d.y[ii[u]];
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const int64_t t = s0 + threadIdx.x + (int64_t)u * TILE_COLS;
            if (t < s1) {
                sv[t - s0] = vv[u];
                sy[t - s0] = yv[u];
            }
        }
        __syncthreads();
    }
    PDBG(2, __builtin_amdgcn_s_memrealtime());
    double acc = 0.0;
    if (j < d.n) {
        if (staged) {
            for (int64_t t = a - s0; t < b - s0; ++t) acc = fma(sv[t], sy[t], acc);
        } else {
            for (int64_t t = a; t < b; ++t) acc = fma(d.cval[t], d.y[d.rind[t]], acc);
        }
    }
    Cand best;
    best.j = -1;
    best.score = 0.0;
    best.d = 0.0;
    best.w = 1.0;
    if (j < d.n) {
        const int8_t vs = vsj;
        if (vs != VS_BASIC && vs != VS_FIXED) {
            const double dj = cj - acc;
            const double wj = cdevex ? devex_weight(d, cdx, j, d.col0 + j, dj, dwj, dpj) : 1.0;
            best = price_cand(vs, dj, wj, cdevex, ctold, d.col0 + j);
        }
    }
    PDBG(3, __builtin_amdgcn_s_memrealtime());
    best = block_best<TILE_COLS>(best, bland, red);
    PDBG(4, __builtin_amdgcn_s_memrealtime());
    if (threadIdx.x == 0) d.cand[blockIdx.x] = best;
}

// CSC: a_R[p] = A[R_p, q] by scattering column q's nonzeros through rpos
// (block-wide; aR zeroed first).  Structural q only.
DEV void scatter_aR_csc(const Dev& d, int q, double* aR, int k) {
    for (int p = threadIdx.x; p < k; p += blockDim.x) aR[p] = 0.0;
    __syncthreads();
    const int64_t jl = (int64_t)q - d.col0;
    for (int64_t t = d.cptr[jl] + threadIdx.x; t < d.cptr[jl + 1]; t += blockDim.x) {
        const int p = d.rpos[d.rind[t]];
        if (p >= 0 && p < k) aR[p] = d.cval[t];
    }
}

// CSC: replace the dense copy of the previous entering column in qcol by
// column q (one workgroup; q < 0 or a slack: just clear)
DEV void scatter_qcol_csc(const Dev& d, int q) {
    DevCtl* c = d.ctl;
    const int prev = c->qcol_var;
    if (prev >= 0 && prev < d.N) {
        const int64_t pl = (int64_t)prev - d.col0;
        for (int64_t t = d.cptr[pl] + threadIdx.x; t < d.cptr[pl + 1]; t += blockDim.x) d.qcol[d.rind[t]] = 0.0;
    }
    __syncthreads();
    if (q >= 0 && q < d.N) {
        const int64_t jl = (int64_t)q - d.col0;
        for (int64_t t = d.cptr[jl] + threadIdx.x; t < d.cptr[jl + 1]; t += blockDim.x) d.qcol[d.rind[t]] = d.cval[t];
    }
    if (threadIdx.x == 0) c->qcol_var = q;
}

// Pricing-launch timer: first start to last end over the stamps of every
// workgroup of the last pricing launch (one workgroup of NT threads), added to
// the control block with the pass's bytes.
template <int NT>
DEV void price_timer_sum(const Dev& d, unsigned long long* red) {
    __syncthreads();  // red may still be read by the preceding reduction
    const int nwg = d.ctl->price_grid;
    unsigned long long lo = ~0ull, hi = 0;
    for (int t = threadIdx.x; t < nwg; t += NT) {
        lo = min(lo, d.pstamp[PSTRIDE * t]);
        hi = max(hi, d.pstamp[PSTRIDE * t + PSTRIDE - 1]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        lo = min(lo, (unsigned long long)__shfl_xor(lo, off));
        hi = max(hi, (unsigned long long)__shfl_xor(hi, off));
    }
    if ((threadIdx.x & 63) == 0) {
        red[2 * (threadIdx.x >> 6)] = lo;
        red[2 * (threadIdx.x >> 6) + 1] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < NT / 64; ++w) {
            lo = min(lo, red[2 * w]);
            hi = max(hi, red[2 * w + 1]);
        }
        DevCtl* c = d.ctl;
        const int ny = c->ny;
        c->price_ticks += hi - lo;
        c->price_timed++;
        c->price_tbytes += price_pass_bytes(d, ny, c->devex);
    }
}

// ============================================================== select
// debug stamps (Dev::dstamp, ELP_STAMPS): s_memrealtime at the phases of workgroup 0
#define RSTAMP(i) do { if (ELP_DIAG && d.dstamp && blockIdx.x == 0 && threadIdx.x == 0) \
    d.dstamp[dslot * DSTAMP_STRIDE + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// k_dual_bfrt's stamps go to LDS (s_st) and out at the end of the launch: a
// global store mid-launch would make the next barrier wait for its ack
#define BSTAMP(i) do { if (ELP_DIAG && s_st && threadIdx.x == 0) s_st[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
constexpr int MAX_P2P = 64;  // ranks a mailbox exchange supports

// xGMI mailbox min-loc (Dev::p2p, column-sharded with A replicated): workgroup
// 0 publishes this rank's best candidate -- with the column's (lb, ub, x, cost)
// when it is one of this shard's structurals -- into slot [parity][rank] of
// every rank's mailbox (fields, system-scope fence, then the sequence word);
// every workgroup waits until all slots of this iteration carry its sequence
// number and reduces them with the candidate total order, so all ranks agree.
// Returns false (status ST_COMMFAIL) if a peer stays silent for Dev::mb_ticks
// (elp_control.mailbox_timeout).
DEV bool p2p_exchange(const Dev& d, Cand& best, int bland, int64_t iter, int64_t epoch, CandX* s_rec,
                      int* s_fail) {
    const int P = d.world;
    const int par = (int)(iter & 1);
    const int64_t want = (epoch << 40) | (iter + 1);
    if (threadIdx.x == 0) *s_fail = 0;
    if (blockIdx.x == 0 && (int)threadIdx.x < P) {  // thread t writes our slot in rank t's mailbox
        CandX x;
        x.c = best;
        x.lb = x.ub = x.x = x.cost = 0.0;
        const int ql = best.j >= 0 && best.j < d.N ? loc_of(d, (int)best.j) : -1;
        if (ql >= 0) {
            x.lb = d.lb[ql];
            x.ub = d.ub[ql];
            x.x = d.xval[ql];
            x.cost = d.cost[ql];
        }
        MboxRec* r = d.mpeers[threadIdx.x] + par * P + d.rank;
        r->x = x;
        __threadfence_system();
        __hip_atomic_store(&r->seq, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    if ((int)threadIdx.x < P) {  // thread t waits for rank t's record, then stages it in LDS
        MboxRec* r = d.mbox + par * P + threadIdx.x;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        while (__hip_atomic_load(&r->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)d.mb_ticks) {  // 100 MHz clock
                ok = false;
                break;
            }
        }
        if (!ok) {
            atomicOr(s_fail, 1);
        } else {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            CandX x;
            x.c.score = __hip_atomic_load(&r->x.c.score, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.c.d = __hip_atomic_load(&r->x.c.d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.c.w = __hip_atomic_load(&r->x.c.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.c.j = __hip_atomic_load(&r->x.c.j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.lb = __hip_atomic_load(&r->x.lb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.ub = __hip_atomic_load(&r->x.ub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.x = __hip_atomic_load(&r->x.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            x.cost = __hip_atomic_load(&r->x.cost, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_rec[threadIdx.x] = x;
        }
    }
    __syncthreads();
    if (*s_fail) {
        if (blockIdx.x == 0 && threadIdx.x == 0) d.ctl->status = ST_COMMFAIL;
        return false;
    }
    int win = 0;
    for (int r = 1; r < P; ++r)
        if (cand_better(s_rec[r].c, s_rec[win].c, bland)) win = r;
    best = s_rec[win].c;
    if (blockIdx.x == 0 && threadIdx.x == 0 && best.j >= 0 && best.j < d.N) {
        const int m = d.m;  // the column's scalars for k_ratio (sharded: read from pkt)
        d.pkt[m] = s_rec[win].lb;
        d.pkt[m + 1] = s_rec[win].ub;
        d.pkt[m + 2] = s_rec[win].x;
        d.pkt[m + 3] = s_rec[win].cost;
    }
    return true;
}

// Min-loc over this shard's tile candidates and the (replicated) slack
// candidates.  One GPU: decide q and form a_R.  Sharded: write the local best
// to cand_xchg[rank] for the all-gather (k_select_global decides).
DEV Cand local_best(const Dev& d, int ncand, Cand* red) {
    const DevCtl* c = d.ctl;
    const int bland = c->bland;
    Cand best;
    best.j = -1;
    best.score = 0.0;
    best.d = 0.0;
    best.w = 1.0;
    for (int t = threadIdx.x; t < ncand; t += 1024) {  // tiles, then the slack workgroups'
        const Cand o = d.cand[t];
        cand_take(best, o, cand_better(o, best, bland));
    }
    return block_best<1024>(best, bland, red);
}

// the statistics of this iteration's pricing pass and of the whole iteration:
// read-modify-writes of control-block fields, so the thread that runs them
// waits a round trip -- kept off the select kernel's critical path (after its
// own bump rows)
DEV void entering_stats(const Dev& d) {
    DevCtl* c = d.ctl;
    const int ny = c->ny;
    // algorithmic bytes of this pricing pass: AR sweep + c + status + y_Y + Yl
    const double pb = price_pass_bytes(d, ny, c->devex);
    c->price_bytes += pb;
    c->price_passes++;
    // the whole iteration: + select 8k^2, FTRAN-z 8mk, ratio
    // 8k^2 + 16n, deferred update 32k^2 + 16m
    const double kk = (double)c->k, mm = (double)d.m, nn = (double)d.n;
    c->iter_bytes += pb + 48.0 * kk * kk + 8.0 * mm * kk + 16.0 * nn + 16.0 * mm;
}
DEV void entering_chosen(const Dev& d, const Cand& best) {
    DevCtl* c = d.ctl;
    c->q = (int)best.j;
    c->dq = best.d;
    c->wq = best.w;
    c->sig = best.d < 0.0 ? 1.0 : -1.0;
}

// a_R = entering column on the bump rows
DEV void gather_aR(const Dev& d, int q, const double* qcol) {
    const int k = d.ctl->k;
    if (q < d.N) {
        for (int p = threadIdx.x; p < k; p += blockDim.x) d.aR[p] = qcol_at(d, qcol, q, d.Rl[p]);
    } else {
        const int i0 = q - d.N;
        for (int p = threadIdx.x; p < k; p += blockDim.x) d.aR[p] = d.Rl[p] == i0 ? 1.0 : 0.0;
    }
}

// dual != 0 (the dual phase): q is k_dual_bfrt's (candidate 0), which also set
// the control block's entering fields and the statistics
__global__ void __launch_bounds__(1024) k_select(Dev d, int ntiles, int nsw, int dual) {
    __shared__ Cand red[16];
    DevCtl* c = d.ctl;
    if (threadIdx.x == 0) c->applied_seq = c->plan_seq;  // the pricing launch applied it
    if (c->status != ST_RUN) return;
    Cand best = local_best(d, ntiles + nsw, red);
    if (d.p2p && !dual) {  // column-sharded: global min-loc over the xGMI mailbox
        __shared__ CandX s_rec[MAX_P2P];
        __shared__ int s_fail;
        if (!p2p_exchange(d, best, c->bland, c->iter, c->mb_epoch, s_rec, &s_fail)) return;
    }
    if (best.j < 0) {
        if (threadIdx.x == 0) c->status = ST_PHASE_OPT;
        return;
    }
    const int q = (int)best.j;
    if (threadIdx.x == 0 && !dual) {
        entering_chosen(d, best);
        entering_stats(d);
    }
    if (ELP_DIAG && d.ptimer) price_timer_sum<1024>(d, reinterpret_cast<unsigned long long*>(red));
    if (d.csc) {  // dense copy of the entering column + a_R through rpos
        scatter_qcol_csc(d, q);
        if (q < d.N) {
            __syncthreads();
            scatter_aR_csc(d, q, d.aR, d.ctl->k);
            return;
        }
    }
    // the full column is read in place by k_ftran_zr / k_update
    gather_aR(d, q, q < d.N ? qcolumn(d, q) : nullptr);
}

// A[Rl[p], q] of a CSC column by binary search over its rows (ascending)
DEV double csc_at(const Dev& d, int64_t jl, int row) {
    int64_t lo = d.cptr[jl], hi = d.cptr[jl + 1] - 1;
    while (lo <= hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int r = d.rind[mid];
        if (r == row) return d.cval[mid];
        if (r < row) lo = mid + 1;
        else hi = mid - 1;
    }
    return 0.0;
}

// CSC, large bump (k_ub > Dev::spf_min): alpha_S = Minv a_R and (dual == 2 with
// flips) fS = Minv a_F[R] from lane-bucketed sparse lists -- a_R from column
// q's rows through rpos, a_F[R] from k_dual_bfrt's list -- one wave per bump
// row (rows pr, pr + 4 nrw, ...), the dense chains' bits (sparse_lane_chain).
// A column with more than SPL entries / no a_F list: the dense chain over an
// operand staged in global memory (d.aR / d.zz; every workgroup writes the same
// final values, no intermediate state)
DEV void select_ftran_sparse(const Dev& d, int q, int k, int pr, int nrw, int dual) {
    __shared__ int s_pos[2][SPL], s_key[SPL], s_sb[2][72], s_scan[4];
    __shared__ double s_val[2][SPL];
    const int tid = threadIdx.x, lane = tid & 63;
    bool dense_a = false;
    {
        bool valid = false;
        int p = 0;
        double v = 0.0;
        if (q < d.N) {
            const int64_t jl = (int64_t)q - d.col0;
            const int64_t t0 = d.cptr[jl], t1 = d.cptr[jl + 1];
            dense_a = t1 - t0 > SPL;
            if (!dense_a && tid < t1 - t0) {
                const int i = d.rind[t0 + tid];
                v = d.cval[t0 + tid];
                p = d.rpos[i];
                valid = p >= 0 && p < k;
            }
        } else if (tid == 0) {
            p = d.rpos[q - d.N];
            v = 1.0;
            valid = p >= 0 && p < k;
        }
        if (dense_a) {
            const int64_t jl = (int64_t)q - d.col0;
            for (int pp = tid; pp < k; pp += 256) d.aR[pp] = csc_at(d, jl, d.Rl[pp]);
        } else {
            spl_build<256>(valid, p, v, s_pos[0], s_val[0], s_sb[0], s_key, s_scan);
        }
    }
    const bool ffs = dual == 2 && d.ctl->nflip > 0;
    const int nf = ffs ? d.afl[0] : -1;
    if (ffs && nf >= 0) {
        for (int t = tid; t < nf; t += 256) {
            s_pos[1][t] = d.afl[AFL_POS + t];
            s_val[1][t] = d.aflv[t];
        }
        if (tid <= 64) s_sb[1][tid] = d.afl[AFL_SB + tid];
    } else if (ffs) {
        for (int pp = tid; pp < k; pp += 256) d.zz[pp] = d.aF[d.Rl[pp]];
    }
    __syncthreads();
    for (int p2 = pr; p2 < k; p2 += 4 * nrw) {
        const double* row = d.Minv + (size_t)p2 * d.ldm;
        const double a =
            wave_tree(dense_a ? lane_chain(row, d.aR, k) : sparse_lane_chain(row, s_pos[0], s_val[0], s_sb[0]));
        if (lane == 0) d.alS[p2] = a;
        if (ffs) {
            const double f =
                wave_tree(nf >= 0 ? sparse_lane_chain(row, s_pos[1], s_val[1], s_sb[1]) : lane_chain(row, d.zz, k));
            if (lane == 0) d.fS[p2] = f;
        }
    }
}

// One GPU, fused select + FTRAN on the bump: every workgroup reduces the tile and
// slack candidates itself (a total order: all agree), gathers a_R into LDS and
// computes alpha_S for its 4 bump rows (one wave per row, wave order).
// Workgroup 0 publishes q.  Saves a launch and the single-workgroup select.
// nrw: the bump-row workgroups (the host's cdiv(k_ub, 4), or Dev::sel_cap):
// workgroup b forms rows 4b + wave, 4b + wave + 4 nrw, ...
// nqz: the staging workgroups after them (Dev::qz; 0: none), QZ_PT rows per thread
constexpr int QZ_PT = 8;
// SP: the CSC sparse FTRAN (select_ftran_sparse) after the min-loc
template <int PFM, bool SP = false>  // Minv values per lane held in registers (k <= 64 PFM): 8 or 16 by the host's bound
__global__ void __launch_bounds__(256) k_select_ftran(Dev d, int ntiles, int nsw, int k_ub, int dslot, int nrw,
                                                      int nqz, int dual) {
    extern __shared__ __attribute__((aligned(16))) double aRs[];  // [k]
    __shared__ Cand red[4];
    RSTAMP(12);
    DevCtl* c = d.ctl;
    // the control block first (vmcnt retires in issue order: the status test
    // then waits for these loads only, not for the prefetch behind them)
    const int32_t st0 = c->status;
    int bland = c->bland, k = c->k;  // (pinned below)
    // (iter / mb_epoch are read by the p2p path only, after the min-loc: loaded
    //  here, their registers were reused before the loads retired -> a full wait)
    const int32_t c_seq = c->plan_seq;
    // Everything that does not depend on the control block or on q goes out
    // first (bounded by the host's k_ub, masked below): the candidates of the
    // tiles and of the slacks (candidates [ntiles, ntiles + nsw), k_price's slack workgroups),
    // this wave's row of Minv, the R list.  After the min-loc only the a_R
    // gather is left.
    constexpr int PFR = 4;  // R-list entries per thread (k <= 1024)
    constexpr int PFC = 4;  // candidates per thread (<= 1023 tiles)
    const int ncand = ntiles + nsw;
    const bool qzw = (int)blockIdx.x >= nrw && (int)blockIdx.x < nrw + nqz;  // a staging workgroup
    const int pr = qzw ? k_ub : blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const bool pfm = k_ub <= 64 * PFM, pfr = k_ub <= 256 * PFR;
    const bool pfc = ncand <= 256 * PFC;
    double mrow[PFM];
    int rl[PFR];
    Cand cc[PFC];
    // (unconditional, no branch around them: a load inside a conditional block
    //  is drained at the block's end; masks are applied where values are used)
#pragma unroll
    for (int t = 0; t < PFC; ++t) cc[t] = ld_clamp(d.cand, tid + 256 * t, ncand);
    {  // (read by the dense register path only: past it every lane loads element 0)
        const int mlim = !SP && pfm ? k_ub : 1;
        const double* row = d.Minv + (size_t)(pr < k_ub ? pr : 0) * d.ldm;
#pragma unroll
        for (int t = 0; t < PFM; ++t) mrow[t] = ld_clamp(row, lane + 64 * t, mlim);
    }
#pragma unroll
    for (int t = 0; t < PFR; ++t) rl[t] = ld_clamp(d.Rl, tid + 256 * t, k_ub);
    __builtin_amdgcn_sched_barrier(0);  // all of the above issued before any use
    asm volatile("" : "+v"(bland), "+v"(k));  // (their scalar copies stay below the prefetch)
    if (blockIdx.x == 0 && threadIdx.x == 0) c->applied_seq = c_seq;  // applied by k_price
    if (st0 != ST_RUN) {
#pragma unroll
        for (int t = 0; t < PFC; ++t) KEEP(cc[t].score);
#pragma unroll
        for (int t = 0; t < PFM; ++t) KEEP(mrow[t]);
#pragma unroll
        for (int t = 0; t < PFR; ++t) KEEP(rl[t]);
        return;
    }
    RSTAMP(13);
    Cand best;
    best.j = -1;
    best.score = 0.0;
    best.d = 0.0;
    best.w = 1.0;
    if (pfc) {
#pragma unroll
        for (int t = 0; t < PFC; ++t)
            cand_take(best, cc[t], tid + 256 * t < ncand && cand_better(cc[t], best, bland));
    } else {  // many tiles (one GPU holding n = 500 000): batches of 8 loads in flight
        for (int t0 = tid; t0 < ncand; t0 += 256 * 8) {
            Cand o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = ld_clamp(d.cand, t0 + 256 * u, ncand);
#pragma unroll
            for (int u = 0; u < 8; ++u) cand_take(best, o[u], t0 + 256 * u < ncand && cand_better(o[u], best, bland));
        }
    }
    best = block_best<256>(best, bland, red);
    if (d.p2p && !dual) {  // column-sharded: global min-loc over the xGMI mailbox
        __shared__ CandX s_rec[MAX_P2P];
        __shared__ int s_fail;
        if (!p2p_exchange(d, best, bland, c->iter, c->mb_epoch, s_rec, &s_fail)) return;
    }
    if (best.j < 0) {
        if (blockIdx.x == 0 && tid == 0) c->status = ST_PHASE_OPT;
        return;
    }
    RSTAMP(14);
    const int q = (int)best.j;
    if (blockIdx.x == 0 && tid == 0 && !dual) entering_chosen(d, best);  // (dual: k_dual_bfrt chose q)
    if (ELP_DIAG && d.ptimer && blockIdx.x == gridDim.x - 1) {  // the extra timer workgroup
        price_timer_sum<256>(d, reinterpret_cast<unsigned long long*>(aRs));
        return;
    }
    if (d.csc && blockIdx.x == gridDim.x - 1 - (ELP_DIAG ? d.ptimer : 0)) {  // CSC: dense entering column
        scatter_qcol_csc(d, q);
        return;
    }
    if (qzw) {  // stage the entering column for k_ftran_zr (QZ_PT loads in flight)
        const int m = d.m;
        const int i0 = (int)(blockIdx.x - nrw) * 256 * QZ_PT + tid;
        if (q < d.N) {
            const double* col = qcolumn(d, q);
            double v[QZ_PT];
#pragma unroll
            for (int t = 0; t < QZ_PT; ++t) v[t] = col[min(i0 + 256 * t, m - 1)];
#pragma unroll
            for (int t = 0; t < QZ_PT; ++t) {
                const int i = i0 + 256 * t;
                if (i < m) d.qz[i] = col == d.pkt ? v[t] : sca(d, v[t], i, q);
            }
        } else {
#pragma unroll
            for (int t = 0; t < QZ_PT; ++t) {
                const int i = i0 + 256 * t;
                if (i < m) d.qz[i] = i == q - d.N ? 1.0 : 0.0;
            }
        }
        return;
    }
    if constexpr (SP) {
        select_ftran_sparse(d, q, k, pr, nrw, dual);
        if (blockIdx.x == 0 && tid == 0 && !dual) entering_stats(d);
        return;
    }
    if (q < d.N && d.csc) {
        scatter_aR_csc(d, q, aRs, k);
    } else if (q < d.N) {
        const double* col = qcolumn(d, q);
        if (pfr) {
            double g[PFR];
#pragma unroll
            for (int t = 0; t < PFR; ++t) g[t] = col[tid + 256 * t < k ? rl[t] : 0];  // straight-line
#pragma unroll
            for (int t = 0; t < PFR; ++t)
                if (tid + 256 * t < k) aRs[tid + 256 * t] = d.srow && col != d.pkt ? sca(d, g[t], rl[t], q) : g[t];
        } else {
            for (int p = tid; p < k; p += 256) aRs[p] = qcol_at(d, col, q, d.Rl[p]);
        }
    } else {
        const int i0 = q - d.N;
        if (pfr) {
#pragma unroll
            for (int t = 0; t < PFR; ++t)
                if (tid + 256 * t < k) aRs[tid + 256 * t] = rl[t] == i0 ? 1.0 : 0.0;
        } else {
            for (int p = tid; p < k; p += 256) aRs[p] = d.Rl[p] == i0 ? 1.0 : 0.0;
        }
    }
    // dual == 2 (CSC dual pivot with the row-wise flip update): the flips' bump
    // FTRAN fS = Minv a_F[R] rides here too (k_dual_flip_bump's chains, the
    // second k_ub doubles of LDS holding a_F[R])
    const bool ffs = dual == 2 && c->nflip > 0;
    double* afr = aRs + k_ub;
    if (ffs)
        for (int p = tid; p < k; p += 256) afr[p] = d.aF[d.Rl[p]];
    __syncthreads();
    const bool stats_here = blockIdx.x == 0 && tid == 0 && !dual;
    if (pr >= k) {
        if (stats_here) entering_stats(d);
        return;
    }
    double acc = 0.0;
    if (pfm) {
#pragma unroll
        for (int t = 0; t < PFM; ++t)
            if (lane + 64 * t < k) acc = fma(mrow[t], aRs[lane + 64 * t], acc);
    } else {
        const double* row = d.Minv + (size_t)pr * d.ldm;
        acc = lane_chain(row, aRs, k);
    }
    acc = wave_tree(acc);
    if (lane == 0) d.alS[pr] = acc;
    if (ffs) {
        const double f = wave_tree(lane_chain(d.Minv + (size_t)pr * d.ldm, afr, k));
        if (lane == 0) d.fS[pr] = f;
    }
    // (capped grid only) the rows past the first 4 nrw, from memory
    for (int p2 = pr + 4 * nrw; p2 < k; p2 += 4 * nrw) {
        double a2 = lane_chain(d.Minv + (size_t)p2 * d.ldm, aRs, k);
        a2 = wave_tree(a2);
        if (lane == 0) d.alS[p2] = a2;
        if (ffs) {
            const double f = wave_tree(lane_chain(d.Minv + (size_t)p2 * d.ldm, afr, k));
            if (lane == 0) d.fS[p2] = f;
        }
    }
    if (stats_here) entering_stats(d);
    RSTAMP(15);
}

__global__ void __launch_bounds__(1024) k_select_local(Dev d, int ntiles, int nsw, int rank) {
    __shared__ Cand red[16];
    DevCtl* c = d.ctl;
    if (threadIdx.x == 0) c->applied_seq = c->plan_seq;  // applied by k_price
    if (c->status != ST_RUN) return;
    const Cand best = local_best(d, ntiles + nsw, red);
    if (threadIdx.x == 0) {
        CandX x;
        x.c = best;
        x.lb = x.ub = x.x = x.cost = 0.0;
        const int ql = best.j >= 0 && best.j < d.N ? loc_of(d, (int)best.j) : -1;
        if (ql >= 0) {
            x.lb = d.lb[ql];
            x.ub = d.ub[ql];
            x.x = d.xval[ql];
            x.cost = d.cost[ql];
        }
        d.cand_xchg[rank] = x;
    }
    if (ELP_DIAG && d.ptimer) price_timer_sum<1024>(d, reinterpret_cast<unsigned long long*>(red));
}

// after the all-gather: global min-loc (same total order on every rank); the
// owner of a structural q packs its column + (lb, ub, x, cost), others zeros
__global__ void __launch_bounds__(256) k_select_global(Dev d) {
    DevCtl* c = d.ctl;
    if (c->status != ST_RUN) return;
    const int bland = c->bland;
    Cand best = d.cand_xchg[0].c;
    for (int r = 1; r < d.world; ++r)
        cand_take(best, d.cand_xchg[r].c, cand_better(d.cand_xchg[r].c, best, bland));
    const int m = d.m;
    if (best.j < 0) {
        for (int i = threadIdx.x; i < m + 4; i += 256) d.pkt[i] = 0.0;
        if (threadIdx.x == 0) c->status = ST_PHASE_OPT;
        return;
    }
    const int q = (int)best.j;
    const int ql = loc_of(d, q);
    const bool own = q < d.N && ql >= 0;
    if (d.Afull) {  // replicated: the column is read in place, pkt carries the scalars
        if (threadIdx.x == 0) {
            int win = 0;
            for (int r = 1; r < d.world; ++r)
                if (cand_better(d.cand_xchg[r].c, d.cand_xchg[win].c, bland)) win = r;
            d.pkt[m] = d.cand_xchg[win].lb;
            d.pkt[m + 1] = d.cand_xchg[win].ub;
            d.pkt[m + 2] = d.cand_xchg[win].x;
            d.pkt[m + 3] = d.cand_xchg[win].cost;
        }
    } else if (own) {
        const double* col = d.A + (size_t)ql * (size_t)m;
        for (int i = threadIdx.x; i < m; i += 256) d.pkt[i] = sca(d, col[i], i, q);
        if (threadIdx.x == 0) {
            d.pkt[m] = d.lb[ql];
            d.pkt[m + 1] = d.ub[ql];
            d.pkt[m + 2] = d.xval[ql];
            d.pkt[m + 3] = d.cost[ql];
        }
    } else {
        for (int i = threadIdx.x; i < m + 4; i += 256) d.pkt[i] = 0.0;
    }
    if (threadIdx.x == 0) {
        entering_chosen(d, best);
        entering_stats(d);
    }
}

// after the all-reduce of pkt: a_R from the exchanged column
__global__ void __launch_bounds__(1024) k_select_finish(Dev d) {
    const DevCtl* c = d.ctl;
    if (c->status != ST_RUN) return;
    gather_aR(d, c->q, c->q < d.N ? qcolumn(d, c->q) : nullptr);
}

// Replicated A, after the all-gather of the ranks' records: every workgroup
// takes the global min-loc (a total order: all agree), reads a_R from its own
// copy of A and forms alpha_S for its 4 bump rows (k_select_ftran's shape).
// Workgroup 0 publishes q and the column's (lb, ub, x, cost) in pkt[m..m+3].
__global__ void __launch_bounds__(256) k_select_xftran(Dev d) {
    extern __shared__ __attribute__((aligned(16))) double aRs[];  // [k]
    DevCtl* c = d.ctl;
    if (c->status != ST_RUN) return;
    const int bland = c->bland, k = c->k, m = d.m;
    int win = 0;
    for (int r = 1; r < d.world; ++r)
        if (cand_better(d.cand_xchg[r].c, d.cand_xchg[win].c, bland)) win = r;
    const Cand best = d.cand_xchg[win].c;
    if (best.j < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) c->status = ST_PHASE_OPT;
        return;
    }
    const int q = (int)best.j;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const CandX& x = d.cand_xchg[win];
        d.pkt[m] = x.lb;
        d.pkt[m + 1] = x.ub;
        d.pkt[m + 2] = x.x;
        d.pkt[m + 3] = x.cost;
        entering_chosen(d, best);
        entering_stats(d);
    }
    if (q < d.N) {
        const double* col = d.Afull + (size_t)q * (size_t)m;
        for (int p = threadIdx.x; p < k; p += 256) aRs[p] = sca(d, col[d.Rl[p]], d.Rl[p], q);
    } else {
        const int i0 = q - d.N;
        for (int p = threadIdx.x; p < k; p += 256) aRs[p] = d.Rl[p] == i0 ? 1.0 : 0.0;
    }
    __syncthreads();
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= k) return;
    const double* row = d.Minv + (size_t)p * d.ldm;
    double acc = lane_chain(row, aRs, k);
    acc = wave_tree(acc);
    if (lane == 0) d.alS[p] = acc;
}

// ============================================================== FTRAN
// out[p] = wave_dot(Minv[p, 0:k], vin[0:k]) -- one wave per bump row
__global__ void __launch_bounds__(256) k_ftran_bump(Dev d, const double* __restrict__ vin,
                                                    double* __restrict__ out, int check_run) {
    if (check_run && d.ctl->status != ST_RUN) return;
    const int k = d.ctl->k;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= k) return;
    const double* row = d.Minv + (size_t)p * d.ldm;
    double acc = 0.0;
    for (int i = lane; i < k; i += 64) acc = fma(row[i], vin[i], acc);
    acc = wave_tree(acc);
    if (lane == 0) out[p] = acc;
}

// zpart[c][i] = sum_{p in chunk c} AS[i][p] * w[p]  (ZCHUNK positions per chunk)
__global__ void __launch_bounds__(256) k_ftran_z(Dev d, const double* __restrict__ wv, int check_run) {
    if (check_run && d.ctl->status != ST_RUN) return;
    const int k = d.ctl->k;
    const int ch = blockIdx.y;
    const int c0 = ch * ZCHUNK;
    if (c0 >= k) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    const int c1 = min(k, c0 + ZCHUNK);
    const double* col = d.AS + (size_t)c0 * (size_t)d.m + i;
    const size_t m = (size_t)d.m;
    double acc = 0.0;
    int p = c0;
    for (; p + 16 <= c1; p += 16) {
        double a[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u] = col[(size_t)(p - c0 + u) * m];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc = fma(a[u], wv[p + u], acc);
    }
    for (; p < c1; ++p) acc = fma(col[(size_t)(p - c0) * m], wv[p], acc);
    d.zpart[(size_t)ch * m + i] = acc;
}

// x_u = sign * (v_i - z_i) on covered rows after a refactor (z from k_ftran_z)
__global__ void k_xr_from_z(Dev d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    const int u = d.cover[i];
    if (u < 0) return;
    const int k = d.ctl->k;
    const int nch = (k + ZCHUNK - 1) / ZCHUNK;
    double z = 0.0;
    for (int ch = 0; ch < nch; ++ch) z = z + d.zpart[(size_t)ch * d.m + i];
    d.xr[i] = unit_sign(d, u, i) * (d.rhs[i] - z);
}

// FTRAN on covered rows fused with Harris pass 1.
// Row tiles: 64 rows x 4 waves; wave w forms the z partials of chunks
// w, w+4, ... (ZCHUNK bump positions each, fma chain in position order) in
// LDS; wave 0 adds them in chunk order (the oracle's zchunk order), forms
// alpha_u = sigma_u (a_iq - z_i), stores it and reduces its Harris pass-1
// ratio.  Bump tiles (after the row tiles) reduce pass 1 over alpha_S.
// One minimum per workgroup goes to blockmin[].
DEV double harris1(double g, double x, double l, double u, double ptol, double pivtol, int bland) {
    if (g > pivtol && l > -HUGE_VAL) return bland ? (x - l) / g : (x - l + ptol) / g;
    if (g < -pivtol && u < HUGE_VAL) return bland ? (u - x) / (-g) : (u - x + ptol) / (-g);
    return HUGE_VAL;
}

// exact (pass-2) ratio of an entry; +inf if it cannot limit the step
DEV double harris2(double g, double x, double l, double u, double pivtol) {
    if (g > pivtol && l > -HUGE_VAL) return (x - l) / g;
    if (g < -pivtol && u < HUGE_VAL) return (u - x) / (-g);
    return HUGE_VAL;
}
// keep entry e as a pass-2 candidate if its exact ratio <= the workgroup's
// pass-1 minimum (the global minimum can only be smaller).  Wave-collective:
// the wave's kept entries are compacted by ballot into its own region and the
// count stored alongside -- no atomic, so nothing waits for a reply.
DEV void emit_wave(const Dev& d, int region, int var, int e, double g, double x, double l, double u, double bmin,
                   double pivtol) {
    const double r = var >= 0 ? harris2(g, x, l, u, pivtol) : HUGE_VAL;
    const bool keep = var >= 0 && r <= bmin && r != HUGE_VAL;
    const unsigned long long mask = __ballot(keep);
    const int lane = threadIdx.x & 63;
    if (keep) {
        const int slot = __popcll(mask & ((1ull << lane) - 1ull));
        RCand cd;
        cd.g = g;
        cd.r = r;
        cd.l = l;
        cd.u = u;
        cd.var = var;
        cd.e = e;
        d.rcand[(size_t)region * RREG + slot] = cd;
    }
    if (lane == 0) d.rcnt[region] = __popcll(mask);
}

// the scalars k_ratio's bookkeeping needs, taken before anything of this
// iteration rewrites them (FTRAN-z's last workgroup; see DevCtl)
DEV void zr_snapshot(const Dev& d, int k, int q) {
    DevCtl* cw = d.ctl;
    const int ny = cw->ny, i0 = q - d.N;
    const int yl = ny > 0 ? d.Yl[ny - 1] : -1;
    cw->snap_ny = ny;
    cw->snap_apos = i0 >= 0 ? d.rpos[i0] : -1;
    cw->snap_ypos0 = i0 >= 0 ? d.ypos[i0] : -1;
    cw->snap_ylast = yl;  // (rpos[yl]: k_ratio loads it itself, one round trip fewer here)
    const int ql = loc_of(d, q);
    const bool pk = ql < 0 || (d.sharded && q < d.N);  // from the exchanged packet
    const int m = d.m, last = k - 1;
    cw->snap_lbq = pk ? d.pkt[m] : d.lb[ql];
    cw->snap_ubq = pk ? d.pkt[m + 1] : d.ub[ql];
    cw->snap_xq = pk ? d.pkt[m + 2] : d.xval[ql];
    cw->snap_cq = pk ? d.pkt[m + 3] : d.cost[ql];
    cw->snap_vsq = ql >= 0 ? d.vstat[ql] : VS_LOWER;
    cw->snap_csl = last >= 0 ? d.cS[last] : 0.0;
    cw->snap_slol = last >= 0 ? d.slo[last] : 0.0;
    cw->snap_shil = last >= 0 ? d.shi[last] : 0.0;
    cw->snap_sllast = last >= 0 ? d.Sl[last] : -1;
    cw->snap_rllast = last >= 0 ? d.Rl[last] : -1;
}

constexpr int SPZ_MAX = 16;  // basic entries of a row the CSC row walk keeps (more: the dense AS walk)

// Row i's entries in basic columns (CSR + spos) as (bump position, value),
// sorted by position: the row's extent r0 / r1 comes preloaded, ZB entries'
// column / value loads go out together and then their spos loads (two
// dependent round trips for a row of <= ZB nonzeros).  *over: more than
// SPZ_MAX basic entries (the caller walks AS densely).
#ifndef ELP_ZB
#define ELP_ZB 16
#endif
constexpr int ZB = ELP_ZB;
// (r05c A/B on the 20 000 x 100 000 phase-1 LP, profiles/r05c_ab_zr_variants.txt:
// the flips' row walk in the same lane as alpha_U's 24.4 us against 25.5 in
// waves of their own, and 28-31 us with 32 entries' loads per batch (ZB = 32:
// 256 VGPRs); r06 removed the one-lane-per-row kernel k_ftran_zr_sp, which
// k_ftran_zr_sq replaced in r05)
DEV int csr_basic(const Dev& d, int64_t r0, int64_t r1, int* pp, double* vv, bool* over) {
    int cnt = 0;
    *over = false;
    for (int64_t t0 = r0; t0 < r1 && !*over; t0 += ZB) {
        int jj[ZB], ps[ZB];
        double vr[ZB];
#pragma unroll
        for (int u = 0; u < ZB; ++u) {
            const int64_t tt = t0 + u < r1 ? t0 + u : r1 - 1;
            jj[u] = d.cind[tt];
            vr[u] = d.rval[tt];
        }
#pragma unroll
        for (int u = 0; u < ZB; ++u) ps[u] = d.spos[jj[u]];
#pragma unroll
        for (int u = 0; u < ZB; ++u) {
            if (t0 + u >= r1 || ps[u] < 0) continue;
            if (cnt == SPZ_MAX) {
                *over = true;
                break;
            }
            pp[cnt] = ps[u];
            vv[cnt] = vr[u];
            ++cnt;
        }
    }
    for (int a = 1; a < cnt; ++a) {  // insertion sort by position (a handful of entries)
        const int p = pp[a];
        const double v = vv[a];
        int b = a - 1;
        while (b >= 0 && pp[b] > p) {
            pp[b + 1] = pp[b];
            vv[b + 1] = vv[b];
            --b;
        }
        pp[b + 1] = p;
        vv[b + 1] = v;
    }
    return cnt;
}
// z = A[i, S] xs from csr_basic's entries in the oracle's zchunk order (an fma
// chain per 32-position chunk, the chunk sums added in order from 0) -- the
// dense AS walk's bits (its zero terms change nothing); over: the dense walk
DEV double zrow_chain(const Dev& d, int i, int k, const int* pp, const double* vv, int cnt, bool over,
                      const double* __restrict__ xs) {
    double z = 0.0;
    if (over) {
        const size_t m = (size_t)d.m;
        for (int c0 = 0; c0 < k; c0 += ZCHUNK) {
            double acc = 0.0;
            const int c1 = min(k, c0 + ZCHUNK);
            for (int p = c0; p < c1; ++p) acc = fma(d.AS[(size_t)p * m + i], xs[p], acc);
            z = z + acc;
        }
        return z;
    }
    double xv[SPZ_MAX];  // the x values, all loads in flight before the chain
#pragma unroll
    for (int e = 0; e < SPZ_MAX; ++e) xv[e] = xs[e < cnt ? pp[e] : 0];
    double acc = 0.0;
    int ch = -1;
#pragma unroll
    for (int e = 0; e < SPZ_MAX; ++e) {
        if (e >= cnt) break;
        const int pc = pp[e] / ZCHUNK;
        if (pc != ch) {
            if (ch >= 0) z = z + acc;
            acc = 0.0;
            ch = pc;
        }
        acc = fma(vv[e], xv[e], acc);
    }
    if (ch >= 0) z = z + acc;
    return z;
}

// FTRAN-z + Harris pass 1 for CSC input (the row walk): four lanes per row --
// a workgroup of 4 waves takes 64 rows, 16 per wave; each lane loads an
// interleaved quarter of its row's entries (<= ZQB per batch: one batch of
// column / value loads, then one of spos loads, for rows of <= 32 nonzeros --
// r05e stamps: the one-lane walk's two batches of 16 scattered loads each took
// ~19 us of the kernel), the quad's basic entries meet in LDS (up to ZSQ per
// row, sorted there by the quad's lane 0), and lane 0 forms alpha_U (and the
// Harris pass-1 entry) while lane 1 forms the flips' x_B update -- each the
// zchunk chains of zrow_chain over the sorted list: the same bits.  One
// pass-2 region and one pass-1 minimum per workgroup (k_ratio's prefetch
// covers 512 regions; a row tile emits <= 64 candidates: one per row); bump
// tiles of 64 positions (the first wave of the workgroup).
constexpr int ZLPR = 4, ZRPW = 64 / ZLPR, ZQB = 8, ZSQ = 32, ZROWS = 4 * ZRPW;
// ordered emission of a workgroup's pass-2 candidates into its region (every
// wave's kept entries compacted by ballot, the waves' counts through LDS)
DEV void emit_block(const Dev& d, int region, int var, int e, double g, double x, double l, double u, double bmin,
                    double pivtol, int* wcnt) {
    const double r = var >= 0 ? harris2(g, x, l, u, pivtol) : HUGE_VAL;
    const bool keep = var >= 0 && r <= bmin && r != HUGE_VAL;
    const unsigned long long mask = __ballot(keep);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wcnt[w] = __popcll(mask);
    __syncthreads();
    int off = 0, tot = 0;
    for (int t = 0; t < (int)blockDim.x / 64; ++t) {
        off += t < w ? wcnt[t] : 0;
        tot += wcnt[t];
    }
    if (keep) {
        const int slot = off + __popcll(mask & ((1ull << lane) - 1ull));
        if (slot < RREG) {
            RCand cd;
            cd.g = g;
            cd.r = r;
            cd.l = l;
            cd.u = u;
            cd.var = var;
            cd.e = e;
            d.rcand[(size_t)region * RREG + slot] = cd;
        }
    }
    if (threadIdx.x == 0) d.rcnt[region] = tot < RREG ? tot : RREG;
}
__global__ void __launch_bounds__(256) k_ftran_zr_sq(Dev d, int nrt, int flip, int dslot) {
    __shared__ int s_p[ZROWS][ZSQ];
    __shared__ double s_v[ZROWS][ZSQ];
    __shared__ double s_min[4];
    __shared__ int s_wc[4];
    RSTAMP(16);
    const DevCtl* c = d.ctl;
    const int32_t st0 = c->status;
    int k = c->k, q = c->q;
    const int bland = c->bland, m = d.m, tid = threadIdx.x;
    const double sig = c->sig, ptol = c->tol_primal, pivtol = c->tol_pivot;
    const int nfl = c->nflip;
    const int r = tid / ZLPR, sub = tid % ZLPR;  // (r: the workgroup's row, 0..63)
    const bool roww = (int)blockIdx.x < nrt;
    const int i = roww ? (int)blockIdx.x * ZROWS + r : 0;
    const int ic = i < m ? i : (m > 0 ? m - 1 : 0);
    int64_t r0 = 0, r1 = 0;
    int u = -1;
    double qi = 0.0, afi = 0.0;
    if (m > 0) {  // (straight-line, masked at use)
        r0 = d.rptr[ic];
        r1 = d.rptr[ic + 1];
        u = d.cover[ic];
        qi = d.qcol[ic];
        afi = d.aF ? d.aF[ic] : 0.0;
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" : "+v"(k), "+v"(q));
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) d.ctl->snap_status = st0;  // for k_ratio
    if (st0 != ST_RUN) {
        KEEP(r0);
        KEEP(u);
        KEEP(qi);
        KEEP(afi);
        return;
    }
    RSTAMP(17);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        d.ctl->snap_k = k;
        d.ctl->snap_bland = bland;
    }
    if (blockIdx.x == gridDim.x - 1) {
        if (threadIdx.x == 0) zr_snapshot(d, k, q);
        return;
    }
    const bool fl = flip && nfl > 0;
    double tmin = HUGE_VAL, ge = 0.0, xe = 0.0, le = 0.0, he = 0.0;
    int ve = -1, e = 0;
    if (roww) {
        const bool act = i < m && u >= 0;
        int cnt = 0;
        for (int64_t t0 = r0; t0 < r1; t0 += ZLPR * ZQB) {  // (trip counts differ per quad)
            int jj[ZQB], ps[ZQB];
            double vr[ZQB];
#pragma unroll
            for (int b = 0; b < ZQB; ++b) {
                const int64_t tt = t0 + sub + ZLPR * b;
                const int64_t tc = tt < r1 ? tt : r1 - 1;
                jj[b] = d.cind[tc];
                vr[b] = d.rval[tc];
            }
#pragma unroll
            for (int b = 0; b < ZQB; ++b) ps[b] = d.spos[jj[b]];
            int mine = 0;
#pragma unroll
            for (int b = 0; b < ZQB; ++b) mine += (t0 + sub + ZLPR * b < r1 && ps[b] >= 0 && ps[b] < k) ? 1 : 0;
            // the quad's offsets (lanes 4r' .. 4r' + 3 of this wave: shuffles within the quad)
            const int qb = (tid & 63) & ~(ZLPR - 1);
            int off = 0, tot = 0;
#pragma unroll
            for (int s2 = 0; s2 < ZLPR; ++s2) {
                const int v = __shfl(mine, qb + s2);
                off += s2 < sub ? v : 0;
                tot += v;
            }
            int o = cnt + off;
#pragma unroll
            for (int b = 0; b < ZQB; ++b)
                if (t0 + sub + ZLPR * b < r1 && ps[b] >= 0 && ps[b] < k) {
                    if (o < ZSQ) {
                        s_p[r][o] = ps[b];
                        s_v[r][o] = vr[b];
                    }
                    ++o;
                }
            cnt += tot;
        }
        __syncthreads();  // (the quads' entries in LDS)
        const bool over = cnt > ZSQ;
        if (act && sub == 0 && !over) {  // insertion sort by position, in LDS (a handful of entries)
            for (int a = 1; a < cnt; ++a) {
                const int p = s_p[r][a];
                const double v = s_v[r][a];
                int b = a - 1;
                while (b >= 0 && s_p[r][b] > p) {
                    s_p[r][b + 1] = s_p[r][b];
                    s_v[r][b + 1] = s_v[r][b];
                    --b;
                }
                s_p[r][b + 1] = p;
                s_v[r][b + 1] = v;
            }
        }
        __syncthreads();
        if (act && (sub == 0 || (sub == 1 && fl))) {
            const double* xs = sub == 0 ? d.alS : d.fS;
            double z = 0.0;
            if (over) {  // the dense walk over AS, 32 positions' loads in flight per chunk
                const size_t mm = (size_t)m;
                for (int c0 = 0; c0 < k; c0 += ZCHUNK) {
                    double a[ZCHUNK], xv[ZCHUNK];
#pragma unroll
                    for (int t = 0; t < ZCHUNK; ++t) {
                        const int p = min(c0 + t, k - 1);
                        a[t] = d.AS[(size_t)p * mm + i];
                        xv[t] = xs[p];
                    }
                    double acc = 0.0;
#pragma unroll
                    for (int t = 0; t < ZCHUNK; ++t)
                        if (c0 + t < k) acc = fma(a[t], xv[t], acc);
                    z = z + acc;
                }
            } else {  // (batches of 8 gathers; static indices only -- no scratch)
                double acc = 0.0;
                int ch = -1;
#pragma unroll
                for (int t0 = 0; t0 < ZSQ; t0 += 8) {
                    if (t0 < cnt) {
                        int pv[8];
                        double xv[8];
#pragma unroll
                        for (int b = 0; b < 8; ++b) {
                            pv[b] = s_p[r][min(t0 + b, cnt - 1)];
                            xv[b] = xs[pv[b]];
                        }
#pragma unroll
                        for (int b = 0; b < 8; ++b)
                            if (t0 + b < cnt) {
                                const int pc = pv[b] / ZCHUNK;
                                if (pc != ch) {
                                    if (ch >= 0) z = z + acc;
                                    acc = 0.0;
                                    ch = pc;
                                }
                                acc = fma(s_v[r][t0 + b], xv[b], acc);
                            }
                    }
                }
                if (ch >= 0) z = z + acc;
            }
            const double sg = unit_sign(d, u, i);
            if (sub == 0) {
                const double aiq = q >= d.N ? (i == q - d.N ? 1.0 : 0.0) : qi;
                const double alU = sg * (aiq - z);
                d.alU[i] = alU;
                RSTAMP(18);
                if (!flip) {
                    ge = sig * alU;
                    xe = d.xr[i];
                    le = d.rlo[i];
                    he = d.rhi[i];
                    ve = u;
                    tmin = harris1(ge, xe, le, he, ptol, pivtol, bland);
                }
            } else {
                d.xr[i] = d.xr[i] - sg * (afi - z);
            }
        }
        e = i;
    } else {  // (64 positions per workgroup: a region holds at most RREG = 64 candidates)
        const int p = (blockIdx.x - nrt) * 64 + tid;
        e = m + p;
        if (tid < 64 && p < k) {
            if (flip) {
                if (fl) d.xs[p] = d.xs[p] - d.fS[p];
            } else {
                ge = sig * d.alS[p];
                xe = d.xs[p];
                le = d.slo[p];
                he = d.shi[p];
                ve = d.Sl[p];
                tmin = harris1(ge, xe, le, he, ptol, pivtol, bland);
            }
        }
    }
    const double bmin = block_min<256>(tmin, s_min);
    if (tid == 0) d.blockmin[blockIdx.x] = bmin;
    emit_block(d, blockIdx.x, ve, e, ge, xe, le, he, bmin, pivtol, s_wc);
    RSTAMP(19);
}

// waves per row tile of k_ftran_zr (ZR_WAVES): 8, or 4 when the row tiles
// outnumber the CUs and every chunk still gets its own half-wave (the kernel
// holds one 8-wave workgroup per CU -- 175 VGPRs -- so 4-wave tiles run two
// per CU: one round of workgroups at m = 10 000 instead of two).  Which wave
// forms a chunk does not change the arithmetic (chunk sums added in order).
constexpr int ZR_ROWS = 32;   // rows per row tile: lane = row + 32 * half; each
                              // half-wave runs whole ZCHUNK chains (its own chunk)
// ALS: alpha_S staged once per workgroup in LDS (after the z partials) instead
// of every lane loading the chunk's 32 values itself (half the VMEM instructions
// and 64 fewer VGPRs); needs k_ub <= ZR_PA * threads
constexpr int ZR_PA = 4;
// XPF: chunks past the 2 ZR_WAVES half-waves' first ones (k > 512 with 8-wave
// tiles: 529 at the end of 10 000 x 500 000 is 17 chunks on 16 half-waves)
// whose values every thread of the row tile prefetches cooperatively (ZR_XR
// per thread, 256-B row segments) before the control block, parked in LDS; the
// owning half-wave then runs its chain from LDS instead of paying a second
// dependent round trip to AS.  Same chain, same order: same bits.
constexpr int ZR_XPF = 2;
template <bool LDSZ, int ZR_WAVES, bool ALS>
__global__ void __launch_bounds__(64 * ZR_WAVES) k_ftran_zr(Dev d, int nrt, int k_ub, int dslot, int qz) {
    extern __shared__ __attribute__((aligned(16))) double zlds[];  // [nch_ub][ZR_ROWS], then (ALS) [k_ub] alpha_S
    __shared__ double red[ZR_WAVES];
    RSTAMP(16);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & (ZR_ROWS - 1), hh = lane >> 5;
    const int i = blockIdx.x * ZR_ROWS + r;
    const size_t mm = (size_t)d.m;
    // The first chunk's AS and alpha_S loads go out before the control block
    // arrives: they are in bounds for any k <= k_ub (host upper bound) and the
    // positions past the real k are dropped below.
    // the control block first (vmcnt retires in issue order: the status test
    // then waits for these loads only)
    const DevCtl* c = d.ctl;
    const int32_t st0 = c->status;
    int k = c->k, q = c->q, bland = c->bland;  // (pinned below)
    const double sig = c->sig, ptol = c->tol_primal, pivtol = c->tol_pivot;
    const int ch0 = 2 * w + hh;
    double a0[ZCHUNK], s0[ALS ? 1 : ZCHUNK], pa[ALS ? ZR_PA : 1];
    const bool row_tile = (int)blockIdx.x < nrt;
    constexpr int XR = ALS ? ZR_XPF * ZCHUNK * ZR_ROWS / (64 * ZR_WAVES) : 1;
    double xv[XR];
    const int nch_ub = (k_ub + ZCHUNK - 1) / ZCHUNK;
    const int nxp = ALS ? min(max(nch_ub - 2 * ZR_WAVES, 0), ZR_XPF) : 0;  // prefetched extra chunks
    if constexpr (ALS) {  // this thread's share of alpha_S, staged in LDS below
#pragma unroll
        for (int t = 0; t < ZR_PA; ++t) pa[t] = ld_clamp(d.alS, (int)threadIdx.x + (int)blockDim.x * t, k_ub);
        // the extra chunks: value v = [chunk x][position][row], rows fastest
        // (clamped addresses, masked when used)
        const int rb = blockIdx.x * ZR_ROWS, mlast = d.m - 1;
#pragma unroll
        for (int t = 0; t < XR; ++t) {
            const int v = (int)threadIdx.x + (int)blockDim.x * t;
            const int x = v / (ZCHUNK * ZR_ROWS), pos = (v / ZR_ROWS) % ZCHUNK, row = v % ZR_ROWS;
            const int cpos = min((2 * ZR_WAVES + x) * ZCHUNK + pos, k_ub - 1);
            xv[t] = d.AS[(size_t)cpos * mm + min(rb + row, mlast)];
        }
    }
    if (row_tile && ch0 * ZCHUNK < k_ub && i < d.m) {
        const double* col = d.AS + (size_t)(ch0 * ZCHUNK) * mm + i;
#pragma unroll
        for (int t = 0; t < ZCHUNK; ++t) {
            const bool in = ch0 * ZCHUNK + t < k_ub;
            a0[t] = in ? col[(size_t)t * mm] : 0.0;
            if constexpr (!ALS) s0[t] = in ? d.alS[ch0 * ZCHUNK + t] : 0.0;
        }
    }
    // likewise wave 0's epilogue operands (independent of q and z)
    double tmin = HUGE_VAL;
    double ge = 0.0, xe = 0.0, le = 0.0, he = 0.0;
    int ve = -1;
    int u = -1;
    double pq = 0.0;  // (qz) a_iq as the select kernel staged it
    if (row_tile && w == 0 && hh == 0 && i < d.m) {
        u = d.cover[i];
        xe = d.xr[i];
        le = d.rlo[i];
        he = d.rhi[i];
        pq = (qz ? d.qz : d.xr)[i];
    }
    __builtin_amdgcn_sched_barrier(0);  // all of the above issued before any use
    // the control-block integers stay vector values up to here: their scalar
    // copies would otherwise be scheduled above the prefetch, which then waits
    // for the control block's round trip (measured: 2.7 us to the status test)
    asm volatile("" : "+v"(k), "+v"(q), "+v"(bland));
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) d.ctl->snap_status = st0;  // for k_ratio
    if (st0 != ST_RUN) {
#pragma unroll
        for (int t = 0; t < ZCHUNK; ++t) KEEP(a0[t]);
        if constexpr (!ALS) {
#pragma unroll
            for (int t = 0; t < ZCHUNK; ++t) KEEP(s0[t]);
        } else {
#pragma unroll
            for (int t = 0; t < ZR_PA; ++t) KEEP(pa[t]);
#pragma unroll
            for (int t = 0; t < XR; ++t) KEEP(xv[t]);
        }
        KEEP(xe);
        KEEP(pq);
        return;
    }
    RSTAMP(17);
    const int m = d.m;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        d.ctl->snap_k = k;
        d.ctl->snap_bland = bland;
    }
    if (blockIdx.x == gridDim.x - 1) {  // the snapshot workgroup (see DevCtl)
        if (threadIdx.x == 0) zr_snapshot(d, k, q);
        return;
    }
    const int nch = (k + ZCHUNK - 1) / ZCHUNK;
    // z partials of this tile's rows: LDS, or (huge bumps) a private slice of zpart
    double* zp = LDSZ ? zlds : d.zpart + (size_t)blockIdx.x * ZR_ROWS * (size_t)nch;
    double* als = zlds + (size_t)nch_ub * ZR_ROWS;  // (ALS)
    double* xz = als + k_ub;                         // (ALS) [nxp][ZCHUNK][ZR_ROWS]
    if constexpr (ALS) {
#pragma unroll
        for (int t = 0; t < ZR_PA; ++t) {
            const int p = (int)threadIdx.x + (int)blockDim.x * t;
            if (p < k) als[p] = pa[t];
        }
#pragma unroll
        for (int t = 0; t < XR; ++t) {
            const int v = (int)threadIdx.x + (int)blockDim.x * t;
            if (v < nxp * ZCHUNK * ZR_ROWS) xz[v] = xv[t];
        }
        __syncthreads();
    }
    if (row_tile) {
        double aiq = 0.0;
        if (u >= 0) aiq = qz ? pq : q >= d.N ? (i == q - d.N ? 1.0 : 0.0) : qcol_at(d, qcolumn(d, q), q, i);
        if (ch0 < nch) {  // the prefetched chunk: fma chain over its real positions
            double acc = 0.0;
            if (i < m) {
                const int len = min(ZCHUNK, k - ch0 * ZCHUNK);
#pragma unroll
                for (int t = 0; t < ZCHUNK; ++t)
                    if (t < len) acc = fma(a0[t], ALS ? als[ch0 * ZCHUNK + t] : s0[t], acc);
            }
            zp[ch0 * ZR_ROWS + r] = acc;
        }
        // later chunks (k > 2 ZR_WAVES ZCHUNK): every load unconditional at a
        // clamped row / position -- a load under a lane or position test is
        // drained at the end of its block, one round trip per position in the
        // last, partial chunk (measured: FTRAN-z 21 us at 10 000 x 500 000, k 529)
        for (int ch = ch0 + 2 * ZR_WAVES; ch < nch; ch += 2 * ZR_WAVES) {
            const int c0 = ch * ZCHUNK, len = min(ZCHUNK, k - c0);
            if (ALS && ch - 2 * ZR_WAVES < nxp) {  // a prefetched extra chunk: from LDS
                const double* xc = xz + (size_t)(ch - 2 * ZR_WAVES) * ZCHUNK * ZR_ROWS + r;
                double acc = 0.0;
                for (int t = 0; t < len; ++t) acc = fma(xc[t * ZR_ROWS], als[c0 + t], acc);
                zp[ch * ZR_ROWS + r] = i < m ? acc : 0.0;
                continue;
            }
            const double* col = d.AS + (size_t)c0 * mm + (i < m ? i : 0);
            double a[ZCHUNK], s[ALS ? 1 : ZCHUNK];  // the whole chunk in flight
#pragma unroll
            for (int t = 0; t < ZCHUNK; ++t) {
                const int tt = t < len ? t : len - 1;
                a[t] = col[(size_t)tt * mm];
                if constexpr (!ALS) s[t] = d.alS[c0 + tt];
            }
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < ZCHUNK; ++t)
                if (t < len) acc = fma(a[t], ALS ? als[c0 + t] : s[t], acc);
            zp[ch * ZR_ROWS + r] = i < m ? acc : 0.0;
        }
        RSTAMP(18);
        __syncthreads();
        if (w == 0) {
            if (hh == 0 && i < m && u >= 0) {
                double z = 0.0;
                for (int ch = 0; ch < nch; ++ch) z = z + zp[ch * ZR_ROWS + r];
                const double alU = unit_sign(d, u, i) * (aiq - z);
                d.alU[i] = alU;
                ge = sig * alU;
                ve = u;
                tmin = harris1(ge, xe, le, he, ptol, pivtol, bland);
            }
            const double bmin = wave_min_f64(tmin);
            if (lane == 0) d.blockmin[blockIdx.x] = bmin;
            emit_wave(d, blockIdx.x, ve, i, ge, xe, le, he, bmin, pivtol);  // region = row tile
            RSTAMP(19);
        }
    } else {
        const int p = (blockIdx.x - nrt) * (64 * ZR_WAVES) + threadIdx.x;
        if (p < k) {
            ge = sig * d.alS[p];
            xe = d.xs[p];
            le = d.slo[p];
            he = d.shi[p];
            ve = d.Sl[p];
            tmin = harris1(ge, xe, le, he, ptol, pivtol, bland);
        }
        double bmin = wave_min_f64(tmin);
        if (lane == 0) red[w] = bmin;
        __syncthreads();
        bmin = red[0];
        for (int ww = 1; ww < ZR_WAVES; ++ww) bmin = fmin(bmin, red[ww]);
        if (threadIdx.x == 0) d.blockmin[blockIdx.x] = bmin;
        // region: nrt + (bump tile) * ZR_WAVES + wave
        emit_wave(d, nrt + (blockIdx.x - nrt) * ZR_WAVES + w, ve, m + p, ge, xe, le, he, bmin, pivtol);
    }
}

// ============================================================== ratio test
struct Leave {
    double ag, r, g, l, u;
    int var, e;
};
DEV bool leave_better(const Leave& a, const Leave& b, int bland) {
    if (a.var < 0) return false;
    if (b.var < 0) return true;
    if (bland) return a.r < b.r || (a.r == b.r && a.var < b.var);
    return a.ag > b.ag || (a.ag == b.ag && a.var < b.var);
}
// field-wise select (see cand_take)
DEV void leave_take(Leave& c, const Leave& o, bool take) {
    c.ag = take ? o.ag : c.ag;
    c.r = take ? o.r : c.r;
    c.g = take ? o.g : c.g;
    c.l = take ? o.l : c.l;
    c.u = take ? o.u : c.u;
    c.var = take ? o.var : c.var;
    c.e = take ? o.e : c.e;
}
// the best leaving candidate of a wave in leave_better's total order, without LDS
DEV Leave wave_best_leave(const Leave& x, int bland) {
    const bool valid = x.var >= 0;
    const unsigned long long vm = __ballot(valid);
    if (vm == 0ull) return x;  // every lane holds "none"
    bool in;
    if (bland) {
        const double rmin = wave_min_f64(valid ? x.r : HUGE_VAL);
        in = valid && x.r == rmin;
    } else {
        const double amax = wave_max_f64(valid ? x.ag : -1.0);
        in = valid && x.ag == amax;
    }
    unsigned long long mask = __ballot(in);
    if (mask == 0ull) {  // (NaN ratios only) the lowest variable among the valid lanes
        in = valid;
        mask = vm;
    }
    const int win = __builtin_amdgcn_readfirstlane(lowest_index_lane(mask, in, x.var));
    Leave r;
    r.ag = readlane_f64(x.ag, win);
    r.r = readlane_f64(x.r, win);
    r.g = readlane_f64(x.g, win);
    r.l = readlane_f64(x.l, win);
    r.u = readlane_f64(x.u, win);
    r.var = __builtin_amdgcn_readlane(x.var, win);
    r.e = __builtin_amdgcn_readlane(x.e, win);
    return r;
}

// Scalars the pivot bookkeeping needs, fetched in parallel at kernel start.
enum { SC_LBQ, SC_UBQ, SC_XVQ, SC_CQ, SC_SLL, SC_CSL, SC_SLOL, SC_SHIL, SC_N };
enum { SI_VSQ, SI_RPOS0, SI_YPOS0, SI_YLAST, SI_SLLAST, SI_RLLAST, SI_RPOSYL, SI_N };

// Harris pass 2 + decision + pivot plan, fused with the B^-1 row of cases B/D.
// Pass 1 came from k_ftran_zr's per-workgroup minima, the candidates from its
// emitted list.  EVERY workgroup repeats the decision (same inputs, total
// orders: all agree); workgroup 0 alone does the bookkeeping; every workgroup
// then forms vvec for its 4 columns when a unit variable leaves.  k and bland
// come from the snapshot (workgroup 0 rewrites them).  The primal update
// x_B -= step * alpha runs in k_update.
// Phase 2 (defer != 0): workgroups [nmain, gridDim.x) copy this pivot's AR rows
// (the only update the next pricing sweep needs), workgroup 0 runs the loop-top
// checks, and the rest of the update is deferred into the next pricing launch.
// PFT: B^-1 row values per lane held in registers (k <= 64 PFT), 8 or 16 by the
// host's bound on k (a longer row is read in a loop)
// DUAL (the dual simplex phase, oracle run_dual): no primal ratio test -- the
// leaving entry is k_dual_row's, the step |x_r - beta_r| / |alpha_rq| on the
// FTRAN column, the leaving variable goes to beta_r; the bookkeeping, the B^-1
// row and the dual update are the primal's (phase 2), the plan carries the dual
// Devex update and the loop-top checks run here (no deferral).
#ifndef ELP_BOOK_WG
#define ELP_BOOK_WG 1
#endif
template <int PFT, bool DUAL = false>
__global__ void __launch_bounds__(256) k_ratio(Dev d, int phase, int nblk, int lds_row, int defer,
                                               int nmain, int k_ub, int dslot, int nreg) {
    extern __shared__ __attribute__((aligned(16))) double asrow_lds[];  // [k]: A[lrow, S]
    __shared__ double dred[4];
    __shared__ Leave lred[4];
    __shared__ double s_wd;
    __shared__ int s_lpos[SPL], s_lkey[SPL], s_lsb[72], s_lscan[4];  // (d.noT: A[lrow, S] as a sparse list)
    __shared__ double s_lval[SPL];
    const int tid = threadIdx.x;
    const int col = blockIdx.x * 4 + (tid >> 6);
    const int lane = tid & 63;
    if (ELP_DIAG && d.stamp_wide && tid == 0) {  // (ELP_STAMPS=2: grid-wide stamps, contended atomics)
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        atomicMin(&d.dstamp[dslot * DSTAMP_STRIDE + 11], t);
        atomicMax(&d.dstamp[dslot * DSTAMP_STRIDE + 8], t);
    }
    RSTAMP(0);
    // ---- the control block first: vmcnt retires loads in issue order, so the
    //      status test below then waits for these alone, not for the prefetch
    DevCtl* c = d.ctl;
    const int32_t st0 = c->snap_status;  // (not c->status: see DevCtl::snap_status)
    const int m = d.m;
    int k = c->snap_k, ny = c->snap_ny, q = c->q;  // (these five pinned below)
    const double sig = c->sig, dq = c->dq, wq = c->wq;
    int bland = c->snap_bland;
    const int devex = c->devex;
    int apos_c = c->snap_apos;
    // the bookkeeping workgroup: a workgroup of its own (ELP_BOOK_WG, grid
    // [nmain main][1 bookkeeping][AR copies]) that skips the B^-1 row and the dual
    // update of bump positions, so its single-lane tail starts at the decision;
    // 0: workgroup 0, after its share of those (r03)
    const bool lead = ELP_BOOK_WG ? (int)blockIdx.x == nmain : blockIdx.x == 0;
    // bookkeeping scalars, snapshot by k_ftran_zr (see DevCtl)
    const double sv_lbq = c->snap_lbq, sv_ubq = c->snap_ubq, sv_xq = c->snap_xq, sv_cq = c->snap_cq;
    const double sv_csl = c->snap_csl, sv_slol = c->snap_slol, sv_shil = c->snap_shil;
    const int sv_vsq = c->snap_vsq, sv_sllast = c->snap_sllast, sv_rllast = c->snap_rllast;
    const int sv_ypos0 = c->snap_ypos0, sv_ylast = c->snap_ylast;
    // ---- loads that depend on neither the control block nor the decision go
    //      out next (bounded by the host's k_ub, masked by the real k below):
    //      the pass-1 minima, this wave's row of MinvT (B^-1 row, cases B / D)
    //      and its bump row R_col (dual update)
    constexpr int PFB = 4;
    const bool main_wg = (int)blockIdx.x < nmain;
    const bool pfb = nblk <= 256 * PFB, pft = k_ub <= 64 * PFT;
    double bm[PFB], trow[PFT];
    // (unconditional, no branch around them: a load inside a conditional block
    //  is drained at the block's end; masks are applied where the values are used)
    // Issue order = the order of first use (vmcnt retires in issue order): Rl
    // (its y is read right after the control block), the pass-1 minima, the
    // pass-2 candidates, then this wave's MinvT row (the B^-1 row, last)
    // entries of Rl past the real k are stale: range-checked before use
    const int rcol = ld_clamp(d.Rl, main_wg ? col : 0, k_ub);
    // (DUAL: no primal ratio test -- the leaving entry is k_dual_row's, so
    //  neither the pass-1 minima nor the pass-2 candidates are read)
#pragma unroll
    for (int t = 0; t < PFB; ++t) bm[t] = DUAL ? HUGE_VAL : ld_clamp(d.blockmin, tid + 256 * t, nblk);
    // the pass-2 candidates k_ftran_zr emitted, one region per emitting wave:
    // thread t takes regions t and t + 256 (PFR), count and first PFQ entries
    // prefetched (clamped, masked by the count at use)
    constexpr int PFQ = 1, PFR = 2;  // (PFQ 4: +0.5 us of k_ratio, rocprof A/B r02)
    int rcn[PFR];
    RCand rq[PFR][PFQ];
#pragma unroll
    for (int s = 0; s < PFR; ++s) {
        const int reg = min(tid + 256 * s, nreg - 1);
        rcn[s] = DUAL ? 0 : d.rcnt[reg];
#pragma unroll
        for (int t = 0; t < PFQ; ++t) {
            if constexpr (DUAL) {
                rq[s][t] = RCand{};
            } else {
                rq[s][t] = d.rcand[(size_t)reg * RREG + t];
            }
        }
    }
    // DUAL: the leaving entry's B^-1 row is k_dual_row's rho_r (same row, same
    // k): its value on this wave's position replaces the MinvT row
    double rho_col = 0.0;
    if constexpr (DUAL) {
        rho_col = ld_clamp(d.rhoR, main_wg ? col : 0, k_ub);
#pragma unroll
        for (int t = 0; t < PFT; ++t) trow[t] = 0.0;
    } else {  // (AR-copy workgroups fetch row 0: harmless)
        // only the register path (k_ub <= 64 PFT, MinvT kept) reads these: past
        // it -- and without MinvT -- every lane loads element 0 (one line), not a
        // row nobody reads (8 KB per wave with arow below: 24 MB per pivot at the
        // CSC feasible-start LP's k ~ 3 000)
        const int tlim = pft && !d.noT ? k_ub : 1;
        const double* row = (d.noT ? d.Minv : d.MinvT) + (size_t)(main_wg && col < k_ub ? col : 0) * d.ldm;
#pragma unroll
        for (int t = 0; t < PFT; ++t) trow[t] = ld_clamp(row, lane + 64 * t, tlim);
    }
    __builtin_amdgcn_sched_barrier(0);  // all of the above issued before any use
    // the control-block integers stay vector values up to here: their scalar
    // copies (loc_of, loop bounds) would otherwise be scheduled above the
    // prefetch, which then waits for the control block
    asm volatile("" : "+v"(q), "+v"(k), "+v"(ny), "+v"(bland), "+v"(apos_c));
    if (st0 != ST_RUN) {  // no plan this iteration: k_update must not re-apply one
        if (blockIdx.x == 0 && threadIdx.x == 0) c->plan.action = ACT_NONE;
#pragma unroll
        for (int t = 0; t < PFB; ++t) KEEP(bm[t]);
#pragma unroll
        for (int t = 0; t < PFT; ++t) KEEP(trow[t]);
        KEEP(rho_col);
        KEEP(rcol);
#pragma unroll
        for (int s = 0; s < PFR; ++s) {
            KEEP(rcn[s]);
#pragma unroll
            for (int t = 0; t < PFQ; ++t) KEEP(rq[s][t].r);
        }
        return;
    }
    RSTAMP(1);
    // workgroup 0 / thread 0 keeps the counters it updates in registers
    // (read once here instead of one dependent round trip per update)
    // (every lane loads them -- one line, broadcast -- so no branch drains them)
    const int64_t cs_iter = c->iter, cs_limit = c->iter_limit, cs_stop = c->iter_stop;
    const int64_t cs_tcap = c->trace_cap, cs_p1 = c->phase1_iters, cs_flips = c->flips;
    const int64_t cs_degen = c->degenerate;
    const int32_t cs_ndegen = c->ndegen, cs_dswitch = c->degen_switch, cs_since = c->since_refactor;
    const int32_t cs_period = c->refactor_period, cs_seq = c->plan_seq;
    // oracle run_phase loop top for the next phase-2 iteration, on the values
    // thread 0 has just written (phase 1: k_btran's)
    auto loop_top = [&](int32_t status, int64_t iter, int32_t since) {
        if (status != ST_RUN) return;
        if (iter >= cs_limit) c->status = ST_ITERCAP;
        else if (iter >= cs_stop) c->status = ST_STOP;
        else if (since >= cs_period) c->status = ST_REFACTOR;
    };
    const int last = k - 1;
    // dual-update operands of this wave's bump row (read unconditionally at a
    // valid index; only used when col < k)
    const int rsafe = (rcol >= 0 && rcol < m) ? rcol : 0;
    const double yold = d.y[rsafe];
    const int ypos_r = d.ypos[rsafe];  // its Y slot (workgroup 0 rewrites no bump row's slot)
    // rpos of the last Y row (the bookkeeping's moved-slot rule): read here, off
    // the snapshot kernel's critical path, and consumed before the barrier
    // below, ahead of the bookkeeping's own rpos stores
    int sv_rposyl = d.rpos[sv_ylast >= 0 ? sv_ylast : 0];
    // ---- parallel prefetch of bookkeeping scalars
    const int ql = loc_of(d, q);  // -1: the entering column lives on another shard
    // case D needs wave_dot(MinvT[apos, :], A[lrow, S]) in every workgroup: wave 0
    // fetches that row now (apos comes with the control block)
    double arow[PFT];
    double rho_a = 0.0, dxsig = 0.0;  // DUAL: rho_r at position apos; the leaving row's sigma
    if constexpr (DUAL) {
        rho_a = d.rhoR[apos_c >= 0 ? apos_c : 0];
        dxsig = c->dr_xsig;
#pragma unroll
        for (int t = 0; t < PFT; ++t) arow[t] = 0.0;
    } else {  // (as trow: read by the register path only)
        const double* row = (d.noT ? d.Minv : d.MinvT) + (size_t)(apos_c >= 0 ? apos_c : 0) * d.ldm;
        const int alim = pft && !d.noT ? k : 1;
#pragma unroll
        for (int t = 0; t < PFT; ++t) arow[t] = ld_clamp(row, lane + 64 * t, alim);
    }
    // ---- pass 1 result: min over the workgroup minima
    const double INF = HUGE_VAL;
    double tmax = INF;
    if (pfb || DUAL) {
#pragma unroll
        for (int t = 0; t < PFB; ++t) tmax = fmin(tmax, tid + 256 * t < nblk ? bm[t] : INF);
    } else {
        for (int b = tid; b < nblk; b += 256) tmax = fmin(tmax, d.blockmin[b]);
    }
    const double theta_max = block_min<256>(tmax, dred);
    RSTAMP(2);
    // ---- pass 2 over the candidates
    Leave best;
    best.var = -1;
    best.ag = best.r = best.g = best.l = best.u = 0.0;
    best.e = -1;
    auto consider = [&](const RCand& cd) {
        if (!(cd.r <= theta_max)) return;
        Leave o;
        o.var = cd.var;
        o.ag = fabs(cd.g);
        o.r = cd.r;
        o.g = cd.g;
        o.l = cd.l;
        o.u = cd.u;
        o.e = cd.e;
        leave_take(best, o, leave_better(o, best, bland));
    };
#pragma unroll
    for (int s = 0; s < PFR; ++s) {
        const int reg = tid + 256 * s;
        if (reg >= nreg) continue;
#pragma unroll
        for (int t = 0; t < PFQ; ++t)
            if (t < rcn[s]) consider(rq[s][t]);
        for (int t = PFQ; t < rcn[s]; ++t) consider(d.rcand[(size_t)reg * RREG + t]);  // long regions
    }
    for (int reg = tid + 256 * PFR; reg < (DUAL ? 0 : nreg); reg += 256) {  // (huge m)
        const int cnt = d.rcnt[reg];
        for (int t = 0; t < cnt; ++t) consider(d.rcand[(size_t)reg * RREG + t]);
    }
    best = wave_best_leave(best, bland);
    if ((tid & 63) == 0) lred[tid >> 6] = best;
    if (sv_ylast < 0) sv_rposyl = -1;
    asm volatile("" : "+v"(sv_rposyl));  // (waited for here, before any rpos store)
    __syncthreads();  // also publishes the prefetched scalars
    {
        int win = 0;
        for (int i = 1; i < 4; ++i)
            if (leave_better(lred[i], lred[win], bland)) win = i;
        best = lred[win];
    }
    RSTAMP(3);
    double dual_acol = 0.0;
    int dual_s = 0;
    double dual_qt = 0.0;
    if constexpr (DUAL) {  // the dual's leaving entry replaces the primal decision
        const int e = c->dr_e;
        dual_acol = e < m ? d.alU[e] : d.alS[e - m];
        const double xe = e < m ? d.xr[e] : d.xs[e - m];  // (after this iteration's flips)
        best.var = c->dr_var;
        best.e = e;
        best.g = sig * dual_acol;
        best.ag = fabs(best.g);
        best.l = c->dr_lb;
        best.u = c->dr_ub;
        best.r = fabs((xe - c->dr_beta) / dual_acol);
        dual_s = c->dr_s;
        dual_qt = c->dq_t;
    }
    // ---- decision (uniform across the block)
    const double lbq = sv_lbq, ubq = sv_ubq;
    const double theta = best.var >= 0 ? (best.r > 0.0 ? best.r : 0.0) : INF;
    const double flip = !DUAL && (lbq > -INF && ubq < INF) ? ubq - lbq : INF;
    int action;
    double step;
    if (flip < INF && flip <= theta) {
        action = ACT_FLIP;
        step = flip;
    } else if (theta == INF) {
        action = ACT_NONE;  // unbounded
        step = 0.0;
    } else {
        action = ACT_PIVOT;
        step = theta;
    }
    if (lead && tid == 0) {
        const int64_t it = cs_iter;
        c->iter = it + 1;
        if (phase == 1 || DUAL) c->phase1_iters = cs_p1 + 1;
        if (DUAL) c->dual_iters++;
        if (action == ACT_NONE) {
            c->status = ST_UNBOUNDED;
            c->unb_var = q;
            c->unb_sig = sig;
        }
        if (it < cs_tcap) {  // leaving: -1 bound flip, -2 unbounded ray
            d.trace[2 * it] = q;
            d.trace[2 * it + 1] = action == ACT_FLIP ? -1 : action == ACT_NONE ? -2 : best.var;
        }
    }
    if (action == ACT_NONE) {
        if (lead && tid == 0) c->plan.action = ACT_NONE;
        return;
    }
    if (action == ACT_FLIP) {
        if (lead && tid == 0) {
            if (ql >= 0) {  // the shard that stores q's status
                if (sv_vsq == VS_LOWER) {
                    d.vstat[ql] = VS_UPPER;
                    d.xval[ql] = ubq;
                } else {
                    d.vstat[ql] = VS_LOWER;
                    d.xval[ql] = lbq;
                }
            }
            c->flips = cs_flips + 1;
            c->ndegen = 0;
            c->bland = 0;
            c->dv_valid = 0;  // a flip changes no reduced cost
            Plan P;
            P.action = ACT_FLIP;
            P.pcase = PC_NONE;
            P.k_old = k;
            P.q = q;
            P.step = step;
            P.sig = sig;
            P.p = P.a = P.b = P.last = P.row = P.i0 = P.lrow = P.lpos = -1;
            P.y_rm_slot = P.y_rm_last = P.y_ap_slot = P.y_ap_row = -1;
            P.piv = 0.0;
            P.xq = 0.0;
            P.dual = P.dre = 0;
            P.dwr = P.darq = 0.0;
            c->plan = P;
            c->plan_seq = cs_seq + 1;
            if (defer) loop_top(ST_RUN, cs_iter + 1, cs_since);
        }
        return;
    }
    if ((int)blockIdx.x >= nmain + ELP_BOOK_WG) {  // deferred flow: this pivot's AR row copies
        if (d.csc) return;
        const int lrow = best.e < m ? best.e : -1;
        const bool leave_art = best.var >= d.N + m;
        int rm_slot = -1, rm_last = -1, ap_slot = -1, ap_row = -1;
        if (q < d.N) {
            if (lrow >= 0 && !leave_art) {  // case B: the leaving unit var's row joins Y
                ap_slot = ny;
                ap_row = lrow;
            }
        } else {  // C, D, E: row i0 leaves Y; D: the leaving slack's row joins it
            rm_slot = sv_ypos0;
            rm_last = ny - 1;
            if (apos_c >= 0 && lrow >= 0 && !leave_art) {
                ap_slot = ny - 1;
                ap_row = lrow;
            }
        }
        if (rm_slot < 0 && ap_slot < 0) return;
        const int64_t tstride = (int64_t)(gridDim.x - nmain - ELP_BOOK_WG) * blockDim.x;
        for (int64_t j = (int64_t)(blockIdx.x - nmain - ELP_BOOK_WG) * blockDim.x + tid; j < d.n; j += tstride) {
            if (rm_slot >= 0 && rm_slot != rm_last) d.AR[ar_at(d, rm_slot, j)] = d.AR[ar_at(d, rm_last, j)];
            if (ap_slot >= 0) d.AR[ar_at(d, ap_slot, j)] = a_row(d, ap_row, j);
        }
        if (ELP_DIAG && d.stamp_wide) {
            __syncthreads();
            if (tid == 0) atomicMax(&d.dstamp[dslot * DSTAMP_STRIDE + 10], __builtin_amdgcn_s_memrealtime());
        }
        return;
    }
    // ---- B^-1 row for a leaving unit variable (cases B, D; E wastes it):
    //      vvec[c] = wave_dot(MinvT[c, 0:k], A[lrow, S]), case B / delta
    const int lrow_all = best.e < m ? best.e : -1;
    double vcol = 0.0;  // vvec[col] (cases B, D)
    // pivot case as workgroup 0's bookkeeping will classify it
    const int lposx = best.e >= m ? best.e - m : -1;
    const int apos = apos_c;
    const int pcx = q < d.N ? (lposx >= 0 ? PC_A : PC_B) : apos < 0 ? PC_E : lposx >= 0 ? PC_C : PC_D;
    // operands of the dual update that need the decision (cases A, C)
    const bool upd = phase == 2 && lane == 0 && col < k && pcx != PC_E &&
                     !((pcx == PC_C || pcx == PC_D) && col == apos);
    const size_t lrowoff = (size_t)(lposx >= 0 ? lposx : 0) * d.ldm;
    const double mpc = d.Minv[lrowoff + (col < k ? col : 0)];
    const double mpiv = d.Minv[lrowoff + (apos >= 0 ? apos : 0)];
    // workgroup 0: what its bookkeeping and the closing vrow / colA copies read
    constexpr int PFV = 4;  // k <= 1024
    const bool pfv = k <= 256 * PFV;
    double vr[PFV], ca[PFV];
    double t0_piv = 0.0, t0_ymoved = 0.0;
    int t0_yposl = -1;
    int8_t t0_rowvs = VS_FIXED, t0_yvslast = VS_FIXED;
    {  // (straight-line; workgroup 0 uses them, the others discard them)
        const size_t rv = (size_t)(lposx >= 0 ? lposx : 0) * d.ldm, ra = (size_t)(apos >= 0 ? apos : 0) * d.ldm;
        // (column a of Minv: row a of MinvT, or a gather with stride ldm without it)
        const double* cab = d.noT ? d.Minv + (apos >= 0 ? apos : 0) : d.MinvT + ra;
        const int64_t cas = d.noT ? d.ldm : 1;
#pragma unroll
        for (int t = 0; t < PFV; ++t) {
            vr[t] = ld_clamp(d.Minv + rv, tid + 256 * t, k);
            ca[t] = cab[(int64_t)(tid + 256 * t < k ? tid + 256 * t : (k > 0 ? k - 1 : 0)) * cas];
        }
        t0_piv = d.Minv[rv + (apos >= 0 ? apos : 0)];
        t0_yposl = d.ypos[lrow_all >= 0 ? lrow_all : 0];
        t0_rowvs = d.rowvs[lrow_all >= 0 ? lrow_all : 0];
        t0_yvslast = d.yvs[ny > 0 ? ny - 1 : 0];
        const int moved = sv_ylast;
        t0_ymoved = d.y[moved >= 0 ? moved : 0];
    }
    // (a separate bookkeeping workgroup forms no B^-1 row entries; it needs
    //  A[lrow, S] only for case D's vvec[a])
    if (DUAL && lrow_all >= 0 && k > 0) {
        // the dual phase leaves on k_dual_row's covered row: rho_r = -(sigma v)
        // with v = row_times_minv(lrow) (wave order), sigma = +-1, so
        // v = -(sigma rho_r) exactly -- no second pass over MinvT
        if (col < k && main_wg) {
            const double acc = -(dxsig * rho_col);
            const double delta = unit_sign(d, best.var, lrow_all) * (sig * best.g);
            vcol = q < d.N ? acc / delta : acc;
            if (lane == 0) d.vvec[col] = vcol;
        }
        if (pcx == PC_D && tid == 0) s_wd = dq / (-(dxsig * rho_a));
        __syncthreads();
    } else if (d.noT && lrow_all >= 0 && k > 0 && !(ELP_BOOK_WG && lead && !(phase == 2 && pcx == PC_D))) {
        // CSC without MinvT: A[lrow, S] as a sparse list from row lrow's CSR
        // entries through spos (the bookkeeping's only spos store in cases B /
        // D is q's, at position k: outside the list), each wave's chain over
        // column col of Minv -- the dense chain's bits (sparse_lane_chain_f);
        // a row with more than SPL entries walks the column with every term
        const int64_t t0 = d.rptr[lrow_all], t1 = d.rptr[lrow_all + 1];
        const bool sl = t1 - t0 <= SPL;
        if (sl) {
            bool valid = false;
            int p = 0;
            double v = 0.0;
            if (tid < t1 - t0) {
                v = d.rval[t0 + tid];
                p = d.spos[d.cind[t0 + tid]];
                valid = p >= 0 && p < k;
            }
            spl_build<256>(valid, p, v, s_lpos, s_lval, s_lsb, s_lkey, s_lscan);
        } else {
            double* asrow = lds_row ? asrow_lds : d.vrow;
            for (int j = tid; j < k; j += 256) asrow[j] = d.AS[(size_t)j * (size_t)m + lrow_all];
            __syncthreads();
        }
        const double* asrow = lds_row ? asrow_lds : d.vrow;
        auto colchain = [&](int cc) {
            auto xf = [&](int qq) { return d.Minv[(size_t)qq * d.ldm + cc]; };
            return wave_tree(sl ? sparse_lane_chain_f(xf, s_lpos, s_lval, s_lsb) : lane_chain_f(xf, asrow, k));
        };
        if (col < k && main_wg) {
            const double acc = colchain(col);
            const double delta = unit_sign(d, best.var, lrow_all) * (sig * best.g);
            vcol = q < d.N ? acc / delta : acc;
            if (lane == 0) d.vvec[col] = vcol;
        }
        if (phase == 2 && pcx == PC_D && tid < 64) {  // vvec[a], redundantly per workgroup
            const double acc = colchain(apos);
            if (tid == 0) s_wd = dq / acc;
        }
        __syncthreads();
    } else if (lrow_all >= 0 && k > 0 && !(ELP_BOOK_WG && lead && !(phase == 2 && pcx == PC_D))) {
        // huge bumps: every workgroup writes the same values to d.vrow (benign)
        double* asrow = lds_row ? asrow_lds : d.vrow;
        for (int j0 = tid; j0 < k; j0 += 1024) {  // 4 loads in flight per thread (k <= 1024: one pass)
            double v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = d.AS[(size_t)min(j0 + 256 * t, k - 1) * (size_t)m + lrow_all];
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (j0 + 256 * t < k) asrow[j0 + 256 * t] = v[t];
        }
        __syncthreads();
        if (col < k) {
            double acc = 0.0;
            if (pft) {
#pragma unroll
                for (int t = 0; t < PFT; ++t)
                    if (lane + 64 * t < k) acc = fma(trow[t], asrow[lane + 64 * t], acc);
            } else {
                const double* row = d.MinvT + (size_t)col * d.ldm;
                acc = lane_chain(row, asrow, k);
            }
            acc = wave_tree(acc);
            // case B delta = acol_i - z_i = sigma_u * sig * g (exact)
            const double delta = unit_sign(d, best.var, lrow_all) * (sig * best.g);
            vcol = q < d.N ? acc / delta : acc;
            if (lane == 0) d.vvec[col] = vcol;
        }
        if (phase == 2 && pcx == PC_D && tid < 64) {  // vvec[a], redundantly per workgroup
            double acc = 0.0;
            if (pft) {
#pragma unroll
                for (int t = 0; t < PFT; ++t)
                    if (lane + 64 * t < k) acc = fma(arow[t], asrow[lane + 64 * t], acc);
            } else {
                const double* row = d.MinvT + (size_t)apos * d.ldm;
                acc = lane_chain(row, asrow, k);
            }
            acc = wave_tree(acc);
            if (tid == 0) s_wd = dq / acc;
        }
        __syncthreads();
    }
    RSTAMP(4);
    // ---- phase 2 dual update y += theta_d rho_r on the bump rows, one wave per
    //      position (oracle run_phase cases A-D); the rows that join or leave R
    //      and the Y slot that moves are workgroup 0's (below)
    const double wD = (phase == 2 && pcx == PC_D) ? s_wd : 0.0;
    if (upd) {
        const int row = rcol;
        const double yo = yold;
        double yn;
        if (pcx == PC_A) {
            yn = fma(dq, mpc / (best.g * sig), yo);
        } else if (pcx == PC_B) {
            yn = fma(-dq, vcol, yo);
        } else if (pcx == PC_C) {
            yn = fma(dq, mpc / mpiv, yo);
        } else {
            yn = fma(wD, vcol, yo);
        }
        d.y[row] = yn;
        // the last Y row moves into the slot of row i0 (cases C, D)
        // (workgroup 0 rewrites ypos only for rows that are not bump rows, the
        //  entering slack's row -- excluded above -- and the moved last row)
        const int slot = (pcx == PC_C || pcx == PC_D) && row == sv_ylast ? sv_ypos0 : ypos_r;
        if (slot >= 0) d.yy[slot] = yn;
    }
    RSTAMP(5);
    if (ELP_DIAG && d.stamp_wide) {
        __syncthreads();
        if (tid == 0) atomicMax(&d.dstamp[dslot * DSTAMP_STRIDE + 9], __builtin_amdgcn_s_memrealtime());
    }
    if (!lead) return;
    // ---- the rows the deferred update reads -- vrow = Minv row p (A) / b (C)
    //      over the pivot, colA = MinvT row a (C, D) -- by the whole workgroup,
    //      from the rows prefetched at the decision, before thread 0's
    //      bookkeeping (which they do not depend on) instead of after it
    {
        const int pc = pcx;
        const double piv = pc == PC_A ? best.g * sig : t0_piv;  // the plan's piv (A: alS[p]; C: Minv[b][a])
        if (pfv) {
#pragma unroll
            for (int t = 0; t < PFV; ++t) {
                const int j = tid + 256 * t;
                if (j >= k) continue;
                if (pc == PC_A || pc == PC_C) d.vrow[j] = vr[t] / piv;
                if (pc == PC_C || pc == PC_D) d.colA[j] = ca[t];
            }
        } else if (pc != PC_B && pc != PC_E) {
            // k > 256 PFV (the CSC bumps): eight entries per thread in flight, the
            // loads ahead of the stores (one at a time, each store waited for the
            // next load: vrow / colA may alias Minv as far as the compiler knows
            // -- ~1 us per entry, the CSC feasible-start LP's k_ratio tail)
            const bool wr = pc == PC_A || pc == PC_C, wc = pc == PC_C || pc == PC_D;
            const size_t rv = (size_t)(lposx >= 0 ? lposx : 0) * d.ldm;
            const int ap = apos >= 0 ? apos : 0;
            for (int j0 = tid; j0 < k; j0 += 256 * 8) {
                double a[8], b[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int j = j0 + 256 * u < k ? j0 + 256 * u : k - 1;
                    a[u] = wr ? d.Minv[rv + j] : 0.0;
                    b[u] = wc ? (d.noT ? d.Minv[(size_t)j * d.ldm + ap] : d.MinvT[(size_t)ap * d.ldm + j]) : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int j = j0 + 256 * u;
                    if (j >= k) break;
                    if (wr) d.vrow[j] = a[u] / piv;
                    if (wc) d.colA[j] = b[u];
                }
            }
        }
    }
    // ---- pivot: bookkeeping, its stores split by destination over the four waves
    //      (a store chain per wave; stores to one address stay in one wave, in order)
    // (each wave's code specialised to its own stores -- wv is a compile-time
    //  constant per instance, so a wave evaluates only what it writes: the
    //  single-lane tail of the kernel is shorter)
    auto book = [&](auto WVc) {
        constexpr int wv = decltype(WVc)::value;  // (0: counters / statuses / control block,
                                                  //  1: bump lists, 2: Y list and covers,
                                                  //  3: plan record and duals)
        // (dual: degenerate when the entering column's dual ratio is not positive)
        if (DUAL ? !(dual_qt > 0.0) : theta == 0.0) {
            if (wv == 0) { c->degenerate = cs_degen + 1; }
            if (wv == 0) { c->ndegen = cs_ndegen + 1; }
            if (wv == 0) { if (cs_ndegen + 1 >= cs_dswitch) c->bland = 1; }
        } else {
            if (wv == 0) { c->ndegen = 0; }
            if (wv == 0) { c->bland = 0; }
        }
        const int lv = best.var;
        const int lrow = best.e < m ? best.e : -1;
        const int lpos = best.e < m ? -1 : best.e - m;
        const double xq = sv_xq + sig * theta;
        const bool at_lower = DUAL ? dual_s > 0 : best.g > 0.0;
        const bool leave_art = lv >= d.N + m;
        const int lvl = loc_of(d, lv);
        if (leave_art) {
            if (wv == 0) { d.lb[lvl] = 0.0; }
            if (wv == 0) { d.ub[lvl] = 0.0; }
            if (wv == 0) { d.vstat[lvl] = VS_FIXED; }
            if (wv == 0) { d.xval[lvl] = 0.0; }
        } else if (lvl >= 0) {  // a structural of another shard keeps no status here
            if (wv == 0) { d.vstat[lvl] = best.l == best.u ? VS_FIXED : at_lower ? VS_LOWER : VS_UPPER; }
            if (wv == 0) { d.xval[lvl] = at_lower ? best.l : best.u; }
        }
        if (wv == 0) { if (ql >= 0) d.vstat[ql] = VS_BASIC; }
        if (devex && wq > DEVEX_RESET) {
            // restart the framework (oracle: every weight 1 now): the next pass
            // sets the weight of each column it prices; a column basic now is
            // priced again only after it leaves, which sets its weight (below)
            if (wv == 0) { if (!leave_art && lvl >= 0) d.dw[lvl] = 1.0; }
            if (wv == 0) { c->dv_valid = 2; }
        } else if (devex) {  // the leaving variable's weight; this pivot for the next pass
            double wl = wq / (best.g * best.g);
            if (wl < 1.0) wl = 1.0;
            if (wl > DEVEX_WMAX) wl = DEVEX_WMAX;
            if (wv == 0) { if (!leave_art && lvl >= 0) d.dw[lvl] = wl; }
            if (wv == 0) { c->dv_valid = 1; }
            if (wv == 0) { c->dv_lv = lv; }
            if (wv == 0) { c->dv_dq = dq; }
            if (wv == 0) { c->dv_wq = wq; }
        }
        const double cq = sv_cq;
        Plan P;
        P.action = ACT_PIVOT;
        P.k_old = k;
        P.q = q;
        P.xq = xq;
        P.p = P.a = P.b = P.last = P.row = P.i0 = -1;
        P.lrow = lrow;
        P.lpos = lpos;
        P.step = step;
        P.sig = sig;
        P.y_rm_slot = P.y_rm_last = P.y_ap_slot = P.y_ap_row = -1;
        P.piv = 0.0;
        P.dual = DUAL && c->ddevex ? 1 : 0;
        P.dre = best.e;
        P.dwr = DUAL ? c->dr_w : 0.0;
        P.darq = dual_acol;
        int nny = ny;
        int newk = k;
        if (q < d.N) {
            if (lpos >= 0) {  // case A
                P.pcase = PC_A;
                P.p = lpos;
                P.piv = best.g * sig;  // alS[lpos]
                if (wv == 1) { d.Sl[lpos] = q; }
                if (wv == 1) { if (d.spos) { d.spos[lv] = -1; d.spos[q] = lpos; } }
                if (wv == 1) { d.cS[lpos] = cq; }
                if (wv == 1) { d.slo[lpos] = lbq; }
                if (wv == 1) { d.shi[lpos] = ubq; }
            } else {  // case B
                const int i = lrow;
                P.pcase = PC_B;
                P.row = i;
                P.p = k;
                // delta = acol_i - z_i = sigma_u * alU_i = sigma_u * sig * g (exact)
                P.piv = unit_sign(d, lv, i) * (sig * best.g);
                if (wv == 1) { d.Rl[k] = i; }
                if (wv == 1) { d.rpos[i] = k; }
                if (wv == 1) { d.Sl[k] = q; }
                if (wv == 1) { if (d.spos) d.spos[q] = k; }
                if (wv == 1) { d.cS[k] = cq; }
                if (wv == 1) { d.slo[k] = lbq; }
                if (wv == 1) { d.shi[k] = ubq; }
                if (wv == 1) { d.cover[i] = -1; }
                newk = k + 1;
                if (!leave_art) {
                    P.y_ap_slot = nny;
                    P.y_ap_row = i;
                    if (wv == 2) { d.Yl[nny] = i; }
                    if (wv == 2) { d.ypos[i] = nny; }
                    if (wv == 2) { d.yvs[nny] = t0_rowvs; }
                    nny++;
                }
            }
        } else {
            const int i0 = q - d.N;
            const int a = apos_c;
            if (a < 0) {  // case E
                P.pcase = PC_E;
                if (wv == 0) { if (lrow != i0) c->status = ST_NUMFAIL; }
            } else if (lpos >= 0) {  // case C
                const int b = lpos;
                P.pcase = PC_C;
                P.a = a;
                P.b = b;
                P.last = last;
                P.piv = t0_piv;  // Minv[b][a]
                if (wv == 1) { if (d.spos) d.spos[lv] = -1; }
                if (b != last) {
                    if (wv == 1) { if (d.spos) d.spos[sv_sllast] = b; }
                    if (wv == 1) { d.Sl[b] = sv_sllast; }
                    if (wv == 1) { d.cS[b] = sv_csl; }
                    if (wv == 1) { d.slo[b] = sv_slol; }
                    if (wv == 1) { d.shi[b] = sv_shil; }
                }
                if (a != last) {
                    const int rl = sv_rllast;
                    if (wv == 1) { d.Rl[a] = rl; }
                    if (wv == 1) { d.rpos[rl] = a; }
                }
                if (wv == 1) { d.rpos[i0] = -1; }
                newk = k - 1;
            } else {  // case D
                const int i1 = lrow;
                P.pcase = PC_D;
                P.a = a;
                P.row = i1;
                if (wv == 1) { d.Rl[a] = i1; }
                if (wv == 1) { d.rpos[i1] = a; }
                if (wv == 1) { d.rpos[i0] = -1; }
                if (wv == 1) { d.cover[i1] = -1; }
            }
            // the entering slack covers row i0
            P.i0 = i0;
            if (wv == 2) { d.cover[i0] = q; }
            if (wv == 2) { d.rlo[i0] = lbq; }
            if (wv == 2) { d.rhi[i0] = ubq; }
            // row i0 leaves Y (its slack is basic now) ...
            const int sl = sv_ypos0, ylast = nny - 1;
            P.y_rm_slot = sl;
            P.y_rm_last = ylast;
            if (sl != ylast) {
                const int moved = sv_ylast;
                if (wv == 2) { d.Yl[sl] = moved; }
                if (wv == 2) { d.ypos[moved] = sl; }
                if (wv == 2) { d.yvs[sl] = t0_yvslast; }
            }
            if (wv == 2) { d.ypos[i0] = -1; }
            nny--;
            // ... and in case D the leaving slack's row joins it
            if (P.pcase == PC_D && !leave_art) {
                P.y_ap_slot = nny;
                P.y_ap_row = lrow;
                if (wv == 2) { d.Yl[nny] = lrow; }
                if (wv == 2) { d.ypos[lrow] = nny; }
                if (wv == 2) { d.yvs[nny] = t0_rowvs; }
                nny++;
            }
        }
        if (phase == 2) {  // dual update: rows joining / leaving R, the moved Y slot
            // Y slot of the leaving unit var's row: the appended slot, or (an
            // artificial left: no append) the slot it already had
            int yslot = P.y_ap_slot >= 0 ? P.y_ap_slot : t0_yposl;
            if (P.y_ap_slot < 0 && P.pcase >= PC_C && P.y_rm_slot != P.y_rm_last &&
                P.lrow == sv_ylast)
                yslot = P.y_rm_slot;  // the leaving row was the last Y row: moved into i0's slot
            if (P.pcase == PC_B) {
                const double yn = dq / P.piv;
                if (wv == 3) { d.y[P.row] = yn; }
                if (wv == 3) { d.yy[yslot] = yn; }
            } else if (P.pcase == PC_C || P.pcase == PC_D) {
                if (wv == 3) { d.y[P.i0] = 0.0; }
                if (P.pcase == PC_D) {
                    if (wv == 3) { d.y[P.row] = -wD; }
                    if (wv == 3) { d.yy[yslot] = -wD; }
                }
            }
            if (P.pcase >= PC_C) {  // C, D, E removed row i0 from Y
                const int sl = sv_ypos0, moved = sv_ylast;
                // the owner wave of a bump row wrote its moved slot already
                const bool owned = P.pcase != PC_E && sv_rposyl >= 0;
                const bool special = P.pcase == PC_D && moved == P.row;
                if (wv == 3) { if (sl != ny - 1 && !owned && !special) d.yy[sl] = t0_ymoved; }
            }
        }
        if (wv == 0) { c->k = newk; }
        if (wv == 0) { c->ny = nny; }
        if (wv == 0) { c->since_refactor = cs_since + 1; }
        if (wv == 3) { c->plan = P; }
        if (wv == 0) { c->plan_seq = cs_seq + 1; }
        if (wv == 0) { if (defer || DUAL) loop_top(P.pcase == PC_E && lrow != q - d.N ? ST_NUMFAIL : ST_RUN, cs_iter + 1, cs_since + 1); }
        };
    if ((tid & 63) == 0) {  // thread 0 of each wave: the same decisions, a quarter of the stores
        switch (tid >> 6) {
            case 0: book(std::integral_constant<int, 0>{}); break;
            case 1: book(std::integral_constant<int, 1>{}); break;
            case 2: book(std::integral_constant<int, 2>{}); break;
            default: book(std::integral_constant<int, 3>{}); break;
        }
    }
    RSTAMP(6);
}

// the pre-update bump inverse: old(r, c) (tr: read from the transpose)
struct OldM {
    const double* M;
    size_t ld;
    bool tr;
    DEV double operator()(int r, int c) const { return tr ? M[(size_t)c * ld + r] : M[(size_t)r * ld + c]; }
};
// The plan k_ratio made: Minv and MinvT update (blocks [0, nb_minv)) + primal
// update x_B -= step*alpha and AS copies (blocks [nb_minv, nb)); with do_ar also
// the AR row copies (phase 1, where nothing is deferred).  Flips only update x_B.
// The rank-one term of every update form: ov - x1 x2, and ov itself when a
// multiplier is zero (the oracle's fma(-x1, x2, ov) returns ov then too, up to
// the sign of a zero ov: -0 + +0 = +0).  The zero rule lets the sparse update
// (apply_minv_sru) leave the untouched entries alone and still give every
// path -- dense, sparse, on the fly -- the same bits; a zero's sign reaches no
// later value or decision (products with it are zeros, sums with a nonzero
// term ignore it, comparisons see +-0 alike, no entry of the inverse is a
// divisor without passing the pivot tolerance), so the traces and solutions
// stay the oracle's.
DEV double r1(double ov, double x1, double x2) { return (x1 == 0.0 || x2 == 0.0) ? ov : fma(-x1, x2, ov); }
// new value of bump-inverse element (i, j) (the sequential path below)
DEV double minv_new(const Dev& d, const Plan& P, int i, int j, const OldM& old) {
    const int k = P.k_old;
    switch (P.pcase) {
        case PC_A:
            return (i == P.p) ? d.vrow[j] : r1(old(i, j), d.alS[i], d.vrow[j]);
        case PC_B:
            if (i < k && j < k) return r1(old(i, j), -d.alS[i], d.vvec[j]);
            if (i < k) return -(d.alS[i] / P.piv);
            if (j < k) return -d.vvec[j];
            return 1.0 / P.piv;
        case PC_C: {
            const int sr = (i == P.b) ? P.last : i;
            const int sc = (j == P.a) ? P.last : j;
            return r1(old(sr, sc), d.colA[sr], d.vrow[sc]);
        }
        default: {  // PC_D
            const double ca = d.colA[i] / d.vvec[P.a];
            return (j == P.a) ? ca : r1(old(i, j), ca, d.vvec[j]);
        }
    }
}
// one element at a time (the dense pricing launch's trailing workgroups, where
// the grouped form below measured slower, r04k / r04m)
DEV void apply_minv_seq(const Dev& d, const Plan& P, int64_t e0, int64_t estride, int kk) {
    const size_t ldm = (size_t)d.ldm;
    const int64_t nel = (int64_t)kk * kk;
    const OldM oM{d.Minv, ldm, false}, oT{d.MinvT, ldm, true};
    const int64_t sq = estride / kk, sr = estride % kk;
    int64_t e = e0;
    if (e < nel) {
        int64_t i = e / kk, j = e % kk;
        for (; e < nel; e += estride) {
            d.Minv[(size_t)i * ldm + (size_t)j] = minv_new(d, P, (int)i, (int)j, oM);
            i += sq;
            j += sr;
            if (j >= kk) {
                j -= kk;
                ++i;
            }
        }
    }
    if (e < 2 * nel && !d.noT) {  // MinvT element (j, i) = new Minv (i, j), f = e - nel = j kk + i
        const int64_t f = e - nel;
        int64_t j = f / kk, i = f % kk;
        for (; e < 2 * nel; e += estride) {
            d.MinvT[(size_t)j * ldm + (size_t)i] = minv_new(d, P, (int)i, (int)j, oT);
            j += sq;
            i += sr;
            if (i >= kk) {
                i -= kk;
                ++j;
            }
        }
    }
}

// the Minv / MinvT part of a plan: element e0, e0 + estride, ... of the 2 kk^2.
// A thread takes its elements MINV_U at a time: every load of the group (the
// old element, the two update operands) goes out before the group's stores --
// the stores alias the old matrix for the compiler, so a plain loop paid one
// memory round trip per element.  Element e -> (row, column) by one division per
// half, then carried along the stride.  Per element (pivot cases A-D, oracle
// update_inverse): A: new = (i == p) ? vrow_j : old - alS_i vrow_j; B (bordered):
// old + alS_i vvec_j inside, -alS_i / piv, -vvec_j, 1 / piv on the border; C:
// old(sr, sc) - colA_sr vrow_sc with the last row / column moved; D: colA_i / vvec_a
// on column a, old - (colA_i / vvec_a) vvec_j elsewhere.
constexpr int MINV_U = 4;  // elements per group
template <bool TR, int U>  // TR false: Minv (row i, column j); true: MinvT, element (j, i)
DEV void apply_minv_half(const Dev& d, const Plan& P, int64_t e, int64_t end, int64_t estride, int64_t base,
                         int kk) {
    const int k = P.k_old, pc = P.pcase;
    const size_t ldm = (size_t)d.ldm;
    double* M = TR ? d.MinvT : d.Minv;
    const OldM old{M, ldm, TR};
    const int64_t sq = estride / kk, sr = estride % kk;
    const int64_t f = e - base;
    int64_t a = f / kk, b = f % kk;  // position in the half's row-major order
    const double va = pc == PC_D ? d.vvec[P.a] : 1.0;
    const int kl = k > 0 ? k - 1 : 0;
    while (e < end) {
        int ii[U], jj[U];
        bool ok[U];
        double ov[U], x1[U], x2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ok[u] = e + (int64_t)u * estride < end;
            ii[u] = (int)(TR ? b : a);
            jj[u] = (int)(TR ? a : b);
            a += sq;
            b += sr;
            if (b >= kk) {
                b -= kk;
                ++a;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {  // the loads (indices clamped; masked by ok at the store)
            const int i = ok[u] ? ii[u] : 0, j = ok[u] ? jj[u] : 0;
            int r = i, c = j;
            int i1 = i, j2 = j;
            if (pc == PC_C) {
                r = (i == P.b) ? P.last : i;
                c = (j == P.a) ? P.last : j;
                i1 = r;
                j2 = c;
            } else if (pc == PC_B) {
                r = i < k ? i : 0;
                c = j < k ? j : 0;
                i1 = i < k ? i : kl;
                j2 = j < k ? j : kl;
            }
            ov[u] = old(r, c);
            x1[u] = pc == PC_C || pc == PC_D ? d.colA[i1] : d.alS[i1];
            x2[u] = pc == PC_B || pc == PC_D ? d.vvec[j2] : d.vrow[j2];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const int i = ii[u], j = jj[u];
            double v;
            if (pc == PC_A) {
                v = (i == P.p) ? x2[u] : r1(ov[u], x1[u], x2[u]);
            } else if (pc == PC_B) {
                if (i < k && j < k) v = r1(ov[u], -x1[u], x2[u]);
                else if (i < k) v = -(x1[u] / P.piv);
                else if (j < k) v = -x2[u];
                else v = 1.0 / P.piv;
            } else if (pc == PC_C) {
                v = r1(ov[u], x1[u], x2[u]);
            } else {  // PC_D
                const double ca = x1[u] / va;
                v = (j == P.a) ? ca : r1(ov[u], ca, x2[u]);
            }
            if (TR) M[(size_t)j * ldm + (size_t)i] = v;
            else M[(size_t)i * ldm + (size_t)j] = v;
        }
        e += (int64_t)U * estride;
    }
}
DEV void apply_minv(const Dev& d, const Plan& P, int64_t e0, int64_t estride, bool batch) {
    if (P.action != ACT_PIVOT || P.pcase == PC_E) return;
    const int k = P.k_old;
    const int kk = P.pcase == PC_B ? k + 1 : P.pcase == PC_C ? k - 1 : k;
    const int64_t nel = (int64_t)kk * kk;
    if (nel == 0) return;
    if (!batch) return apply_minv_seq(d, P, e0, estride, kk);
    if (e0 < nel) {
        apply_minv_half<false, MINV_U>(d, P, e0, nel, estride, 0, kk);
        // this thread's first MinvT element: the first e0 + t estride >= nel
        e0 += (nel - e0 + estride - 1) / estride * estride;
    }
    if (e0 < 2 * nel && !d.noT) apply_minv_half<true, MINV_U>(d, P, e0, 2 * nel, estride, nel, kk);
}

// The sparse rank-one update (Dev::sru_on, CSC): workgroup wg of nwg.  The
// bump inverse of a sparse LP is sparse (the 20 000 x 100 000 KKT LP's final
// bump is triangular after permutation: ~1.6 nonzeros per row of its
// inverse), and so are the update's multipliers x1 (alpha_S / column a of the
// inverse) and x2 (the pivot row / v): r05 counts 87 / 100 nonzeros of 2000 per
// dual pivot there; the feasible-start LP's primal pivots reach ~50 % at bumps
// of ~3000.  By the zero rule of r1 only the rows with a nonzero multiplier
// change (and in them the entries with a nonzero x2), plus the border the case
// rewrites (A: row p; B: row and column k; C: row b and column a, moved from
// the last ones; D: column a).  One workgroup per row (the host launches one
// per bump position up to SRU_WG_MAX; more rows: strided): one load tells
// whether its multiplier is zero -- then it is done -- else the row and x2 go
// out SRU_U per thread together (the row is read whole, so one round trip per
// batch) and only the changed entries are stored.  The border is strided over
// the whole launch.  Every entry written is written by the dense update too,
// with the same bits.
constexpr int SRU_U = 8;
constexpr unsigned SRU_WG_MAX = 4096;
constexpr int SRU_RPW = 1;  // rows per workgroup (r05ze: 4 -- their multipliers in one round trip -- measured slower)
constexpr unsigned sru_wgs(int k_ub) {
    return (unsigned)((k_ub + SRU_RPW) / SRU_RPW) < SRU_WG_MAX ? (unsigned)((k_ub + SRU_RPW) / SRU_RPW) : SRU_WG_MAX;
}
template <int NT>
DEV void apply_minv_sru(const Dev& d, const Plan& P, int wg, int nwg) {
    if (P.action != ACT_PIVOT || P.pcase == PC_E || nwg <= 0) return;
    const int k = P.k_old, pc = P.pcase, tid = threadIdx.x;
    const int kk = pc == PC_B ? k + 1 : pc == PC_C ? k - 1 : k;
    if (kk <= 0) return;
    const int nl = pc == PC_B ? k : kk;  // the rank-one part's index range
    const double* x1 = (pc == PC_C || pc == PC_D) ? d.colA : d.alS;
    const double* x2 = (pc == PC_B || pc == PC_D) ? d.vvec : d.vrow;
    const int ex1 = pc == PC_A ? P.p : pc == PC_C ? P.b : -1;  // (the row / column the border rewrites)
    const int ex2 = (pc == PC_C || pc == PC_D) ? P.a : -1;
    const size_t ldm = (size_t)d.ldm;
    double* M = d.Minv;
    double* MT = d.noT ? nullptr : d.MinvT;
    const double va = pc == PC_D ? d.vvec[P.a] : 1.0;
    // rows wg, wg + nwg, ...: SRU_RPW multipliers loaded together per group
    for (int i0 = wg; i0 < nl; i0 += nwg * SRU_RPW) {
      double a1s[SRU_RPW];
#pragma unroll
      for (int u = 0; u < SRU_RPW; ++u) {
          const int i = i0 + u * nwg;
          a1s[u] = x1[i < nl ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < SRU_RPW; ++u) {
        const int i = i0 + u * nwg;
        if (i >= nl || i == ex1) continue;
        double a1 = a1s[u];
        if (pc == PC_B) a1 = -a1;
        else if (pc == PC_D) a1 = a1 / va;
        if (a1 == 0.0) continue;
        double* row = M + (size_t)i * ldm;
        for (int j0 = tid; j0 < nl; j0 += NT * SRU_U) {
            double bb[SRU_U], ov[SRU_U];
#pragma unroll
            for (int u = 0; u < SRU_U; ++u) {
                const int j = min(j0 + u * NT, nl - 1);
                bb[u] = x2[j];
                ov[u] = row[j];
            }
#pragma unroll
            for (int u = 0; u < SRU_U; ++u) {
                const int j = j0 + u * NT;
                if (j >= nl || j == ex2 || bb[u] == 0.0) continue;
                const double v = fma(-a1, bb[u], ov[u]);
                row[j] = v;
                if (MT) MT[(size_t)j * ldm + i] = v;
            }
        }
      }
    }
    // ---- the border, strided over the launch
    auto put = [&](int i, int j, double v) {
        M[(size_t)i * ldm + j] = v;
        if (MT) MT[(size_t)j * ldm + i] = v;
    };
    const int64_t g = (int64_t)wg * NT + tid, G = (int64_t)nwg * NT;
    switch (pc) {
        case PC_A:
            for (int64_t j = g; j < k; j += G) put(P.p, (int)j, d.vrow[j]);
            break;
        case PC_B:
            for (int64_t t = g; t < 2 * (int64_t)k + 1; t += G) {
                if (t < k) put((int)t, k, -(d.alS[t] / P.piv));
                else if (t < 2 * k) put(k, (int)(t - k), -d.vvec[t - k]);
                else put(k, k, 1.0 / P.piv);
            }
            break;
        case PC_C: {
            const int last = P.last, b = P.b, a = P.a;
            if (b != last)
                for (int64_t j = g; j < kk; j += G) {
                    const int sc = (int)j == a ? last : (int)j;
                    put(b, (int)j, r1(M[(size_t)last * ldm + sc], d.colA[last], d.vrow[sc]));
                }
            if (a != last)
                for (int64_t i = g; i < kk; i += G)
                    if ((int)i != b) put((int)i, a, r1(M[(size_t)i * ldm + last], d.colA[i], d.vrow[last]));
            break;
        }
        default:  // PC_D
            for (int64_t i = g; i < k; i += G) put((int)i, P.a, d.colA[i] / va);
            break;
    }
}

// the primal update and the AS (/ AR) copies of a plan: thread t0 of tstride
DEV void apply_copy(const Dev& d, const Plan& P, int64_t t0, int64_t tstride, bool do_ar) {
    const int k = P.k_old;
    if (P.dual && P.action == ACT_PIVOT) {
        // dual Devex (oracle run_dual): the basic entries of the old basis other
        // than the leaving one take max(w, (alpha_e / alpha_rq)^2 w_r), the
        // entering variable max(w_r / alpha_rq^2, 1); above DEVEX_RESET every
        // weight restarts at 1.  Entries are read through the new lists (k_ratio
        // rewrote them): the entering slack's row (i0) and the removed bump
        // position are skipped, case C's moved position keeps alpha_S[last].
        const double wr = P.dwr, arq = P.darq;
        double wq = wr / (arq * arq);
        if (wq < 1.0) wq = 1.0;
        if (wq > DEVEX_WMAX) wq = DEVEX_WMAX;
        if (wq > DEVEX_RESET) {
            for (int64_t t = t0; t < (int64_t)d.N + d.m; t += tstride) d.ddw[t] = 1.0;
        } else {
            auto upd = [&](int var, double ae) {
                const double r = ae / arq;
                double wn = (r * r) * wr;
                if (wn > DEVEX_WMAX) wn = DEVEX_WMAX;
                if (wn > d.ddw[var]) d.ddw[var] = wn;
            };
            for (int64_t t = t0; t < d.m; t += tstride) {
                if (t == P.i0 || t == P.lrow) continue;
                const int u = d.cover[t];
                if (u >= 0) upd(u, d.alU[t]);
            }
            for (int64_t p = t0; p < k; p += tstride) {
                if (p == P.lpos) continue;  // (A, C: the leaving structural)
                if (P.pcase == PC_C && p == P.last) upd(d.Sl[P.b], d.alS[P.last]);  // (moved to b)
                else upd(d.Sl[p], d.alS[p]);
            }
            if (t0 == 0) d.ddw[P.q] = wq;
        }
    }
    // ---- primal update (oracle order: x -= step * (sig * alpha), then the
    //      entering value / compaction of the pivot case)
    const size_t m = (size_t)d.m;
    const double step = P.step, sg = P.sig;
    for (int64_t t = t0; t < d.m; t += tstride) {
        if (t == P.i0) d.xr[t] = P.xq;       // entering slack's row (C, D, E)
        else if (t == P.lrow) continue;      // leaving unit var's row (B, D)
        else if (d.cover[t] >= 0) d.xr[t] = fma(-step, sg * d.alU[t], d.xr[t]);
    }
    for (int64_t p = t0; p < k; p += tstride) {
        if (P.pcase == PC_A && p == P.lpos) d.xs[p] = P.xq;
        else if (P.pcase == PC_C && p == P.last) continue;  // removed position
        else if (P.pcase == PC_C && p == P.b)
            d.xs[p] = fma(-step, sg * d.alS[P.last], d.xs[P.last]);
        else d.xs[p] = fma(-step, sg * d.alS[p], d.xs[p]);
    }
    if (P.action != ACT_PIVOT) return;
    if (P.pcase == PC_B && t0 == 0) d.xs[k] = P.xq;
    // ---- copies: thread t covers row t of AS and column t of AR
    for (int64_t t = t0; t < d.m; t += tstride) {
        if (P.pcase == PC_A || P.pcase == PC_B) {
            const int pos = P.pcase == PC_A ? P.p : k;
            d.AS[(size_t)pos * m + t] = qcol_at(d, qcolumn(d, P.q), P.q, t);
        } else if (P.pcase == PC_C && P.b != P.last) {
            d.AS[(size_t)P.b * m + t] = d.AS[(size_t)P.last * m + t];
        }
    }
    if (do_ar && !d.csc && (P.y_rm_slot >= 0 || P.y_ap_slot >= 0)) {  // CSC prices from the columns
        for (int64_t j = t0; j < d.n; j += tstride) {
            if (P.y_rm_slot >= 0 && P.y_rm_slot != P.y_rm_last)
                d.AR[ar_at(d, P.y_rm_slot, j)] = d.AR[ar_at(d, P.y_rm_last, j)];
            if (P.y_ap_slot >= 0) d.AR[ar_at(d, P.y_ap_slot, j)] = a_row(d, P.y_ap_row, j);
        }
    }
}

DEV void apply_plan(const Dev& d, const Plan& P, int blk, int nb, int nb_minv, bool do_ar, bool batch) {
    if (blk < nb_minv) {
        apply_minv(d, P, (int64_t)blk * blockDim.x + threadIdx.x, (int64_t)nb_minv * blockDim.x, batch);
        return;
    }
    apply_copy(d, P, (int64_t)(blk - nb_minv) * blockDim.x + threadIdx.x, (int64_t)(nb - nb_minv) * blockDim.x,
               do_ar);
}

// ---- the dual phase's deferred update (one GPU, Dev::dual_defer; DESIGN.md
// 2.3).  k_ratio's plan of iteration t is applied during iteration t + 1: x_B,
// the dual Devex weights, the AS column (dense: AR rows) in k_dual_chuzr, entry
// by entry by the thread that then scores the entry (dual_copy_entry); MinvT in
// trailing workgroups of the pricing launch and Minv in those of the ratio-test
// launch (apply_minv_part); k_dual_row in between reads the new inverse on the
// fly (minv_new: the update's own arithmetic, so the same bits).  copy_seq and
// applied_seq mark the two parts applied (k_dual_row, the select kernel).
DEV bool copy_pending(const DevCtl* c) {
    return c->plan_seq != c->copy_seq && c->plan.action == ACT_PIVOT && c->status != ST_NUMFAIL;
}
DEV bool minv_pending(const DevCtl* c) {
    return c->plan_seq != c->applied_seq && c->plan.action == ACT_PIVOT && c->plan.pcase != PC_E &&
           c->status != ST_NUMFAIL;
}
// part 0: Minv, part 1: MinvT -- elements t0, t0 + tstride, ... of that half
DEV void apply_minv_part(const Dev& d, const Plan& P, int part, int64_t t0, int64_t tstride) {
    const int k = P.k_old;
    const int kk = P.pcase == PC_B ? k + 1 : P.pcase == PC_C ? k - 1 : k;
    const int64_t nel = (int64_t)kk * kk;
    if (d.sru_on) return;  // (the sparse update: all of it by the pricing launch's apply_minv_sru)
    if (nel == 0 || t0 >= nel) return;
    if (d.noT) {  // no MinvT: the two launches split Minv (rows [h, kk) here in part 0, [0, h) in part 1)
        const int64_t h = (int64_t)(kk / 2) * kk;
        if (part == 0) apply_minv_half<false, MINV_U>(d, P, h + t0, nel, tstride, 0, kk);
        else if (t0 < h) apply_minv_half<false, MINV_U>(d, P, t0, h, tstride, 0, kk);
        return;
    }
    if (part == 0) apply_minv_half<false, MINV_U>(d, P, t0, nel, tstride, 0, kk);
    else apply_minv_half<true, MINV_U>(d, P, nel + t0, 2 * nel, tstride, nel, kk);
}
// the dual Devex weight and x of the variable now basic at entry e (row e < m,
// else bump position e - m of the new basis) -- apply_copy's arithmetic, per
// entry: every basic variable but the entering one takes max(w, (alpha / a_rq)^2
// w_r) from the alpha of its old entry (case C: position b's from alS[last]);
// the entering one max(w_r / a_rq^2, 1); reset: every weight 1 (*wout = 1)
DEV void dual_copy_entry(const Dev& d, const Plan& P, int e, int k_new, double* wout) {
    const int m = d.m;
    const double step = P.step, sg = P.sig;
    const double wr = P.dwr, arq = P.darq;
    double wq = wr / (arq * arq);
    if (wq < 1.0) wq = 1.0;
    if (wq > DEVEX_WMAX) wq = DEVEX_WMAX;
    const bool reset = wq > DEVEX_RESET;
    int var = -1;
    double ae = 0.0;
    if (e < m) {
        const int t = e, u = d.cover[t];
        if (t == P.i0) d.xr[t] = P.xq;
        else if (t != P.lrow && u >= 0) d.xr[t] = fma(-step, sg * d.alU[t], d.xr[t]);
        var = u;
        if (u >= 0 && u != P.q) ae = d.alU[t];
    } else if (e - m < k_new) {
        const int p = e - m;
        const bool moved = P.pcase == PC_C && p == P.b;  // (b != last: the last position moved to b)
        if ((P.pcase == PC_A && p == P.lpos) || (P.pcase == PC_B && p == P.k_old)) d.xs[p] = P.xq;
        else if (moved) d.xs[p] = fma(-step, sg * d.alS[P.last], d.xs[P.last]);
        else d.xs[p] = fma(-step, sg * d.alS[p], d.xs[p]);
        var = d.Sl[p];
        if (var != P.q) ae = moved ? d.alS[P.last] : d.alS[p];
    }
    *wout = -1.0;  // (not updated: read d.ddw)
    if (!P.dual || var < 0) return;
    if (reset) {
        *wout = 1.0;
    } else if (var == P.q) {
        d.ddw[var] = wq;
        *wout = wq;
    } else {
        const double r = ae / arq;
        double wn = (r * r) * wr;
        if (wn > DEVEX_WMAX) wn = DEVEX_WMAX;
        const double w0 = d.ddw[var];
        const double w = wn > w0 ? wn : w0;
        if (wn > w0) d.ddw[var] = wn;
        *wout = w;
    }
}
// the rest of the copy part, strided over the launch: the AS column (A, B: the
// entering column at its position; C: the last column moved to b), AR rows
// (dense), every dual Devex weight 1 on a reset
DEV void dual_copy_rest(const Dev& d, const Plan& P, int64_t t0, int64_t tstride) {
    const int64_t m = d.m;
    const int k = P.k_old;
    if (P.pcase == PC_A || P.pcase == PC_B) {
        const int pos = P.pcase == PC_A ? P.p : k;
        const double* qc = qcolumn(d, P.q);
        for (int64_t t = t0; t < m; t += tstride) d.AS[(size_t)pos * m + t] = qcol_at(d, qc, P.q, t);
    } else if (P.pcase == PC_C && P.b != P.last) {
        for (int64_t t = t0; t < m; t += tstride) d.AS[(size_t)P.b * m + t] = d.AS[(size_t)P.last * m + t];
    }
    if (!d.csc && (P.y_rm_slot >= 0 || P.y_ap_slot >= 0)) {
        for (int64_t j = t0; j < d.n; j += tstride) {
            if (P.y_rm_slot >= 0 && P.y_rm_slot != P.y_rm_last)
                d.AR[ar_at(d, P.y_rm_slot, j)] = d.AR[ar_at(d, P.y_rm_last, j)];
            if (P.y_ap_slot >= 0) d.AR[ar_at(d, P.y_ap_slot, j)] = a_row(d, P.y_ap_row, j);
        }
    }
    if (P.dual) {
        double wq = P.dwr / (P.darq * P.darq);
        if (wq < 1.0) wq = 1.0;
        if (wq > DEVEX_WMAX) wq = DEVEX_WMAX;
        if (wq > DEVEX_RESET)
            for (int64_t t = t0; t < (int64_t)d.N + m; t += tstride) d.ddw[t] = 1.0;
    }
}

// Standalone update.  mode 0 (phase 1): the plan k_ratio just made, AR included.
// mode 1 (phase 2, host poll): a deferred plan still pending; its AR rows were
// copied by k_ratio already.  mode 2 (the dual phase's deferred plan at a host
// poll): the parts k_dual_chuzr / the trailing workgroups have not applied.
__global__ void __launch_bounds__(256) k_update(Dev d, int nb_minv, int mode) {
    const DevCtl* c = d.ctl;
    if (mode == 2) {
        const bool cp = copy_pending(c), mp = minv_pending(c);
        const Plan P = c->plan;
        const int blk = blockIdx.x, nb = gridDim.x;
        if (blk < nb_minv) {
            if (mp) apply_minv(d, P, (int64_t)blk * blockDim.x + threadIdx.x, (int64_t)nb_minv * blockDim.x);
        } else if (cp) {
            apply_copy(d, P, (int64_t)(blk - nb_minv) * blockDim.x + threadIdx.x,
                       (int64_t)(nb - nb_minv) * blockDim.x, true);
        }
        return;
    }
    if (mode == 1 && !plan_pending(c)) return;
    const Plan P = c->plan;
    if (P.action == ACT_NONE || c->status == ST_NUMFAIL) return;
    apply_plan(d, P, blockIdx.x, gridDim.x, nb_minv, mode == 0);
}

// ============================================================== refactor
__global__ void k_gj_init(Dev d, int k) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < (int64_t)k * k) {
        const int a = (int)(e / k), cc = (int)(e % k);
        d.W0[e] = d.AS[(size_t)cc * (size_t)d.m + d.Rl[a]];
    }
    if (e < k) d.pivstep[e] = 0x7fffffff;
}

// one Gauss-Jordan column step, two launches, in place on W (r05; r04: W -> W2
// every step).  The oracle's step with its zero rule (gauss_jordan): pivot p =
// the unused row with the largest |W[r][c]| (lowest row on ties); row p becomes
// q_j = W[p][j] / piv (1 / piv at c); column c becomes -(f_r / piv) with f_r =
// W[r][c]; every other entry W[r][j] -= f_r q_j -- left alone when f_r or q_j
// is zero.  k_gj_pivot (one workgroup) finds p, writes row p and column c in
// place and leaves f (all rows) and q (row p) in side buffers, with lists of
// the rows with f != 0 and the columns with q != 0; k_gj_elim updates those
// pairs only (a sparse bump's GJ touches a handful of rows per step), or sweeps
// every entry, tested, when the pairs are more than an eighth of k^2.
// Side buffers in W1: q [0, k), f [k, 2k), the rows' f [2k, 3k), rows (int)
// [3k, 4k), columns (int) [4k, 5k), the two counts at 5k.
constexpr int GJ_PT = 4;
struct GjSide {
    double *q, *f, *fv;
    int *rows, *cols, *cnt;
};
DEV GjSide gj_side(double* W1, int k) {
    GjSide g;
    g.q = W1;
    g.f = W1 + k;
    g.fv = W1 + 2 * (size_t)k;
    g.rows = reinterpret_cast<int*>(W1 + 3 * (size_t)k);
    g.cols = reinterpret_cast<int*>(W1 + 4 * (size_t)k);
    g.cnt = reinterpret_cast<int*>(W1 + 5 * (size_t)k);
    return g;
}
__global__ void __launch_bounds__(1024) k_gj_pivot(Dev d, int k, int col, double* __restrict__ W) {
    __shared__ double sv[16];
    __shared__ int sr[16], s_nr, s_nc;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const GjSide g = gj_side(d.W1, k);
    double bv = -1.0;
    int br = 0x7fffffff;
    // column c's entries of this thread's rows (up to GJ_RPT kept in registers
    // for the factors below; the loads and the used-row flags go out together)
    constexpr int GJ_RPT = 4;
    double cv[GJ_RPT];
    int ps[GJ_RPT];
#pragma unroll
    for (int u = 0; u < GJ_RPT; ++u) {
        const int r = min(tid + 1024 * u, k - 1);
        cv[u] = W[(size_t)r * k + col];
        ps[u] = d.pivstep[r];
    }
#pragma unroll
    for (int u = 0; u < GJ_RPT; ++u) {
        const int r = tid + 1024 * u;
        if (r >= k || ps[u] < col) continue;  // (used in an earlier step)
        const double v = fabs(cv[u]);
        if (v > bv || (v == bv && r < br)) {
            bv = v;
            br = r;
        }
    }
    for (int r = tid + 1024 * GJ_RPT; r < k; r += 1024) {
        if (d.pivstep[r] < col) continue;
        const double v = fabs(W[(size_t)r * k + col]);
        if (v > bv || (v == bv && r < br)) {
            bv = v;
            br = r;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double ov = __shfl_xor(bv, off);
        const int orr = __shfl_xor(br, off);
        if (ov > bv || (ov == bv && orr < br)) {
            bv = ov;
            br = orr;
        }
    }
    if (lane == 0) {
        sv[w] = bv;
        sr[w] = br;
    }
    if (tid == 0) {
        s_nr = 0;
        s_nc = 0;
    }
    __syncthreads();
    double v0 = sv[0];
    int p = sr[0];
    for (int i = 1; i < 16; ++i)
        if (sv[i] > v0 || (sv[i] == v0 && sr[i] < p)) {
            v0 = sv[i];
            p = sr[i];
        }
    if (p >= k) p = 0;  // (no unused row: k steps never ask for more)
    const double piv = W[(size_t)p * k + col];
    if (tid == 0) {
        d.perm[col] = p;
        d.pivstep[p] = col;
        if (!(fabs(piv) > d.tol_singular)) d.ctl->status = ST_NUMFAIL;
    }
    // row p's quotients and column c's factors, read before either is rewritten
    for (int j = tid; j < k; j += 1024) {
        const double q = j == col ? 0.0 : W[(size_t)p * k + j] / piv;
        g.q[j] = q;
        if (q != 0.0) g.cols[atomicAdd(&s_nc, 1)] = j;  // (any order: the pairs are independent)
    }
    for (int r = tid, u = 0; r < k; r += 1024, ++u) {
        const double f = u < GJ_RPT ? cv[u < GJ_RPT ? u : 0] : W[(size_t)r * k + col];
        g.f[r] = r == p ? 0.0 : f;
        if (r != p && f != 0.0) {
            const int o = atomicAdd(&s_nr, 1);
            g.rows[o] = r;
            g.fv[o] = f;
        }
    }
    __syncthreads();  // (every read of row p and column c is done)
    for (int j = tid; j < k; j += 1024)
        if (j != col) W[(size_t)p * k + j] = g.q[j];
    for (int r = tid; r < k; r += 1024) W[(size_t)r * k + col] = r == p ? 1.0 / piv : -(g.f[r] / piv);
    if (tid == 0) {
        g.cnt[0] = s_nr;
        g.cnt[1] = s_nc;
    }
}

__global__ void __launch_bounds__(256) k_gj_elim(Dev d, int k, int col, double* __restrict__ W) {
    const GjSide g = gj_side(d.W1, k);
    const int nr = g.cnt[0], nc = g.cnt[1];
    const int64_t np = (int64_t)nr * nc, kk = (int64_t)k * k;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, T = (int64_t)gridDim.x * blockDim.x;
    if (np * 8 <= kk) {  // the pairs of nonzero factors
        for (int64_t e = t0; e < np; e += T) {
            const int a = (int)(e / nc), b = (int)(e % nc);
            const int r = g.rows[a], j = g.cols[b];
            double* x = W + (size_t)r * k + j;
            *x = fma(-g.fv[a], g.q[j], *x);
        }
        return;
    }
    const int p = d.perm[col];
    for (int64_t e0 = t0 * GJ_PT; e0 < kk; e0 += T * GJ_PT) {  // every entry, tested
#pragma unroll
        for (int u = 0; u < GJ_PT; ++u) {
            const int64_t e = e0 + u;
            if (e >= kk) break;
            const int r = (int)(e / k), j = (int)(e % k);
            if (r == p || j == col) continue;
            const double f = g.f[r], q = g.q[j];
            if (f != 0.0 && q != 0.0) W[e] = fma(-f, q, W[e]);
        }
    }
}

__global__ void k_gj_final(Dev d, int k, const double* __restrict__ W) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)k * k) return;
    const int a = (int)(e / k), cc = (int)(e % k);
    const double v = W[(size_t)d.perm[a] * k + cc];
    d.Minv[(size_t)a * d.ldm + d.perm[cc]] = v;
    if (!d.noT) d.MinvT[(size_t)d.perm[cc] * d.ldm + a] = v;
}

// rhs_i = (b_i - sum_{nz} a_ij x_j) - s_i  and a_R for the bump solve
__global__ void k_refactor_rhs(Dev d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    double r = d.b[i] - d.ract[i];
    if (d.vstat[d.n + i] != VS_BASIC) r = r - d.xval[d.n + i];
    d.rhs[i] = r;
    const int p = d.rpos[i];
    if (p >= 0) d.aR[p] = r;
}

// ------------------------------------------------------------ Newton-Schulz
// Register-blocked fp64 GEMMs (r04): a 64 x 64 output tile per 256-thread
// workgroup, thread (tx, ty) owning outputs (ty + 16 u, tx + 16 v), u, v < 4;
// operands staged through LDS 16 values of l at a time.  Every output is still
// ONE fma chain over l in order (oracle newton_schulz: the same bits); per l the
// thread reads 4 + 4 values for 16 fmas instead of 2 per fma (r03's 32 x 32
// tiles, one output per thread: ~3 TFLOP/s, 5 ms at k = 2000).
// NS_R outputs per thread and dimension: 4 (64 x 64 tiles) below NS_R8_MIN
// positions, 8 (128 x 128 tiles, 251 VGPRs) from there -- r05: 1.57 -> 1.36 ms
// per call on the feasible-start KKT LP's bumps of ~3 000; small bumps keep the
// smaller tiles' workgroup count
constexpr int NS_L = 16, NS_R8_MIN = 1536;
template <int MODE, int NS_R = 4>  // 0: E = I - M Minv (M[i][l] = AS[l][Rl[i]]) into W0; 1: W1 = Minv + Minv E
__global__ void __launch_bounds__(256) k_ns_gemm(Dev d, int k) {
    constexpr int NS_T = 16 * NS_R;
    // thread (tx, ty) owns rows i0 + NS_R ty + u and columns j0 + NS_R tx + v:
    // its operands are NS_R consecutive doubles of an LDS row (16-byte loads;
    // the row pitch NS_T + 2 keeps them aligned)
    __shared__ __attribute__((aligned(16))) double At[NS_L][NS_T + 2];  // At[l][r]: operand A(i0 + r, l0 + l)
    __shared__ __attribute__((aligned(16))) double Bt[NS_L][NS_T + 2];  // Bt[l][c]: operand B(l0 + l, j0 + c)
    __shared__ double red[4];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int i0 = blockIdx.y * NS_T, j0 = blockIdx.x * NS_T;
    const size_t ldm = (size_t)d.ldm, m = (size_t)d.m;
    double acc[NS_R][NS_R];
#pragma unroll
    for (int u = 0; u < NS_R; ++u)
#pragma unroll
        for (int v = 0; v < NS_R; ++v) {
            const int i = i0 + NS_R * ty + u, j = j0 + NS_R * tx + v;
            acc[u][v] = (MODE == 1 && i < k && j < k) ? d.Minv[(size_t)i * ldm + j] : 0.0;
        }
    // the next chunk's operands are loaded into registers while this chunk's
    // fmas run (r05: one exposed global round trip per 16 values of l before)
    constexpr int NS_PT = NS_T * NS_L / 256;
    double na[NS_PT], nb[NS_PT];
    auto load_chunk = [&](int l0) {
#pragma unroll
        for (int t = 0; t < NS_PT; ++t) {
            const int e = tid + 256 * t;
            const int r = e / NS_L, c = e % NS_L;  // A: row r, l c
            const int i = i0 + r, l = l0 + c;
            double a = 0.0;
            if (i < k && l < k) a = MODE == 0 ? d.AS[(size_t)l * m + d.Rl[i]] : d.Minv[(size_t)i * ldm + l];
            na[t] = a;
            const int rb = e / NS_T, cb = e % NS_T;  // B: l rb, column cb
            const int lb = l0 + rb, j = j0 + cb;
            double b = 0.0;
            if (lb < k && j < k) b = MODE == 0 ? d.Minv[(size_t)lb * ldm + j] : d.W0[(size_t)lb * k + j];
            nb[t] = b;
        }
    };
    load_chunk(0);
    for (int l0 = 0; l0 < k; l0 += NS_L) {
#pragma unroll
        for (int t = 0; t < NS_PT; ++t) {
            const int e = tid + 256 * t;
            At[e % NS_L][e / NS_L] = na[t];
            Bt[e / NS_T][e % NS_T] = nb[t];
        }
        __syncthreads();
        if (l0 + NS_L < k) load_chunk(l0 + NS_L);
        const int lend = min(NS_L, k - l0);
        for (int ll = 0; ll < lend; ++ll) {
            double a[NS_R], b[NS_R];
            const double2* ap = reinterpret_cast<const double2*>(&At[ll][NS_R * ty]);
            const double2* bp = reinterpret_cast<const double2*>(&Bt[ll][NS_R * tx]);
#pragma unroll
            for (int u = 0; u < NS_R / 2; ++u) {
                const double2 x = ap[u], y = bp[u];
                a[2 * u] = x.x;
                a[2 * u + 1] = x.y;
                b[2 * u] = y.x;
                b[2 * u + 1] = y.y;
            }
#pragma unroll
            for (int u = 0; u < NS_R; ++u)
#pragma unroll
                for (int v = 0; v < NS_R; ++v) acc[u][v] = fma(a[u], b[v], acc[u][v]);
        }
        __syncthreads();
    }
    double emax = 0.0;
#pragma unroll
    for (int u = 0; u < NS_R; ++u)
#pragma unroll
        for (int v = 0; v < NS_R; ++v) {
            const int i = i0 + NS_R * ty + u, j = j0 + NS_R * tx + v;
            if (i >= k || j >= k) continue;
            if (MODE == 0) {
                const double e = (i == j ? 1.0 : 0.0) - acc[u][v];
                d.W0[(size_t)i * k + j] = e;
                emax = fmax(emax, fabs(e));
            } else {
                d.W1[(size_t)i * k + j] = acc[u][v];
            }
        }
    if (MODE == 0) {
        const double am = block_max<256>(emax, red);
        if (tid == 0) atomicMax(&d.ctl->ns_emax_bits, (unsigned long long)__double_as_longlong(am));
    }
}

// CSC: the same residual E = I - M Minv with M's row i = A[R_i, S] taken from
// row R_i's CSR entries in basic columns (spos), ascending position: each
// E[i][j] is k_ns_gemm<0>'s sequential fma chain over l without its zero terms
// -- the same bits at O(nnz(M) k) instead of O(k^3).  One workgroup per row i,
// a thread per column j (coalesced rows of Minv); a row with more than 256
// basic entries runs every l.
__global__ void __launch_bounds__(256) k_ns_resid_sp(Dev d, int k) {
    __shared__ int s_l[256], s_scan[4];
    __shared__ double s_v[256], red[4];
    const int tid = threadIdx.x, i = blockIdx.x;
    const int r = d.Rl[i];
    const int64_t t0 = d.rptr[r], t1 = d.rptr[r + 1];
    const bool sp = t1 - t0 <= 256;
    int n = 0;
    if (sp) {
        int l = -1;
        double v = 0.0;
        if (tid < t1 - t0) {
            v = d.rval[t0 + tid];
            l = d.spos[d.cind[t0 + tid]];
        }
        const bool valid = l >= 0 && l < k;
        int excl;
        n = block_scan_excl<256>(valid ? 1 : 0, &excl, s_scan);
        if (valid) s_l[excl] = l;
        __syncthreads();
        int rk = 0;
        if (valid)
            for (int t = 0; t < n; ++t) rk += s_l[t] < l ? 1 : 0;
        __syncthreads();
        if (valid) {
            s_l[rk] = l;
            s_v[rk] = v;
        }
        __syncthreads();
    }
    const size_t ldm = (size_t)d.ldm, m = (size_t)d.m;
    double emax = 0.0;
    for (int j = tid; j < k; j += 256) {
        double acc = 0.0;
        if (sp) {
            for (int t = 0; t < n; ++t) acc = fma(s_v[t], d.Minv[(size_t)s_l[t] * ldm + j], acc);
        } else {
            for (int l = 0; l < k; ++l) acc = fma(d.AS[(size_t)l * m + r], d.Minv[(size_t)l * ldm + j], acc);
        }
        const double e = (i == j ? 1.0 : 0.0) - acc;
        d.W0[(size_t)i * k + j] = e;
        emax = fmax(emax, fabs(e));
    }
    const double am = block_max<256>(emax, red);
    if (tid == 0) atomicMax(&d.ctl->ns_emax_bits, (unsigned long long)__double_as_longlong(am));
}

// Minv = W1, MinvT = W1^T (transposed through LDS, both stores coalesced)
__global__ void __launch_bounds__(1024) k_ns_store(Dev d, int k) {
    __shared__ double T[32][33];
    const int tx = threadIdx.x, ty = threadIdx.y;
    const int i = blockIdx.y * 32 + ty, j = blockIdx.x * 32 + tx;
    double v = 0.0;
    if (i < k && j < k) {
        v = d.W1[(size_t)i * k + j];
        d.Minv[(size_t)i * d.ldm + j] = v;
    }
    T[ty][tx] = v;
    __syncthreads();
    const int ti = blockIdx.y * 32 + tx, tj = blockIdx.x * 32 + ty;  // MinvT[tj][ti]
    if (ti < k && tj < k && !d.noT) d.MinvT[(size_t)tj * d.ldm + ti] = T[tx][ty];
}

// ============================================================== phase 2 / extract
// a phase start: the reference framework is the current nonbasic set
__global__ void k_devex_reset(Dev d) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < (int64_t)d.n + d.m) d.dw[j] = 1.0;
    if (d.ddw && d.ddw != d.dw && j < (int64_t)d.N + d.m) d.ddw[j] = 1.0;  // (sharded: global ids)
    if (j == 0) d.ctl->dv_valid = 0;
}

__global__ void k_phase2(Dev d) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < d.m) {
        const int av = d.n + d.m + t;
        d.cost[d.n + t] = 0.0;  // (a MIP node's warm start may have shifted a slack's cost)
        d.cost[av] = 0.0;
        d.lb[av] = 0.0;
        d.ub[av] = 0.0;
        if (d.cover[t] == d.N + d.m + t) {
            d.rlo[t] = 0.0;
            d.rhi[t] = 0.0;
        }
    }
    if (t < d.n) d.cost[t] = d.maximize ? -d.obj[t] : d.obj[t];
}
// c_S after the phase-2 costs are in place
__global__ void k_phase2_cS(Dev d) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < d.ctl->k) {
        const double o = d.objg[d.Sl[p]];
        d.cS[p] = d.maximize ? -o : o;
    }
}

__global__ void k_extract(Dev d, double* __restrict__ xout) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.n) return;
    xout[j] = d.xval[j];  // basic columns are overwritten by k_extract_basic
}
__global__ void k_extract_basic(Dev d, double* __restrict__ xout) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= d.ctl->k) return;
    const int64_t j = (int64_t)d.Sl[p] - d.col0;
    if (j >= 0 && j < d.n) xout[j] = d.xs[p];
}

// ============================================================== sensitivity
// Sensitivity report of the final basis (R/class.R:613-646; conventions in
// oracle/elp_oracle.c sensitivity()).  The two dense contractions -- alpha =
// Minv * A[R,:] (objective ranging of the basic structurals) and
// G = A[:,S] * Minv (columns of B^-1 for the binding rows, rhs ranging) -- run
// on the fp64 matrix cores (v_mfma_f64_16x16x4f64) with the ratio tests fused
// into the epilogue, so neither k x n nor m x k product is ever stored.

// reduced costs of the structurals (0 for basic): dense = wave order over all
// m rows (one wave per column), CSC = the column chain
__global__ void __launch_bounds__(256) k_sens_redcost(Dev d, double* __restrict__ dred) {
    const int lane = threadIdx.x & 63;
    if (d.csc) {
        const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
        if (j >= d.n) return;
        double acc = 0.0;
        for (int64_t t = d.cptr[j]; t < d.cptr[j + 1]; ++t) acc = fma(d.cval[t], d.y[d.rind[t]], acc);
        dred[j] = d.vstat[j] == VS_BASIC ? 0.0 : d.cost[j] - acc;
        return;
    }
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= d.n) return;
    const double* col = d.A + (size_t)j * (size_t)d.m;
    double acc = 0.0;
    for (int i = lane; i < d.m; i += 64) acc = fma(sca(d, col[i], i, d.col0 + j), d.y[i], acc);
    acc = wave_tree(acc);
    if (lane == 0) dred[j] = d.vstat[j] == VS_BASIC ? 0.0 : d.cost[j] - acc;
}

// TR[c][j] = A[R_c, j]  (k x n row-major; TR zeroed beforehand for CSC)
__global__ void k_sens_gather_rows(Dev d, double* __restrict__ TR, int k) {
    const int c = blockIdx.y;
    if (c >= k) return;
    const int i = d.Rl[c];
    if (d.csc) {
        for (int64_t t = d.rptr[i] + threadIdx.x; t < d.rptr[i + 1]; t += blockDim.x)
            TR[(size_t)c * (size_t)d.n + d.cind[t]] = d.rval[t];
        return;
    }
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d.n; j += (int64_t)gridDim.x * blockDim.x)
        TR[(size_t)c * (size_t)d.n + (size_t)j] = sca(d, d.A[(size_t)j * (size_t)d.m + (size_t)i], i, d.col0 + j);
}

// ratio-interval update: keep l <= x + t g <= u  ->  t in [lo, hi]
DEV void primal_interval(double g, double x, double l, double u, double tol, double& lo, double& hi) {
    if (g > tol) {
        hi = fmin(hi, (u - x) / g);
        lo = fmax(lo, (l - x) / g);
    } else if (g < -tol) {
        hi = fmin(hi, (l - x) / g);
        lo = fmax(lo, (u - x) / g);
    }
}
// reduced-cost interval: keep s (d - t a) >= 0 for nonbasic status vs
DEV void dual_interval(double a, double dk, int8_t vs, double tol, double& lo, double& hi) {
    if (vs == VS_BASIC || vs == VS_FIXED) return;
    const double r = dk / a;
    if (vs == VS_FREE) {
        if (fabs(a) > tol) {
            hi = fmin(hi, r);
            lo = fmax(lo, r);
        }
        return;
    }
    const double sa = vs == VS_LOWER ? a : -a;
    if (sa > tol) hi = fmin(hi, r);
    if (sa < -tol) lo = fmax(lo, r);
}

typedef double dbl4 __attribute__((ext_vector_type(4)));

// C = X (M x K) * Y (K x N) on the fp64 MFMA, X(r, kk) = X[r*xrs + kk*xcs],
// Y(kk, c) = Y[kk*yrs + c*ycs].  Workgroup = 4 waves = a 64 x 64 tile, wave w
// owns rows 16w..16w+15 (four 16x16 accumulators).  Epilogue:
//   MODE 0 (objective): rows = bump positions p, columns = structurals j;
//          interval of t = delta c_{S_p} from dual_interval(alpha, d_j) reduced
//          over the tile's columns -> plo/phi[p * gridDim.x + blockIdx.x]
//   MODE 1 (rhs): rows = covered rows i, columns = R positions c;
//          g = -sigma_u G(i, c), primal_interval on the covering unit variable,
//          reduced over the tile's rows -> plo/phi[c * gridDim.y + blockIdx.y]
template <int MODE>
__global__ void __launch_bounds__(256) k_sens_mfma(Dev d, const double* __restrict__ X, int64_t xrs,
                                                   int64_t xcs, const double* __restrict__ Y,
                                                   int64_t yrs, int64_t ycs, int M, int N, int K,
                                                   const double* __restrict__ dred, double* plo,
                                                   double* phi) {
    __shared__ double slo[4][64], shi[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = (MODE == 0 ? blockIdx.y : blockIdx.y) * 64 + 16 * w;
    const int c0 = blockIdx.x * 64;
    const int ar = r0 + (lane & 15);
    const int kq = lane >> 4;
    dbl4 acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < K; k0 += 4) {
        const int kk = k0 + kq;
        const double a = (ar < M && kk < K) ? X[(size_t)ar * xrs + (size_t)kk * xcs] : 0.0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int cc = c0 + 16 * b + (lane & 15);
            const double bv = (cc < N && kk < K) ? Y[(size_t)kk * yrs + (size_t)cc * ycs] : 0.0;
            acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv, acc[b], 0, 0, 0);
        }
    }
    const double tol = d.ctl->tol_pivot, INF = HUGE_VAL;
    // lane holds (row r0 + (lane>>4) + 4*reg, column c0 + 16b + (lane&15))
    if (MODE == 0) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            double lo = -INF, hi = INF;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = c0 + 16 * b + (lane & 15);
                if (j < N) dual_interval(acc[b][reg], dred[j], d.vstat[j], tol, lo, hi);
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                lo = fmax(lo, __shfl_xor(lo, off));
                hi = fmin(hi, __shfl_xor(hi, off));
            }
            const int p = r0 + (lane >> 4) + 4 * reg;
            if ((lane & 15) == 0 && p < M) {
                plo[(size_t)p * gridDim.x + blockIdx.x] = lo;
                phi[(size_t)p * gridDim.x + blockIdx.x] = hi;
            }
        }
    } else {
        double lo[4], hi[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            lo[b] = -INF;
            hi[b] = INF;
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int i = r0 + (lane >> 4) + 4 * reg;
            if (i >= M) continue;
            const int u = d.cover[i];
            if (u < 0) continue;
            const double x = d.xr[i], l = d.rlo[i], h = d.rhi[i], sg = unit_sign(d, u, i);
#pragma unroll
            for (int b = 0; b < 4; ++b) primal_interval(-sg * acc[b][reg], x, l, h, tol, lo[b], hi[b]);
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            lo[b] = fmax(lo[b], __shfl_xor(lo[b], 16));
            lo[b] = fmax(lo[b], __shfl_xor(lo[b], 32));
            hi[b] = fmin(hi[b], __shfl_xor(hi[b], 16));
            hi[b] = fmin(hi[b], __shfl_xor(hi[b], 32));
            if (lane < 16) {
                slo[w][16 * b + lane] = lo[b];
                shi[w][16 * b + lane] = hi[b];
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            const int c = c0 + threadIdx.x;
            double L = slo[0][threadIdx.x], H = shi[0][threadIdx.x];
            for (int ww = 1; ww < 4; ++ww) {
                L = fmax(L, slo[ww][threadIdx.x]);
                H = fmin(H, shi[ww][threadIdx.x]);
            }
            if (c < N) {
                plo[(size_t)c * gridDim.y + blockIdx.y] = L;
                phi[(size_t)c * gridDim.y + blockIdx.y] = H;
            }
        }
    }
}

// per bump position: reduce the column-tile partials, add the slack columns of
// the R rows (alpha = Minv[p][c]) -> olo/ohi (delta of c_{S_p}); and per R
// position c: reduce the row-tile partials, add the bump part (g = Minv[p][c]
// on x_S) -> rlo/rhi (delta of b_{R_c})
__global__ void k_sens_final(Dev d, int k, int ntc, int ntr, const double* __restrict__ plo,
                             const double* __restrict__ phi, const double* __restrict__ qlo,
                             const double* __restrict__ qhi, double* olo, double* ohi, double* rlo,
                             double* rhi) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * k) return;
    const double tol = d.ctl->tol_pivot, INF = HUGE_VAL;
    double lo = -INF, hi = INF;
    if (t < k) {
        const int p = t;
        for (int b = 0; b < ntc; ++b) {
            lo = fmax(lo, plo[(size_t)p * ntc + b]);
            hi = fmin(hi, phi[(size_t)p * ntc + b]);
        }
        for (int c = 0; c < k; ++c) {
            const int i = d.Rl[c];
            const int sv = d.n + i;  // the slack of an R row is nonbasic
            dual_interval(d.Minv[(size_t)p * d.ldm + c], -d.y[i], d.vstat[sv], tol, lo, hi);
        }
        olo[p] = lo;
        ohi[p] = hi;
    } else {
        const int c = t - k;
        for (int b = 0; b < ntr; ++b) {
            lo = fmax(lo, qlo[(size_t)c * ntr + b]);
            hi = fmin(hi, qhi[(size_t)c * ntr + b]);
        }
        for (int p = 0; p < k; ++p)
            primal_interval(d.Minv[(size_t)p * d.ldm + c], d.xs[p], d.slo[p], d.shi[p], tol, lo, hi);
        rlo[c] = lo;
        rhi[c] = hi;
    }
}

// ============================================================== dual simplex
// Phase 1 by the dual simplex (lp_solve's default SIMPLEX_DUAL_PRIMAL; oracle
// run_dual, whose arithmetic every kernel here reproduces bit for bit).  One
// iteration (launch_dual_iteration): k_dual_chuzr (leaving-row partials) ->
// k_dual_row (leaving row, rho_r on the bump positions) -> k_dual_price (ONE
// sweep of the Y rows for both d_j = c_j - y'a_j and the pivot row alpha_j =
// rho_r'a_j, Harris candidates compacted per tile) -> k_dual_bfrt (bound-
// flipping ratio test over the compacted candidates, one workgroup) ->
// k_dual_flip_* (a_F = sum of the flipped columns, its FTRAN, x_B -= B^-1 a_F)
// -> the primal iteration's select-FTRAN, FTRAN-z and k_ratio (DUAL: the
// leaving entry is the dual's) -> k_update (also the dual Devex weights).

// oracle solve_core's dual start: cost (minimisation form), boxed columns at
// the bound their cost sign asks for, zero cost where no bound is dual feasible
__global__ void k_dual_setup_cols(Dev d) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.n) return;
    const double cj = d.maximize ? -d.obj[j] : d.obj[j];
    d.cost[j] = cj;
    const double l = d.lb[j], u = d.ub[j];
    if (l > -HUGE_VAL && u < HUGE_VAL && l != u) {
        d.vstat[j] = cj < 0.0 ? VS_UPPER : VS_LOWER;
        d.xval[j] = cj < 0.0 ? u : l;
    }
    const int8_t vs = d.vstat[j];
    if (l != u && ((vs == VS_LOWER && cj < 0.0) || (vs == VS_UPPER && cj > 0.0) || (vs == VS_FREE && cj != 0.0))) {
        d.cost[j] = 0.0;
        atomicAdd(reinterpret_cast<unsigned long long*>(&d.ctl->dflat), 1ull);
    }
}

// every row covered by its slack, feasible or not (after k_init_rows and the
// row activities of the placement above); no artificial, Y empty
__global__ void k_dual_init_rows(Dev d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.m) return;
    const int n = d.n, m = d.m, sv = n + i, av = n + m + i;
    d.vstat[sv] = VS_BASIC;
    d.cover[i] = d.N + i;
    d.xr[i] = d.b[i] - d.ract[i];
    d.xval[sv] = 0.0;
    d.rlo[i] = d.lb[sv];
    d.rhi[i] = d.ub[sv];
    d.lb[av] = 0.0;
    d.ub[av] = 0.0;
    d.cost[av] = 0.0;
    d.vstat[av] = VS_FIXED;
    d.xval[av] = 0.0;
    d.asgn[i] = 1.0;
    d.rpos[i] = -1;
    d.ypos[i] = -1;
    if (i == 0) {
        d.ctl->ny = 0;
        d.ctl->k = 0;
    }
}

// CHUZR total order: the larger infeasibility score, then the lower variable
// id; Bland: the lower variable id
DEV bool chz_better(const ChzRec& a, const ChzRec& b, int bland) {
    if (a.var < 0) return false;
    if (b.var < 0) return true;
    if (bland) return a.var < b.var;
    return a.score > b.score || (a.score == b.score && a.var < b.var);
}
DEV void chz_take(ChzRec& c, const ChzRec& o, bool take) {  // (field-wise, see cand_take)
    c.score = take ? o.score : c.score;
    c.x = take ? o.x : c.x;
    c.beta = take ? o.beta : c.beta;
    c.var = take ? o.var : c.var;
    c.e = take ? o.e : c.e;
    c.s = take ? o.s : c.s;
}
DEV void chz_none(ChzRec& r) {
    r.score = r.x = r.beta = 0.0;
    r.var = r.e = -1;
    r.s = r.pad = 0;
}
// block-wide best of NT records in chz_better's total order (the records' ids
// are distinct): each wave's best by DPP reductions -- the largest score, then
// the lowest id among the lanes holding it (Bland: the lowest id) -- then the
// NT / 64 wave bests through LDS, one barrier (r05; r04: an 8-level LDS tree,
// a barrier per level)
template <int NT>
DEV ChzRec block_best_chz(ChzRec r, int bland, ChzRec* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool valid = r.var >= 0;
    bool in = valid;
    if (!bland) {
        const double smax = wave_max_f64(valid ? r.score : -HUGE_VAL);
        in = valid && r.score == smax;
    }
    const int vmin = wave_min_i32(in ? r.var : 0x7fffffff);
    ChzRec b;
    chz_none(b);
    if (vmin != 0x7fffffff) {
        const int win = __ffsll((long long)__ballot(in && r.var == vmin)) - 1;
        b.score = readlane_f64(r.score, win);
        b.x = readlane_f64(r.x, win);
        b.beta = readlane_f64(r.beta, win);
        b.var = __builtin_amdgcn_readlane(r.var, win);
        b.e = __builtin_amdgcn_readlane(r.e, win);
        b.s = __builtin_amdgcn_readlane(r.s, win);
    }
    if (lane == 0) lds[w] = b;
    __syncthreads();
    ChzRec out = lds[0];
    for (int i = 1; i < NT / 64; ++i) {
        const ChzRec o = lds[i];
        chz_take(out, o, chz_better(o, out, bland));
    }
    __syncthreads();  // (lds may be rewritten by the caller)
    return out;
}

// CHUZR partials: one basic entry per thread (covered rows, then bump positions)
// defer (Dev::dual_defer): first the last plan's x_B / dual Devex / AS part --
// each thread updates the entry it scores (dual_copy_entry), the AS / AR
// copies and a weight reset strided over the launch -- whatever the status
__global__ void __launch_bounds__(256) k_dual_chuzr(Dev d, int defer) {
    __shared__ ChzRec red[256];
    const DevCtl* c = d.ctl;
    const int e = blockIdx.x * 256 + threadIdx.x;
    double wnew = -1.0;  // the entry's updated dual Devex weight (-1: read ddw)
    if (defer && copy_pending(c)) {
        const Plan P = c->plan;
        dual_copy_entry(d, P, e, c->k, &wnew);
        dual_copy_rest(d, P, e, (int64_t)gridDim.x * 256);
    }
    if (c->status != ST_RUN) return;
    const int m = d.m, k = c->k, bland = c->bland, dvx = c->ddevex;
    const double ptol = c->tol_primal;
    ChzRec r;
    chz_none(r);
    int var = -1;
    double x = 0.0, l = 0.0, u = 0.0;
    if (e < m) {
        const int cv = d.cover[e];
        if (cv >= 0) {
            var = cv;
            x = d.xr[e];
            l = d.rlo[e];
            u = d.rhi[e];
        }
    } else if (e - m < k) {
        const int p = e - m;
        var = d.Sl[p];
        x = d.xs[p];
        l = d.slo[p];
        u = d.shi[p];
    }
    if (var >= 0) {
        double delta = 0.0, beta = 0.0;
        int sd = 0;
        if (x < l - ptol) {
            delta = l - x;
            beta = l;
            sd = 1;
        } else if (x > u + ptol) {
            delta = x - u;
            beta = u;
            sd = -1;
        }
        if (sd) {
            r.var = var;
            r.e = e;
            r.x = x;
            r.beta = beta;
            r.s = sd;
            r.score = dvx ? (delta * delta) / (wnew >= 0.0 ? wnew : d.ddw[var]) : delta;
        }
    }
    r = block_best_chz<256>(r, bland, red);
    if (threadIdx.x == 0) d.dchz[blockIdx.x] = r;
}

// The leaving row (every workgroup reduces the CHUZR partials: a total order,
// all agree) and rho_r on the bump positions, one wave per position:
// Minv row p for bump position p; -sigma (A[i,S] Minv)_c for the slack covering
// row i (the oracle's row_times_minv in wave order).  Written in position order
// (rhoR) and on the Y slots (rr, the dense sweep's operand).
// sp (CSC, large bump): A[i, S] from row i's nonzeros in basic columns (CSR +
// spos) as a sparse list, rho_c = sparse_lane_chain over row c of MinvT (the
// dense chain's bits; a row with more than SPL entries takes the dense walk)
// defer (Dev::dual_defer): the last plan's inverse update is still pending --
// rho_r reads the new inverse through minv_new -- and k_dual_chuzr applied its
// copy part (copy_seq)
__global__ void __launch_bounds__(256) k_dual_row(Dev d, int nchz, int lds_row, int sp, int defer) {
    extern __shared__ __attribute__((aligned(16))) double asrow_lds[];  // [k]: A[i, S]
    __shared__ ChzRec red[256];
    __shared__ int s_pos[SPL], s_key[SPL], s_sb[72], s_scan[4];
    __shared__ double s_val[SPL];
    DevCtl* c = d.ctl;
    const bool pend = defer && minv_pending(c);
    const Plan P = c->plan;
    if (defer && blockIdx.x == 0 && threadIdx.x == 0) c->copy_seq = c->plan_seq;
    if (c->status != ST_RUN) return;
    const int m = d.m, k = c->k, bland = c->bland;
    const int tid = threadIdx.x, lane = tid & 63;
    ChzRec r;
    chz_none(r);
    for (int t = tid; t < nchz; t += 256) {
        const ChzRec o = d.dchz[t];
        chz_take(r, o, chz_better(o, r, bland));
    }
    r = block_best_chz<256>(r, bland, red);
    if (r.var < 0) {  // primal feasible: the dual phase is done (the host re-checks)
        if (blockIdx.x == 0 && tid == 0) c->status = ST_PHASE_OPT;
        return;
    }
    const int xrow = r.e < m ? r.e : -1;
    const double xsig = xrow >= 0 ? unit_sign(d, r.var, xrow) : 0.0;
    if (blockIdx.x == 0 && tid == 0) {
        // (a leaving structural's bounds from its bump position: on column-sharded
        //  ranks it may live on another shard; the values are the same)
        const int lv = loc_of(d, r.var);
        c->dr_var = r.var;
        c->dr_e = r.e;
        c->dr_s = r.s;
        c->dr_xrow = xrow;
        c->dr_x = r.x;
        c->dr_beta = r.beta;
        c->dr_lb = xrow >= 0 ? d.lb[lv] : d.slo[r.e - m];
        c->dr_ub = xrow >= 0 ? d.ub[lv] : d.shi[r.e - m];
        c->dr_w = d.ddw[r.var];
        c->dr_xsig = xsig;
    }
    double* asrow = lds_row ? asrow_lds : d.zz;  // (huge bumps: every workgroup writes the same values)
    bool spl = false;
    if (xrow >= 0 && (sp || d.noT)) {  // (no MinvT: always the list when it fits)
        const int64_t t0 = d.rptr[xrow], t1 = d.rptr[xrow + 1];
        spl = t1 - t0 <= SPL;
        if (spl) {
            bool valid = false;
            int p = 0;
            double v = 0.0;
            if (tid < t1 - t0) {
                v = d.rval[t0 + tid];
                p = d.spos[d.cind[t0 + tid]];
                valid = p >= 0 && p < k;
            }
            spl_build<256>(valid, p, v, s_pos, s_val, s_sb, s_key, s_scan);
        }
    }
    if (xrow >= 0 && !spl) {
        for (int p = tid; p < k; p += 256) asrow[p] = d.AS[(size_t)p * (size_t)m + xrow];
        __syncthreads();
    }
    const int lrp = r.e - m;  // (bump position of a leaving structural)
    for (int cc = blockIdx.x * 4 + (tid >> 6); cc < k; cc += gridDim.x * 4) {
        double v;
        if (xrow >= 0) {
            double acc;
            if (pend) {  // row cc of the new MinvT: element (q, cc) of the new Minv
                const OldM oT = d.noT ? OldM{d.Minv, (size_t)d.ldm, false} : OldM{d.MinvT, (size_t)d.ldm, true};
                auto xf = [&](int q) { return minv_new(d, P, q, cc, oT); };
                acc = spl ? sparse_lane_chain_f(xf, s_pos, s_val, s_sb) : lane_chain_f(xf, asrow, k);
            } else if (d.noT) {  // column cc of Minv
                auto xf = [&](int q) { return d.Minv[(size_t)q * d.ldm + cc]; };
                acc = spl ? sparse_lane_chain_f(xf, s_pos, s_val, s_sb) : lane_chain_f(xf, asrow, k);
            } else {
                const double* mrow = d.MinvT + (size_t)cc * d.ldm;
                acc = spl ? sparse_lane_chain(mrow, s_pos, s_val, s_sb) : lane_chain(mrow, asrow, k);
            }
            acc = wave_tree(acc);
            v = -(xsig * acc);
        } else {
            v = pend ? minv_new(d, P, lrp, cc, OldM{d.Minv, (size_t)d.ldm, false}) : d.Minv[(size_t)lrp * d.ldm + cc];
        }
        if (lane == 0) {
            d.rhoR[cc] = v;
            const int slot = d.ypos[d.Rl[cc]];  // (R = Y in the dual phase: every R row has a slot)
            if (slot >= 0) d.rr[slot] = v;
        }
    }
}

// MIP node warm start (oracle warm_core): the nonbasic column's status and
// value under its new bounds, then dual feasibility -- a boxed column whose
// reduced cost has the wrong sign moves to its other bound, anything still
// dual infeasible beyond tol_dual has its cost shifted by -d_j for the dual
// phase (k_phase2 restores the costs).  Slacks: the shift only.
DEV void warm_fix(const Dev& d, int jl, bool structural, double dj, double dtol) {
    int8_t vs = d.vstat[jl];
    if (vs == VS_BASIC) return;
    const double l = d.lb[jl], u = d.ub[jl];
    if (l == u) {
        if (structural) {
            d.vstat[jl] = VS_FIXED;
            d.xval[jl] = l;
        }
        return;
    }
    if (structural) {
        const bool lo_ok = l > -HUGE_VAL, up_ok = u < HUGE_VAL;
        if (vs == VS_FIXED) vs = VS_LOWER;  // (fixed in the last node: the oracle's "lower")
        if (vs == VS_LOWER && !lo_ok) vs = up_ok ? VS_UPPER : VS_FREE;
        else if (vs == VS_UPPER && !up_ok) vs = lo_ok ? VS_LOWER : VS_FREE;
        else if (vs == VS_FREE && (lo_ok || up_ok)) vs = lo_ok ? VS_LOWER : VS_UPPER;
        if (vs == VS_LOWER && dj < -dtol && up_ok) vs = VS_UPPER;
        else if (vs == VS_UPPER && dj > dtol && lo_ok) vs = VS_LOWER;
        d.vstat[jl] = vs;
        d.xval[jl] = vs == VS_LOWER ? l : vs == VS_UPPER ? u : 0.0;
    }
    if ((vs == VS_LOWER && dj < -dtol) || (vs == VS_UPPER && dj > dtol) || (vs == VS_FREE && fabs(dj) > dtol)) {
        d.cost[jl] = d.cost[jl] - dj;
        atomicAdd(reinterpret_cast<unsigned long long*>(&d.ctl->dflat), 1ull);
    }
}

// the node's bounds of the local structurals (scaled; lo / up hold all N
// columns by global id), the real costs, and the bump positions' cached bounds /
// costs; lower > upper on any column flags the node infeasible (every
// column-sharded rank checks all N, so all agree)
__global__ void k_warm_bounds(Dev d, const double* __restrict__ lo, const double* __restrict__ up) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < d.n) {
        d.lb[t] = lo[d.col0 + t];
        d.ub[t] = up[d.col0 + t];
        d.cost[t] = d.maximize ? -d.obj[t] : d.obj[t];
    }
    if (t < d.N && lo[t] > up[t]) atomicOr(&d.ctl->infeasible_bounds, 1);
    if (t < d.m) d.cost[d.n + t] = 0.0;
    if (t < d.ctl->k) {
        const int j = d.Sl[t];  // (a global id)
        d.slo[t] = lo[j];
        d.shi[t] = up[j];
        const double o = d.objg[j];
        d.cS[t] = d.maximize ? -o : o;
    }
}

// a priced column's ratio-test record (oracle run_dual): side +1 acts at its
// lower bound (needs ah < -tol_pivot), -1 at its upper (ah > tol_pivot)
DEV bool dual_candidate(int8_t vs, double a, double dj, double lb, double ub, int rs, int bland, double dtol,
                        double pivtol, int j, double xj, double cj, DualCand& o) {
    if (vs == VS_BASIC || vs == VS_FIXED) return false;
    const double ah = rs * a;
    int side = 0;
    if (vs == VS_LOWER || (vs == VS_FREE && ah < 0.0)) side = ah < -pivtol ? 1 : 0;
    else if (vs == VS_UPPER || (vs == VS_FREE && ah > 0.0)) side = ah > pivtol ? -1 : 0;
    if (!side) return false;
    o.t = side > 0 ? dj / (-ah) : (-dj) / ah;
    o.b = bland ? o.t : side > 0 ? (dj + dtol) / (-ah) : (dtol - dj) / ah;
    o.a = a;
    o.r = (lb > -HUGE_VAL && ub < HUGE_VAL) ? ub - lb : HUGE_VAL;
    o.d = dj;
    o.j = j;
    o.side = side;
    o.lb = lb;
    o.ub = ub;
    o.x = xj;
    o.c = cj;
    o.c0 = 0;
    o.len = -1;
    o.pad = 0;
    return true;
}

// ordered emission of a workgroup's candidates into its region: `flag` per
// thread in thread order (plus a second one right behind it: two columns per
// lane), counts per wave in LDS
template <int NT>
DEV void emit_region(const Dev& d, int region, bool f0, const DualCand& c0, bool f1, const DualCand& c1,
                     int* wcnt) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long b0 = __ballot(f0), b1 = __ballot(f1);
    const unsigned long long below = (1ull << lane) - 1ull;
    const int before = __popcll(b0 & below) + __popcll(b1 & below);
    if (lane == 0) wcnt[w] = __popcll(b0) + __popcll(b1);
    __syncthreads();
    int off = 0, tot = 0;
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) off += wcnt[i];
        tot += wcnt[i];
    }
    DualCand* base = d.dcand + (size_t)region * DREG;
    if (f0) base[off + before] = c0;
    if (f1) base[off + before + (f0 ? 1 : 0)] = c1;
    if (threadIdx.x == 0) d.dcnt[region] = tot;
}

// the slack columns of the Y rows (cost 0: d = -y, alpha = rho on the slot)
template <int NT>
DEV void dual_slacks(const Dev& d, int region, int s, int nsw, int* wcnt, int warm) {
    const DevCtl* c = d.ctl;
    const int ny = c->ny, bland = c->bland, rs = c->dr_s;
    const double dtol = c->tol_dual, pivtol = c->tol_pivot;
    const int p = s * NT + threadIdx.x;  // (the host sizes nsw for one slot per thread)
    DualCand o;
    bool f = false;
    if (warm) {
        if (p < ny) {
            const int sv = d.n + d.Yl[p];
            warm_fix(d, sv, false, d.cost[sv] - d.yy[p], dtol);
        }
        return;
    }
    if (p < ny) {
        const int8_t v = d.yvs[p];
        const int i = d.Yl[p];
        const int sv = d.n + i;
        f = dual_candidate(v, d.rr[p], d.cost[sv] - d.yy[p], d.lb[sv], d.ub[sv], rs, bland, dtol, pivtol, d.N + i,
                           d.xval[sv], d.cost[sv], o);
    }
    emit_region<NT>(d, region, f, o, false, o, wcnt);
}

// Dense pivot row + pricing: one sweep of the tile's Y rows with both y and
// rho (wave w: slot class p = w mod 4, fma chains in slot order; the classes
// added in order), then wave 0 finishes columns 2 lane, 2 lane + 1: d_j,
// alpha_j (+ sigma a_ij of a covered leaving row i, last), the candidates.
// Grid: [nsw slack workgroups][ntiles tiles].
// warm != 0 (MIP node warm start): the same pass for d_j alone (rho = 0), each
// nonbasic column re-placed by warm_fix instead of a candidate
// (+ napply trailing workgroups: the deferred plan's MinvT update, dual_defer)
__global__ void __launch_bounds__(PRICE_THREADS) k_dual_price(Dev d, int nsw, int warm, int napply) {
    __shared__ double pd[PRICE_SPLIT][TILE_COLS], pa[PRICE_SPLIT][TILE_COLS];
    __shared__ int wcnt[PRICE_SPLIT];
    const DevCtl* c = d.ctl;
    if (napply > 0 && (int)blockIdx.x >= (int)gridDim.x - napply) {
        if (minv_pending(c)) {
            const Plan P = c->plan;
            const int wg = (int)blockIdx.x - ((int)gridDim.x - napply);
            apply_minv_part(d, P, 1, (int64_t)wg * blockDim.x + threadIdx.x, (int64_t)napply * blockDim.x);
        }
        return;
    }
    if (c->status != ST_RUN) return;
    if ((int)blockIdx.x < nsw) {
        dual_slacks<PRICE_THREADS>(d, d.ntiles + blockIdx.x, blockIdx.x, nsw, wcnt, warm);
        return;
    }
    const int64_t tile = (int64_t)blockIdx.x - nsw;
    const int tw = d.tile_w, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ny = c->ny;
    const int lcol = 2 * lane < tw ? 2 * lane : ((tw - 1) & ~1);
    const double* col = d.AR + (size_t)tile * (size_t)d.arcap * (size_t)tw + lcol;
    double d0 = 0.0, d1 = 0.0, a0 = 0.0, a1 = 0.0;
    constexpr int U = 8;
    int p = w;
    for (; p + PRICE_SPLIT * (U - 1) < ny; p += PRICE_SPLIT * U) {
        dbl2 v[U];
        double yv[U], rv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = *reinterpret_cast<const dbl2*>(col + (size_t)(p + PRICE_SPLIT * u) * (size_t)tw);
            yv[u] = d.yy[p + PRICE_SPLIT * u];
            rv[u] = d.rr[p + PRICE_SPLIT * u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            d0 = fma(v[u].x, yv[u], d0);
            d1 = fma(v[u].y, yv[u], d1);
            a0 = fma(v[u].x, rv[u], a0);
            a1 = fma(v[u].y, rv[u], a1);
        }
    }
    for (; p < ny; p += PRICE_SPLIT) {
        const dbl2 v = *reinterpret_cast<const dbl2*>(col + (size_t)p * (size_t)tw);
        const double yv = d.yy[p], rv = d.rr[p];
        d0 = fma(v.x, yv, d0);
        d1 = fma(v.y, yv, d1);
        a0 = fma(v.x, rv, a0);
        a1 = fma(v.y, rv, a1);
    }
    pd[w][2 * lane] = d0;
    pd[w][2 * lane + 1] = d1;
    pa[w][2 * lane] = a0;
    pa[w][2 * lane + 1] = a1;
    __syncthreads();
    // wave 0 finishes the tile's columns; waves 1..3 only take part in the
    // emission's barrier (no candidates of their own)
    const int xrow = warm ? -1 : c->dr_xrow, rs = c->dr_s, bland = c->bland;
    const double xsig = c->dr_xsig, dtol = c->tol_dual, pivtol = c->tol_pivot;
    DualCand o[2];
    bool f[2] = {false, false};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int64_t j = tile * tw + 2 * lane + h;
        if (w != 0 || 2 * lane + h >= tw || j >= d.n) continue;
        const int8_t vs = d.vstat[j];
        if (warm) {
            if (vs == VS_BASIC) continue;
            double td = 0.0;
#pragma unroll
            for (int ww = 0; ww < PRICE_SPLIT; ++ww) td = td + pd[ww][2 * lane + h];
            warm_fix(d, (int)j, true, d.cost[j] - td, dtol);
            continue;
        }
        if (vs == VS_BASIC || vs == VS_FIXED) continue;
        double td = 0.0, ta = 0.0;
#pragma unroll
        for (int ww = 0; ww < PRICE_SPLIT; ++ww) {
            td = td + pd[ww][2 * lane + h];
            ta = ta + pa[ww][2 * lane + h];
        }
        const double dj = d.cost[j] - td;
        const double aj = xrow >= 0 ? fma(xsig, a_row(d, xrow, j), ta) : ta;
        f[h] = dual_candidate(vs, aj, dj, d.lb[j], d.ub[j], rs, bland, dtol, pivtol, (int)(d.col0 + j), d.xval[j],
                              d.cost[j], o[h]);
    }
    if (warm) return;
    emit_region<PRICE_THREADS>(d, (int)tile, f[0], o[0], f[1], o[1], wcnt);
}

// CSC pivot row + pricing: one column chain per thread over its nonzeros in
// ascending rows with the dense y and rho (rho_i from the bump positions
// through rpos, sigma on a covered leaving row)
__global__ void __launch_bounds__(TILE_COLS) k_dual_price_csc(Dev d, int nsw, int warm, int napply) {
    __shared__ int wcnt[TILE_COLS / 64];
    const DevCtl* c = d.ctl;
    if (napply > 0 && (int)blockIdx.x >= (int)gridDim.x - napply) {
        if (minv_pending(c)) {
            const Plan P = c->plan;
            const int wg = (int)blockIdx.x - ((int)gridDim.x - napply);
            if (d.sru_on) apply_minv_sru<TILE_COLS>(d, P, wg, napply);
            else apply_minv_part(d, P, 1, (int64_t)wg * blockDim.x + threadIdx.x, (int64_t)napply * blockDim.x);
        }
        return;
    }
    const int64_t tile = (int64_t)blockIdx.x - nsw;
    const int64_t j = tile * TILE_COLS + threadIdx.x;
    // the column's record and the control fields, issued with the status
    // (straight-line: one round trip, not two)
    const int64_t jc = j < 0 ? 0 : j < d.n ? j : (d.n > 0 ? d.n - 1 : 0);
    const int8_t vsj = d.vstat[jc];
    const int64_t ta = d.cptr[jc], tb = d.cptr[jc + 1];
    const double cj = d.cost[jc], lbj = d.lb[jc], ubj = d.ub[jc], xj = d.xval[jc];
    const int xrow = warm ? -1 : c->dr_xrow, rs = c->dr_s, bland = c->bland;
    const double xsig = c->dr_xsig, dtol = c->tol_dual, pivtol = c->tol_pivot;
    __builtin_amdgcn_sched_barrier(0);
    if (c->status != ST_RUN) {
        KEEP(ta);
        KEEP(cj);
        KEEP(xj);
        return;
    }
    if ((int)blockIdx.x < nsw) {
        dual_slacks<TILE_COLS>(d, d.ntiles + blockIdx.x, blockIdx.x, nsw, wcnt, warm);
        return;
    }
    DualCand o;
    bool f = false;
    if (warm) {
        if (j < d.n && d.vstat[j] != VS_BASIC) {
            double ad = 0.0;
            for (int64_t t = d.cptr[j]; t < d.cptr[j + 1]; ++t) ad = fma(d.cval[t], d.y[d.rind[t]], ad);
            warm_fix(d, (int)j, true, d.cost[j] - ad, dtol);
        }
        return;
    }
    if (j < d.n) {
        const int8_t vs = vsj;
        if (vs != VS_BASIC && vs != VS_FIXED) {
            // batches of DPB entries: each level of the row index -> rpos / y ->
            // rho_R gathers in flight together (one round trip per level, not
            // three per nonzero), the chains in ascending rows as before
            constexpr int DPB = 1;  // (r05: batches of 4 measured slower, 13.1 -> 15.3 us)
            double ad = 0.0, aa = 0.0;
            const int64_t t1 = tb;
            for (int64_t t0 = ta; t0 < t1; t0 += DPB) {
                int ii[DPB], rp[DPB];
                double vv[DPB], yv[DPB], rh[DPB];
#pragma unroll
                for (int b = 0; b < DPB; ++b) {
                    const int64_t tt = t0 + b < t1 ? t0 + b : t1 - 1;
                    ii[b] = d.rind[tt];
                    vv[b] = d.cval[tt];
                }
#pragma unroll
                for (int b = 0; b < DPB; ++b) {
                    rp[b] = d.rpos[ii[b]];
                    yv[b] = d.y[ii[b]];
                }
#pragma unroll
                for (int b = 0; b < DPB; ++b) rh[b] = d.rhoR[rp[b] >= 0 ? rp[b] : 0];
#pragma unroll
                for (int b = 0; b < DPB; ++b)
                    if (t0 + b < t1) {
                        const double rho = rp[b] >= 0 ? rh[b] : (ii[b] == xrow ? xsig : 0.0);
                        ad = fma(vv[b], yv[b], ad);
                        aa = fma(vv[b], rho, aa);
                    }
            }
            f = dual_candidate(vs, aa, cj - ad, lbj, ubj, rs, bland, dtol, pivtol, (int)j, xj, cj, o);
            o.c0 = ta;
            o.len = (int)(t1 - ta < (1 << 30) ? t1 - ta : (1 << 30));
        }
    }
    emit_region<TILE_COLS>(d, (int)tile, f, o, false, o, wcnt);
}

// Bound-flipping Harris ratio test (oracle run_dual), one workgroup: compacts
// the regions' candidates (region order = ascending structural id, then the
// slacks), then takes bunches -- the live candidates whose exact ratio is
// within the smallest Harris bound -- flipping a bunch while all of it is boxed
// and the slope (x_r's infeasibility) stays above tol_primal past the sum of
// its |alpha| (u - l) in ascending id, else letting the bunch's largest |alpha|
// enter (Bland: the smallest ratio).  Each thread owns a contiguous run of the
// compacted candidates, so ordered compactions are one block scan.
constexpr int BF_NT = 1024;
constexpr int BF_BUN = 1024;  // bunch entries staged in LDS for the flip sum (16 KiB)
constexpr int BF_RR = 4;      // candidates per thread held in registers (N <= 4096)
// ELP_BFRT_REG (test hook): 0 every candidate set takes the workgroup path from
// global memory, 1 the workgroup path from registers (up to 4096 candidates),
// 2 (default) also the one-wave path for up to 64 * BF_RR candidates
static int bfrt_reg() {
    static const int mode = [] {
        const char* e = std::getenv("ELP_BFRT_REG");
        return e ? std::atoi(e) : 2;
    }();
    return mode;
}
// the regions' candidates in region order into dst[0, total): region counts
// scanned in chunks of BF_NT regions, then the chunk's records copied by the
// whole workgroup (output slot o -> its region by a binary search over the
// scanned offsets in LDS), so the copies are independent loads in flight
// instead of one thread walking a region's records one after another (a
// region holds up to DREG)
// s_rec (k_dual_bfrt's fast tail; one chunk of regions): when the regions hold
// <= 64 candidates they go to s_rec in LDS instead of dst -- no global stores
// for the barrier after the compaction to wait on, no reload (r05: loading
// every region's first record with its count, to save the second round trip,
// measured 1 us slower: ~900 scattered 80-byte records)
DEV int compact_regions(const Dev& d, int nreg, DualCand* dst, int* scan_lds, DualCand* s_rec = nullptr) {
    __shared__ int s_off[BF_NT];
    const int tid = threadIdx.x;
    int total = 0;
    for (int r0 = 0; r0 < nreg; r0 += BF_NT) {
        const int r = r0 + tid;
        const int cnt = r < nreg ? d.dcnt[r] : 0;
        int excl;
        const int tot = block_scan_excl<BF_NT>(cnt, &excl, scan_lds);
        s_off[tid] = excl;
        __syncthreads();
        for (int o = tid; o < tot; o += BF_NT) {
            // the last region whose offset is <= o (empty regions share their
            // successor's offset; regions past nreg sit at tot > o)
            int lo = 0, hi = BF_NT - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_off[mid] <= o) lo = mid;
                else hi = mid - 1;
            }
            const DualCand* src = d.dcand + (size_t)(r0 + lo) * DREG + (o - s_off[lo]);
            if (s_rec && tot <= 64) s_rec[o] = *src;  // (uniform: one chunk, nreg <= BF_NT)
            else dst[total + o] = *src;
        }
        total += tot;
        __syncthreads();  // (s_off is rewritten by the next chunk)
    }
    return total;
}

// column-sharded ranks: this shard's candidates (and the last rank's slack
// candidates) packed into dsend -- record 0 carries the count
__global__ void __launch_bounds__(BF_NT) k_dual_pack(Dev d, int nreg) {
    __shared__ int scan_lds[BF_NT / 64];
    if (d.ctl->status != ST_RUN) return;
    const int total = compact_regions(d, nreg, d.dsend + 1, scan_lds);
    if (threadIdx.x == 0) d.dsend[0].j = total;
}

// Up to 64 candidates (the common case: ~42 per dual pivot on the 20 000 x
// 100 000 KKT LP): one per lane, so a bunch round is a DPP minimum, one ballot
// and the flip sum as lane 0's fma chain over the members' (|alpha|, u - l)
// read lane by lane in lane order -- no LDS, no register slots to scan (r05:
// ~0.8 us per round in bfrt_wave, mostly dependent latency of its four-slot
// bookkeeping).  The same decisions in the same order.
// out (k_dual_bfrt's fast tail, one GPU CSC): the records are in s_rec (LDS);
// the flips' ids / dx go to ofj / ofdx from the lanes that hold them
DEV void bfrt_wave1(const Dev& d, int N, int bland, double ptol, double slope, int* nflip_out, int* qidx_out,
                    int* s_flip, unsigned long long* s_st, bool out = false, DualCand* s_rec = nullptr,
                    int* ofj = nullptr, double* ofdx = nullptr) {
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    const double INF = HUGE_VAL;
    double rt = 0.0, rb = 0.0, ra = 0.0, rw = 0.0;
    int rj = 0;
    bool live = lane < N;
    if (live) {  // (out: the compaction left the records in s_rec)
        const DualCand* o = out ? s_rec + lane : d.dcomp + lane;
        rt = o->t;
        rb = o->b;
        ra = fabs(o->a);
        rw = o->r;
        rj = o->j;
    }
    int nflip = 0, qidx = -1, rounds = 0;
    BSTAMP(7);
    for (;;) {
        ++rounds;
        if (!__any(live)) break;  // nothing left: the dual ray (q = -1)
        const double thmax = wave_min_f64(live ? rb : INF);
        const bool mem = live && rt <= thmax;
        const unsigned long long mm = __ballot(mem);
        if (mm == 0ull) break;  // (NaN ratios only: no candidate qualifies -- the ray)
        const bool boxed = __all(!mem || rw != INF);
        double sum = 0.0;
        if (boxed)  // |alpha| (u - l) in lane order (= the compacted order)
            for (unsigned long long mk = mm; mk; mk &= mk - 1ull) {
                const int l = __ffsll((long long)mk) - 1;
                sum = fma(readlane_f64(ra, l), readlane_f64(rw, l), sum);
            }
        if (boxed && sum < slope - ptol) {  // flip the bunch
            slope = slope - sum;
            if (mem) {
                const int pos = nflip + __popcll(mm & below);
                s_flip[pos] = lane;
                if (out) {  // dx = +-(u - l) (LDS only: k_dual_bfrt stores the flips after its last barrier)
                    const DualCand& o = s_rec[lane];
                    ofj[pos] = o.j;
                    ofdx[pos] = o.side > 0 ? o.ub - o.lb : o.lb - o.ub;
                }
            }
            nflip += __popcll(mm);
            live = live && !mem;
            continue;
        }
        // the bunch's best enters: the largest |alpha| (Bland: the smallest
        // ratio), then the lowest id
        const double key = mem ? (bland ? -rt : ra) : -INF;
        const double kmax = wave_max_f64(key);
        const bool at = mem && key == kmax;
        const unsigned long long w = __ballot(at);
        qidx = w ? lowest_index_lane(w, at, rj) : lowest_index_lane(mm, mem, rj);
        break;
    }
    BSTAMP(9);
    if (ELP_DIAG && threadIdx.x == 0) s_st[15] = (unsigned long long)rounds;
    *nflip_out = nflip;
    *qidx_out = qidx;
}

// Small candidate sets (N <= 64 * BF_RR, the usual case: ~36 candidates per
// dual pivot on kkt_2000x10000, ~5 bunch rounds) run the bunch rounds in one
// wave: lane l holds its run of the compacted candidates in registers, the
// round's minimum, prefix count, all-boxed test and entering choice are wave
// shuffles (no workgroup barrier per step), the flip sum is lane 0's in-order
// fma chain over the bunch staged in LDS.  Same decisions as the block path.
DEV void bfrt_wave(const Dev& d, int N, int bland, double ptol, double slope, double* s_bun, int* nflip_out,
                   int* qidx_out, int* s_flip, int dslot) {
    const int lane = threadIdx.x & 63;
    const int run = (N + 63) / 64;
    const int lo = min(N, lane * run), hi = min(N, lo + run);
    const double INF = HUGE_VAL;
    const unsigned long long below = (1ull << lane) - 1ull;
    double rt[BF_RR], rb[BF_RR], ra[BF_RR], rw[BF_RR];
    int rj[BF_RR];
    unsigned ral = 0;
#pragma unroll
    for (int q = 0; q < BF_RR; ++q) {
        rt[q] = rb[q] = ra[q] = rw[q] = 0.0;
        rj[q] = 0;
        if (lo + q < hi) {
            const DualCand& o = d.dcomp[lo + q];
            rt[q] = o.t;
            rb[q] = o.b;
            ra[q] = fabs(o.a);
            rw[q] = o.r;
            rj[q] = o.j;
            ral |= 1u << q;
        }
    }
    int nflip = 0, qidx = -1, rounds = 0;
    RSTAMP(27);
    for (;;) {
        ++rounds;
        if (!__any(ral != 0)) break;  // nothing left: the dual ray (q = -1)
        double bmin = INF;
#pragma unroll
        for (int q = 0; q < BF_RR; ++q)
            if (ral >> q & 1u) bmin = fmin(bmin, rb[q]);
        const double thmax = wave_min_f64(bmin);  // (DPP; uniform)
        unsigned rbun = 0;
        int allbox = 1;
#pragma unroll
        for (int q = 0; q < BF_RR; ++q)
            if ((ral >> q & 1u) && rt[q] <= thmax) {
                rbun |= 1u << q;
                if (rw[q] == INF) allbox = 0;
            }
        // the bunch in order (lane-major runs = ascending id): this lane's
        // members' ranks from one ballot per register slot
        int before = 0, nq = 0;
#pragma unroll
        for (int q = 0; q < BF_RR; ++q) {
            const unsigned long long bq = __ballot((rbun >> q & 1u) != 0u);
            before += __popcll(bq & below);
            nq += __popcll(bq);
        }
        const bool boxed = __all(allbox);
        // (|alpha|, u - l) to LDS for the sum, compact indices to the flip list
        // in LDS; this lane's best member for the entering choice
        double ba = -1.0, bt = INF;
        int bj = -1, bi = -1;
        int o = before;
#pragma unroll
        for (int q = 0; q < BF_RR; ++q)
            if (rbun >> q & 1u) {
                s_bun[2 * o] = ra[q];
                s_bun[2 * o + 1] = rw[q];
                s_flip[nflip + o] = lo + q;
                ++o;
                const bool take = bi < 0 || (bland ? (rt[q] < bt || (rt[q] == bt && rj[q] < bj))
                                                   : (ra[q] > ba || (ra[q] == ba && rj[q] < bj)));
                if (take) {
                    ba = ra[q];
                    bt = rt[q];
                    bj = rj[q];
                    bi = lo + q;
                }
            }
        if (nq == 0) break;  // (NaN ratios only: no candidate qualifies -- the ray)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double sum = 0.0;
        if (lane == 0 && boxed)  // |alpha| (u - l) in ascending id (nq <= N <= 64 BF_RR < BF_BUN)
            for (int t = 0; t < nq; ++t) sum = fma(s_bun[2 * t], s_bun[2 * t + 1], sum);
        sum = readlane_f64(sum, 0);
        __builtin_amdgcn_wave_barrier();  // (s_bun is rewritten by the next round)
        if (boxed && sum < slope - ptol) {  // flip the bunch
            slope = slope - sum;
            ral &= ~rbun;
            nflip += nq;
            continue;
        }
        // the bunch's best enters: the largest |alpha| (Bland: the smallest
        // ratio), then the lowest id -- each lane holds its own runs' best, and
        // ids ascend with the lane, so the lowest lane among the best values
        const bool has = bi >= 0;
        const double key = has ? (bland ? -bt : ba) : -INF;
        const double kmax = wave_max_f64(key);
        // (the lowest id among the lanes at the best value: slack candidates
        //  follow the Y slots, not ascending id)
        const bool at = has && key == kmax;
        const unsigned long long w = __ballot(at);
        const int win = w ? lowest_index_lane(w, at, bj) : lowest_index_lane(__ballot(has), has, bj);
        qidx = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(bi, win));
        break;
    }
    if (ELP_DIAG && d.dstamp && threadIdx.x == 0) d.dstamp[dslot * DSTAMP_STRIDE + 28] = (unsigned long long)rounds;
    *nflip_out = nflip;
    *qidx_out = qidx;
}

// CSC (one GPU): a_F = sum of the flipped columns times their dx, each row one
// fma chain in flip order (oracle run_dual).  Up to AF_PAR entries of flipped
// columns: one thread per entry, the first entry of each row runs that row's
// chain over the entries after it (rows of a column are distinct, so the
// entries in flip order are the chain's terms in order); only the last a_F's
// support is cleared first (Dev::afs), and a_F[R] leaves as the select
// kernel's sparse list (Dev::afl).  More: the flips one after the other, a
// barrier each, after clearing all of a_F (r04's path).
constexpr int AF_PAR = 256;
// The flips' entries grouped by row (bfrt_flip_column, bfrt_flip_lds): an
// open-addressed LDS table of the rows (E <= AF_PAR < AF_HT entries: probing
// ends) holding each row's entries as a bit set over the entry index, so the
// row's first entry runs the chain over the row's own entries in ascending
// index -- flip order, the same terms in the same order -- instead of every
// thread scanning all E entries twice (r05zk: 29 us per launch at ~83
// entries, against 12 us for the one-wave path).  Clear before a barrier,
// insert before the next, chain after it.
constexpr int AF_HT = 2 * AF_PAR, AF_W = AF_PAR / 64;
DEV int* af_hkey() {
    __shared__ int k[AF_HT];
    return k;
}
DEV unsigned long long* af_hbit() {
    __shared__ unsigned long long b[AF_HT * AF_W];
    return b;
}
DEV void af_tab_clear() {
    int* hk = af_hkey();
    unsigned long long* hb = af_hbit();
    for (int t = threadIdx.x; t < AF_HT; t += blockDim.x) {
        hk[t] = -1;
#pragma unroll
        for (int w = 0; w < AF_W; ++w) hb[t * AF_W + w] = 0ull;
    }
}
// entry e (< AF_PAR) of row `row` (>= 0) into the table; returns its slot
DEV int af_tab_insert(int row, int e) {
    int* hk = af_hkey();
    int slot = (int)(((unsigned)row * 2654435761u) >> 23) & (AF_HT - 1);
    for (;;) {
        const int pr = atomicCAS(&hk[slot], -1, row);
        if (pr == -1 || pr == row) break;
        slot = (slot + 1) & (AF_HT - 1);
    }
    atomicOr(&af_hbit()[slot * AF_W + (e >> 6)], 1ull << (e & 63));
    return slot;
}
// entry e leads its row when it is the row's first; the lead's chain in acc
DEV bool af_tab_chain(int slot, int e, const double* s_v, const double* s_dx, double& acc) {
    const unsigned long long* hb = af_hbit() + slot * AF_W;
    unsigned long long bw[AF_W];
#pragma unroll
    for (int w = 0; w < AF_W; ++w) bw[w] = hb[w];
    int first = -1;
#pragma unroll
    for (int w = AF_W - 1; w >= 0; --w)
        if (bw[w]) first = 64 * w + __ffsll((long long)bw[w]) - 1;
    if (first != e) return false;
#pragma unroll
    for (int w = 0; w < AF_W; ++w)
        for (unsigned long long mk = bw[w]; mk; mk &= mk - 1ull) {
            const int x = 64 * w + __ffsll((long long)mk) - 1;
            acc = fma(s_v[x], s_dx[x], acc);
        }
    return true;
}
// (myj / mydx: thread t's flip t, t < nflip <= BF_NT -- its column and dx)
DEV void bfrt_flip_column(const Dev& d, int nflip, int k, int myj, double mydx) {
    __shared__ int s_off[BF_NT], s_lpos[SPL], s_lkey[SPL], s_lsb[72], s_scan[BF_NT / 64];
    __shared__ double s_v[AF_PAR], s_dx[AF_PAR], s_lval[SPL];
    __shared__ int64_t s_c0[BF_NT];
    __shared__ double s_fdx[BF_NT];
    const int tid = threadIdx.x, m = d.m;
    af_tab_clear();
    int len = 0;
    if (tid < nflip) {
        const int64_t c0 = d.cptr[myj];
        len = (int)(d.cptr[myj + 1] - c0);
        s_c0[tid] = c0;
        s_fdx[tid] = mydx;
    }
    __syncthreads();  // (also: the flip ids / dx written above, for the sequential path)
    int excl = 0, E = AF_PAR + 1;
    if (nflip <= BF_NT) E = block_scan_excl<BF_NT>(len, &excl, s_scan);
    const bool par = E <= AF_PAR;
    const int pn = d.afs[0];
    if (pn < 0 || !par) {
        for (int i = tid; i < m; i += BF_NT) d.aF[i] = 0.0;
    } else {
        for (int t = tid; t < pn; t += BF_NT) d.aF[d.afs[1 + t]] = 0.0;
    }
    if (!par) {
        __syncthreads();
        for (int f = 0; f < nflip; ++f) {
            const int j = d.dflip[f];
            const double dx = d.dflipdx[f];
            for (int64_t t = d.cptr[j] + tid; t < d.cptr[j + 1]; t += BF_NT) {
                const int i = d.rind[t];
                d.aF[i] = fma(d.cval[t], dx, d.aF[i]);
            }
            __syncthreads();
        }
        if (tid == 0) {
            d.afs[0] = -1;
            d.afl[0] = -1;
        }
        return;
    }
    if (tid < nflip) s_off[tid] = excl;
    __syncthreads();  // (also orders the clear before the chains' stores)
    int row = -1, slot = 0;
    if (tid < E) {
        int lo = 0, hi = nflip - 1;  // the last flip whose offset is <= tid
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= tid) lo = mid;
            else hi = mid - 1;
        }
        const int64_t t = s_c0[lo] + (tid - s_off[lo]);
        row = d.rind[t];
        s_v[tid] = d.cval[t];
        s_dx[tid] = s_fdx[lo];
        slot = af_tab_insert(row, tid);
    }
    __syncthreads();
    bool lead = false;
    double acc = 0.0;
    int p = -1;
    if (tid < E) {
        lead = af_tab_chain(slot, tid, s_v, s_dx, acc);
        if (lead) {
            d.aF[row] = acc;
            p = d.rpos[row];
        }
    }
    int lex;
    const int nl = block_scan_excl<BF_NT>(lead ? 1 : 0, &lex, s_scan);
    if (lead) d.afs[1 + lex] = row;
    const int n = spl_build<BF_NT>(lead && p >= 0 && p < k, p, acc, s_lpos, s_lval, s_lsb, s_lkey, s_scan);
    for (int t = tid; t < n; t += BF_NT) {
        d.afl[AFL_POS + t] = s_lpos[t];
        d.aflv[t] = s_lval[t];
    }
    if (tid <= 64) d.afl[AFL_SB + tid] = s_lsb[tid];
    if (tid == 0) {
        d.afs[0] = nl;
        d.afl[0] = n;
    }
}

// The fast tail's a_F (one GPU, CSC, <= 64 candidates): the candidates'
// columns -- up to BF_ENT entries each, with the rows' bump positions -- were
// loaded into LDS by waves 1-8 while wave 0 ran the bunch rounds, and a_F's
// old support was cleared then too (k_dual_bfrt), so after the decision the
// chains, the support list and the a_F[R] list come from LDS: bfrt_flip_column's
// arithmetic without its four dependent global round trips.  Returns false
// (uniform) when a flipped column is longer than BF_ENT or the flips hold more
// than AF_PAR entries: the caller then runs bfrt_flip_column.
constexpr int BF_ENT = 8;
DEV bool bfrt_flip_lds(const Dev& d, int nflip, int k, const int* s_flip, const int* s_clen, const int* s_erow,
                       const double* s_eval, const int* s_erp, const double* s_fdx, unsigned long long* s_st) {
    __shared__ int s_off[64], s_lpos[SPL], s_lkey[SPL], s_lsb[72], s_scan[BF_NT / 64];
    __shared__ double s_v[AF_PAR], s_dx[AF_PAR], s_lval[SPL];
    __shared__ int s_bad;
    const int tid = threadIdx.x;
    af_tab_clear();  // (the entries grouped by row)
    int len = 0;
    if (tid == 0) s_bad = 0;
    if (tid < nflip) len = s_clen[s_flip[tid]];
    int excl;
    const int E = block_scan_excl<BF_NT>(len > 0 ? len : 0, &excl, s_scan);
    if (len < 0) s_bad = 1;  // (a slack or an overlong column)
    if (tid < nflip) s_off[tid] = excl;
    __syncthreads();
    BSTAMP(10);
    if (s_bad || E > AF_PAR) return false;
    int row = -1, rp = -1, slot = 0;
    if (tid < E) {
        int lo = 0, hi = nflip - 1;  // the last flip whose offset is <= tid
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= tid) lo = mid;
            else hi = mid - 1;
        }
        const int sl = s_flip[lo] * BF_ENT + (tid - s_off[lo]);
        row = s_erow[sl];
        rp = s_erp[sl];
        s_v[tid] = s_eval[sl];
        s_dx[tid] = s_fdx[lo];
        slot = af_tab_insert(row, tid);
    }
    __syncthreads();
    bool lead = false;
    double acc = 0.0;
    if (tid < E) lead = af_tab_chain(slot, tid, s_v, s_dx, acc);
    // (every global store after the last barrier: a barrier waits for the
    //  workgroup's outstanding stores)
    BSTAMP(11);
    int lex;
    const int nl = block_scan_excl<BF_NT>(lead ? 1 : 0, &lex, s_scan);
    BSTAMP(12);
    const int n = spl_build<BF_NT>(lead && rp >= 0 && rp < k, rp, acc, s_lpos, s_lval, s_lsb, s_lkey, s_scan);
    BSTAMP(13);
    if (lead) {
        d.aF[row] = acc;
        d.afs[1 + lex] = row;
    }
    for (int t = tid; t < n; t += BF_NT) {
        d.afl[AFL_POS + t] = s_lpos[t];
        d.aflv[t] = s_lval[t];
    }
    if (tid <= 64) d.afl[AFL_SB + tid] = s_lsb[tid];
    if (tid == 0) {
        d.afs[0] = nl;
        d.afl[0] = n;
    }
    return true;
}

// The fast tail's a_F when the flips hold <= 64 entries (the usual case: ~23):
// wave 0 alone, no barrier -- entry t in lane t (its flip by the offsets'
// scan in registers), the first lane of each row runs that row's chain over
// the later lanes in flip order (readlane: the same terms in the same order as
// bfrt_flip_column), the support list by ballot, and the a_F[R] list ranked by
// (position mod 64, position) and bucketed as spl_build's, straight to memory.
// r05t stamps: the block-level version spent ~6 us in its O(E) LDS loops.
DEV void bfrt_flip_wave(const Dev& d, int nflip, int E, int k, const int* s_flip, const int* s_clen,
                        const int* s_erow, const double* s_eval, const int* s_erp, const double* s_fdx,
                        unsigned long long* s_st) {
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    const int len = lane < nflip ? s_clen[s_flip[lane]] : 0;
    int incl = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off);
        if (lane >= off) incl += u;
    }
    const int excl = incl - len;
    int f = 0;  // this entry's flip: the last one whose offset is <= lane
    for (int g = 1; g < nflip; ++g)
        if (__builtin_amdgcn_readlane(excl, g) <= lane) f = g;
    const bool has = lane < E;
    int row = -1, rp = -1;
    double v = 0.0, dx = 0.0;
    if (has) {
        const int sl = s_flip[f] * BF_ENT + (lane - __shfl(excl, f));
        row = s_erow[sl];
        rp = s_erp[sl];
        v = s_eval[sl];
        dx = s_fdx[f];
    }
    BSTAMP(11);
    // the entries grouped by row through the row table (af_tab_*; 128 slots and
    // one mask word here: E <= 64): the row's first lane walks its own lanes in
    // ascending order -- flip order, the same chain -- instead of E readlane
    // steps on every lane (~37 ns each, r05zj).  One wave: its LDS operations
    // complete in order, so no barrier between the clear, the inserts and the reads.
    __shared__ double w_v[64], w_dx[64];
    int* hk = af_hkey();
    unsigned long long* hb = af_hbit();
    hk[lane] = -1;
    hk[64 + lane] = -1;
    hb[lane * AF_W] = 0ull;
    hb[(64 + lane) * AF_W] = 0ull;
    w_v[lane] = v;
    w_dx[lane] = dx;
    int slot = 0;
    if (has) {
        slot = (int)(((unsigned)row * 2654435761u) >> 25);
        for (;;) {
            const int pr = atomicCAS(&hk[slot], -1, row);
            if (pr == -1 || pr == row) break;
            slot = (slot + 1) & 127;
        }
        atomicOr(&hb[slot * AF_W], 1ull << lane);
    }
    bool lead = false;
    double acc = 0.0;
    if (has) {
        const unsigned long long bw = hb[slot * AF_W];
        lead = __ffsll((long long)bw) - 1 == lane;
        if (lead)
            for (unsigned long long mk = bw; mk; mk &= mk - 1ull) {
                const int e = __ffsll((long long)mk) - 1;
                acc = fma(w_v[e], w_dx[e], acc);
            }
    }
    BSTAMP(12);
    const unsigned long long lm = __ballot(lead);
    const bool val = lead && rp >= 0 && rp < k;
    const unsigned long long vm = __ballot(val);
    const int key = ((rp & 63) << 25) | (rp & 0x1ffffff);
    int r = 0, b = 0;  // rank among the listed entries; bucket start of bucket `lane`
    for (unsigned long long mk = vm; mk; mk &= mk - 1ull) {
        const int kl = __builtin_amdgcn_readlane(key, __ffsll((long long)mk) - 1);
        r += kl < key ? 1 : 0;
        b += (kl >> 25) < lane ? 1 : 0;
    }
    const int n = __popcll(vm);
    if (lead) {
        d.aF[row] = acc;
        d.afs[1 + __popcll(lm & below)] = row;
    }
    if (val) {
        d.afl[AFL_POS + r] = rp;
        d.aflv[r] = acc;
    }
    d.afl[AFL_SB + lane] = b;
    if (lane == 0) {
        d.afl[AFL_SB + 64] = n;
        d.afs[0] = __popcll(lm);
        d.afl[0] = n;
    }
}

// gathered: P = world ranks' packed records in drecv (rank order) instead of
// this launch's regions
// (workgroups 1 .. gridDim.x - 1: the deferred plan's Minv update, dual_defer)
__global__ void __launch_bounds__(BF_NT) k_dual_bfrt(Dev d, int nreg, int gathered, int reg_ok, int dslot) {
    __shared__ double s_bun[2 * BF_BUN];
    __shared__ int scan_lds[BF_NT / 64];
    __shared__ double red[BF_NT / 64];
    __shared__ int s_int[4];
    __shared__ double s_dbl[2];
    __shared__ int s_flip[64 * BF_RR];  // (the one-wave path's flip list: compact indices)
    // the fast tail (one GPU, CSC, <= 64 candidates): the candidates' ids and
    // columns (BF_ENT entries each, with the rows' bump positions), the flips'
    // ids / dx and the entering record, all in LDS
    __shared__ int s_clen[64], s_erow[64 * BF_ENT], s_erp[64 * BF_ENT], s_fj[64];
    __shared__ double s_eval[64 * BF_ENT], s_fdx[64];
    __shared__ DualCand s_rec[64];
    __shared__ unsigned long long s_stb[16];
    unsigned long long* s_st = (ELP_DIAG && d.dstamp) ? s_stb : nullptr;
    DevCtl* c = d.ctl;
    if (blockIdx.x > 0) {
        if (minv_pending(c)) {
            const Plan P = c->plan;
            apply_minv_part(d, P, 0, (int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x,
                            (int64_t)(gridDim.x - 1) * blockDim.x);
        }
        return;
    }
    BSTAMP(0);
    if (ELP_DIAG && s_st && threadIdx.x == 0) s_st[4] = __builtin_amdgcn_s_memtime();  // (shader clock)
    // (the counters the tail updates, read now: nothing else writes them during the launch)
    const int64_t pf_flips = c->flips, pf_pp = c->price_passes;
    const double pf_pb = c->price_bytes, pf_ib = c->iter_bytes;
    const int pf_k = c->k, pf_ny = c->ny;
    const int tid = threadIdx.x;
    // (CSC: the last a_F's support count and this thread's first entry of it,
    //  for the clearing waves of the fast tail -- read now, beside the
    //  compaction's loads, not two dependent round trips after it; afs holds
    //  1 + 1024 entries, the speculative index stays below 1 + 448)
    int pf_afn = 0, pf_afr = 0;
    if (d.csc && tid >= 64 + 64 * BF_ENT) {
        pf_afn = d.afs[0];
        pf_afr = d.afs[1 + tid - (64 + 64 * BF_ENT)];
    }
    if (c->status != ST_RUN) return;
    const int bland = c->bland;
    // ---- compaction (one GPU: the regions; sharded: the ranks' records, in
    //      rank order = ascending structural id, the last rank's slacks last)
    int total = 0;
    const bool lds_rec = !gathered && d.csc && nreg <= BF_NT && reg_ok >= 2;
    if (!gathered) {
        total = compact_regions(d, nreg, d.dcomp, scan_lds, lds_rec ? s_rec : nullptr);
    } else {
        for (int r = 0; r < d.world; ++r) {
            const DualCand* src = d.drecv + (size_t)r * ((size_t)d.dcap + 1);
            const int cnt = src[0].j;
            for (int t = tid; t < cnt; t += BF_NT) d.dcomp[total + t] = src[1 + t];
            total += cnt;
        }
    }
    __syncthreads();  // (the compacted array is read by other threads below)
    BSTAMP(1);
    const int N = total;
    const double ptol = c->tol_primal;
    int nflip = 0, qidx = -1;
    const bool wave = reg_ok >= 2 && N <= 64 * BF_RR;  // (bfrt_wave: the usual case)
    // fast: wave 0 runs the rounds and leaves the flips / the entering record
    // in LDS while waves 1-8 load the candidates' columns and waves 9-15
    // clear the last a_F's support (every thread here is otherwise idle)
    const bool fast = lds_rec && N <= 64;  // (then the records are in s_rec only)
    if (wave) {
        if (tid < 64) {
            if (N <= 64)
                bfrt_wave1(d, N, bland, ptol, fabs(c->dr_x - c->dr_beta), &nflip, &qidx, s_flip, s_st, fast, s_rec,
                           s_fj, s_fdx);
            else bfrt_wave(d, N, bland, ptol, fabs(c->dr_x - c->dr_beta), s_bun, &nflip, &qidx, s_flip, dslot);
        } else if (fast && tid < 64 + 64 * BF_ENT) {
            const int sl = tid - 64, cc = sl / BF_ENT, e = sl % BF_ENT;
            if (cc < N) {
                const int j = s_rec[cc].j;
                const int jl = j < d.N ? loc_of(d, j) : -1;
                int len = -1;  // (a slack: no column to scatter; it never flips -- no finite range)
                if (jl >= 0) {  // (the column's extent from its record: the pricing pass's cptr)
                    const int64_t c0 = s_rec[cc].c0;
                    len = s_rec[cc].len;
                    if (e < len && len <= BF_ENT) {
                        const int row = d.rind[c0 + e];
                        s_eval[sl] = d.cval[c0 + e];
                        s_erow[sl] = row;
                        s_erp[sl] = d.rpos[row];
                    }
                }
                if (e == 0) s_clen[cc] = len <= BF_ENT ? len : -1;
            }
        } else if (fast) {  // the last a_F's support back to zero (or all of a_F)
            const int t0 = tid - (64 + 64 * BF_ENT), T = BF_NT - (64 + 64 * BF_ENT);
            const int pn = pf_afn;
            if (pn < 0) {
                for (int i = t0; i < d.m; i += T) d.aF[i] = 0.0;
            } else {
                for (int t = t0; t < pn; t += T) d.aF[t == t0 ? pf_afr : d.afs[1 + t]] = 0.0;
            }
        }
        if (tid == 0) {
            s_int[2] = nflip;
            s_int[3] = qidx;
        }
        __syncthreads();
        nflip = s_int[2];
        qidx = s_int[3];
    }
    // the workgroup path: thread t's candidates [lo, hi) (none when the wave ran)
    const int run = wave ? 0 : (N + BF_NT - 1) / BF_NT;
    const int lo = min(N, tid * run), hi = min(N, lo + run);
    // up to BF_RR candidates per thread (N <= BF_RR * BF_NT) are held in
    // registers for the bunch rounds (fully unrolled: no scratch); larger
    // candidate sets walk dcomp / dalive in global memory
    const bool reg = reg_ok >= 1 && run <= BF_RR;
    double rt[BF_RR], rb[BF_RR], ra[BF_RR], rw[BF_RR];
    int rj[BF_RR];
    unsigned ral = 0;  // live mask of the register candidates
    if (reg) {
#pragma unroll
        for (int q = 0; q < BF_RR; ++q) {
            rt[q] = rb[q] = ra[q] = rw[q] = 0.0;
            rj[q] = 0;
            if (lo + q < hi) {
                const DualCand& o = d.dcomp[lo + q];
                rt[q] = o.t;
                rb[q] = o.b;
                ra[q] = fabs(o.a);
                rw[q] = o.r;
                rj[q] = o.j;
                ral |= 1u << q;
            }
        }
    } else {
        for (int t = lo; t < hi; ++t) d.dalive[t] = 1;
    }
    double slope = fabs(c->dr_x - c->dr_beta);
    const double INF = HUGE_VAL;
    for (;;) {
        if (wave) break;
        // smallest Harris bound among the live candidates
        double bmin = INF;
        int live = 0;
        if (reg) {
#pragma unroll
            for (int q = 0; q < BF_RR; ++q)
                if (ral >> q & 1u) bmin = fmin(bmin, rb[q]);
            live = ral != 0;
        } else {
            for (int t = lo; t < hi; ++t)
                if (d.dalive[t]) {
                    live = 1;
                    bmin = fmin(bmin, d.dcomp[t].b);
                }
        }
        const double thmax = block_min<BF_NT>(bmin, red);
        if (tid == 0) s_int[0] = 0;
        __syncthreads();
        if (live) s_int[0] = 1;
        __syncthreads();
        if (!s_int[0]) break;  // nothing left: the dual ray (q = -1)
        // the bunch, in order, into dflip[nflip ...) (a flip list in the making)
        int cnt = 0, allbox = 1;
        unsigned rbun = 0;  // (register path: the bunch's members)
        if (reg) {
#pragma unroll
            for (int q = 0; q < BF_RR; ++q)
                if ((ral >> q & 1u) && rt[q] <= thmax) {
                    rbun |= 1u << q;
                    cnt++;
                    if (rw[q] == INF) allbox = 0;
                }
        } else {
            for (int t = lo; t < hi; ++t)
                if (d.dalive[t] && d.dcomp[t].t <= thmax) {
                    cnt++;
                    if (d.dcomp[t].r == INF) allbox = 0;
                }
        }
        int excl;
        const int nq = block_scan_excl<BF_NT>(cnt, &excl, scan_lds);
        if (tid == 0) s_int[1] = 1;
        __syncthreads();
        if (!allbox) s_int[1] = 0;
        // the bunch's (|alpha|, u - l) in bunch order into LDS for thread 0's sum;
        // this thread's best member (largest |alpha| (Bland: smallest ratio),
        // lowest id -- a total order: ids are distinct) for the entering choice
        double ba = -1.0, bt = INF;
        int bj = -1, bi = -1;
        if (reg) {
            int o = nflip + excl;
#pragma unroll
            for (int q = 0; q < BF_RR; ++q)
                if (rbun >> q & 1u) {
                    if (o - nflip < BF_BUN) {
                        s_bun[2 * (o - nflip)] = ra[q];
                        s_bun[2 * (o - nflip) + 1] = rw[q];
                    }
                    d.dflip[o++] = lo + q;  // (compact index for now)
                    const bool take = bi < 0 || (bland ? (rt[q] < bt || (rt[q] == bt && rj[q] < bj))
                                                       : (ra[q] > ba || (ra[q] == ba && rj[q] < bj)));
                    if (take) {
                        ba = ra[q];
                        bt = rt[q];
                        bj = rj[q];
                        bi = lo + q;
                    }
                }
        } else {
            for (int t = lo, o = nflip + excl; t < hi; ++t)
                if (d.dalive[t] && d.dcomp[t].t <= thmax) {
                    const DualCand& e = d.dcomp[t];
                    const double ea = fabs(e.a);
                    if (o - nflip < BF_BUN) {
                        s_bun[2 * (o - nflip)] = ea;
                        s_bun[2 * (o - nflip) + 1] = e.r;
                    }
                    d.dflip[o++] = t;
                    const bool take = bi < 0 || (bland ? (e.t < bt || (e.t == bt && e.j < bj))
                                                       : (ea > ba || (ea == ba && e.j < bj)));
                    if (take) {
                        ba = ea;
                        bt = e.t;
                        bj = e.j;
                        bi = t;
                    }
                }
        }
        __syncthreads();
        if (tid == 0) {  // |alpha| (u - l) summed in ascending id (the bunch's order): from LDS,
                         // not two dependent global loads per entry (r03: ~1 us each)
            double sum = 0.0;
            if (s_int[1])
                for (int t = 0; t < nq; ++t) {
                    if (t < BF_BUN) {
                        sum = fma(s_bun[2 * t], s_bun[2 * t + 1], sum);
                    } else {
                        const DualCand& o = d.dcomp[d.dflip[nflip + t]];
                        sum = fma(fabs(o.a), o.r, sum);
                    }
                }
            s_dbl[0] = sum;
        }
        __syncthreads();
        const double sum = s_dbl[0];
        if (nq == 0) break;  // (NaN ratios only: no candidate qualifies -- the ray)
        if (s_int[1] && sum < slope - ptol) {  // flip the bunch (x_r still out past it)
            slope = slope - sum;
            if (reg) {
                ral &= ~rbun;
            } else {
                for (int t = nflip + tid; t < nflip + nq; t += BF_NT) d.dalive[d.dflip[t]] = 0;
            }
            nflip += nq;
            __syncthreads();
            continue;
        }
        // the bunch's best enters: block argmax of the threads' best members
        // in the same total order, keys through LDS (s_bun is free again)
        __shared__ int s_bi[BF_NT], s_bj[BF_NT];
        s_bun[tid] = ba;
        s_bun[BF_NT + tid] = bt;
        s_bi[tid] = bi;
        s_bj[tid] = bj;
        __syncthreads();
        for (int h = BF_NT / 2; h >= 1; h >>= 1) {
            if (tid < h) {
                const int y = s_bi[tid + h];
                if (y >= 0) {
                    const double ya = s_bun[tid + h], yt = s_bun[BF_NT + tid + h];
                    const int yj = s_bj[tid + h];
                    const bool take = s_bi[tid] < 0 ||
                                      (bland ? (yt < s_bun[BF_NT + tid] || (yt == s_bun[BF_NT + tid] && yj < s_bj[tid]))
                                             : (ya > s_bun[tid] || (ya == s_bun[tid] && yj < s_bj[tid])));
                    if (take) {
                        s_bun[tid] = ya;
                        s_bun[BF_NT + tid] = yt;
                        s_bi[tid] = y;
                        s_bj[tid] = yj;
                    }
                }
            }
            __syncthreads();
        }
        qidx = s_bi[0];
        break;
    }
    __syncthreads();
    BSTAMP(2);
    // the flips: compact indices -> ids and dx = +-(u - l) (the record's range)
    // (the new status and value from the record's bounds: the column's own)
    int myj = -1;
    double mydx = 0.0;
    if (fast && tid < nflip) {  // (wave 0 stored them already)
        myj = s_fj[tid];
        mydx = s_fdx[tid];
    }
    for (int t = fast ? BF_NT : tid; t < nflip; t += BF_NT) {
        const DualCand o = d.dcomp[wave ? s_flip[t] : d.dflip[t]];
        const bool at_lower = o.side > 0;  // (boxed columns act at their current bound)
        const double dx = at_lower ? o.ub - o.lb : o.lb - o.ub;
        d.dflipdx[t] = dx;
        d.dflip[t] = o.j;
        if (t == tid) {
            myj = o.j;
            mydx = dx;
        }
        const int jl = loc_of(d, o.j);
        if (jl < 0) continue;  // (column-sharded: another shard's column)
        const bool up = dx > 0.0;
        d.vstat[jl] = up ? VS_UPPER : VS_LOWER;
        d.xval[jl] = up ? o.ub : o.lb;
    }
    // CSC (one GPU): a_F = sum of the flipped columns times their dx here, in
    // place of a one-workgroup k_dual_flip_col launch -- each row's entries in
    // flip order, the same fma chain
    int dbg_E = 0, dbg_path = 0;  // (diagnostic builds: the flips' entries and the a_F path taken)
    if (d.csc && !gathered && qidx >= 0 && nflip > 0) {
        const int kq = pf_k;
        int E = 0;  // (the flips' entries, every thread alike: the wave path or a block path, uniformly)
        bool bad = false;
        if (fast)
            for (int f = 0; f < nflip; ++f) {
                const int l = s_clen[s_flip[f]];
                bad = bad || l < 0;
                E += l > 0 ? l : 0;
            }
        dbg_E = bad ? -1 : E;
        dbg_path = fast && !bad && E <= 64 ? 1 : fast ? 2 : 3;
        if (fast && !bad && E <= 64) {  // wave 0 alone; the other waves are done
            if (tid >= 64) return;
            BSTAMP(10);
            bfrt_flip_wave(d, nflip, E, kq, s_flip, s_clen, s_erow, s_eval, s_erp, s_fdx, s_st);
            BSTAMP(13);
        } else if (!(fast && bfrt_flip_lds(d, nflip, kq, s_flip, s_clen, s_erow, s_eval, s_erp, s_fdx, s_st))) {
            if (ELP_DIAG) dbg_path = 3;
            if (fast && tid < nflip) {  // (the sequential path reads the flip list from memory; its first barrier orders these)
                d.dflip[tid] = s_fj[tid];
                d.dflipdx[tid] = s_fdx[tid];
            }
            bfrt_flip_column(d, nflip, kq, myj, mydx);
        }
    } else {
        __syncthreads();  // (the flip list is read by the other threads below / in later launches)
    }
    if (fast && tid < nflip) {  // the flips' list, status and value (after the last barrier)
        const DualCand& o = s_rec[s_flip[tid]];
        const double dx = s_fdx[tid];
        d.dflip[tid] = o.j;
        d.dflipdx[tid] = dx;
        const int jl = loc_of(d, o.j);
        if (jl >= 0) {
            d.vstat[jl] = dx > 0.0 ? VS_UPPER : VS_LOWER;
            d.xval[jl] = dx > 0.0 ? o.ub : o.lb;
        }
    }
    if (tid != 0) return;
    BSTAMP(3);
    if (ELP_DIAG && s_st) s_st[5] = __builtin_amdgcn_s_memtime();
    if (ELP_DIAG && d.dstamp) {  // the LDS stamps out: 20-23 start / compacted / decided / tail end,
                                 // 27 records loaded, 29 rounds done, 30-33 the LDS a_F phases; counts 24-26, 28
        unsigned long long* o = d.dstamp + (size_t)dslot * DSTAMP_STRIDE;
        o[20] = s_st[0];
        o[21] = s_st[1];
        o[22] = s_st[2];
        o[23] = s_st[3];
        o[27] = s_st[7];
        o[29] = s_st[9];
        for (int t = 0; t < 4; ++t) o[30 + t] = fast && nflip > 0 && qidx >= 0 ? s_st[10 + t] : 0ull;
        o[24] = (unsigned long long)N;
        o[25] = (unsigned long long)nflip;
        o[26] = wave ? 1ull : 0ull;
        o[28] = N <= 64 ? s_st[15] : 0ull;
        o[34] = s_st[5] - s_st[4];  // shader clocks over the launch (s_memtime)
        o[35] = (unsigned long long)(long long)dbg_E;
        o[36] = (unsigned long long)dbg_path;
    }
    const int64_t it = c->iter;
    if (qidx < 0) {  // dual unbounded: the LP is infeasible (oracle: trace -2, the leaving variable)
        c->iter = it + 1;
        c->phase1_iters++;
        c->dual_iters++;
        if (it < c->trace_cap) {
            d.trace[2 * it] = -2;
            d.trace[2 * it + 1] = c->dr_var;
        }
        c->nflip = 0;
        c->status = ST_DUALINF;
        return;
    }
    const DualCand* qp = fast ? s_rec + qidx : d.dcomp + qidx;
    const DualCand q = *qp;
    if (d.sharded) {  // the entering column's scalars, wherever it lives (k_ftran_zr's snapshot)
        d.pkt[d.m] = q.lb;
        d.pkt[d.m + 1] = q.ub;
        d.pkt[d.m + 2] = q.x;
        d.pkt[d.m + 3] = q.c;
    }
    c->q = q.j;
    c->dq = q.d;
    c->wq = 1.0;
    c->sig = q.side > 0 ? 1.0 : -1.0;
    c->dq_t = q.t;
    c->nflip = nflip;
    c->flips = pf_flips + nflip;
    Cand e;
    e.score = 1.0;
    e.d = q.d;
    e.w = 1.0;
    e.j = q.j;
    d.cand[0] = e;
    // (statistics: the pricing pass and the whole iteration's bytes)
    const double kk = (double)pf_k, mm = (double)d.m;
    const double pb = price_pass_bytes(d, pf_ny, 0) + 8.0 * (double)pf_ny;  // (+ rho on the slots)
    c->price_bytes = pf_pb + pb;
    c->price_passes = pf_pp + 1;
    c->iter_bytes = pf_ib + pb + 48.0 * kk * kk + 8.0 * mm * kk * (nflip > 0 ? 2.0 : 1.0) + 16.0 * (double)d.n + 16.0 * mm;
}

// a_F = sum over the flips (in list order) of a_j dx_j, dense A: one row per
// thread (the oracle's per-row fma chain).  CSC: k_dual_bfrt's tail scatters
// the flipped columns one after the other (rows of a column are distinct, so
// each row sees the same chain)
__global__ void __launch_bounds__(256) k_dual_flip_col(Dev d) {
    const DevCtl* c = d.ctl;
    const int nf = c->nflip;
    if (c->status != ST_RUN || nf == 0) return;
    const int m = d.m;  // (dense A only: CSC builds a_F in k_dual_bfrt)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double acc = 0.0;
    for (int f = 0; f < nf; ++f) {  // (qcolumn: this shard's A, or the replicated A when sharded)
        const int j = d.dflip[f];
        acc = fma(qcol_at(d, qcolumn(d, j), j, i), d.dflipdx[f], acc);
    }
    d.aF[i] = acc;
}

// column-only shards (no replicated A): the owner of a structural entering
// column packs it (scaled) into pkt[0, m), every other rank zeros -- the host
// all-reduces pkt[0, m), an exact copy; k_dual_bfrt wrote pkt[m, m + 4) on all
// ranks.  a_F starts at 0 for the flips' chain (k_dual_flip_part)
__global__ void __launch_bounds__(256) k_dual_qpack(Dev d) {
    const DevCtl* c = d.ctl;
    if (c->status != ST_RUN) return;
    const int i = blockIdx.x * 256 + threadIdx.x, m = d.m;
    if (i >= m) return;
    const int q = c->q;
    const int ql = q < d.N ? loc_of(d, q) : -1;
    d.pkt[i] = ql >= 0 ? sca(d, d.A[(size_t)ql * (size_t)m + i], i, q) : 0.0;
    d.aF[i] = 0.0;
}

// a_F's per-row chain over this shard's flips (the flip list ascends by
// global id, so the shards' runs follow each other in rank order): continued
// from the a_F the previous rank broadcast -- the one-GPU chain's bits
__global__ void __launch_bounds__(256) k_dual_flip_part(Dev d) {
    const DevCtl* c = d.ctl;
    const int nf = c->nflip;
    if (c->status != ST_RUN || nf == 0) return;
    const int m = d.m;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double acc = d.aF[i];
    for (int f = 0; f < nf; ++f) {
        const int j = d.dflip[f];
        const int jl = loc_of(d, j);
        if (jl < 0) continue;
        acc = fma(sca(d, d.A[(size_t)jl * (size_t)m + i], i, j), d.dflipdx[f], acc);
    }
    d.aF[i] = acc;
}

// fS = Minv a_F[R] (one wave per bump row, wave order)
__global__ void __launch_bounds__(256) k_dual_flip_bump(Dev d, int lds_row) {
    extern __shared__ __attribute__((aligned(16))) double afr_lds[];
    const DevCtl* c = d.ctl;
    if (c->status != ST_RUN || c->nflip == 0) return;
    const int k = c->k;
    double* afr = lds_row ? afr_lds : d.zz;  // (huge bumps: every workgroup writes the same values)
    for (int p = threadIdx.x; p < k; p += 256) afr[p] = d.aF[d.Rl[p]];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int p = blockIdx.x * 4 + (threadIdx.x >> 6); p < k; p += gridDim.x * 4) {
        double acc = lane_chain(d.Minv + (size_t)p * d.ldm, afr, k);
        acc = wave_tree(acc);
        if (lane == 0) d.fS[p] = acc;
    }
}

// x_B -= B^-1 a_F: covered rows x -= sigma (a_F,i - A[i,S] fS) (zchunk order:
// a chain per 32-position chunk, the chunk sums added in order from 0), bump
// positions x -= fS.  FTRAN-z's shape: row tiles of 32 rows x 8 waves, half-wave
// h of wave w runs chunks 2w + h, + 16, ... with the chunk's AS values all in
// flight, partials through LDS (LDSZ) or a slice of zpart (huge bumps); then
// tiles of 512 bump positions.  (r03: one thread per row walking all k
// positions -- ~90 workgroups, 317 us per call at m = 20 000, k <= 2000.)
template <bool LDSZ>
__global__ void __launch_bounds__(512) k_dual_flip_apply(Dev d, int nrt) {
    extern __shared__ __attribute__((aligned(16))) double fzl[];  // [nch][32]
    const DevCtl* c = d.ctl;
    if (c->status != ST_RUN || c->nflip == 0) return;
    const int m = d.m, k = c->k;
    if ((int)blockIdx.x >= nrt) {
        const int p = (blockIdx.x - nrt) * 512 + threadIdx.x;
        if (p < k) d.xs[p] = d.xs[p] - d.fS[p];
        return;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
    const int i = blockIdx.x * ZR_ROWS + r;
    const int nch = (k + ZCHUNK - 1) / ZCHUNK;
    double* zp = LDSZ ? fzl : d.zpart + (size_t)blockIdx.x * ZR_ROWS * (size_t)nch;
    const double* col0 = d.AS + (i < m ? i : 0);
    for (int ch = 2 * w + hh; ch < nch; ch += 16) {
        const int c0 = ch * ZCHUNK, len = min(ZCHUNK, k - c0);
        double a[ZCHUNK];
#pragma unroll
        for (int t = 0; t < ZCHUNK; ++t) a[t] = col0[(size_t)(c0 + (t < len ? t : len - 1)) * (size_t)m];
        double acc = 0.0;
#pragma unroll
        for (int t = 0; t < ZCHUNK; ++t)
            if (t < len) acc = fma(a[t], d.fS[c0 + t], acc);
        zp[ch * ZR_ROWS + r] = acc;
    }
    __syncthreads();
    if (w == 0 && hh == 0 && i < m) {
        const int u = d.cover[i];
        if (u >= 0) {
            double tot = 0.0;
            for (int ch = 0; ch < nch; ++ch) tot = tot + zp[ch * ZR_ROWS + r];
            d.xr[i] = d.xr[i] - unit_sign(d, u, i) * (d.aF[i] - tot);
        }
    }
}

// ============================================================== launchers
static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch_generate(const Dev& d, uint64_t seed, int64_t col0, int64_t n_global, double* A,
                           double* b, double* c, hipStream_t st) {
    const int m = d.m;
    const int64_t ncols = d.n;
    if (m > 0 && A) {
        dim3 g(cdiv(m, 256), (unsigned)(ncols < 65535 ? ncols : 65535));
        k_gen_A<<<g, 256, 0, st>>>(seed, m, ncols, col0, A);
    }
    const int64_t mx = m > ncols ? m : ncols;
    k_gen_bc<<<cdiv(mx, 256), 256, 0, st>>>(seed, m, ncols, col0, n_global, b, c);
    return hipGetLastError();
}

hipError_t launch_init_cols(const Dev& d, const double* lo, const double* up, hipStream_t st) {
    k_init_cols<<<cdiv(d.n, 256), 256, 0, st>>>(d, lo, up);
    return launch_nzlist(d, st);
}

hipError_t launch_fill_AR(const Dev& d, hipStream_t st) {
    if (d.m > 0 && !d.csc) {
        dim3 g(cdiv(d.n, 256), (unsigned)(d.m < 4096 ? d.m : 4096));
        k_fill_AR<<<g, 256, 0, st>>>(d);
    }
    return hipGetLastError();
}

hipError_t launch_ar_relayout(const Dev& d, const double* old_ar, int64_t old_cap, int rows,
                              hipStream_t st) {
    if (rows > 0) k_ar_relayout<<<2048, 256, 0, st>>>(d, old_ar, old_cap, rows);
    return hipGetLastError();
}

hipError_t launch_scale_init(int m, int64_t ncols, int32_t* rho, int32_t* gam, int32_t* rmn, int32_t* rmx,
                             hipStream_t st) {
    const int64_t mx = m > ncols ? m : ncols;
    k_scale_init<<<cdiv(mx > 0 ? mx : 1, 256), 256, 0, st>>>(m, ncols, rho, gam, rmn, rmx);
    return hipGetLastError();
}
hipError_t launch_scale_rows(int m, int64_t ncols, const double* A, const int32_t* gam, int32_t* rmn, int32_t* rmx,
                             hipStream_t st) {
    if (m > 0 && ncols > 0)
        k_scale_row_part<<<dim3(cdiv(m, 256), cdiv(ncols, SCALE_RCOLS)), 256, 0, st>>>(m, ncols, A, gam, rmn, rmx);
    return hipGetLastError();
}
hipError_t launch_scale_row_final(int m, int32_t* rmn, int32_t* rmx, int32_t* rho, int32_t* changed, hipStream_t st) {
    if (m > 0) k_scale_row_final<<<cdiv(m, 256), 256, 0, st>>>(m, rmn, rmx, rho, changed);
    return hipGetLastError();
}
hipError_t launch_scale_cols(int m, int64_t ncols, const double* A, const int32_t* rho, int32_t* gam, int equilibrate,
                             int32_t* changed, hipStream_t st) {
    if (m > 0 && ncols > 0) {
        const unsigned g = (unsigned)(ncols < 65536 ? ncols : 65536);
        k_scale_col<<<g, 256, 0, st>>>(m, ncols, A, rho, gam, equilibrate, changed);
    }
    return hipGetLastError();
}
hipError_t launch_scale_apply(int m, int64_t ncols, double* A, const int32_t* rho, const int32_t* gam,
                              hipStream_t st) {
    if (m > 0 && ncols > 0) {
        dim3 g(cdiv(m, 256), (unsigned)(ncols < 65535 ? ncols : 65535));
        k_scale_apply<<<g, 256, 0, st>>>(m, ncols, A, rho, gam);
    }
    return hipGetLastError();
}


hipError_t launch_nzlist(const Dev& d, hipStream_t st) {
    const unsigned nb = (unsigned)cdiv(d.n > 0 ? d.n : 1, NZ_CHUNK);
    k_nzlist_count<<<nb, 1024, 0, st>>>(d);
    k_nzlist<<<nb, 1024, 0, st>>>(d);
    return hipGetLastError();
}

hipError_t launch_row_chain(const Dev& d, hipStream_t st) {
    if (d.m > 0 && d.csc) k_row_chain_csr<<<cdiv(d.m, 256), 256, 0, st>>>(d);
    else if (d.m > 0) k_row_chain<<<cdiv(d.m, 256), 256, 0, st>>>(d);
    return hipGetLastError();
}


// the dense pricing kernel for a launch: non-temporal sweep loads or not, timed or not
typedef void (*PriceFn)(Dev d, int, int, int, int);
static PriceFn price_kernel(bool nt, bool timed) {
    if (timed) return nt ? k_price<1, TILE_COLS, true> : k_price<0, TILE_COLS, true>;
    return nt ? k_price<1, TILE_COLS> : k_price<0, TILE_COLS>;
}

hipError_t launch_ptimer_reduce(const Dev& d, int nslots, hipStream_t st) {
    if (nslots > 0 && d.ptst) k_ptimer_reduce<<<nslots, 256, 0, st>>>(d);
    return hipGetLastError();
}

hipError_t launch_init_rows(const Dev& d, const double* rhs, hipStream_t st) {
    if (d.m > 0) {
        k_init_rows<<<cdiv(d.m, 256), 256, 0, st>>>(d, rhs);
        k_init_Y<<<1, 1024, 0, st>>>(d);
    } else {
        k_init_Y<<<1, 1024, 0, st>>>(d);
    }
    return hipGetLastError();
}

// workgroups of a plan application for bumps up to k_ub: nb_minv for Minv /
// MinvT, the rest for x_B, AS (and AR rows: with_ar)
// apply_plan grid: nb_minv workgroups for Minv / MinvT (per_thread elements
// per thread), then the x_B / AS (/ AR) copy workgroups; threads = the
// launch's workgroup size
// Workgroup caps on the Minv / MinvT share (only large bumps reach them): the
// pricing launch's trailing apply (ELP_APPLY_PT elements per thread) takes up
// to ELP_MINV_WG_MAX -- 8192 (2048 until r04x) measured 2 % faster on the
// 20 000 x 100 000 feasible-start LP (k 2000) -- while k_update (one element per
// thread, its x_B / AS copy workgroups dispatched after them) keeps
// ELP_UPDATE_WG_MAX = 2048: 8192 there slowed it 21.7 -> 28.1 us at k 2000
#ifndef ELP_MINV_WG_MAX
#define ELP_MINV_WG_MAX 8192
#endif
#ifndef ELP_UPDATE_WG_MAX
#define ELP_UPDATE_WG_MAX 2048
#endif
static void update_grid(const Dev& d, int k_ub, bool with_ar, unsigned* nb_minv, unsigned* nb,
                        int threads = 256, int per_thread = 1, unsigned wg_max = ELP_UPDATE_WG_MAX) {
    const int64_t kk = (d.noT ? 1 : 2) * (int64_t)(k_ub + 1) * (k_ub + 1);
    *nb_minv = cdiv(kk, threads * per_thread);
    if (*nb_minv > wg_max) *nb_minv = wg_max;
    const int64_t cw = with_ar ? (d.m > d.n ? d.m : d.n) : (d.m > k_ub + 1 ? d.m : k_ub + 1);
    unsigned nb_copy = cdiv(cw, threads);
    if (nb_copy > 1024) nb_copy = 1024;
    *nb = *nb_minv + nb_copy;
}

// CSC: A[i, S] v from the rows' nonzeros (csr_basic + zrow_chain) once the dense walk over AS
// would stream more than ELP_SPZ_MIN_MB (16) MB -- below that the dense walk's
// independent loads beat the row walk's dependent ones (1000 x 10 000 packing
// LP, k <= 877: 0.53 s dense against 0.85 s sparse, r04m)
static bool use_spz(const Dev& d, int k_ub) {
    static const double thr = [] {
        const char* e = std::getenv("ELP_SPZ_MIN_MB");
        return e ? std::atof(e) * 1e6 : 16e6;
    }();
    return d.csc && d.spos && 8.0 * (double)d.m * (double)k_ub > thr;
}

// CSC: sparse FTRAN / B^-1 rows once the bump exceeds Dev::spf_min positions
static bool use_spf(const Dev& d, int k_ub) { return d.csc && d.spf_min > 0 && k_ub > d.spf_min; }

// slack workgroups of the pricing launch for |Y| <= ny_ub
static int slack_wgs(const Dev& d, int ny_ub) {
    return (int)cdiv(ny_ub > 0 ? ny_ub : 1, d.csc ? TILE_COLS : PRICE_THREADS);
}

// non-temporal sweep loads above this many sweep bytes (ELP_SWEEP_NT: 0 never,
// 1 always, unset: 192 MB -- beyond the Infinity Cache's share the sweep can keep)
static bool sweep_nt(double bytes) {
    static const double thr = [] {
        const char* e = std::getenv("ELP_SWEEP_NT");
        if (!e) return 192.0e6;
        const int v = std::atoi(e);
        return v == 0 ? 1e300 : v == 1 ? 0.0 : (double)v * 1e6;
    }();
    return bytes > thr;
}

static hipError_t launch_btran_price(const Dev& d, int k_ub, int ny_ub, int phase, hipStream_t st,
                                     hipEvent_t ev0, hipEvent_t ev1, int tslot) {
    const int m = d.m;
    const double* tv = d.cS;
    if (phase == 1) {
        if (m > 0) k_ycov<<<cdiv(m, 256), 256, 0, st>>>(d);
        if (k_ub > 0) k_btran_t<<<cdiv(k_ub, 4), 256, 0, st>>>(d);
        tv = d.t;
    }
    if (phase == 1) {  // phase 2 keeps y by the dual update (k_ratio)
        unsigned g = cdiv(k_ub > 0 ? k_ub : 1, 4);
        if (g > 1024) g = 1024;
        k_btran<<<g, 256, 0, st>>>(d, phase, tv);
    }
    const unsigned ntiles = cdiv(d.n, TILE_COLS);
    // phase 2: the previous iteration's plan is applied by trailing workgroups
    // of the pricing launch (it touches nothing the sweep reads)
    unsigned nb_minv = 0, napply = 0;
    // (the apply workgroups ride beside the sweep: a few elements per thread
    // keeps their count, and the launch's dispatch tail, small)
    #ifndef ELP_APPLY_PT
#define ELP_APPLY_PT 4
#endif
    if (phase == 2 && d.csc) {
        update_grid(d, k_ub, false, &nb_minv, &napply, TILE_COLS, ELP_APPLY_PT, ELP_MINV_WG_MAX);
        if (d.sru_on) {  // (the sparse update: sru_wgs workgroups instead of the dense share)
            napply = napply - nb_minv + sru_wgs(k_ub);
            nb_minv = sru_wgs(k_ub);
        }
    }
    // the dense deferred plan in trailing workgroups of the launch (r02's
    // layout, the default again since r04: 3 x 3 interleaved A/B at 5000 x 50000,
    // 25.4k against 24.7k iterations/s with the tiles' waves 1-3 applying it)
    unsigned dnapply = 0, dnb_minv = 0;
    if (phase == 2 && !d.csc) update_grid(d, k_ub, false, &dnb_minv, &dnapply, PRICE_THREADS, ELP_APPLY_PT, ELP_MINV_WG_MAX);
    // + nsw: the slack workgroups (candidates [ntiles, ntiles + nsw)); the dense
    // sweep applies the deferred plan inside its tiles (price_body)
    const int nsw = slack_wgs(d, ny_ub);
    const unsigned grid = (d.csc ? ntiles + napply : (unsigned)d.ntiles + dnapply) + nsw;
    const bool nt = !d.csc && sweep_nt(8.0 * (double)ny_ub * (double)d.n);
    // tslot >= 0: the timed variant (in-kernel stamps, k_ptimer_reduce)
    const bool timed = tslot >= 0 && d.ptst && tslot < d.ptslots;
    if (!timed) tslot = 0;
    if (ev0) {
        // profiling (ELP_PROFILE_EVENTS): events bound to the dispatch itself
        // (the CP's start / end timestamps of this launch, as a kernel trace
        // reports them; no marker packets between the kernels)
        if (d.csc)
            hipExtLaunchKernelGGL(timed ? k_price_csc<true> : k_price_csc<false>, dim3(grid), dim3(TILE_COLS), 0, st,
                                  ev0, ev1, 0, d, (int)napply, (int)nb_minv, nsw, tslot);
        else
            hipExtLaunchKernelGGL(price_kernel(nt, timed), dim3(grid), dim3(PRICE_THREADS), 0, st, ev0,
                                  ev1, 0, d, nsw, (int)dnapply, (int)dnb_minv, tslot);
        return hipGetLastError();
    }
    if (d.csc) {
        if (timed) k_price_csc<true><<<grid, TILE_COLS, 0, st>>>(d, (int)napply, (int)nb_minv, nsw, tslot);
        else k_price_csc<false><<<grid, TILE_COLS, 0, st>>>(d, (int)napply, (int)nb_minv, nsw, tslot);
    } else {
        hipLaunchKernelGGL(price_kernel(nt, timed), dim3(grid), dim3(PRICE_THREADS), 0, st, d,
                           nsw, (int)dnapply, (int)dnb_minv, tslot);
    }
    return hipGetLastError();
}

hipError_t launch_apply_pending(const Dev& d, int k_ub, hipStream_t st, bool dual) {
    unsigned nb_minv, nb;
    update_grid(d, k_ub, dual, &nb_minv, &nb);
    k_update<<<nb, 256, 0, st>>>(d, (int)nb_minv, dual ? 2 : 1);
    return hipGetLastError();
}

hipError_t launch_iteration_tail(const Dev& d, int k_ub, int phase, hipStream_t st, bool bump_ftran,
                                 int dslot, int qz) {
    const int m = d.m;
    // phase 3: the dual phase (k_update applies its plan at once); 4: the dual
    // phase with the plan deferred into the next iteration (Dev::dual_defer)
    const bool dskip = phase == 4;
    if (phase >= 3) phase = 3;
    if (bump_ftran && k_ub > 0) k_ftran_bump<<<cdiv(k_ub, 4), 256, 0, st>>>(d, d.aR, d.alS, 1);
    // CSC with a large bump: FTRAN-z from the rows of A (k_ftran_zr_sq: 64 rows
    // per 4-wave workgroup, 64-position bump tiles); else k_ftran_zr's 32-row
    // tiles over AS
    const bool spz = use_spz(d, k_ub);
    const int nrt = spz ? (int)cdiv(m > 0 ? m : 1, 64) : (int)cdiv(m > 0 ? m : 1, ZR_ROWS);
    // z partials: 256 B per chunk of ZCHUNK bump positions in LDS (<= 64 KiB,
    // k <= 8192); larger bumps use a private slice of zpart per row tile
    const size_t lds = (size_t)cdiv(k_ub, ZCHUNK) * ZR_ROWS * sizeof(double);
    const bool ldsz = lds <= 64 * 1024 && !d.force_select;
    int zw = (ldsz && nrt > 256 && cdiv(k_ub, ZCHUNK) <= 8) ? 4 : 8;  // waves per row tile
    if (spz) zw = 1;
    const int nbt = (int)cdiv(k_ub, 64 * zw);  // bump tiles (k_ftran_zr_sq: 64 positions per workgroup)
    // alpha_S in LDS beside the z partials when the half-waves run more than one
    // chunk each (k_ub > 2 zw ZCHUNK) and it fits the prefetch (ZR_PA per thread):
    // 10 000 x 500 000 at k 529: 18.8 -> 16.3 us; with one chunk per half-wave the
    // registers win (the LDS round trip cost 0.8 us at 5000 x 50000, r02)
    const int nxp = (int)std::min<int64_t>(std::max<int64_t>((int64_t)cdiv(k_ub, ZCHUNK) - 2 * zw, 0), ZR_XPF);
    const size_t lds_als = lds + (size_t)k_ub * sizeof(double) + (size_t)nxp * ZCHUNK * ZR_ROWS * sizeof(double);
    const bool als = ldsz && k_ub > 2 * zw * ZCHUNK && k_ub <= ZR_PA * 64 * zw && lds_als <= 64 * 1024;
    if (spz) {
        // (the dual phase: + nrt waves for the flips' x_B update, before the snapshot one)
        k_ftran_zr_sq<<<nrt + nbt + 1, 256, 0, st>>>(d, nrt, phase == 3 ? 1 : 0, dslot);
    } else {
        // + 1: the snapshot workgroup
        if (als) {
            if (zw == 4) k_ftran_zr<true, 4, true><<<nrt + nbt + 1, 256, lds_als, st>>>(d, nrt, k_ub, dslot, qz);
            else k_ftran_zr<true, 8, true><<<nrt + nbt + 1, 512, lds_als, st>>>(d, nrt, k_ub, dslot, qz);
        } else if (zw == 4) {
            k_ftran_zr<true, 4, false><<<nrt + nbt + 1, 256, lds, st>>>(d, nrt, k_ub, dslot, qz);
        } else if (ldsz) {
            k_ftran_zr<true, 8, false><<<nrt + nbt + 1, 512, lds, st>>>(d, nrt, k_ub, dslot, qz);
        } else {
            k_ftran_zr<false, 8, false><<<nrt + nbt + 1, 512, 0, st>>>(d, nrt, k_ub, dslot, qz);
        }
    }
    // ratio test + (cases B/D) B^-1 row: one workgroup per 4 bump columns;
    // phase 2 adds the AR-copy workgroups and defers the rest of the update
    const int defer = phase == 2;  // (phase 3, the dual: applied right away by k_update)
    {
        const size_t lds = (size_t)k_ub * sizeof(double);
        const int lds_row = lds <= 48 * 1024 && !d.force_select;
        const unsigned nmain = cdiv(k_ub > 0 ? k_ub : 1, 4);
        unsigned nar = 0;
        if (defer && !d.csc) {
#ifndef ELP_NAR_MAX
#define ELP_NAR_MAX 512
#endif
#ifndef ELP_NAR_COLS
#define ELP_NAR_COLS 768
#endif
            // the AR-copy workgroups work only when Y changes, but every one of
            // them prefetches and repeats the decision: 3 columns per thread
            // (66 workgroups at n = 50 000, was 196 -- +1-2 % over the C3
            // solve, r03 A/B) and at most 512 (n = 500 000, where a copy that
            // long wants the parallelism)
            nar = cdiv(d.n, ELP_NAR_COLS);
            if (nar > ELP_NAR_MAX) nar = ELP_NAR_MAX;
        }
        // (8 B^-1 values per lane in registers; for k > 512 the row is read in a
        //  loop after the decision -- 16 per lane measured slower at 10 000 x
        //  500 000 (16.5 vs 14.7 us, r01), 10 as well (12.01 vs 11.75 us at k
        //  529, r03 A/B over the last 2000 iterations))
        const unsigned nbk = ELP_BOOK_WG;  // (the bookkeeping workgroup after the main ones)
        // (past the register path -- k > 512 -- the row registers only cost
        //  occupancy: the <1> instance, 135 -> ~107 VGPRs, four waves per SIMD
        //  instead of three, so the ~k/4 workgroups of a CSC bump all fit at once)
        if (phase == 3)
            k_ratio<8, true><<<nmain + nbk, 256, lds_row ? lds : 0, st>>>(d, 2, nrt + nbt, lds_row, 0,
                                                                         (int)nmain, k_ub, dslot, nrt + nbt * zw);
        else if (k_ub > 64 * 8)
            k_ratio<1><<<nmain + nbk + nar, 256, lds_row ? lds : 0, st>>>(d, phase, nrt + nbt, lds_row,
                                                                         defer, (int)nmain, k_ub, dslot,
                                                                         nrt + nbt * zw);
        else
            k_ratio<8><<<nmain + nbk + nar, 256, lds_row ? lds : 0, st>>>(d, phase, nrt + nbt, lds_row,
                                                                         defer, (int)nmain, k_ub, dslot,
                                                                         nrt + nbt * zw);
    }
    if (!defer && !dskip) {
        unsigned nb_minv, nb;
        update_grid(d, k_ub, true, &nb_minv, &nb);
        k_update<<<nb, 256, 0, st>>>(d, (int)nb_minv, 0);
    }
    return hipGetLastError();
}

hipError_t launch_iteration(const Dev& d, int k_ub, int ny_ub, int phase, hipStream_t st,
                            hipEvent_t ev0, hipEvent_t ev1, int dslot, int tslot) {
    hipError_t e = launch_btran_price(d, k_ub, ny_ub, phase, st, ev0, ev1, tslot);
    if (e != hipSuccess) return e;
    const int ntiles = d.ntiles, nsw = slack_wgs(d, ny_ub);
    const size_t lds = (size_t)k_ub * sizeof(double);
    const bool sp = use_spf(d, k_ub);
    if ((sp || lds <= 48 * 1024) && !d.force_select) {  // fused select + bump FTRAN
        const size_t ldsz = sp ? 64 : lds > 64 ? lds : 64;  // the timer workgroup reduces in it
        // + the timer workgroup, + the CSC column-scatter workgroup
        unsigned nrw = cdiv(k_ub > 0 ? k_ub : 1, 4);
        if (d.sel_cap > 0 && nrw > (unsigned)d.sel_cap) nrw = (unsigned)d.sel_cap;
        // (ranks sharing a device, sel_cap > 0: no staging workgroups -- they would
        //  spin on the mailbox beside the capped bump rows; FTRAN-z reads the column)
        const unsigned nqz = d.qz && !d.csc && d.sel_cap == 0 ? cdiv(d.m, 256 * QZ_PT) : 0;
        const unsigned g = nrw + nqz + (d.ptimer ? 1 : 0) + (d.csc ? 1 : 0);
        // Minv row values per lane in registers: 8 (k <= 512), 10 (k <= 640: the
        // last 4 000 iterations of 10 000 x 500 000, k 529; 16 measured no faster
        // there, r01 -- fewer waves per SIMD), else the row is read after a_R
        if (sp)
            k_select_ftran<1, true><<<g, 256, ldsz, st>>>(d, ntiles, nsw, k_ub, dslot, (int)nrw, (int)nqz, 0);
        else if (k_ub > 512 && k_ub <= 640)
            k_select_ftran<10><<<g, 256, ldsz, st>>>(d, ntiles, nsw, k_ub, dslot, (int)nrw, (int)nqz, 0);
        else
            k_select_ftran<8><<<g, 256, ldsz, st>>>(d, ntiles, nsw, k_ub, dslot, (int)nrw, (int)nqz, 0);
        return launch_iteration_tail(d, k_ub, phase, st, false, dslot, nqz > 0 ? 1 : 0);
    }
    k_select<<<1, 1024, 0, st>>>(d, ntiles, nsw, 0);
    return launch_iteration_tail(d, k_ub, phase, st, true, dslot);
}

hipError_t launch_dual_setup_cols(const Dev& d, hipStream_t st) {
    if (d.n > 0) k_dual_setup_cols<<<cdiv(d.n, 256), 256, 0, st>>>(d);
    return launch_nzlist(d, st);  // (columns moved to their upper bound: the row activities' list)
}

hipError_t launch_dual_init_rows(const Dev& d, hipStream_t st) {
    if (d.m > 0) k_dual_init_rows<<<cdiv(d.m, 256), 256, 0, st>>>(d);
    return hipGetLastError();
}

// CHUZR, rho_r and the pivot row + pricing of this shard's columns (+ the
// slack candidates where d.dslack); returns the candidate regions' count
// the deferred inverse update's share of a launch (dual_defer): workgroups of
// `threads` for one half (Minv or MinvT) of a bump up to k_ub + 1 positions,
// MINV_U elements per thread per pass, at most `cap`
static unsigned defer_wgs(int k_ub, int threads, unsigned cap) {
    const int64_t kk = (int64_t)(k_ub + 1) * (k_ub + 1);
    unsigned nb = cdiv(kk, (int64_t)threads * 4);
    return nb > cap ? cap : nb;
}

// defer: the one-GPU dual_defer flow (the last plan applied by this
// iteration's CHUZR and trailing workgroups, no k_update); 0 on sharded ranks
static int dual_head(const Dev& d, int k_ub, int ny_ub, hipStream_t st, int defer = 0) {
    const int m = d.m;
    const unsigned nchz = cdiv((int64_t)m + k_ub, 256);
    k_dual_chuzr<<<nchz, 256, 0, st>>>(d, defer);
    const size_t lds = (size_t)k_ub * sizeof(double);
    const int lds_row = lds <= 48 * 1024;
    unsigned nrw = cdiv(k_ub > 0 ? k_ub : 1, 4);
    if (nrw > 1024) nrw = 1024;
    const int sp = use_spf(d, k_ub) ? 1 : 0;
    k_dual_row<<<nrw, 256, lds_row && !sp ? lds : 0, st>>>(d, (int)nchz, lds_row && !sp, sp, defer);
    const int nsw = d.dslack ? slack_wgs(d, ny_ub) : 0;
    if (d.csc) {
        const int na = defer ? (d.sru_on ? (int)sru_wgs(k_ub) : (int)defer_wgs(k_ub, TILE_COLS, 8192)) : 0;
        k_dual_price_csc<<<d.ntiles + nsw + na, TILE_COLS, 0, st>>>(d, nsw, 0, na);
    } else {
        const int na = defer ? (int)defer_wgs(k_ub, PRICE_THREADS, 4096) : 0;
        k_dual_price<<<d.ntiles + nsw + na, PRICE_THREADS, 0, st>>>(d, nsw, 0, na);
    }
    return d.ntiles + nsw;
}

static hipError_t dual_tail(const Dev& d, int k_ub, hipStream_t st, bool flip_col = true, int defer = 0, int dslot = 0);

hipError_t launch_dual_iteration_head(const Dev& d, int k_ub, int ny_ub, hipStream_t st) {
    const int nreg = dual_head(d, k_ub, ny_ub, st);
    k_dual_pack<<<1, BF_NT, 0, st>>>(d, nreg);
    return hipGetLastError();
}

hipError_t launch_dual_iteration_tail(const Dev& d, int k_ub, hipStream_t st) {
    k_dual_bfrt<<<1, BF_NT, 0, st>>>(d, 0, 1, bfrt_reg(), 0);
    return dual_tail(d, k_ub, st);
}

// column-only shards: the ratio test over the gathered candidates, then the
// owner's entering column into pkt[0, m) (others: zeros) and a_F cleared
hipError_t launch_dual_ratio_shards(const Dev& d, hipStream_t st) {
    k_dual_bfrt<<<1, BF_NT, 0, st>>>(d, 0, 1, bfrt_reg(), 0);
    k_dual_qpack<<<cdiv(d.m > 0 ? d.m : 1, 256), 256, 0, st>>>(d);
    return hipGetLastError();
}
hipError_t launch_dual_flip_part(const Dev& d, hipStream_t st) {
    k_dual_flip_part<<<cdiv(d.m > 0 ? d.m : 1, 256), 256, 0, st>>>(d);
    return hipGetLastError();
}
hipError_t launch_dual_iteration_finish(const Dev& d, int k_ub, hipStream_t st) {
    return dual_tail(d, k_ub, st, false);
}

hipError_t launch_dual_iteration(const Dev& d, int k_ub, int ny_ub, hipStream_t st, int dslot) {
    const int defer = d.dual_defer ? 1 : 0;
    const int nreg = dual_head(d, k_ub, ny_ub, st, defer);
    // (dual_defer: + the Minv half of the last plan's update beside the ratio test)
    // (the sparse update: none -- the pricing launch's workgroups took all of it)
    const unsigned nbf = defer && !(d.csc && d.sru_on) ? defer_wgs(k_ub, BF_NT, 1024) : 0;
    k_dual_bfrt<<<1 + nbf, BF_NT, 0, st>>>(d, nreg, 0, bfrt_reg(), dslot);
    return dual_tail(d, k_ub, st, true, defer, dslot);
}

// the bound flips' FTRAN and x_B update, then FTRAN of a_q and the pivot
// (flip_col false: a_F was formed by the column-only shards' chain already)
static hipError_t dual_tail(const Dev& d, int k_ub, hipStream_t st, bool flip_col, int defer, int dslot) {
    const int m = d.m;
    const size_t lds = (size_t)k_ub * sizeof(double);
    const int lds_row = lds <= 48 * 1024;
    unsigned nrw = cdiv(k_ub > 0 ? k_ub : 1, 4);
    if (nrw > 1024) nrw = 1024;
    if (flip_col && !d.csc) k_dual_flip_col<<<cdiv(m > 0 ? m : 1, 256), 256, 0, st>>>(d);  // (CSC: k_dual_bfrt)
    const bool spz = use_spz(d, k_ub), sp = use_spf(d, k_ub);
    // CSC with the row-wise update: the flips' bump FTRAN inside k_select_ftran
    // (dual = 2; a_R and a_F[R] side by side in LDS, or sparse lists: sp)
    const bool fold_fs = spz && (sp || 2 * lds <= 64 * 1024) && !d.force_select;
    if (k_ub > 0 && !fold_fs) k_dual_flip_bump<<<nrw, 256, lds_row ? lds : 0, st>>>(d, lds_row);
    if (spz) {
        // (the row-wise x_B update runs inside k_ftran_zr_sq, below)
    } else {
        const unsigned nrt = cdiv(m > 0 ? m : 1, ZR_ROWS), nbt = cdiv(k_ub > 0 ? k_ub : 1, 512);
        const size_t zl = (size_t)cdiv(k_ub > 0 ? k_ub : 1, ZCHUNK) * ZR_ROWS * sizeof(double);
        if (zl <= 48 * 1024) k_dual_flip_apply<true><<<nrt + nbt, 512, zl, st>>>(d, (int)nrt);
        else k_dual_flip_apply<false><<<nrt + nbt, 512, 0, st>>>(d, (int)nrt);
    }
    // the entering column q (k_dual_bfrt's, candidate 0): a_R, alpha_S (+ staging)
    if (fold_fs || ((sp || lds <= 48 * 1024) && !d.force_select)) {
        const size_t ldsz = sp ? 64 : fold_fs ? (2 * lds > 64 ? 2 * lds : 64) : (lds > 64 ? lds : 64);
        const int dual = fold_fs ? 2 : 1;
        const unsigned nqz = d.qz && !d.csc ? cdiv(m, 256 * QZ_PT) : 0;
        const unsigned g = nrw + nqz + (d.csc ? 1 : 0);
        if (sp)
            k_select_ftran<1, true><<<g, 256, ldsz, st>>>(d, 1, 0, k_ub, 0, (int)nrw, (int)nqz, dual);
        else if (k_ub > 512 && k_ub <= 640)
            k_select_ftran<10><<<g, 256, ldsz, st>>>(d, 1, 0, k_ub, 0, (int)nrw, (int)nqz, dual);
        else
            k_select_ftran<8><<<g, 256, ldsz, st>>>(d, 1, 0, k_ub, dslot, (int)nrw, (int)nqz, dual);
        return launch_iteration_tail(d, k_ub, defer ? 4 : 3, st, false, dslot, nqz > 0 ? 1 : 0);
    }
    k_select<<<1, 1024, 0, st>>>(d, 1, 0, 1);
    return launch_iteration_tail(d, k_ub, defer ? 4 : 3, st, true, dslot);
}

hipError_t launch_warm_start(const Dev& d, const double* lo, const double* up, int k, int ny, hipStream_t st) {
    const int64_t mx = std::max<int64_t>(std::max<int64_t>(d.N, d.m), 1);
    k_warm_bounds<<<cdiv(mx, 256), 256, 0, st>>>(d, lo, up);
    const hipError_t e = launch_btran_exact(d, k, st);  // y = B^-T c_B (the real costs)
    if (e != hipSuccess) return e;
    const int nsw = slack_wgs(d, ny);
    if (d.csc) k_dual_price_csc<<<d.ntiles + nsw, TILE_COLS, 0, st>>>(d, nsw, 1, 0);
    else k_dual_price<<<d.ntiles + nsw, PRICE_THREADS, 0, st>>>(d, nsw, 1, 0);
    return hipGetLastError();
}

hipError_t launch_iteration_head(const Dev& d, int k_ub, int ny_ub, int phase, int rank,
                                 hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, int tslot) {
    hipError_t e = launch_btran_price(d, k_ub, ny_ub, phase, st, ev0, ev1, tslot);
    if (e != hipSuccess) return e;
    k_select_local<<<1, 1024, 0, st>>>(d, d.ntiles, slack_wgs(d, ny_ub), rank);
    return hipGetLastError();
}

hipError_t launch_select_global(const Dev& d, hipStream_t st) {
    k_select_global<<<1, 256, 0, st>>>(d);
    return hipGetLastError();
}

bool launch_select_xftran(const Dev& d, int k_ub, hipStream_t st, hipError_t* err) {
    const size_t lds = (size_t)k_ub * sizeof(double);
    if (lds > 48 * 1024 || d.force_select) return false;
    k_select_xftran<<<cdiv(k_ub > 0 ? k_ub : 1, 4), 256, lds > 64 ? lds : 64, st>>>(d);
    *err = hipGetLastError();
    return true;
}

hipError_t launch_select_finish(const Dev& d, hipStream_t st) {
    k_select_finish<<<1, 1024, 0, st>>>(d);
    return hipGetLastError();
}

hipError_t launch_refactor_ns_resid(const Dev& d, int k, hipStream_t st) {
    if (k <= 0) return hipSuccess;
    if (d.csc && d.spos) {  // (M is sparse: k_ns_resid_sp, the same bits)
        k_ns_resid_sp<<<k, 256, 0, st>>>(d, k);
        return hipGetLastError();
    }
    if (k >= NS_R8_MIN) k_ns_gemm<0, 8><<<dim3(cdiv(k, 128), cdiv(k, 128)), 256, 0, st>>>(d, k);
    else k_ns_gemm<0, 4><<<dim3(cdiv(k, 64), cdiv(k, 64)), 256, 0, st>>>(d, k);
    return hipGetLastError();
}

hipError_t launch_refactor_ns_update(const Dev& d, int k, hipStream_t st) {
    if (k <= 0) return hipSuccess;
    if (k >= NS_R8_MIN) k_ns_gemm<1, 8><<<dim3(cdiv(k, 128), cdiv(k, 128)), 256, 0, st>>>(d, k);
    else k_ns_gemm<1, 4><<<dim3(cdiv(k, 64), cdiv(k, 64)), 256, 0, st>>>(d, k);
    dim3 g(cdiv(k, 32), cdiv(k, 32));
    k_ns_store<<<g, dim3(32, 32), 0, st>>>(d, k);
    return hipGetLastError();
}

hipError_t launch_refactor_gj(const Dev& d, int k, hipStream_t st) {
    if (k <= 0) return hipSuccess;
    const int64_t kk = (int64_t)k * k;
    k_gj_init<<<cdiv(kk > k ? kk : k, 256), 256, 0, st>>>(d, k);
    double* W = d.W0;  // (in place; d.W1 holds the step's side buffers)
    unsigned ge = cdiv(kk, 256 * GJ_PT);
    if (ge > 2048) ge = 2048;
    for (int c = 0; c < k; ++c) {
        k_gj_pivot<<<1, 1024, 0, st>>>(d, k, c, W);
        k_gj_elim<<<ge, 256, 0, st>>>(d, k, c, W);
    }
    k_gj_final<<<cdiv(kk, 256), 256, 0, st>>>(d, k, W);
    return hipGetLastError();
}

hipError_t launch_btran_exact(const Dev& d, int k, hipStream_t st) {
    unsigned g = cdiv(k > 0 ? k : 1, 4);
    const unsigned gm = cdiv(d.m > 0 ? d.m : 1, 256);
    if (g < gm) g = gm;
    if (g > 1024) g = 1024;
    k_btran_exact<<<g, 256, 0, st>>>(d);
    return hipGetLastError();
}

hipError_t launch_refactor_primal(const Dev& d, int k, hipStream_t st) {
    if (d.m > 0) {
        k_refactor_rhs<<<cdiv(d.m, 256), 256, 0, st>>>(d);
        if (k > 0) {
            k_ftran_bump<<<cdiv(k, 4), 256, 0, st>>>(d, d.aR, d.xs, 0);
            dim3 g(cdiv(d.m, 256), cdiv(k, ZCHUNK));
            k_ftran_z<<<g, 256, 0, st>>>(d, d.xs, 0);
        }
        k_xr_from_z<<<cdiv(d.m, 256), 256, 0, st>>>(d);
    }
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_fill32(Fill32List l) {
    const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x, T = (int64_t)gridDim.x * 256;
    for (int b = 0; b < l.count; ++b) {
        uint32_t* p = static_cast<uint32_t*>(l.f[b].p);
        const int64_t nw = l.f[b].words;
        const uint32_t v = l.f[b].val;
        for (int64_t i = t0; i < nw; i += T) p[i] = v;
    }
}
hipError_t launch_fill32(const Fill32List& l, hipStream_t st) {
    if (l.count <= 0) return hipSuccess;
    int64_t mx = 1;
    for (int b = 0; b < l.count; ++b) mx = std::max<int64_t>(mx, l.f[b].words);
    const int64_t g = std::min<int64_t>(cdiv(mx, 256), 2048);
    k_fill32<<<(unsigned)g, 256, 0, st>>>(l);
    return hipGetLastError();
}

hipError_t launch_devex_reset(const Dev& d, hipStream_t st) {
    k_devex_reset<<<cdiv((int64_t)(d.N > d.n ? d.N : d.n) + d.m, 256), 256, 0, st>>>(d);
    return hipGetLastError();
}

hipError_t launch_phase2(const Dev& d, hipStream_t st) {
    const int64_t mx = d.m > d.n ? d.m : d.n;
    k_phase2<<<cdiv(mx, 256), 256, 0, st>>>(d);
    if (d.m > 0) k_phase2_cS<<<cdiv(d.m, 256), 256, 0, st>>>(d);
    return launch_devex_reset(d, st);
}

hipError_t launch_extract(const Dev& d, double* xout, hipStream_t st) {
    k_extract<<<cdiv(d.n, 256), 256, 0, st>>>(d, xout);
    if (d.m > 0) k_extract_basic<<<cdiv(d.m, 256), 256, 0, st>>>(d, xout);
    return hipGetLastError();
}

hipError_t launch_sensitivity(const Dev& d, int k, double* dred, double* TR, double* plo,
                              double* phi, double* qlo, double* qhi, double* out4, hipStream_t st) {
    const int n = d.n, m = d.m;
    if (d.csc) k_sens_redcost<<<cdiv(n, 256), 256, 0, st>>>(d, dred);
    else k_sens_redcost<<<cdiv(n, 4), 256, 0, st>>>(d, dred);
    if (k > 0) {
        if (d.csc) (void)hipMemsetAsync(TR, 0, (size_t)k * (size_t)n * sizeof(double), st);
        dim3 gg(d.csc ? 1 : cdiv(n, 256) < 64 ? cdiv(n, 256) : 64, (unsigned)k);
        k_sens_gather_rows<<<gg, 256, 0, st>>>(d, TR, k);
        const int ntc = (int)cdiv(n, 64), ntr = (int)cdiv(m, 64);
        // alpha = Minv (k x k, row-major ldm) * TR (k x n, row-major)
        k_sens_mfma<0><<<dim3(ntc, cdiv(k, 64)), 256, 0, st>>>(d, d.Minv, d.ldm, 1, TR, n, 1, k, n, k,
                                                                dred, plo, phi);
        // G = AS (m x k, column-major ld m) * Minv (k x k)
        k_sens_mfma<1><<<dim3(cdiv(k, 64), ntr), 256, 0, st>>>(d, d.AS, 1, m, d.Minv, d.ldm, 1, m, k, k,
                                                               dred, qlo, qhi);
        k_sens_final<<<cdiv(2 * k, 256), 256, 0, st>>>(d, k, ntc, ntr, plo, phi, qlo, qhi, out4,
                                                       out4 + k, out4 + 2 * k, out4 + 3 * k);
    }
    return hipGetLastError();
}

}  // namespace elp
