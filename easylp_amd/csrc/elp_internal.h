// elp_internal.h -- device state shared by the gfx950 kernels and the host
// driver of the dense revised simplex (see DESIGN.md for the data layout).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Diagnostic builds (tools/build_variant.sh NAME "-DELP_DIAG=1"): the
// ELP_STAMPS phase stamps and the ELP_PROFILE_PRICE device-clock pricing
// timer.  Off in the product build: their run-time tests sat at the head of
// the latency kernels, each a dependent scalar load before the control block.
#ifndef ELP_DIAG
#define ELP_DIAG 0
#endif

namespace elp {

// variable status (same codes as oracle/elp_oracle.c)
// VS_FIXED: nonbasic with lb == ub (never enters; pricing then needs no bounds)
enum : int8_t { VS_BASIC = 0, VS_LOWER = 1, VS_UPPER = 2, VS_FREE = 3, VS_FIXED = 4 };

// device loop status
enum : int32_t {
    ST_RUN = 0,
    ST_PHASE_OPT = 1,  // no entering candidate: current phase optimal
    ST_UNBOUNDED = 2,
    ST_REFACTOR = 3,   // refactor period reached at loop top
    ST_ITERCAP = 4,
    ST_P1DONE = 5,     // phase-1 artificial sum within tolerance at loop top
    ST_NUMFAIL = 6,
    ST_STOP = 7,       // elp_iterate budget reached at loop top
    ST_COMMFAIL = 8,   // xGMI mailbox: a peer's record did not arrive in time
    ST_DUALINF = 9,    // dual simplex: no entering candidate for the leaving row (primal infeasible)
    ST_TIMEOUT = 10,   // resident solver: elp_control.time_limit reached at a loop top
};

// pivot cases (oracle/elp_oracle.c "case A".."case E")
enum : int32_t { PC_NONE = 0, PC_A = 1, PC_B = 2, PC_C = 3, PC_D = 4, PC_E = 5 };
enum : int32_t { ACT_NONE = 0, ACT_FLIP = 1, ACT_PIVOT = 2 };

#ifndef ELP_PRICE_SPLIT
#define ELP_PRICE_SPLIT 4
#endif
// slot chunks per pricing tile (one per wave); the oracle's PRICE_SPLIT must match
constexpr int PRICE_SPLIT = ELP_PRICE_SPLIT;
constexpr int ZCHUNK = 32;      // bump positions per FTRAN-z partial
constexpr int DSTAMP_STRIDE = 40;  // ELP_STAMPS slots per chunk iteration (k_ratio 0-11, select 12-15, FTRAN-z 16-19, dual BFRT 20-23;
                                    // 24-26, 28: the dual BFRT's counts -- candidates, flips, one-wave path,
                                    // bunch rounds; 27: its records loaded, 29: rounds done, 30-33: the LDS a_F phases)
constexpr int RREG = 64;  // pass-2 candidate slots per k_ftran_zr wave region
constexpr int TILE_COLS = 128;  // columns per pricing workgroup (2 per lane)

struct Plan {
    int32_t action, pcase, k_old, p;
    int32_t a, b, last, row;      // row: B leaving-cover row / D leaving row i1
    int32_t q, i0;                // i0: row of an entering slack (-1 otherwise)
    int32_t lrow, lpos;           // leaving entry: covered row / bump position
    double step, sig;             // x_B -= step * sig * alpha
    int32_t y_rm_slot, y_rm_last; // -1: no removal
    int32_t y_ap_slot, y_ap_row;  // -1: no append
    double piv;                   // A: alS[p]; B: delta; C: Minv[b][a]
    double xq;
    // dual simplex (phase 3): dual Devex weights of the basic entries are
    // updated with the plan (apply_copy): w_r of the leaving variable, the
    // pivot alpha_rq of the FTRAN column, the leaving entry (row / m + position)
    int32_t dual, dre;
    double dwr, darq;
};

struct DevCtl {
    int32_t status, phase, k, ny;
    int64_t iter, iter_limit, iter_stop;
    int32_t since_refactor, refactor_period;
    int32_t ndegen, bland, degen_switch, unb_var;
    int64_t phase1_iters, flips, degenerate;
    double tol_inf, unb_sig;
    double tol_primal, tol_dual, tol_pivot, art_sum;
    int32_t q, ntiles;
    double dq, sig;
    Plan plan;
    int64_t trace_cap;
    int32_t infeasible_bounds, pad1;
    double price_bytes;    // algorithmic bytes of every pricing pass that ran
    int64_t price_passes;
    double iter_bytes;     // algorithmic bytes of the whole iterations
    unsigned long long ns_emax_bits;  // max|I - M Minv| of the last refactor (bits of a double >= 0)
    int32_t price_grid, pad3;         // workgroups of the last pricing launch (Dev::ptimer)
    int32_t snap_k, snap_bland;       // k, bland as k_ratio's workgroups must see them
                                      // (workgroup 0 rewrites k / bland meanwhile)
    // likewise the bookkeeping entries k_ratio's dual update reads (k_ftran_zr's
    // snapshot workgroup): |Y|, rpos / ypos of the entering slack's row, the
    // last Y row and its bump position
    int32_t snap_ny, snap_apos, snap_ypos0, snap_ylast, snap_pad;
    // the status k_ratio's workgroups act on: workgroup 0 may already have
    // written the next loop-top status (refactor / stop / cap) when another
    // workgroup of the same launch starts and reads the control block
    int32_t snap_status;
    // ... and the scalars of the pivot bookkeeping, so k_ratio reads them with
    // the control block: q's (lb, ub, x, cost) and status; the last bump
    // position's (cost, lo, hi), structural and row
    double snap_lbq, snap_ubq, snap_xq, snap_cq, snap_csl, snap_slol, snap_shil;
    int32_t snap_vsq, snap_sllast, snap_rllast, pad7;
    // pricing-kernel timer (Dev::ptimer): s_memrealtime ticks (100 MHz) from the
    // first workgroup's start to the last one's end -- every workgroup of the
    // launch: tiles, slack candidates and the deferred-update appliers, i.e. what
    // a kernel trace times -- summed over timed passes
    unsigned long long price_ticks;
    int64_t price_timed;
    double price_tbytes;
    int32_t qcol_var, pad6;  // CSC: the variable whose column is scattered in Dev::qcol
    // phase-2 deferred update: k_ratio bumps plan_seq with every plan it makes;
    // the next pricing launch applies it (Minv / MinvT / x_B / AS) and the next
    // select kernel marks it applied; the host applies a plan still pending at
    // a poll (k_update) -- see DESIGN.md "Iteration pipeline"
    int32_t plan_seq, applied_seq;
    // the dual phase's deferred update (one GPU): the plan whose x_B / dual
    // Devex / AS part k_dual_chuzr applied (its inverse part: applied_seq)
    int32_t copy_seq;
    int32_t pad9;
    int64_t mb_epoch;  // xGMI mailbox: loads so far (seq = epoch << 40 | iteration + 1)
    // Devex pricing (elp_control.pricing): the last pivot as the next pricing
    // pass needs it -- entering reduced cost and weight, leaving variable;
    // dv_valid: 0 no update (phase start, bound flip), 1 update from the last
    // pivot, 2 the reference framework restarts (oracle run_phase)
    int32_t devex, dv_valid;
    int32_t dv_lv, pad8;
    double dv_dq, dv_wq;
    double wq;  // weight of the entering candidate (select kernels)
    // dual simplex phase 1 (h->phase 3, oracle run_dual): the leaving row of
    // this iteration as k_dual_row chose it -- basic variable, entry (covered
    // row, or m + bump position), direction s (+1 below its lower bound), the
    // covered row whose own entry the pivot row adds (-1: a bump position) and
    // its sign; value, target bound, bounds, dual Devex weight
    int32_t dr_var, dr_e, dr_s, dr_xrow;
    double dr_x, dr_beta, dr_lb, dr_ub, dr_w, dr_xsig;
    double dq_t;              // the entering column's exact dual ratio (<= 0: degenerate)
    int32_t nflip, ddevex;    // bound flips of this iteration; dual Devex pricing on
    int64_t dual_iters, dflat;  // dual iterations; columns whose cost the phase zeroed
};

// dual simplex candidates (k_dual_price -> k_dual_bfrt): exact ratio t, Harris
// bound b, pivot-row alpha (signed), range u - l (+inf: not boxed), reduced cost
struct DualCand {
    double t, b, a, r, d;
    int32_t j, side;  // global id; +1 acts at its lower bound, -1 at its upper
    // the column's bounds, value and cost (scaled): what the other shards need
    // when it enters (column-sharded ranks exchange the candidates)
    double lb, ub, x, c;
    // CSC: the column's first entry and length (cptr, as the pricing pass read
    // it), so k_dual_bfrt's fast tail loads a flipped column without cptr's
    // round trip; len -1: no column (a slack, or not a CSC record)
    int64_t c0;
    int32_t len, pad;
};
// a dual CHUZR partial (k_dual_chuzr, one per workgroup)
struct ChzRec {
    double score, x, beta;
    int32_t var, e, s, pad;
};
constexpr int DREG = 256;  // DualCand slots per k_dual_price region (one region per workgroup)

// Harris pass-2 candidate (a superset of the global candidates: exact ratio
// <= its workgroup's pass-1 minimum)
struct RCand {
    double g, r, l, u;
    int32_t var, e;
};

struct Cand {
    double score, d, w;  // w: the column's Devex weight (1 under Dantzig)
    int64_t j;           // -1: none
};

// a rank's best candidate as exchanged between shards: with every rank holding
// all of A (Dev::Afull) the record also carries the column's (lb, ub, x, cost),
// so the entering column never travels
struct CandX {
    Cand c;
    double lb, ub, x, cost;
};

// one mailbox slot: a rank's record for iteration seq - 1 (seq written last)
struct MboxRec {
    CandX x;
    int64_t seq;
};

// Everything a kernel needs, passed by value (pointers into device memory).
// Variable ids: replicated state (cover, Sl, candidates, q, trace) holds GLOBAL
// ids -- structural j < N, slack N + i, artificial N + m + i; per-variable
// arrays (lb, ub, cost, xval, vstat) are indexed by the shard-LOCAL id --
// structural j - col0 < n, slack n + i, artificial n + m + i (loc_of()).
// With one GPU, col0 = 0 and n = N, so both coincide.
struct Dev {
    int32_t m, n, nv, N;  // n: local columns; N: global columns
    int64_t col0;         // first global column of this shard
    int32_t world;        // ranks sharing the columns
    int32_t sharded;      // 1: column-sharded solve (world > 1 or a test transport)
    int64_t ldm;   // Minv leading dimension (= max(m,1))
    int64_t ldr;   // AR row length: ntiles x tile_w (a tile's rows are tile_w apart)
    int32_t tile_w, ntiles;  // pricing tiles: tile_w (even, <= TILE_COLS) columns each
    int64_t arcap; // AR rows per column tile (capacity)
    const double* A;  // column-major m x n (this shard's columns)
    const double* Afull;  // sharded + replicated: all N columns (A = Afull + col0*m);
                          // null: the entering column comes in the exchanged pkt
    double* AR;       // Y rows, tile-major: [ntiles][arcap rows][tile_w cols]
                      // (a pricing wave streams one contiguous run of rows)
    double* AS;       // basic structural columns, column-major (m x m capacity)
    double* Minv;     // bump inverse, row-major ldm x ldm
    double* MinvT;    // its transpose (BTRAN and B^-1 rows read rows of it)
    double *W0, *W1;  // Gauss-Jordan work (k x k each)
    double *b, *obj, *lb, *ub, *cost, *xval, *asgn;
    double *xr, *xs, *y, *yy, *t, *acol, *aR, *alS, *alU, *zz, *zpart;  // yy: y on Y slots
    double *vrow, *vvec, *colA, *rhs;
    double *cS, *slo, *shi;  // per bump position: cost, bounds of S_p
    double* blockmin;        // per-workgroup Harris pass-1 minima (k_ftran_zr)
    double* pkt;             // entering column + (lb, ub, x, cost) exchanged across shards
    double* objg;            // global objective (N), for c_S of foreign basic columns
    double* ract;            // row activities sum_j a_ij x_j of nonzero nonbasic columns
    CandX* cand_xchg;        // [world] local best candidates (all-gathered)
    RCand* rcand;            // pass-2 candidates: one region of RREG slots per emitting
                             // k_ftran_zr wave (row tile: wave 0; bump tile: every wave)
    int32_t* rcnt;           // candidates in each region (written every iteration, no atomics)
    int32_t rregs;           // regions allocated
    double *rlo, *rhi;       // per covered row: bounds of the covering unit variable
    int8_t* vstat;
    int8_t* rowvs;  // per row: the status its slack has whenever it is nonbasic
                    // (<=: lower, >=: upper, ==: fixed -- a slack never flips)
    int8_t* yvs;    // per Y slot: rowvs of the slot's row (select reads it in slot order)
    int32_t *cover, *rpos, *Rl, *Sl, *spos, *Yl, *ypos, *perm, *pivstep, *nzlist, *nzcount;
    int32_t* nzchunk;  // per-chunk counts of the nzlist compaction
    Cand* cand;
    unsigned long long* pstamp;  // [workgroup][2] start / end stamps of the last pricing launch
    int32_t ptimer, pad3;        // 1: k_price stamps, the select kernels sum them
    DevCtl* ctl;
    int64_t* trace;
    int32_t maximize, pad2;
    double infinity;
    double tol_singular;  // Gauss-Jordan: |pivot| <= this -> ST_NUMFAIL (elp_control)
    // on-the-fly scaling (elp_load_dense_device with scaling on: the caller's A
    // is read-only and is not copied): every read of A / Afull / the exchanged
    // column multiplies by 2^(srow[i] + scol[j]) (j global; exact, so the values
    // are those of a scaled copy); null when A itself holds the scaled values
    const int32_t* srow;
    const int32_t* scol;
    int64_t mb_ticks;     // xGMI mailbox wait limit in s_memrealtime ticks (100 MHz)
    // CSC input (elp_load_csc, one GPU): A is null, columns live in cptr/rind/cval
    // (rows ascending), a CSR copy serves the row activities, and the entering
    // column is scattered into the dense qcol each iteration
    int32_t csc, force_select;  // force_select: test hook (ELP_FORCE_SELECT), large-bump launch shape
    // bump-row workgroups of the fused select kernel, at most (0: one per 4 rows):
    // ranks that share a device (ngpu on fewer devices) spin in that kernel on
    // the peer mailbox, and P - 1 ranks' spinning grids must leave the device
    // room for the last rank's pricing launch (else it never starts)
    int32_t sel_cap, sel_pad;
    int64_t nnz;
    const int64_t* cptr;
    const int32_t* rind;
    const double* cval;
    const int64_t* rptr;
    const int32_t* cind;
    const double* rval;
    double* qcol;
    // dense, one-GPU select path: the entering column as FTRAN-z reads it
    // (a_iq per row, scaled; the unit column of an entering slack), written by
    // the select kernel's staging workgroups so k_ftran_zr can load it at
    // kernel start instead of one round trip after its control block
    double* qz;
    // debug (ELP_STAMPS): s_memrealtime stamps of k_ratio, 16 per chunk slot
    unsigned long long* dstamp;
    int32_t stamp_wide, pad_sw;  // ELP_STAMPS=2: also the grid-wide (atomic) stamps
    // xGMI mailbox exchange (Comm::enable_p2p): the select kernel publishes this
    // rank's best candidate into every peer's slot and waits for all of them
    MboxRec* mbox;          // this rank's mailbox [2 parities][world]
    MboxRec* const* mpeers; // every rank's mailbox as mapped in this process
    int32_t p2p, rank;
    // Devex: weight and last reduced cost per local structural (j < n) and
    // slack (n + i); the dual phase keeps its reference weights of the basic
    // variables in dw
    double *dw, *dprev;
    // dual simplex phase 1 (single GPU): rho_r on the bump positions and on the
    // Y slots, the CHUZR partials, the ratio-test candidate regions and their
    // counts, the compacted candidates and their live flags, the bound flips
    // (ids, dx), the flip column a_F and its bump FTRAN
    double *rhoR, *rr;
    ChzRec* dchz;
    DualCand *dcand, *dcomp;
    int32_t* dcnt;
    int8_t* dalive;
    int32_t* dflip;
    double *dflipdx, *aF, *fS;
    int32_t dregs, dchzn;
    // the dual Devex weights of the basic variables, indexed by GLOBAL variable
    // id (N + 2m): dw itself on one GPU (local = global ids), a replicated array
    // on column-sharded ranks (a basic structural may live on another shard)
    double* ddw;
    // column-sharded dual phase (replicated A): this rank's compacted ratio-test
    // candidates [header][dcap records] (header.j = count) and every rank's,
    // all-gathered in rank order; dslack: this rank emits the slack candidates
    // (one GPU, or the last rank -- so the gathered order is the one-GPU order:
    // structurals by ascending id, then the slacks)
    DualCand *dsend, *drecv;
    int32_t dcap, dslack;
    // CSC dual phase (one GPU): the support of the last a_F (afs[0] rows, -1:
    // unknown -- clear all m; the rows in afs[1 ..]) and a_F[R] as a
    // lane-bucketed sparse list for the select kernel's fS (afl[0] = n, -1: use
    // the dense a_F; afl[1 .. 66) bucket starts; afl[66 ..) positions; aflv the
    // values), both written by k_dual_bfrt's tail
    int32_t* afs;
    int32_t* afl;
    double* aflv;
    // CSC: bumps above this many positions take the sparse FTRAN / B^-1-row
    // paths (ELP_SPF_MIN; 0 never)
    int32_t spf_min, spf_pad;
    // release pricing timer (k_price<.., TIMED>): [ptslots][ptcap][start, end]
    // s_memrealtime stamps per workgroup, the grid of each slot's launch
    unsigned long long* ptst;
    int32_t* ptgrid;
    int32_t ptcap, ptslots;
    // one GPU, dual phase: k_ratio's plan applied during the next iteration
    // (k_dual_chuzr, the pricing / ratio-test launches' trailing workgroups)
    // instead of by a k_update launch (ELP_DUAL_DEFER=0: the launch)
    int32_t dual_defer;
    // CSC loads keep no MinvT (ELP_CSC_MINVT=1 restores it): every product
    // that read a row of MinvT reads a column of Minv -- a handful of entries
    // (sparse lists) or a gather -- and the per-pivot inverse update moves half
    // the bytes; MinvT is then null
    int32_t noT;
    // CSC: the per-pivot inverse update touches only the pairs of nonzero
    // multipliers (apply_minv_sru: the bump inverse of a sparse LP is sparse),
    // in trailing workgroups of the pricing launch, one per SRU_ROWS rows
    // (ELP_SRU=0: the dense update over all k^2 entries)
    int32_t sru_on;
};
constexpr int AFL_SB = 1;    // afl: bucket starts [1, 66)
constexpr int AFL_POS = 66;  // afl: positions [66, 66 + SPL)

// ---------------------------------------------------------------- launches
// Each returns hipGetLastError() of its launch.
hipError_t launch_generate(const Dev& d, uint64_t seed, int64_t col0, int64_t n_global,
                           double* A, double* b, double* c, hipStream_t st);
// init in two parts: columns (+ nonzero list), then rows once ract is complete
// several buffers filled with a 32-bit pattern in one launch (the load's
// zeroed / -1 buffers: one launch instead of one hipMemsetAsync each)
struct Fill32 {
    void* p;
    int64_t words;  // 32-bit words
    uint32_t val;
    int32_t pad;
};
constexpr int FILL32_MAX = 12;
struct Fill32List {
    Fill32 f[FILL32_MAX];
    int32_t count, pad;
};
hipError_t launch_fill32(const Fill32List& l, hipStream_t st);
hipError_t launch_init_cols(const Dev& d, const double* lo, const double* up, hipStream_t st);
hipError_t launch_init_rows(const Dev& d, const double* rhs, hipStream_t st);
hipError_t launch_fill_AR(const Dev& d, hipStream_t st);  // AR rows for the initial Y
// copy the first `rows` rows of every tile from an AR with capacity old_cap
hipError_t launch_ar_relayout(const Dev& d, const double* old_ar, int64_t old_cap, int rows,
                              hipStream_t st);
// ev0/ev1 (may be null): events recorded around the pricing kernel
// tslot >= 0: the timed pricing variant into stamp slot tslot (launch_ptimer_reduce)
hipError_t launch_iteration(const Dev& d, int k_ub, int ny_ub, int phase, hipStream_t st,
                            hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, int dslot = 0, int tslot = -1);
// the pricing timer of the chunk's timed slots [0, nslots) into DevCtl::price_ticks
hipError_t launch_ptimer_reduce(const Dev& d, int nslots, hipStream_t st);
// sharded iteration: head (BTRAN, pricing, local min-loc into cand_xchg[rank]),
// then the host all-gathers cand_xchg, select_global packs pkt, the host
// all-reduces pkt, then tail (a_R, FTRAN, ratio test, update)
hipError_t launch_iteration_head(const Dev& d, int k_ub, int ny_ub, int phase, int rank,
                                 hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, int tslot = -1);
hipError_t launch_select_global(const Dev& d, hipStream_t st);
// phase 2, at a host poll: apply a plan the last iteration left pending
// dual: the dual phase's deferred plan (the parts not applied yet, AR included)
hipError_t launch_apply_pending(const Dev& d, int k_ub, hipStream_t st, bool dual = false);
// replicated A: global min-loc + a_R + bump FTRAN in one launch (false: the
// bump is too large for it; use select_global + select_finish + tail(bump_ftran))
bool launch_select_xftran(const Dev& d, int k_ub, hipStream_t st, hipError_t* err);
hipError_t launch_select_finish(const Dev& d, hipStream_t st);
hipError_t launch_iteration_tail(const Dev& d, int k_ub, int phase, hipStream_t st,
                                 bool bump_ftran = true, int dslot = 0, int qz = 0);
// row activities: ract = chain(ract, local nonzero nonbasic columns)
hipError_t launch_row_chain(const Dev& d, hipStream_t st);
// refactor = ns_resid; (host reads ns_emax) ns_update | gauss_jordan; primal
constexpr double NS_TOL = 1e-6;
// (NS_TOL, NS_TOL2]: a correction and, if the residual is then within NS_TOL,
// a second one instead of a Gauss-Jordan rebuild (oracle refactor())
constexpr double NS_TOL2 = 1e-2;
hipError_t launch_refactor_ns_resid(const Dev& d, int k, hipStream_t st);
hipError_t launch_refactor_ns_update(const Dev& d, int k, hipStream_t st);
hipError_t launch_refactor_gj(const Dev& d, int k, hipStream_t st);
hipError_t launch_btran_exact(const Dev& d, int k, hipStream_t st);  // phase-2 duals
hipError_t launch_refactor_primal(const Dev& d, int k, hipStream_t st);  // needs ract
hipError_t launch_nzlist(const Dev& d, hipStream_t st);
// scaling (elp_control.scaling): exponents rho (m rows), gamma (ncols columns);
// rmn / rmx: per-row work (m each: max of -e, max of e; rmx must follow rmn in
// one 2m buffer so shards combine them with one all-reduce max); changed: set
// when a pass moved a factor
constexpr int SCALE_PASSES = 20;  // geometric row + column passes at most
hipError_t launch_scale_init(int m, int64_t ncols, int32_t* rho, int32_t* gam, int32_t* rmn, int32_t* rmx,
                             hipStream_t st);
hipError_t launch_scale_rows(int m, int64_t ncols, const double* A, const int32_t* gam, int32_t* rmn, int32_t* rmx,
                             hipStream_t st);
hipError_t launch_scale_row_final(int m, int32_t* rmn, int32_t* rmx, int32_t* rho, int32_t* changed, hipStream_t st);
hipError_t launch_scale_cols(int m, int64_t ncols, const double* A, const int32_t* rho, int32_t* gam, int equilibrate,
                             int32_t* changed, hipStream_t st);
hipError_t launch_scale_apply(int m, int64_t ncols, double* A, const int32_t* rho, const int32_t* gam,
                              hipStream_t st);
hipError_t launch_phase2(const Dev& d, hipStream_t st);  // (includes devex_reset)
hipError_t launch_devex_reset(const Dev& d, hipStream_t st);  // weights 1, dv_valid 0
// sensitivity (final basis, k = bump dimension): dred[n] reduced costs; TR
// (k x n), plo/phi (k x ceil(n/64)), qlo/qhi (k x ceil(m/64)) work; out4 =
// [olo(k) ohi(k) rlo(k) rhi(k)]: intervals of delta c_{S_p} and delta b_{R_c}
hipError_t launch_sensitivity(const Dev& d, int k, double* dred, double* TR, double* plo,
                              double* phi, double* qlo, double* qhi, double* out4, hipStream_t st);
// x of the local shard into xout[0:n) (basic values from the replicated S list)
hipError_t launch_extract(const Dev& d, double* xout, hipStream_t st);

// dual simplex phase 1 (elp_kernels.hip "dual simplex" section; oracle run_dual)
// load: the dual-feasible start -- boxed columns at the bound their cost sign
// asks for, costs of the columns no bound makes dual feasible zeroed (run
// before the row activities), then every row covered by its slack
hipError_t launch_dual_setup_cols(const Dev& d, hipStream_t st);
hipError_t launch_dual_init_rows(const Dev& d, hipStream_t st);
// one iteration: CHUZR, rho_r, pivot row + pricing, bound-flipping ratio test,
// the flips' FTRAN and x_B update, FTRAN of a_q, pivot bookkeeping, update
hipError_t launch_dual_iteration(const Dev& d, int k_ub, int ny_ub, hipStream_t st, int dslot = 0);
// column-sharded ranks (replicated A): head = CHUZR, rho_r, the pivot row and
// pricing of this shard, its candidates packed into dsend; the host all-gathers
// dsend into drecv; tail = the bound-flipping ratio test over every rank's
// candidates (identical on all ranks) and the rest of the iteration
hipError_t launch_dual_iteration_head(const Dev& d, int k_ub, int ny_ub, hipStream_t st);
hipError_t launch_dual_iteration_tail(const Dev& d, int k_ub, hipStream_t st);
// column-only shards (A not replicated): ratio test + the owner's entering
// column into pkt[0, m) (the host all-reduces it), then per rank in rank order
// its part of a_F's chain (the host broadcasts a_F from that rank), then the rest
hipError_t launch_dual_ratio_shards(const Dev& d, hipStream_t st);
hipError_t launch_dual_flip_part(const Dev& d, hipStream_t st);
hipError_t launch_dual_iteration_finish(const Dev& d, int k_ub, hipStream_t st);
// MIP node warm start (oracle warm_core): new column bounds lo / up (local,
// scaled), real costs, y, and every nonbasic column re-placed for the node
// (k, ny: the kept basis's bump dimension and |Y|); the host then refactors
hipError_t launch_warm_start(const Dev& d, const double* lo, const double* up, int k, int ny, hipStream_t st);

// resident small-LP solver (elp_resident.hip): the whole simplex loop of an LP
// whose state fits in LDS, one wave, one launch.  phase: the host's h->phase
// (1 primal phase 1, 2 primal phase 2, 3 dual phase 1); price_rule: 1 Devex,
// 0 Dantzig (for the phase-2 start); tick_budget: s_memrealtime ticks (100 MHz)
// the launch may run before it stops with ST_TIMEOUT (0: no limit)
struct ResOut {
    int64_t refactors, gj_refactors, devex_resets, ticks;
    double emax_max;
    int32_t phase, pad;
    int64_t stage[8], stage2[8], stage3[8];  // diagnostic builds (-DELP_RES_PROF=1): shader cycles per loop stage
};
// warm: a branch-and-bound node's warm start runs first (reload_bounds_warm's
// device part: real costs, BTRAN, every nonbasic column re-placed, the dual
// weights reset, a refactor); xout: the structurals' values (scaled, n) at exit
struct ResArgs {
    int32_t phase, price_rule, refactor_mode, warm;
    int64_t tick_budget;
    ResOut* out;
    double* xout;
};
size_t resident_lds_bytes(int m, int n);
hipError_t launch_resident(const Dev& d, const ResArgs& a, size_t lds, hipStream_t st);

}  // namespace elp
