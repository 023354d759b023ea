/*
 * easylp_hip.h -- C ABI of the MI355X dense revised-simplex solver.
 *
 * Drop-in seam: the body of easylp$solve() at /root/reference/R/class.R:260-278
 * (and the sensitivity read-back at :624, :641) hands a dense LP to lp_solve
 * through lpSolveAPI.  These entry points are what an R .Call() shim (see
 * INTEGRATION.md) binds instead; each one cites the lpSolveAPI call(s) it
 * replaces.  Plain C types only: pointers, sizes, int32/int64, double.
 *
 * Error convention: functions return 0 on success and a negative ELP_E_* code
 * on usage / device error (elp_last_error() explains).  The LP outcome is
 * reported separately in lp_solve's numbering so R/class.R:279-295 is unchanged:
 * 0 optimal, 1 sub-optimal (iteration cap), 2 infeasible, 3 unbounded,
 * 5 numerical failure, 7 timeout.  Infinite values are accepted as +-Inf or as
 * |v| >= control.infinity (1e30, lp_solve's infinity) and are reported back as
 * +-1e30, so R/utils.R:172-176 (large_to_infinity) still applies.
 */
#ifndef EASYLP_HIP_H
#define EASYLP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ELP_ABI_VERSION 7  /* 7: elp_control.resident, elp_stats.resident / resident_launches /
                             resident_ticks (were reserved / lu_nnz / eta_nnz); 6: elp_stats.price_seconds_stamps / price_stamped_launches; 3: elp_stats.iter_bytes appended; 4: elp_control.exchange /
                             basis, elp_load_dense_device_multi, elp_stats.exchange /
                             h2d_bytes / basis; 5: elp_control.simplex,
                             elp_stats.exchange_rtt_us / dual_iterations / simplex */

/* row directions, mirroring R/class.R:272 ("==" -> "=") and the "<"/">"
 * spellings accepted by R/methods.R:215-219 */
#define ELP_LE 1
#define ELP_GE 2
#define ELP_EQ 3

/* lp_solve status numbering (R/class.R:279-295) */
#define ELP_OPTIMAL 0
#define ELP_SUBOPTIMAL 1
#define ELP_INFEASIBLE 2
#define ELP_UNBOUNDED 3
#define ELP_NUMFAILURE 5
#define ELP_TIMEOUT 7

/* usage / device errors (negative return values) */
#define ELP_E_ARG -1
#define ELP_E_STATE -2
#define ELP_E_NOMEM -3
#define ELP_E_HIP -4
#define ELP_E_COMM -5
#define ELP_E_UNSUPPORTED -6

typedef struct elp_handle elp_handle;

#define ELP_PRICE_DANTZIG 0 /* elp_control.pricing */
#define ELP_PRICE_DEVEX 1

typedef struct elp_control {
    double tol_primal;       /* Harris primal feasibility tolerance    (1e-9)  */
    double tol_dual;         /* optimality tolerance on |d_j|          (1e-9)  */
    double tol_pivot;        /* |alpha| below this never limits a step (1e-9)  */
    double infinity;         /* lp_solve infinity                      (1e30)  */
    double time_limit;       /* seconds, <= 0: none   (lp.control timeout)     */
    int64_t max_iter;        /* <= 0: 100*(m+n)+10000                          */
    int32_t refactor_period; /* pivots between refactors (250, lp_solve maxpivot) */
    int32_t degen_switch;    /* degenerate pivots before Bland's rule  (50)    */
    int32_t device;          /* HIP device ordinal for this handle     (0)     */
    int32_t sync_every;      /* iterations launched between host polls (32)    */
    int32_t verbose;         /* 0 quiet; ELP_PROFILE_PRICE: time pricing kernel */
    int32_t refactor_mode;   /* 0: Newton-Schulz correction, Gauss-Jordan when
                                max|I - M Minv| > 1e-6; 1: always Gauss-Jordan */
    int32_t replicate;       /* column-sharded solves (elp_comm_init*): 0 auto --
                                every rank keeps all of A when m*n*8 <= 64 GiB, so
                                the entering column is read locally and only the
                                min-loc record is exchanged; 1 always; 2 never
                                (each rank holds its shard, the entering column
                                travels in an all-reduce) */
    int32_t max_nodes;       /* branch and bound: node limit, <= 0 unlimited   */
    int32_t pricing;         /* ELP_PRICE_DEVEX (default): largest d_j^2 / w_j
                                with Devex reference weights, lp_solve's default
                                pricer (lp.control(pivoting = "devex"));
                                ELP_PRICE_DANTZIG: largest |d_j|               */
    int32_t ngpu;            /* devices this handle drives in ONE process (the
                                R caller stays one process): <= 1 one GPU; P > 1
                                shards the columns over devices device ..
                                device+P-1 (mod the visible count) with one host
                                thread per device and an in-process
                                communicator (RCCL over xGMI when the devices
                                are distinct).  Excludes elp_comm_init*.
                                P > n: ELP_E_ARG (a rank prices >= 1 column). */
    int32_t scaling;         /* ELP_SCALE_* bits (lp.control(scaling = ...)):
                                0 none; ELP_SCALE_GEOMETRIC | ELP_SCALE_EQUILIBRATE
                                (default, lp_solve's "geometric" + "equilibrate");
                                factors are powers of 2 so scaling is exact     */
    int32_t exchange;        /* per-iteration min-loc of a column-sharded solve
                                with A replicated:  0 (default) -- an ngpu
                                handle writes each rank's record straight into
                                every peer's device memory (peer access, no IPC)
                                and polls its own mailbox inside the select
                                kernel, when every device maps every peer and a
                                probe round trip succeeds at elp_create; else,
                                and with A not replicated, the collective
                                (RCCL all-gather / in-process transport).
                                Multi-process handles (elp_comm_init*) use the
                                collective unless elp_comm_enable_p2p.
                                1: always the collective */
    double tol_singular;     /* |pivot| <= this in a Gauss-Jordan refactor is a
                                singular basis -> status 5            (1e-13)  */
    double mailbox_timeout;  /* xGMI mailbox: seconds a rank waits for a peer's
                                record before the solve fails (ELP_E_COMM) (2) */
    int32_t basis;           /* basis representation (lp_solve's bfp):
                                ELP_BASIS_AUTO (default) = ELP_BASIS_INVERSE:
                                unit columns + the explicit inverse of the
                                structural bump (k basic structurals: O(m k +
                                k^2) device memory, grown with k);
                                ELP_BASIS_LU: refused (ELP_E_UNSUPPORTED) -- the
                                r03-r04 sparse-LU engine measured 150x slower
                                than the bump inverse and was removed in r05
                                 */
    int32_t simplex;         /* lp.control(simplextype = ...), lp_solve's
                                set_simplextype numbering: ELP_SIMPLEX_DUAL_PRIMAL
                                (6) -- phase 1 by the dual simplex when the slack
                                basis is primal infeasible, phase 2 primal;
                                ELP_SIMPLEX_PRIMAL_PRIMAL (5) -- phase 1 primal on
                                artificials.  0: the default = lp_solve's,
                                DUAL_PRIMAL where the dual phase exists (one
                                GPU, or column-sharded ranks holding all of A,
                                with the bump inverse), else PRIMAL_PRIMAL;
                                elp_stats.simplex reports what ran */
    int32_t resident;        /* the resident small-LP solver: the
                                whole simplex loop of an LP whose state fits in
                                one CU's LDS in ONE launch of one wave instead
                                of 4-7 launches per pivot.  0 (default): when it
                                fits (one GPU, no column shards); 1: the same
                                (force: the tests); 2: never (the multi-workgroup
                                pipeline).  Same pivots, same bits either way;
                                branch-and-bound nodes warm-start inside the
                                same launch; elp_stats.resident reports what ran */
    int32_t pad_resident;
} elp_control;

#define ELP_SIMPLEX_PRIMAL_PRIMAL 5  /* elp_control.simplex (lp_solve's SIMPLEX_*) */
#define ELP_SIMPLEX_DUAL_PRIMAL 6

#define ELP_BASIS_AUTO 0     /* elp_control.basis */
#define ELP_BASIS_INVERSE 1
#define ELP_BASIS_LU 2

#define ELP_SCALE_GEOMETRIC 4   /* elp_control.scaling bits (lp_solve's numbering) */
#define ELP_SCALE_EQUILIBRATE 64

typedef struct elp_stats {
    int64_t iterations;        /* simplex iterations, both phases             */
    int64_t phase1_iterations;
    int64_t bound_flips;
    int64_t degenerate;
    int64_t refactors;
    int64_t bump_dim;          /* k: basic structural columns at exit          */
    int64_t y_rows;            /* |Y|: rows with a nonbasic slack at exit      */
    int64_t host_polls;
    double seconds_total;      /* elp_solve wall time                          */
    double seconds_loop;       /* simplex loop only (excludes load / H2D)      */
    double seconds_load;       /* elp_load_* (H2D + device canonicalisation)  */
    double price_bytes;        /* algorithmic bytes of the pricing sweeps      */
    int32_t world_size;        /* ranks sharing the column partition           */
    int32_t rank;
    int64_t col0, ncols;       /* this rank's column shard                     */
    /* pricing-kernel timing.  control.verbose & ELP_PROFILE_EVENTS: HIP events
     * bound to every pricing dispatch (hipExtLaunchKernelGGL: the launch's
     * start / end timestamps, as a kernel trace reports them) of the chunks
     * between host polls in which every launch priced.  ELP_PROFILE_PRICE
     * instead: every workgroup of the pricing kernel stamps s_memrealtime (the
     * GPU's 100 MHz constant clock) at start and end; first start -> last end
     * per pass that chose an entering variable. */
    double price_seconds;      /* sum of timed pricing-kernel durations        */
    double price_timed_bytes;  /* algorithmic bytes of those launches          */
    int64_t price_timed_launches;
    int64_t gj_refactors;      /* refactors that needed a Gauss-Jordan rebuild */
    int64_t mip_nodes;         /* branch-and-bound nodes (LP relaxations) solved */
    int64_t mip_lp_iterations; /* simplex iterations over all of them           */
    int64_t price_launches;    /* pricing-kernel launches enqueued (profilers:
                                  the dispatches of this handle's pricing kernel) */
    double max_inv_resid;      /* drift of the maintained bump inverse: the
                                  largest max|I - M Minv| a refactor measured
                                  before correcting it (refactor_mode 0)        */
    double iter_bytes;         /* algorithmic bytes of the whole iterations:
                                  price_bytes + 48k^2 + 8mk + 16n + 16m each
                                  (select, FTRAN-z, ratio test, update)         */
    int32_t exchange;          /* min-loc transport of the last load: 0 none
                                  (one rank), 1 peer mailbox, 2 collective      */
    int32_t resident;          /* 1: the last solve ran in the resident solver */
    double seconds_h2d;        /* elp_load_dense: host -> device copy of A     */
    double h2d_bytes;          /* bytes of A read from host memory (once, also
                                  when several devices receive them)            */
    int64_t resident_launches; /* resident-solver launches of the last solve     */
    int64_t resident_ticks;    /* their device time (s_memrealtime, 100 MHz)   */
    int32_t basis;             /* the representation the last load used
                                  (ELP_BASIS_INVERSE)                           */
    int32_t simplex;           /* the phase-1 method the last solve ran
                                  (ELP_SIMPLEX_DUAL_PRIMAL / _PRIMAL_PRIMAL)    */
    double exchange_rtt_us;    /* peer mailbox (exchange 1): one exchange round
                                  between all ranks, measured by the set-up
                                  probe with every rank's kernel running        */
    int64_t dual_iterations;   /* iterations of the dual simplex (phase 1)     */
    /* ABI 6: the same sampled pricing launches timed by the kernel itself --
     * every workgroup stamps s_memrealtime (the GPU's 100 MHz constant clock)
     * at entry and exit; first start -> last end per launch (no marker packets,
     * no dispatch gap: VERDICT r04 #2) */
    double price_seconds_stamps;
    int64_t price_stamped_launches;
} elp_stats;

#define ELP_PROFILE_PRICE 2   /* elp_control.verbose bit: device-clock pricing timer */
#define ELP_PROFILE_EVENTS 4  /* elp_control.verbose bit: HIP events on each pricing dispatch */
#define ELP_PROFILE_SAMPLE 8  /* elp_control.verbose bit: the same on every 8th chunk between polls */

/* Fill *c with defaults. */
void elp_default_control(elp_control* c);

/* make.lp(nrow = 0, ncol = n) + lp.control(...)      R/class.R:260, :262
 * m rows, n structural columns (n >= 1, m >= 0).  ctl may be NULL. */
int elp_create(elp_handle** h, int64_t m, int64_t n, const elp_control* ctl);

/* set.objfn / lp.control(sense=) / set.bounds / add.constraint   R/class.R:261-274
 * A: column-major m x n host array (lda = m, R's native matrix layout).
 * dir[m] in {ELP_LE, ELP_GE, ELP_EQ}; rhs[m]; obj[n]; lo[n], up[n] (NULL:
 * 0 and +inf).  maximize != 0 for sense "max".  Inputs are copied. */
int elp_load_dense(elp_handle* h, const double* A, const int32_t* dir, const double* rhs,
                   const double* obj, const double* lo, const double* up, int32_t maximize);

/* Same, with A already in device memory on the handle's device (lda = m);
 * the solver reads it in place and never writes it; the caller keeps it alive
 * until elp_destroy. The small vectors are host arrays. */
int elp_load_dense_device(elp_handle* h, const double* dA, const int32_t* dir, const double* rhs,
                          const double* obj, const double* lo, const double* up,
                          int32_t maximize);

/* Single-process multi-device (elp_control.ngpu = P > 1) with A already
 * resident on every device: dA[r] is the full m x n column-major A (lda = m)
 * in the memory of rank r's device (device + r mod the visible count), count =
 * P.  Rank r reads its copy in place -- all of it when A is replicated
 * (elp_control.replicate), else only its column shard -- so no device-to-device
 * copy happens at load.  The caller keeps every dA[r] alive until elp_destroy.
 * On a one-device handle count must be 1 (then = elp_load_dense_device). */
int elp_load_dense_device_multi(elp_handle* h, const double* const* dA, int32_t count, const int32_t* dir,
                                const double* rhs, const double* obj, const double* lo, const double* up,
                                int32_t maximize);

/* Sparse A in compressed sparse columns (BASELINE config 5;
 * the bump inverse with hypersparse FTRAN / B^-1 rows):
 * colptr[n+1] (colptr[0] = 0, colptr[n] = nnz), rowind[nnz] strictly increasing
 * within each column, val[nnz] finite.  Same problem semantics as
 * elp_load_dense; pricing then sweeps the nonzeros (12 bytes each) instead of
 * dense rows.  One GPU only (ELP_E_UNSUPPORTED after elp_comm_init*).  Inputs
 * are copied. */
int elp_load_csc(elp_handle* h, const int64_t* colptr, const int32_t* rowind, const double* val,
                 const int32_t* dir, const double* rhs, const double* obj, const double* lo,
                 const double* up, int32_t maximize);

/* Synthetic dense LP of SURVEY.md 8d generated on the device (bench / tests):
 * maximize c'x, A x <= b, x >= 0, A_ij, c_j ~ U[0,1), b_i = n/8 + U n/4,
 * counter-based (seed, stream, global index) so every rank / the oracle
 * regenerate the same numbers. */
int elp_load_generated(elp_handle* h, uint64_t seed);

/* The same synthetic LP written into caller memory instead of a handle (bench
 * and tests: A stays resident in HBM and every solve loads it with
 * elp_load_dense_device, so load is timed and generation is not).  dA: device
 * memory on `device`, m x n column-major (lda = m); b[m], c[n]: host arrays
 * (either may be NULL). */
int elp_generate_dense(int32_t device, uint64_t seed, int64_t m, int64_t n, double* dA, double* b,
                       double* c);

/* set.type(prob, columns, "integer" | "binary")        R/class.R:265
 * is_int[n] != 0 marks integer columns (binary = integer with bounds [0, 1]);
 * NULL clears.  Call after elp_load_*, before elp_solve, which then runs a
 * depth-first branch and bound over GPU LP relaxations (lowest-index
 * fractional column, ceiling branch first, as lp_solve's defaults) and reports
 * the incumbent through elp_get_solution. */
int elp_set_int(elp_handle* h, const int32_t* is_int);

/* solve(prob)                                          R/class.R:276 */
int elp_solve(elp_handle* h, int32_t* lp_status);

/* Run at most `iters` more simplex iterations (bench steps); *lp_status is
 * ELP_SUBOPTIMAL while the solve is still in progress. */
int elp_iterate(elp_handle* h, int64_t iters, int32_t* lp_status);

/* get.objective / get.variables (+ duals and basis)    R/class.R:277-278
 * Any output pointer may be NULL.  x[n], y[m] (duals in the user's sense),
 * basis[m] sorted basic variable ids: j < n structural, n+i slack of row i,
 * n+m+i artificial of row i.  After a MIP solve (elp_set_int) objval and x
 * are the incumbent's as the search found it; y and basis belong to no LP of
 * the tree and are zeroed / set to -1 (R reads only the objective and the
 * variables, R/class.R:277-278). */
int elp_get_solution(elp_handle* h, double* objval, double* x, double* y, int64_t* basis);

int elp_get_stats(elp_handle* h, elp_stats* st);

/* get.sensitivity.obj / get.sensitivity.rhs             R/class.R:613-646
 * Sensitivity report of the final basis of an OPTIMAL solve (ELP_E_STATE
 * otherwise, as R's stop("Problem is not optimal"); one GPU, an ngpu handle or
 * a rank of elp_comm_init* -- each rank ranges its own columns, the report is
 * the one-GPU report bit for bit; after elp_comm_init* it is a collective that
 * every rank calls and each receives the full report).  Any output
 * may be NULL.  objfrom[n] / objtill[n]: range of each objective coefficient
 * over which the basis stays optimal; duals[m+n]: constraint duals then reduced
 * costs (user sense); dualsfrom / dualstill[m+n]: range of each constraint's rhs
 * over which the duals stay valid (variable entries -1e30 / 1e30).  Infinite
 * limits are reported as +-1e30 (R/utils.R:172-176 maps them back). */
int elp_sensitivity(elp_handle* h, double* objfrom, double* objtill, double* duals,
                    double* dualsfrom, double* dualstill);

/* Pivot trace for parity tests: (entering, leaving) per iteration, leaving
 * = -1 for a bound flip, -2 for the unbounded ray.  Enable before elp_solve with capacity > 0. */
int elp_set_trace(elp_handle* h, int64_t capacity);
int elp_get_trace(elp_handle* h, int64_t* pairs, int64_t capacity, int64_t* count);

/* Multi-GPU column sharding: one process per GPU.  Rank 0
 * calls elp_comm_unique_id, ships the 128-byte id to every rank (e.g. over
 * torch.distributed), every rank calls elp_comm_init with it BEFORE
 * elp_load_*.  Rank r then owns columns [r*n/P, (r+1)*n/P). */
int elp_comm_unique_id(uint8_t id[128]);
int elp_comm_init(elp_handle* h, const uint8_t id[128], int32_t world_size, int32_t rank);

/* Per-iteration min-loc over xGMI without a collective launch: every rank
 * allocates a small uncached mailbox, the IPC handles are exchanged once over
 * the communicator, and from then on the select kernel writes its candidate
 * record straight into every peer's mailbox and waits for theirs (2 s timeout
 * -> ELP_E_COMM).  Call after elp_comm_init* and before elp_load_*; needs A
 * replicated (elp_control.replicate).  No-op on one rank. */
int elp_comm_enable_p2p(elp_handle* h);

/* Same sharded algorithm over caller-provided host transports instead of RCCL
 * (every rank may then share one GPU; used by the multi-rank tests).  Buffers
 * are host memory; return 0 on success.  allgather: recv holds world*bytes.
 * allreduce dtype: 0 = float64 sum, 1 = int32 max. */
typedef int (*elp_host_allgather_fn)(const void* send, void* recv, size_t bytes, void* user);
typedef int (*elp_host_allreduce_fn)(void* buf, size_t count, int32_t dtype, void* user);
typedef int (*elp_host_bcast_fn)(void* buf, size_t bytes, int32_t root, void* user);
int elp_comm_init_host(elp_handle* h, int32_t world_size, int32_t rank, elp_host_allgather_fn ag,
                       elp_host_allreduce_fn ar, elp_host_bcast_fn bc, void* user);

/* R finalizer for self$pointer (R/class.R:300; EasyLP's finalize at
 * R/class.R:497-501 is empty, this one frees device memory).  A one-GPU
 * handle leaves its stream, device buffers and pinned blocks to the next
 * elp_create on the same device (a bounded cache, ELP_NO_SPARE=1: off), so
 * R's one-handle-per-solve pattern pays no stream creation after the first. */
void elp_destroy(elp_handle* h);

/* Thread-local description of the last negative return. */
const char* elp_last_error(void);

int32_t elp_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
