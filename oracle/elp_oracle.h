/*
 * elp_oracle.h -- CPU restatement of the dense revised-simplex hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library.  The product path
 * (easylp_amd/, libeasylp_hip.so) never links or calls it.
 *
 * What it restates: the LP solve that EasyLP hands to lp_solve at
 * /root/reference/R/class.R:260-278 (make.lp / set.objfn / lp.control /
 * set.bounds / add.constraint / solve / get.objective / get.variables),
 * including the status numbering of R/class.R:279-295, the lower>upper
 * override of R/class.R:297-298 and lp_solve's 1e30 "infinity" that
 * R/utils.R:172-176 maps back to +-Inf.  lp_solve 5.5 itself is a
 * third-party dependency that is absent from /root/reference (lpSolveAPI,
 * unversioned, DESCRIPTION:18-21); its numbers are pinned instead by the
 * reference's own LP tests (tests/testthat/test-DOP.R:53,
 * tests/testthat/test-unbounded.R:8-9), the README LP (README.md:14-38),
 * vignette LPs, and HiGHS-generated fixtures (tests/golden/).
 *
 * The floating-point order of every reduction here is the one the HIP
 * kernels use (see DESIGN.md "Reduction order contract"), so the GPU and
 * this oracle walk the same pivot sequence on the same input.
 */
#ifndef ELP_ORACLE_H
#define ELP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_control {
    double tol_primal;     /* Harris primal feasibility tolerance            */
    double tol_dual;       /* reduced-cost optimality tolerance              */
    double tol_pivot;      /* |alpha| below this never limits the step       */
    double infinity;       /* |v| >= infinity is treated as infinite (1e30)  */
    int64_t max_iter;      /* <=0: default 100*(m+n)+10000                   */
    int32_t refactor_period;
    int32_t degen_switch;  /* consecutive degenerate pivots before Bland     */
    int64_t t_mark_iter;   /* record the wall time when this many iterations
                              have run (stats.seconds_at_mark); <0: never     */
    int32_t refactor_mode; /* 0 Newton-Schulz (GJ fallback), 1 always GJ     */
    int32_t price_mode;    /* 0 dense: chunked AR sweep over the Y rows;
                              1 CSC path: one fma chain per column over its
                              nonzero rows in ascending order (elp_load_csc)  */
    int32_t price_rule;    /* 0 Dantzig (largest |d_j|), 1 Devex reference
                              weights (largest d_j^2 / w_j; run_phase)        */
    int32_t scaling;       /* 4 geometric | 64 equilibrate (elp_control.scaling):
                              power-of-2 factors, scale_factors()           */
    double tol_singular;   /* Gauss-Jordan |pivot| <= this: numerical failure */
    int32_t simplex;       /* phase 1 when the slack basis is infeasible:
                              6 dual simplex (lp_solve SIMPLEX_DUAL_PRIMAL),
                              5 primal on artificials (SIMPLEX_PRIMAL_PRIMAL);
                              0: the default (= elp_control.simplex's)       */
    int32_t pad0;
} orc_control;

typedef struct orc_stats {
    int64_t iterations;
    int64_t phase1_iterations;
    int64_t bound_flips;
    int64_t degenerate;
    int64_t refactors;
    int64_t bump_dim;      /* k at exit: basic structurals                   */
    int64_t y_rows;        /* |Y| at exit: rows with a nonbasic slack         */
    double seconds;
    double price_bytes;    /* sum over iterations of 8*(|Y|*n + n + |Y|)      */
    double seconds_at_mark;
    int64_t gj_refactors;  /* refactors that fell back to Gauss-Jordan      */
    int64_t devex_resets;  /* Devex reference-framework restarts            */
    double max_inv_resid;  /* largest max|I - M Minv| a refactor measured    */
    int64_t lu_nnz;        /* (reserved: the r03-r04 sparse-LU restatement)   */
    int64_t eta_nnz;       /* (reserved)                                       */
    int64_t dual_iterations; /* phase-1 iterations of the dual simplex        */
    int64_t flattened;     /* columns whose cost the dual phase zeroed        */
} orc_stats;

void orc_default_control(orc_control* c);

/* Solve  min/max obj'x  s.t.  A x (dir) rhs,  lo <= x <= up.
 * A: column-major m x n (lda = m).  dir: 1 '<=', 2 '>=', 3 '=='.
 * Outputs (caller-allocated, may be NULL): x[n], y[m] duals, basis[m]
 * (sorted basic variable ids: j<n structural, n+i slack, n+m+i artificial).
 * trace (may be NULL): up to trace_cap entries of (entering, leaving) per
 * iteration; leaving = -1 for a bound flip, -2 for the unbounded ray.
 * Returns lp_solve status: 0 optimal, 1 sub-optimal (iteration cap),
 * 2 infeasible, 3 unbounded, 5 numerical failure.  Negative = usage error. */
int orc_solve_dense(int64_t m, int64_t n, const double* A, const int32_t* dir,
                    const double* rhs, const double* obj, const double* lo,
                    const double* up, int32_t maximize, const orc_control* ctl,
                    double* objval, double* x, double* y, int64_t* basis,
                    int64_t* trace, int64_t trace_cap, orc_stats* st);

/* orc_solve_dense plus, when the LP is solved to optimality and sens != NULL,
 * the sensitivity report of the final basis (R/class.R:613-646; conventions in
 * elp_oracle.c sensitivity()): sens = objfrom[n] objtill[n] duals[m+n]
 * dualsfrom[m+n] dualstill[m+n] (5n + 3m doubles, user sense, +-1e30 = inf). */
int orc_solve_dense_sens(int64_t m, int64_t n, const double* A, const int32_t* dir,
                         const double* rhs, const double* obj, const double* lo,
                         const double* up, int32_t maximize, const orc_control* ctl,
                         double* objval, double* x, double* y, int64_t* basis,
                         int64_t* trace, int64_t trace_cap, orc_stats* st, double* sens);

/* orc_solve_dense on the synthetic LP of orc_generate_dense(seed, m, n) (all
 * rows <=, x >= 0, maximize) without materialising A: every entry is
 * regenerated from the counter-based generator when the algorithm reads it, so
 * the 10000 x 500000 config (40 GB) runs in the memory of its Y rows (AR), the
 * bump inverse and O(m + n) vectors.  Dense pricing order only (price_mode 0). */
int orc_solve_generated(uint64_t seed, int64_t m, int64_t n, const orc_control* ctl, double* objval,
                        double* x, double* y, int64_t* basis, int64_t* trace, int64_t trace_cap,
                        orc_stats* st);

/* Mixed-integer LP (is_int[n] != 0: integer column; binary = integer in
 * [0, 1]) by depth-first branch and bound over orc_solve_dense relaxations
 * (rules in elp_oracle.c).  max_nodes <= 0: unlimited.  Returns 0 optimal,
 * 1 node limit (x = best found, if any), 2 infeasible, 3 unbounded. */
int orc_solve_mip(int64_t m, int64_t n, const double* A, const int32_t* dir, const double* rhs,
                  const double* obj, const double* lo, const double* up, int32_t maximize,
                  const int32_t* is_int, const orc_control* ctl, int64_t max_nodes,
                  double* objval, double* x, int64_t* nodes, int64_t* lp_iters);

/* Counter-based synthetic dense LP:
 * maximize c'x, A x <= b, x >= 0; A_ij, c_j ~ U[0,1), b_i = n/8 + U[0,1) n/4.
 * Columns [col0, col0+ncols) of the m x n instance are written to A
 * (column-major, lda = m).  c (ncols) and b (m) may be NULL. */
void orc_generate_dense(uint64_t seed, int64_t m, int64_t n, int64_t col0,
                        int64_t ncols, double* A, double* b, double* c);

/* Scaling exponents (control.scaling bits: 4 geometric, 64 equilibrate) of a
 * dense column-major m x n A: the solver works on a_ij * 2^(rho_i + gam_j). */
void orc_scale_factors(int64_t m, int64_t n, const double* A, int32_t mode, int32_t* rho, int32_t* gam);

/* Rows rows[0..nrows) of the same instance, row-major (out[r * n + j]). */
void orc_generate_rows(uint64_t seed, int64_t m, int64_t n, const int64_t* rows, int64_t nrows,
                       double* out);

#ifdef __cplusplus
}
#endif
#endif
