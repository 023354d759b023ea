// elp_lu_factor.h -- host side of the sparse-LU basis of the CSC path
// (elp_control.basis = ELP_BASIS_LU): the Markowitz
// factorization P B Q = L U of the whole basis at a refactor, and the level
// schedules the single-workgroup GPU solves walk.  Plain C++ (no HIP), so the
// CPU tests compile this file alone and compare its factors with the oracle's
// restatement (oracle/elp_oracle_lu.c lu_factor), bit for bit.
#pragma once
#include <stdint.h>

#include <vector>

namespace elp {

// basis column source: position p holds variable head[p] -- structural j < n
// (CSC column, scaled values), slack n + i (e_i), artificial n + m + i (asgn_i e_i)
struct LuColumns {
    int64_t m, n;
    const int64_t* cp;
    const int32_t* ri;
    const double* cv;
    const double* asgn;
};

// one triangular solve as the GPU walks it: rows in level order (a row's
// dependencies all lie in earlier levels), each row's entries (step index,
// value) in ascending step order -- the oracle's fma-chain order
struct LuSched {
    std::vector<int32_t> lvptr;  // nlev + 1: level l = rows [lvptr[l], lvptr[l+1])
    std::vector<int32_t> row;    // step s of each scheduled row
    std::vector<int32_t> ptr;    // entries of scheduled row i: [ptr[i], ptr[i+1])
    std::vector<int32_t> j;      // step index of each entry
    std::vector<double> v;       // value of each entry
    int32_t nlev() const { return (int32_t)lvptr.size() - 1; }
};

struct LuFactors {
    int64_t m = 0;
    std::vector<int32_t> prow, pcol, rstep;  // step -> pivot row / position; row -> step
    std::vector<double> ud;                  // U diagonal per step
    // L rows (s' < s), U rows (s' > s) and their transposes, ascending s'
    std::vector<int64_t> Lp, Up, LTp, UTp;
    std::vector<int32_t> Lj, Uj, LTj, UTj;
    std::vector<double> Lv, Uv, LTv, UTv;
    // schedules: L forward, U backward, U^T forward, L^T backward
    LuSched sL, sU, sUT, sLT;
    int64_t nnz() const { return (int64_t)Lj.size() + (int64_t)Uj.size() + m; }
};

// Markowitz LU with threshold partial pivoting (the oracle's lu_factor: the
// same pivot rule -- column singleton, row singleton, then the first
// LU_SEARCH columns in (count, column) order -- and the same arithmetic).
// Returns 0, or -1 for a singular basis.
int lu_factor(LuFactors& f, const LuColumns& a, const int32_t* head, double tol_singular);

// level schedules of the four solves (after lu_factor)
void lu_schedules(LuFactors& f);

}  // namespace elp
