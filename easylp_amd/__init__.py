"""easylp_amd -- MI355X-native dense revised-simplex solver behind EasyLP's solve().

The compute path is libeasylp_hip.so (hand-written gfx950 HIP kernels behind the
C ABI in include/easylp_hip.h).  `easylp_amd.solver` mirrors the hand-off of
easylp$solve() (/root/reference/R/class.R:251-302): dense A (`solve_dense`),
sparse A through the CSC path (`solve_sparse`).
"""
from .solver import (  # noqa: F401
    STATUS_TEXT, Problem, Solution, csc_arrays, dir_codes, generate_dense_device, large_to_infinity,
    solve_dense, solve_sparse, status_text,
)

__all__ = ["Problem", "Solution", "solve_dense", "solve_sparse", "csc_arrays", "generate_dense_device",
           "large_to_infinity", "status_text", "STATUS_TEXT"]
