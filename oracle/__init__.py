"""CPU oracle for the dense revised-simplex hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product (easylp_amd, libeasylp_hip.so) never touches it.
"""
from .binding import (  # noqa: F401
    OracleResult, generate_dense, generate_rows, load, scale_factors, solve_dense, solve_generated, solve_mip,
)
