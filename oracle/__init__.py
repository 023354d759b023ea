"""CPU oracle for the dense revised-simplex hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product (easylp_amd, libeasylp_hip.so) never touches it.
"""
from .binding import OracleResult, generate_dense, load, solve_dense, solve_mip  # noqa: F401
