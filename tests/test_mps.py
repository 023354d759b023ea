"""CPU: the MPS reader / writer (easylp_amd/mps.py) -- section handling, ranged
rows, bound types, integer markers, objective constant and sense -- and the
parsed LP solved by the oracle in the CSC order against SciPy-HiGHS."""
import numpy as np
import pytest

from easylp_amd.mps import MpsError, read_mps, write_mps

TEXT = """\
* a small LP exercising every section
NAME          TESTLP
OBJSENSE
    MAX
ROWS
 N  COST
 L  LIM1
 G  LIM2
 E  MYEQN
 L  R4
 E  R5
COLUMNS
    X1        COST         1.0   LIM1         1.0
    X1        LIM2         1.0   R4           2.0
    X2        COST         2.0   LIM1         1.0
    X2        MYEQN       -1.0
    X3        COST        -1.0   MYEQN        1.0
    X3        R5           1.0
    X4        COST         1.5   LIM2         1.0
    X4        R4          -1.0   R5           1.0
RHS
    RHS       COST        -3.5
    RHS       LIM1         4.0   LIM2         1.0
    RHS       MYEQN        1.0   R4           6.0
    RHS       R5           2.0
RANGES
    RNG       LIM1         2.5   R5          -1.5
    RNG       R4           3.0
BOUNDS
 UP BND       X1           4.0
 LO BND       X2          -1.0
 UP BND       X2           1.0
 MI BND       X3
 UP BND       X3           8.0
 FX BND       X4           0.5
ENDATA
"""


def test_parse_sections():
    p = read_mps(TEXT, text=True)
    assert p.name == "TESTLP" and p.maximize and p.objective_constant == 3.5
    assert p.col_names == ["X1", "X2", "X3", "X4"]
    # LIM1 ranged (L, R=2.5) -> [1.5, 4]; R4 (L, 3) -> [3, 6]; R5 (E, -1.5) -> [0.5, 2]
    assert p.row_names == ["LIM1_lo", "LIM1_hi", "LIM2", "MYEQN", "R4_lo", "R4_hi", "R5_lo", "R5_hi"]
    np.testing.assert_array_equal(p.dirs, [2, 1, 2, 3, 2, 1, 2, 1])
    np.testing.assert_array_equal(p.rhs, [1.5, 4.0, 1.0, 1.0, 3.0, 6.0, 0.5, 2.0])
    np.testing.assert_array_equal(p.obj, [1.0, 2.0, -1.0, 1.5])
    np.testing.assert_array_equal(p.lo, [0.0, -1.0, -np.inf, 0.5])
    np.testing.assert_array_equal(p.up, [4.0, 1.0, 8.0, 0.5])
    A = p.dense()
    np.testing.assert_array_equal(A[:, 0], [1, 1, 1, 0, 2, 2, 0, 0])
    np.testing.assert_array_equal(A[:, 3], [0, 0, 1, 0, -1, -1, 1, 1])
    assert not p.is_int.any()


def _highs(p):
    from scipy.optimize import linprog
    A = p.dense()
    c = -p.obj if p.maximize else p.obj
    ub = [(A[i], p.rhs[i]) if d == 1 else (-A[i], -p.rhs[i]) for i, d in enumerate(p.dirs) if d != 3]
    eq = [(A[i], p.rhs[i]) for i, d in enumerate(p.dirs) if d == 3]
    kw = {}
    if ub:
        kw.update(A_ub=np.array([u[0] for u in ub]), b_ub=[u[1] for u in ub])
    if eq:
        kw.update(A_eq=np.array([e[0] for e in eq]), b_eq=[e[1] for e in eq])
    bounds = [(None if not np.isfinite(l) else l, None if not np.isfinite(u) else u)
              for l, u in zip(p.lo, p.up)]
    r = linprog(c, bounds=bounds, method="highs-ds", **kw)
    return r.status, (-r.fun if p.maximize else r.fun)


def test_parsed_lp_oracle_vs_highs():
    from oracle import solve_dense as orc
    p = read_mps(TEXT, text=True)
    o = orc(p.dense(), p.dirs, p.rhs, p.obj, p.lo, p.up, p.maximize, price_mode=1)
    st, ref = _highs(p)
    assert st == 0 and o.status == 0
    assert abs(o.objval - ref) <= 1e-9 * max(1.0, abs(ref))


def test_round_trip():
    p = read_mps(TEXT, text=True)
    q = read_mps(write_mps(p), text=True)
    for f in ("dirs", "rhs", "obj", "lo", "up", "colptr", "rowind", "val"):
        np.testing.assert_array_equal(getattr(p, f), getattr(q, f))
    assert q.maximize and q.objective_constant == p.objective_constant


def test_integer_markers_and_bv():
    t = """NAME INTS
ROWS
 N obj
 L c1
COLUMNS
    MARKER 'MARKER' 'INTORG'
    y obj 1 c1 1
    MARKER 'MARKER' 'INTEND'
    z obj 2 c1 1
    w obj 1 c1 1
RHS
    rhs c1 3
BOUNDS
 BV bnd w
 UI bnd z 5
ENDATA
"""
    p = read_mps(t, text=True)
    np.testing.assert_array_equal(p.is_int, [True, True, True])
    np.testing.assert_array_equal(p.up, [np.inf, 5.0, 1.0])
    q = read_mps(write_mps(p), text=True)
    np.testing.assert_array_equal(q.is_int, p.is_int)


def test_errors():
    with pytest.raises(MpsError, match="unknown row"):
        read_mps("NAME X\nROWS\n N obj\nCOLUMNS\n    x nope 1\nENDATA\n", text=True)
    with pytest.raises(MpsError, match="bad number"):
        read_mps("NAME X\nROWS\n N obj\n L r\nCOLUMNS\n    x r abc\nENDATA\n", text=True)


def test_free_rows_dropped_with_their_entries():
    """N rows after the first are free rows: their COLUMNS / RHS / RANGES
    entries are skipped, not reported as unknown rows."""
    t = """NAME FREE
ROWS
 N obj
 N FREE
 L c1
 N FREE2
COLUMNS
    x obj 1 FREE 7
    x c1 1 FREE2 -2
    y obj 2 c1 1
    y FREE 3
RHS
    rhs c1 4 FREE 9
RANGES
    rng FREE2 1
ENDATA
"""
    p = read_mps(t, text=True)
    assert p.row_names == ["c1"]
    np.testing.assert_array_equal(p.obj, [1.0, 2.0])
    np.testing.assert_array_equal(p.rhs, [4.0])
    np.testing.assert_array_equal(p.dense(), [[1.0, 1.0]])
    with pytest.raises(MpsError, match="unknown row"):
        read_mps(t.replace("y FREE 3", "y NOPE 3"), text=True)
