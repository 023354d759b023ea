"""GPU parity on the seeded fuzz LPs (tests/fuzz_lps.py: every row direction
and bound kind, empty / one-row / one-column models, degenerate integer
matrices, badly scaled rows and columns, infeasible and unbounded outcomes;
the oracle itself is checked against HiGHS on the same set in
tests/test_fuzz_oracle.py).  Each LP goes through the HIP path and the oracle
with the same controls: status, pivot trace and basis identical, objective and
x bit-identical (asserted within 1e-12), the unbounded ray's +-1e30 values
exact.  Variants: the default (Devex, scaling on, dense), Dantzig pricing,
scaling off, the CSC path (oracle price_mode 1) and two ranks in one process
(elp_control.ngpu = 2, column-sharded); the sensitivity report of every
optimal LP; branch and bound on the fuzz MIPs (node for node)."""
import numpy as np
import pytest

from fuzz_lps import fuzz_mip, fuzz_set

pytestmark = pytest.mark.gpu

FUZZ = fuzz_set(120)
IDS = [f"f{r['seed']}_{r['m']}x{r['n']}" for r in FUZZ]

# (name, GPU controls, oracle controls, subset of the set)
VARIANTS = [
    ("devex", {}, {}, slice(None)),
    ("dantzig", {"pricing": 0}, {"price_rule": 0}, slice(0, None, 2)),
    ("unscaled", {"scaling": 0}, {"scaling": 0}, slice(1, None, 2)),
]


def _same(g, o):
    assert g.status == o.status, (g.status, o.status)
    np.testing.assert_array_equal(g.trace, o.trace)
    if g.status in (0, 1):
        np.testing.assert_array_equal(g.basis, o.basis)
        assert abs(g.objval - o.objval) <= 1e-12 * max(1.0, abs(o.objval))
        if len(o.x):
            np.testing.assert_allclose(g.x, o.x, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(o.x).max()))
    if g.status == 3:
        assert g.objval == o.objval
        np.testing.assert_array_equal(g.x, o.x)


def _run(gpu, rec, sparse=False, gctl=None, octl=None):
    from oracle import solve_dense as orc
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
    solve = gpu.solve_sparse if sparse else gpu.solve_dense
    g = solve(*args, trace=100000, **(gctl or {}), **({"basis": 1} if sparse else {}))
    o = orc(*args, trace_cap=100000, **(octl or {}), **({"price_mode": 1} if sparse else {}))
    _same(g, o)
    return g


@pytest.mark.parametrize("name,gctl,octl,sub", VARIANTS, ids=[v[0] for v in VARIANTS])
def test_fuzz_dense(gpu, name, gctl, octl, sub):
    seen = set()
    for rec, rid in zip(FUZZ[sub], IDS[sub]):
        try:
            seen.add(_run(gpu, rec, gctl=gctl, octl=octl).status)
        except Exception as e:  # name the LP
            raise AssertionError(f"{rid}: {type(e).__name__}: {e}") from None
    assert {0, 2, 3} <= seen, seen


def test_fuzz_csc(gpu):
    seen = set()
    for rec, rid in zip(FUZZ, IDS):
        try:
            seen.add(_run(gpu, rec, sparse=True).status)
        except Exception as e:  # name the LP
            raise AssertionError(f"{rid}: {type(e).__name__}: {e}") from None
    assert {0, 2, 3} <= seen, seen


def test_fuzz_two_ranks(gpu):
    """ngpu = 2: columns split over two rank handles (sharing the test GPU);
    a one-column model cannot be split and is refused (ELP_E_ARG)."""
    for rec, rid in list(zip(FUZZ, IDS))[::4]:
        if rec["n"] < 2:
            from easylp_amd._lib import ElpError
            with pytest.raises(ElpError, match="ngpu exceeds n"):
                _run(gpu, rec, gctl={"ngpu": 2})
            continue
        try:
            g = _run(gpu, rec, gctl={"ngpu": 2})
        except Exception as e:  # name the LP
            raise AssertionError(f"{rid}: {type(e).__name__}: {e}") from None
        assert g.stats["world_size"] == 2


def test_fuzz_sensitivity(gpu):
    """elp_sensitivity (fp64 MFMA, fused ranging) against the oracle's
    sequential restatement on every optimal fuzz LP: 1e-9 relative to the
    report's scale (north_star's 1e-8), +-1e30 limits exact."""
    from oracle import solve_dense as orc
    done = 0
    for rec, rid in zip(FUZZ, IDS):
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        o = orc(*args, sens=True)
        if o.status != 0:
            continue
        g = gpu.solve_dense(*args, sensitivity=True)
        try:
            assert g.status == 0
            np.testing.assert_array_equal(g.basis, o.basis)
            for key in ("objfrom", "objtill", "duals", "dualsfrom", "dualstill"):
                a, b = np.asarray(g.sens[key]), np.asarray(o.sens[key])
                ia, ib = np.abs(a) >= 1e30, np.abs(b) >= 1e30
                np.testing.assert_array_equal(ia, ib, err_msg=key)
                np.testing.assert_array_equal(a[ia], b[ib], err_msg=key)
                scale = max(1.0, float(np.abs(b[~ib]).max(initial=0.0)))
                np.testing.assert_allclose(a[~ia], b[~ib], rtol=1e-9, atol=1e-9 * scale, err_msg=key)
        except AssertionError as e:
            raise AssertionError(f"{rid}: {e}") from None
        done += 1
    assert done >= 40, done


@pytest.mark.parametrize("path", ["dense", "csc"])
def test_fuzz_mip(gpu, path):
    """The GPU tree equals the oracle's (same LPs bit for bit, same rules):
    status, node count, LP iterations, incumbent and objective."""
    from oracle import solve_mip
    for s in range(40):
        rec = fuzz_mip(s)
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        solve = gpu.solve_dense if path == "dense" else gpu.solve_sparse
        g = solve(*args, is_int=rec["is_int"], **({"basis": 1} if path == "csc" else {}))
        o = solve_mip(*args, rec["is_int"], price_mode=1 if path == "csc" else 0)
        assert (g.status, g.stats["mip_nodes"], g.stats["mip_lp_iterations"]) == (
            o.status, o.stats["nodes"], o.stats["lp_iterations"]), f"mip{s}"
        if o.status == 0:
            assert g.objval == o.objval, f"mip{s}"
            np.testing.assert_array_equal(g.x, o.x, err_msg=f"mip{s}")
