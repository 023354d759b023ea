"""MPS reader / writer for the CSC path (BASELINE config 5).

lp_solve reads MPS through lpSolveAPI's `read.lp(file, type = "mps" | "free")`;
EasyLP itself builds its models in R (R/class.R:251-302), so this is the one
file format the solver boundary accepts directly.  Both the fixed and the free
MPS dialects are read (whitespace-separated fields; names without spaces):

    NAME / OBJSENSE (MIN|MAX, also "OBJSENSE MAX" on one line) / ROWS (N L G E)
    COLUMNS (with MARKER INTORG / INTEND) / RHS (a value on the objective row is
    minus the objective constant) / RANGES / BOUNDS (UP LO FX FR MI PL BV LI UI)
    / ENDATA

The result maps onto the C ABI's arrays: a ranged row becomes two rows (>= and
<=) because elp_load_* takes one direction per row; the objective constant is
returned separately (EasyLP adds its `objective_add` outside the solver too,
R/class.R:593-597).  The first N row is the objective; other N rows (free rows)
are dropped, and their COLUMNS / RHS / RANGES entries with them.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

INF = np.inf


@dataclass
class MpsProblem:
    name: str
    row_names: list
    col_names: list
    colptr: np.ndarray
    rowind: np.ndarray
    val: np.ndarray
    dirs: np.ndarray          # 1 <=, 2 >=, 3 ==
    rhs: np.ndarray
    obj: np.ndarray
    lo: np.ndarray
    up: np.ndarray
    maximize: bool = False
    objective_constant: float = 0.0
    is_int: np.ndarray = field(default_factory=lambda: np.zeros(0, bool))

    @property
    def shape(self):
        return len(self.rhs), len(self.obj)

    def dense(self) -> np.ndarray:
        m, n = self.shape
        A = np.zeros((m, n))
        for j in range(n):
            s, e = self.colptr[j], self.colptr[j + 1]
            A[self.rowind[s:e], j] += self.val[s:e]
        return A


class MpsError(ValueError):
    pass


def _num(tok: str, what: str, lineno: int) -> float:
    try:
        return float(tok)
    except ValueError:
        raise MpsError(f"line {lineno}: bad number {tok!r} in {what}") from None


def read_mps(path_or_text: str, *, text: bool = False) -> MpsProblem:
    """Parse an MPS file (fixed or free format) into CSC arrays."""
    if text:
        lines = path_or_text.splitlines()
    else:
        with open(path_or_text) as f:
            lines = f.read().splitlines()
    name = ""
    section = None
    maximize = False
    rows = {}          # name -> index (constraint rows)
    row_type = []      # 'L' 'G' 'E'
    row_names = []
    obj_row = None
    free_rows = set()  # N rows after the first: dropped with their entries
    cols = {}          # name -> index
    col_names = []
    entries = []       # (row, col, value)
    obj = []
    is_int = []
    in_int = False
    rhs_vals = {}
    rng_vals = {}
    obj_const = 0.0
    bounds = []        # (type, col, value)

    for lineno, raw in enumerate(lines, 1):
        line = raw.rstrip()
        if not line or line.lstrip().startswith("*"):
            continue
        toks = line.split()
        head = line[0] not in " \t"
        if head:
            key = toks[0].upper()
            if key == "NAME":
                name = " ".join(toks[1:])
                section = None
                continue
            if key == "OBJSENSE":
                section = "OBJSENSE"
                if len(toks) > 1:
                    maximize = toks[1].upper() in ("MAX", "MAXIMIZE")
                continue
            if key in ("ROWS", "COLUMNS", "RHS", "RANGES", "BOUNDS"):
                section = key
                continue
            if key == "ENDATA":
                break
            if key == "OBJSENSE" or section == "OBJSENSE":
                maximize = key in ("MAX", "MAXIMIZE")
                continue
            raise MpsError(f"line {lineno}: unknown section {toks[0]!r}")
        if section == "OBJSENSE":
            maximize = toks[0].upper() in ("MAX", "MAXIMIZE")
        elif section == "ROWS":
            if len(toks) < 2:
                raise MpsError(f"line {lineno}: ROWS entry needs a type and a name")
            t, rn = toks[0].upper(), toks[1]
            if t == "N":
                if obj_row is None:
                    obj_row = rn
                else:
                    free_rows.add(rn)
                continue
            if t not in ("L", "G", "E"):
                raise MpsError(f"line {lineno}: row type {t!r}")
            if rn in rows:
                raise MpsError(f"line {lineno}: duplicate row {rn!r}")
            rows[rn] = len(row_type)
            row_type.append(t)
            row_names.append(rn)
        elif section == "COLUMNS":
            if len(toks) >= 3 and toks[1].strip("'").upper() == "MARKER":
                mk = toks[2].strip("'").upper()
                if mk == "INTORG":
                    in_int = True
                elif mk == "INTEND":
                    in_int = False
                continue
            cn = toks[0]
            if cn not in cols:
                cols[cn] = len(col_names)
                col_names.append(cn)
                obj.append(0.0)
                is_int.append(in_int)
            j = cols[cn]
            pairs = toks[1:]
            if len(pairs) % 2:
                raise MpsError(f"line {lineno}: COLUMNS entry needs (row, value) pairs")
            for a in range(0, len(pairs), 2):
                rn, v = pairs[a], _num(pairs[a + 1], "COLUMNS", lineno)
                if rn == obj_row:
                    obj[j] += v
                elif rn in rows:
                    entries.append((rows[rn], j, v))
                elif rn in free_rows:
                    continue
                else:
                    raise MpsError(f"line {lineno}: unknown row {rn!r}")
        elif section in ("RHS", "RANGES"):
            pairs = toks[1:] if len(toks) % 2 == 1 else toks  # the set name is optional
            for a in range(0, len(pairs), 2):
                rn, v = pairs[a], _num(pairs[a + 1], section, lineno)
                if section == "RHS" and rn == obj_row:
                    obj_const = -v
                elif rn in rows:
                    (rhs_vals if section == "RHS" else rng_vals)[rows[rn]] = v
                elif rn in free_rows or rn == obj_row:
                    continue
                else:
                    raise MpsError(f"line {lineno}: unknown row {rn!r}")
        elif section == "BOUNDS":
            t = toks[0].upper()
            if t in ("FR", "MI", "PL", "BV"):
                if len(toks) < 2:
                    raise MpsError(f"line {lineno}: bound needs a column")
                cn = toks[2] if len(toks) >= 3 and toks[2] in cols else toks[1] if toks[1] in cols else toks[-1]
                v = 0.0
            else:
                if len(toks) < 3:
                    raise MpsError(f"line {lineno}: bound needs a column and a value")
                cn, v = (toks[2], _num(toks[3], "BOUNDS", lineno)) if len(toks) >= 4 else (
                    toks[1], _num(toks[2], "BOUNDS", lineno))
            if cn not in cols:
                raise MpsError(f"line {lineno}: unknown column {cn!r}")
            bounds.append((t, cols[cn], v))
        else:
            raise MpsError(f"line {lineno}: data outside a section")

    n = len(col_names)
    lo = np.zeros(n)
    up = np.full(n, INF)
    is_int = np.array(is_int, dtype=bool)
    for j in np.nonzero(is_int)[0]:
        up[j] = INF  # lp_solve: integer columns from markers keep [0, inf)
    for t, j, v in bounds:
        if t == "UP":
            up[j] = v
            if v < 0 and lo[j] == 0.0:  # the classic MPS rule for a negative UP
                lo[j] = -INF
        elif t == "LO":
            lo[j] = v
        elif t == "FX":
            lo[j] = up[j] = v
        elif t == "FR":
            lo[j], up[j] = -INF, INF
        elif t == "MI":
            lo[j] = -INF
        elif t == "PL":
            up[j] = INF
        elif t == "BV":
            lo[j], up[j] = 0.0, 1.0
            is_int[j] = True
        elif t == "LI":
            lo[j] = v
            is_int[j] = True
        elif t == "UI":
            up[j] = v
            is_int[j] = True
        else:
            raise MpsError(f"bound type {t!r}")

    # rows: ranged rows split into a >= and a <= row
    out_dirs, out_rhs, out_names, row_map = [], [], [], []
    for i, t in enumerate(row_type):
        b = rhs_vals.get(i, 0.0)
        if i in rng_vals:
            r = rng_vals[i]
            if t == "E":
                lo_r, hi_r = (b, b + abs(r)) if r >= 0 else (b - abs(r), b)
            elif t == "L":
                lo_r, hi_r = b - abs(r), b
            else:
                lo_r, hi_r = b, b + abs(r)
            row_map.append([len(out_dirs), len(out_dirs) + 1])
            out_dirs += [2, 1]
            out_rhs += [lo_r, hi_r]
            out_names += [row_names[i] + "_lo", row_names[i] + "_hi"]
        else:
            row_map.append([len(out_dirs)])
            out_dirs.append({"L": 1, "G": 2, "E": 3}[t])
            out_rhs.append(b)
            out_names.append(row_names[i])
    cols_entries = [[] for _ in range(n)]
    for i, j, v in entries:
        for r in row_map[i]:
            cols_entries[j].append((r, v))
    colptr = np.zeros(n + 1, dtype=np.int64)
    rowind, val = [], []
    for j in range(n):
        acc = {}
        for r, v in cols_entries[j]:
            acc[r] = acc.get(r, 0.0) + v
        for r in sorted(acc):
            rowind.append(r)
            val.append(acc[r])
        colptr[j + 1] = len(rowind)
    return MpsProblem(name, out_names, col_names, colptr, np.array(rowind, dtype=np.int32),
                      np.array(val, dtype=np.float64), np.array(out_dirs, dtype=np.int32),
                      np.array(out_rhs, dtype=np.float64), np.array(obj, dtype=np.float64),
                      lo, up, maximize, obj_const, is_int)


def write_mps(p: MpsProblem, path: str | None = None) -> str:
    """Free-format MPS of a problem (rows keep their direction; no RANGES)."""
    fmt = repr
    out = [f"NAME {p.name or 'EASYLP'}"]
    if p.maximize:
        out += ["OBJSENSE", "    MAX"]
    out.append("ROWS")
    out.append(" N  OBJ")
    for i, d in enumerate(p.dirs):
        out.append(f" {'LGE'[int(d) - 1]}  {p.row_names[i]}")
    out.append("COLUMNS")
    marker = False
    for j, cn in enumerate(p.col_names):
        if len(p.is_int) and p.is_int[j] != marker:
            marker = bool(p.is_int[j])
            out.append(f"    M{j} 'MARKER' '{'INTORG' if marker else 'INTEND'}'")
        if p.obj[j] != 0.0:
            out.append(f"    {cn} OBJ {fmt(float(p.obj[j]))}")
        for t in range(p.colptr[j], p.colptr[j + 1]):
            out.append(f"    {cn} {p.row_names[p.rowind[t]]} {fmt(float(p.val[t]))}")
        if not p.colptr[j + 1] > p.colptr[j] and p.obj[j] == 0.0:
            out.append(f"    {cn} OBJ 0.0")
    if marker:
        out.append("    MEND 'MARKER' 'INTEND'")
    out.append("RHS")
    if p.objective_constant != 0.0:
        out.append(f"    RHS OBJ {fmt(-float(p.objective_constant))}")
    for i, b in enumerate(p.rhs):
        if b != 0.0:
            out.append(f"    RHS {p.row_names[i]} {fmt(float(b))}")
    out.append("BOUNDS")
    for j, cn in enumerate(p.col_names):
        lo, up = p.lo[j], p.up[j]
        if lo == up:
            out.append(f" FX BND {cn} {fmt(float(lo))}")
            continue
        if lo == -INF and up == INF:
            out.append(f" FR BND {cn}")
            continue
        if lo == -INF:
            out.append(f" MI BND {cn}")
        elif lo != 0.0:
            out.append(f" LO BND {cn} {fmt(float(lo))}")
        if up != INF:
            out.append(f" UP BND {cn} {fmt(float(up))}")
    out.append("ENDATA")
    s = "\n".join(out) + "\n"
    if path:
        with open(path, "w") as f:
            f.write(s)
    return s


def solve_mps(path: str, **control):
    """Read an MPS file and solve it through the CSC path on the GPU (a MIP when
    it has integer columns).  Returns
    (problem, Solution); Solution.objval excludes the objective constant, as
    lp_solve's get.objective does for EasyLP's addend (R/class.R:593-597)."""
    from .solver import Problem
    p = read_mps(path)
    m, n = p.shape
    with Problem(m, n, **control) as pr:
        pr.load_csc(p.colptr, p.rowind, p.val, p.dirs, p.rhs, p.obj, p.lo, p.up, p.maximize)
        if p.is_int.any():  # integer markers / BV / LI / UI: branch and bound
            pr.set_int(p.is_int)
        st = pr.solve()
        return p, pr.solution(st)
