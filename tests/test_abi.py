"""CPU checks of the drop-in boundary: the library loads and exports every
symbol include/easylp_hip.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "easylp_hip.h")


def _torch_first():
    """On a GPU box torch must start the HIP runtime before the library is
    loaded (the gpu fixture's rule, tests/conftest.py): loading the library
    first breaks every later GPU test of the same process."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(elp_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_expected_surface():
    from easylp_amd._lib import EXPORTS
    assert sorted(EXPORTS) == declared()


def test_library_exports_every_declared_symbol():
    from easylp_amd import build
    _torch_first()
    lib_path = build.build()
    lib = ctypes.CDLL(lib_path)
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_abi_version_and_defaults():
    from easylp_amd._lib import ABI_VERSION, ElpControl, load
    _torch_first()
    lib = load()
    assert lib.elp_abi_version() == ABI_VERSION == 7
    c = ElpControl()
    lib.elp_default_control(ctypes.byref(c))
    assert c.infinity == 1e30 and c.refactor_period == 250 and c.sync_every == 32
    assert c.tol_singular == 1e-13 and c.mailbox_timeout == 2.0 and c.ngpu == 1
    assert c.resident == 0  # (auto: the resident solver when the LP fits in LDS)


def _c_layout(struct, fields, tmp_path):
    """sizeof / offsetof of a header struct, from gcc (the ctypes mirror must match)."""
    import subprocess
    src = tmp_path / "lay.c"
    body = "".join(f'printf("%zu\\n", offsetof({struct}, {f}));' for f in fields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{HEADER}"\n'
                   f'int main(void){{printf("%zu\\n", sizeof({struct}));{body}return 0;}}\n')
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    return int(out[0]), [int(v) for v in out[1:]]


@pytest.mark.parametrize("which", ["elp_control", "elp_stats"])
def test_struct_layout_matches_header(which, tmp_path):
    from easylp_amd._lib import ElpControl, ElpStats
    cls = ElpControl if which == "elp_control" else ElpStats
    names = [f for f, _ in cls._fields_]
    size, offs = _c_layout(which, names, tmp_path)
    assert ctypes.sizeof(cls) == size
    assert [getattr(cls, f).offset for f in names] == offs


def test_usage_errors_without_gpu():
    from easylp_amd._lib import load
    _torch_first()
    lib = load()
    h = ctypes.c_void_p()
    assert lib.elp_create(ctypes.byref(h), -1, 5, None) == -1
    assert b"m >= 0" in lib.elp_last_error()
    assert lib.elp_create(None, 1, 1, None) == -1


def test_status_text_matches_reference_switch():
    from easylp_amd import status_text
    assert status_text(0) == "optimal"
    assert status_text(2) == "unfeasible"
    assert status_text(3) == "unbounded"
    assert status_text(7) == "timeout"
    assert status_text(42) == "undocumented status"
