"""CPU checks of the drop-in boundary: the library loads and exports every
symbol include/easylp_hip.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "easylp_hip.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(elp_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_expected_surface():
    from easylp_amd._lib import EXPORTS
    assert sorted(EXPORTS) == declared()


def test_library_exports_every_declared_symbol():
    from easylp_amd import build
    lib_path = build.build()
    lib = ctypes.CDLL(lib_path)
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_abi_version_and_defaults():
    from easylp_amd._lib import ElpControl, load
    lib = load()
    assert lib.elp_abi_version() == 1
    c = ElpControl()
    lib.elp_default_control(ctypes.byref(c))
    assert c.infinity == 1e30 and c.refactor_period == 100 and c.sync_every == 32


def test_control_struct_size_matches_header():
    # 5 doubles + int64 + 8 int32 fields + 4 reserved int32 = 96 bytes
    from easylp_amd._lib import ElpControl, ElpStats
    assert ctypes.sizeof(ElpControl) == 96
    assert ctypes.sizeof(ElpStats) == 8 * 8 + 4 * 8 + 4 + 4 + 16 + 8 + 8 + 8 + 8 + 16


def test_usage_errors_without_gpu():
    from easylp_amd._lib import load
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
