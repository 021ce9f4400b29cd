"""The C-ABI library loads on a GPU-less host and exports every symbol include/vbn_hip.h
declares; the ctypes mirror of the argument struct matches the C layout."""
import ctypes
import os
import re

from conftest import REPO


def _declared():
    hdr = open(os.path.join(REPO, "include", "vbn_hip.h")).read()
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(vbn_hip_\w+)\s*\(", hdr, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert {"vbn_hip_walk", "vbn_hip_normalize_weights", "vbn_hip_abi_version"} <= set(names)


def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  (bind torch's HIP runtime first, as the package does)
    from vectorizedbayesiannetwork_amd import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_declared()) == set(_lib.EXPORTS)
    assert lib.vbn_hip_abi_version() == _lib.ABI_VERSION
    assert lib.vbn_hip_struct_size(0) == ctypes.sizeof(_lib.VbnWalkArgs)
    assert lib.vbn_hip_struct_size(1) == 32 * 4


def test_bad_arguments_fail_before_any_launch():
    from vectorizedbayesiannetwork_amd import _lib
    lib = _lib.load()
    a = _lib.VbnWalkArgs()                       # all NULL / zero
    rc = lib.vbn_hip_walk(ctypes.byref(a), None)
    assert rc == 1001
    assert b"bad arguments" in lib.vbn_hip_last_error()
    assert lib.vbn_hip_normalize_weights(None, None, None, 0, 0, 1, 0.0, None) == 1001
    assert lib.vbn_hip_lds_bytes(12, 2) == (12 + 2) * 64 * 4
