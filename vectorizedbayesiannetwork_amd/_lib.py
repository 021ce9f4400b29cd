"""Loader for ``libvbn_hip.so`` (the C-ABI of include/vbn_hip.h) via ctypes.

The library is built in-tree by ``__graft_entry__.build()`` / ``make -C
vectorizedbayesiannetwork_amd/csrc``.  There is no CPU fallback: if the library is missing
or cannot be loaded, every accelerated entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VBN_HIP_LIB", os.path.join(HERE, "libvbn_hip.so"))
ABI_VERSION = 13

# exported symbols declared in include/vbn_hip.h
EXPORTS = (
    "vbn_hip_abi_version",
    "vbn_hip_last_error",
    "vbn_hip_walk",
    "vbn_hip_normalize_weights",
    "vbn_hip_normalize_weights_ex",
    "vbn_hip_rb_epilogue",
    "vbn_hip_resample",
    "vbn_hip_posterior_stats",
    "vbn_hip_posterior_stats_merge",
    "vbn_hip_normalize_weights_stats",
    "vbn_hip_discrete_posterior",
    "vbn_hip_discrete_posterior_typed",
    "vbn_hip_lds_bytes",
    "vbn_hip_struct_size",
    "vbn_hip_walk_kind_set",
    "vbn_hip_module_load",
    "vbn_hip_walk_module",
    "vbn_hip_module_unload",
    "vbn_hip_module_chain_waves",
)


class VbnWalkArgs(ctypes.Structure):
    """Mirror of ``vbn_walk_args`` (include/vbn_hip.h)."""

    _fields_ = [
        ("steps", ctypes.c_void_p),
        ("in_cols", ctypes.c_void_p),
        ("params", ctypes.c_void_p),
        ("fixed", ctypes.c_void_p),
        ("noise", ctypes.c_void_p),
        ("out_cols", ctypes.c_void_p),
        ("out_lp", ctypes.c_void_p),
        ("out_x", ctypes.c_void_p),
        ("n_queries", ctypes.c_int64),
        ("n_samples", ctypes.c_int32),
        ("n_steps", ctypes.c_int32),
        ("n_slots", ctypes.c_int32),
        ("max_out", ctypes.c_int32),
        ("fixed_ld", ctypes.c_int32),
        ("fixed_per_particle", ctypes.c_int32),
        ("noise_b", ctypes.c_int32),
        ("dmax", ctypes.c_int32),
        ("n_out_cols", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("kind_mask", ctypes.c_int32),
        ("q_base", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("offset", ctypes.c_uint64),
        ("state", ctypes.c_void_p),
        ("state_flags", ctypes.c_int32),
        ("gibbs_iters", ctypes.c_int32),
        ("gibbs_burn_in", ctypes.c_int32),
        ("gibbs_thin", ctypes.c_int32),
        ("n_noise", ctypes.c_int32),
        ("wbuf_floats", ctypes.c_int32),
        ("wave_particles", ctypes.c_int32),
        ("precomp_q", ctypes.c_void_p),
        ("run_if", ctypes.c_void_p),
        ("stats_part", ctypes.c_void_p),
    ]


class VbnHipError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None


def load(path: str = None) -> ctypes.CDLL:
    """Load and type the library (torch must be imported first so the HIP runtime that
    torch bundles is the one the library binds to)."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise VbnHipError(
                f"HIP library not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(no CPU fallback exists for the accelerated path)")
        import torch  # noqa: F401  (binds libamdhip64 first)
        lib = ctypes.CDLL(p)
        for name in EXPORTS:
            if not hasattr(lib, name):
                raise VbnHipError(f"{p} does not export {name}")
        lib.vbn_hip_abi_version.restype = ctypes.c_int
        lib.vbn_hip_last_error.restype = ctypes.c_char_p
        lib.vbn_hip_walk.argtypes = [ctypes.POINTER(VbnWalkArgs), ctypes.c_void_p]
        lib.vbn_hip_walk.restype = ctypes.c_int
        lib.vbn_hip_normalize_weights.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
            ctypes.c_int32, ctypes.c_float, ctypes.c_void_p]
        lib.vbn_hip_normalize_weights.restype = ctypes.c_int
        lib.vbn_hip_normalize_weights_ex.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
            ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p]
        lib.vbn_hip_normalize_weights_ex.restype = ctypes.c_int
        lib.vbn_hip_rb_epilogue.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        lib.vbn_hip_rb_epilogue.restype = ctypes.c_int
        lib.vbn_hip_resample.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        lib.vbn_hip_resample.restype = ctypes.c_int
        lib.vbn_hip_posterior_stats.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_void_p]
        lib.vbn_hip_posterior_stats.restype = ctypes.c_int
        lib.vbn_hip_posterior_stats_merge.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.vbn_hip_posterior_stats_merge.restype = ctypes.c_int
        lib.vbn_hip_normalize_weights_stats.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
            ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p]
        lib.vbn_hip_normalize_weights_stats.restype = ctypes.c_int
        lib.vbn_hip_discrete_posterior.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        lib.vbn_hip_discrete_posterior.restype = ctypes.c_int
        lib.vbn_hip_discrete_posterior_typed.argtypes = [
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        lib.vbn_hip_discrete_posterior_typed.restype = ctypes.c_int
        lib.vbn_hip_lds_bytes.argtypes = [ctypes.c_int32, ctypes.c_int32]
        lib.vbn_hip_lds_bytes.restype = ctypes.c_int64
        lib.vbn_hip_walk_kind_set.argtypes = [ctypes.POINTER(VbnWalkArgs)]
        lib.vbn_hip_walk_kind_set.restype = ctypes.c_int
        lib.vbn_hip_module_load.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_void_p)]
        lib.vbn_hip_module_load.restype = ctypes.c_int
        lib.vbn_hip_walk_module.argtypes = [ctypes.c_void_p, ctypes.POINTER(VbnWalkArgs), ctypes.c_void_p]
        lib.vbn_hip_walk_module.restype = ctypes.c_int
        lib.vbn_hip_module_unload.argtypes = [ctypes.c_void_p]
        lib.vbn_hip_module_unload.restype = ctypes.c_int
        lib.vbn_hip_module_chain_waves.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.vbn_hip_module_chain_waves.restype = ctypes.c_int
        lib.vbn_hip_struct_size.argtypes = [ctypes.c_int]
        lib.vbn_hip_struct_size.restype = ctypes.c_int
        if lib.vbn_hip_struct_size(0) != ctypes.sizeof(VbnWalkArgs) or lib.vbn_hip_struct_size(1) != 128:
            raise VbnHipError(f"{p}: struct layout differs from the ctypes mirror")
        v = lib.vbn_hip_abi_version()
        if v != ABI_VERSION:
            raise VbnHipError(f"{p}: ABI version {v}, expected {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().vbn_hip_last_error().decode(errors="replace")
        raise VbnHipError(f"{what} failed ({rc}): {msg}")
