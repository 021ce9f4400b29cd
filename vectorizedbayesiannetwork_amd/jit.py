"""Plan-specialised walks: the walk kernel compiled at run time for one step table.

The step-table interpreter (csrc ``vbn_walk_kernel``) reads every step's fields, parent slots
and LDS staging schedule from memory and branches on role / kind / flags per step.  For a
query signature whose plan is reused (the plan cache of :mod:`.engines`), this module writes
the step table as compile-time constants in front of ``csrc/vbn_walk_plan.h``, compiles that
translation unit for gfx950 with hiprtc, loads the code object (``vbn_hip_module_load``) and
launches it with the same arguments, grid and LDS as the interpreter
(``vbn_hip_walk_module``): same device functions, same operation order, bit-identical
outputs, no per-step loads or dispatch (cfg2 walk 1.01 -> 0.88 ms, cfg3 3.83 -> 3.05 ms).

Compiled code objects are cached per process and on disk (``$VBN_HIP_CACHE``, default the
package's ``plan_cache/``, which ``scripts/precompile_plans.py`` fills on the build host for the
benchmark workloads), keyed by the source, the options, the hiprtc version and the headers.  Only lean
full-wave walks are specialised (production MCM / IS / LW / ancestral); by default only
launches of at least ``JIT_MIN_PARTICLES`` particles (a compile takes seconds) --
``VBN_PLAN_JIT=0`` disables it, the engines' ``plan_jit=True`` forces it.  Without hiprtc, or
when a compile fails, the interpreter runs (a warning is printed once).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import sys
import threading
import time
from typing import Dict, Optional, Tuple

import numpy as np

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
JIT_MIN_PARTICLES = 1 << 20
KERNEL = "vbn_walk_plan"
OPTIONS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast-honor-pragmas",
           "-fno-slp-vectorize", "-fno-vectorize")

_lock = threading.Lock()
_modules: Dict[Tuple[int, str], int] = {}        # (device, key) -> module handle
_failed: Dict[str, str] = {}
_rtc = None
_warned = False
STATS = {"compiled": 0, "compile_s": 0.0, "disk_hits": 0, "loaded": 0}


def enabled() -> bool:
    return os.environ.get("VBN_PLAN_JIT", "1") != "0"


def plan_source(steps: np.ndarray, in_cols: np.ndarray, kind_set: int, levels=None) -> str:
    """The translation unit of one plan-specialised walk (csrc/vbn_walk_plan.h).  ``levels``
    (plan.gibbs_levels: per level, per wave, step ranges) makes it a Gibbs sweep on chain
    workgroups of ``len(levels[0])`` waves."""
    rows = []
    for r in np.asarray(steps, np.int32).reshape(-1, 32):
        v = [int(x) for x in r]
        rows.append("  {" + ", ".join(map(str, v[:24])) + ", {" + ", ".join(map(str, v[24:])) + "}},")
    ic = [int(x) for x in np.asarray(in_cols, np.int32).reshape(-1)] or [0]
    chain, sweep = [], []
    if levels:
        chain = [f"#define VBN_PLAN_CHAIN_WAVES {len(levels[0])}"]
        sweep = ["template <unsigned KM>",
                 "__device__ __forceinline__ void vbn_plan_sweep_levels(const vbn_walk_args& A, "
                 "const float* __restrict__ params, int wave, Lane& L, float& lp) {"]
        for lv, waves in enumerate(levels):
            sweep.append(f"  // level {lv}")
            first = True
            for w, ranges in enumerate(waves):
                idx = [i for b, e in ranges for i in range(b, e)]
                if not idx:
                    continue
                seq = ", ".join(map(str, idx))
                sweep.append(f"  {'if' if first else 'else if'} (wave == {w}) "
                             f"vbn_plan_run<KM>(A, params, L, lp, vbn_seq<int, {seq}>{{}});")
                first = False
            sweep.append("  __syncthreads();")
        sweep.append("}")
    return "\n".join([
        "// plan-specialised walk (vectorizedbayesiannetwork_amd/jit.py)",
        '#include "vbn_walk_impl.h"',
        f"#define VBN_PLAN_N_STEPS {len(rows)}",
        *chain,
        "constexpr vbn_step VBN_PLAN_STEPS[VBN_PLAN_N_STEPS] = {",
        *rows,
        "};",
        f"__constant__ int32_t VBN_PLAN_IC[{len(ic)}] = {{{', '.join(map(str, ic))}}};",
        '#include "vbn_walk_plan.h"',
        *sweep,
        f'extern "C" __global__ void __launch_bounds__(WG_MAX_WAVES * WAVE) '
        f"__attribute__((amdgpu_waves_per_eu(VBN_WPE))) {KERNEL}(const vbn_walk_args A, "
        f"const float* __restrict__ params) {{ vbn_walk_plan_body<{int(kind_set)}u>(A, params); }}",
        "",
    ])


def _hiprtc():
    global _rtc
    if _rtc is None:
        for name in ("/opt/rocm/lib/libhiprtc.so", "libhiprtc.so"):
            try:
                _rtc = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _rtc is None:
            raise OSError("libhiprtc not found")
    return _rtc


def compile_source(src: str) -> bytes:
    """hiprtc: source -> gfx950 code object (raises RuntimeError with the compiler log)."""
    rtc = _hiprtc()
    prog = ctypes.c_void_p()
    rc = rtc.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"vbn_walk_plan.hip", 0, None, None)
    if rc != 0:
        raise RuntimeError(f"hiprtcCreateProgram failed ({rc})")
    try:
        opts = [o.encode() for o in OPTIONS] + [f"-I{CSRC}".encode(), f"-I{INCLUDE}".encode()]
        arr = (ctypes.c_char_p * len(opts))(*opts)
        rc = rtc.hiprtcCompileProgram(prog, len(opts), arr)
        n = ctypes.c_size_t()
        if rc != 0:
            rtc.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
            log = ctypes.create_string_buffer(max(n.value, 1))
            rtc.hiprtcGetProgramLog(prog, log)
            raise RuntimeError(f"hiprtc compile failed ({rc}):\n{log.value.decode(errors='replace')[-4000:]}")
        rtc.hiprtcGetCodeSize(prog, ctypes.byref(n))
        code = ctypes.create_string_buffer(n.value)
        rtc.hiprtcGetCode(prog, code)
        return code.raw
    finally:
        rtc.hiprtcDestroyProgram(ctypes.byref(prog))


def _cache_dir() -> Optional[str]:
    # default: in the package tree, so code objects precompiled on the build host
    # (scripts/precompile_plans.py, __graft_entry__.build) travel with the built library
    d = os.environ.get("VBN_HIP_CACHE") or os.path.join(HERE, "plan_cache")
    try:
        os.makedirs(d, exist_ok=True)
        return d if os.access(d, os.W_OK) else None
    except OSError:
        return None


def _version_tag() -> str:
    try:
        rtc = _hiprtc()
        a, b = ctypes.c_int(), ctypes.c_int()
        rtc.hiprtcVersion(ctypes.byref(a), ctypes.byref(b))
        return f"hiprtc{a.value}.{b.value}"
    except OSError:
        return "hiprtc?"


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in (os.path.join(CSRC, "vbn_walk_impl.h"), os.path.join(CSRC, "vbn_walk_plan.h"),
              os.path.join(INCLUDE, "vbn_hip.h"), os.path.join(INCLUDE, "vbn_hip_types.h")):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def code_object(steps: np.ndarray, in_cols: np.ndarray, kind_set: int, levels=None) -> Tuple[str, bytes]:
    """(cache key, code object) of a plan, from the disk cache or compiled."""
    src = plan_source(steps, in_cols, kind_set, levels)
    key = hashlib.sha256("\n".join([src, " ".join(OPTIONS), _version_tag(), _headers_digest()]).encode()
                         ).hexdigest()[:32]
    d = _cache_dir()
    path = os.path.join(d, f"{key}.hsaco") if d else None
    if path and os.path.exists(path):
        with open(path, "rb") as f:
            STATS["disk_hits"] += 1
            return key, f.read()
    t0 = time.perf_counter()
    code = compile_source(src)
    STATS["compiled"] += 1
    STATS["compile_s"] += time.perf_counter() - t0
    if path:
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(code)
        os.replace(tmp, path)
    return key, code


def module_for(steps: np.ndarray, in_cols: np.ndarray, kind_set: int, device_index: int,
               plan_key: str, chain_waves: int = 0) -> Optional[int]:
    """Loaded module handle for (plan, kind set, device), compiling on first use; None if the
    plan cannot be specialised here (the caller runs the interpreter).  ``chain_waves`` > 0:
    a Gibbs sweep table run on chain workgroups of that many waves (plan.gibbs_levels)."""
    global _warned
    mk = (device_index, f"{plan_key}:{kind_set}:{chain_waves}")
    h = _modules.get(mk)
    if h is not None:
        return h
    with _lock:
        h = _modules.get(mk)
        if h is not None:
            return h
        if mk[1] in _failed:
            return None
        try:
            levels = None
            if chain_waves > 0:
                from .plan import gibbs_levels
                levels = gibbs_levels(steps, in_cols, chain_waves)
            _, code = code_object(steps, in_cols, kind_set, levels)
            lib = _lib.load()
            handle = ctypes.c_void_p()
            buf = ctypes.create_string_buffer(code, len(code))
            _lib.check(lib.vbn_hip_module_load(buf, KERNEL.encode(), kind_set, len(steps), ctypes.byref(handle)),
                       "vbn_hip_module_load")
            if chain_waves > 0:
                _lib.check(lib.vbn_hip_module_chain_waves(handle, chain_waves), "vbn_hip_module_chain_waves")
            _modules[mk] = handle.value
            STATS["loaded"] += 1
            return handle.value
        except (OSError, RuntimeError, _lib.VbnHipError) as e:
            _failed[mk[1]] = str(e)
            if not _warned:
                print(f"[vbn_hip] plan-specialised walk unavailable, running the step-table interpreter: {e}",
                      file=sys.stderr)
                _warned = True
            return None


def walk_kind_set(plan, n_queries: int, n_samples: int, precomp: bool = False, wave_particles: int = 0) -> int:
    """The kind-set instantiation a lean launch of ``plan`` runs (host only: the C-ABI's
    vbn_hip_walk_kind_set on a descriptor with placeholder pointers)."""
    lib = _lib.load()
    a = _lib.VbnWalkArgs()
    a.steps = 16                                   # placeholders: the shape logic never dereferences
    a.params = 16
    a.in_cols = 16
    a.n_queries = n_queries
    a.n_samples = n_samples
    a.n_steps = plan.n_steps
    a.n_slots = plan.n_slots
    a.max_out = plan.max_out
    a.mode = plan.mode
    a.kind_mask = plan.kind_mask
    a.wbuf_floats = int(plan.wbuf)
    a.wave_particles = wave_particles
    if precomp:
        a.state = 16
        a.state_flags = 4
    km = lib.vbn_hip_walk_kind_set(ctypes.byref(a))
    if km <= 0:
        _lib.check(-km if km < 0 else 1, "vbn_hip_walk_kind_set")
    return km


def precompile(plan, n_queries: int, n_samples: int, precomp: bool = False) -> Tuple[str, float]:
    """Compile (or find in the disk cache) the specialised walk of a lean launch of ``plan``;
    returns (cache key, seconds spent compiling)."""
    km = walk_kind_set(plan, n_queries, n_samples, precomp)
    steps, ic, _ = plan.steps._vbn_host
    t0 = STATS["compile_s"]
    key, _ = code_object(steps, ic, km)
    return key, STATS["compile_s"] - t0
