"""Plan-specialised walks: the walk kernel compiled at run time for one step table.

The step-table interpreter (csrc ``vbn_walk_kernel``) reads every step's fields, parent slots
and LDS staging schedule from memory and branches on role / kind / flags per step.  For a
query signature whose plan is reused (the plan cache of :mod:`.engines`), this module writes
the step table as compile-time constants in front of ``csrc/vbn_walk_plan.h``, compiles that
translation unit for gfx950 with hiprtc, loads the code object (``vbn_hip_module_load``) and
launches it with the same arguments, grid and LDS as the interpreter
(``vbn_hip_walk_module``): same device functions, same operation order, bit-identical
outputs, no per-step loads or dispatch (cfg2 walk 1.01 -> 0.88 ms, cfg3 3.83 -> 3.05 ms).

Compiled code objects are cached per process and on disk (``$VBN_HIP_CACHE``, the package's
``plan_cache/`` -- which ``scripts/precompile_plans.py`` fills on the build host for the
benchmark workloads -- and a per-user fallback for read-only installs), keyed by the source, the
options, the hiprtc version and the headers.  In the engines' default ("auto") mode a launch
runs the specialised walk whenever its code object is at hand; a launch of at least
``JIT_MIN_PARTICLES`` particles whose plan is not compiled yet starts the compile on a
background thread and runs the interpreter meanwhile (same outputs, bit for bit), so a new
query signature never waits for hiprtc (12-50 s); :func:`wait_pending` joins the compiles and
``VBN.precompile`` compiles a list of signatures ahead of time.  ``VBN_PLAN_JIT=0`` disables
specialisation, the engines' ``plan_jit=True`` forces it (compiling in the call).  Without
hiprtc, or when a compile fails, the interpreter runs (a warning is printed once).
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
_stats_lock = threading.Lock()
_bg_slots = threading.BoundedSemaphore(2)       # background hiprtc compiles at a time
_modules: Dict[Tuple[int, str], int] = {}        # (device, key) -> module handle
_codes: Dict[str, bytes] = {}                    # source key -> code object (this process)
_jobs: Dict[str, "_Job"] = {}                    # source key -> background compile
_failed: Dict[str, str] = {}
_rtc = None
_warned = False
STATS = {"compiled": 0, "compile_s": 0.0, "disk_hits": 0, "loaded": 0, "background": 0}


def enabled() -> bool:
    return os.environ.get("VBN_PLAN_JIT", "1") != "0"


def plan_source(steps: np.ndarray, in_cols: np.ndarray, kind_set: int, schedule=None) -> str:
    """The translation unit of one plan-specialised walk (csrc/vbn_walk_plan.h).  ``schedule``
    (plan.gibbs_schedule: (phases, n_rows), per phase the ops of each wave) makes it a Gibbs
    sweep on chain workgroups of ``len(phases[0])`` waves."""
    rows = []
    for r in np.asarray(steps, np.int32).reshape(-1, 32):
        v = [int(x) for x in r]
        rows.append("  {" + ", ".join(map(str, v[:24])) + ", {" + ", ".join(map(str, v[24:])) + "}},")
    ic = [int(x) for x in np.asarray(in_cols, np.int32).reshape(-1)] or [0]
    chain, sweep = [], []
    if schedule:
        phases, n_rows = schedule
        chain = [f"#define VBN_PLAN_CHAIN_WAVES {len(phases[0])}"]
        # split levels (plan.gibbs_schedule): a LATENT / child step scores into its own LDS row
        # (from 0), the SELECT step adds the rows in sweep order
        sweep = [f"__shared__ float vbn_lp_rows[{max(int(n_rows), 1)} * WAVE];",
                 "template <unsigned KM, int I, int ROW>",
                 "__device__ __forceinline__ void vbn_plan_step_lpout(const vbn_walk_args& A, "
                 "const float* __restrict__ params, Lane& L) {",
                 "  float t = 0.f;",
                 "  vbn_plan_step_direct<KM, I>(A, params, L, t);",
                 "  vbn_lp_rows[ROW * WAVE + L.lane] = t;",
                 "}",
                 "template <unsigned KM, int I, int R0, int... R>",
                 "__device__ __forceinline__ void vbn_plan_step_select(const vbn_walk_args& A, "
                 "const float* __restrict__ params, Lane& L) {",
                 "  float t = vbn_lp_rows[R0 * WAVE + L.lane];",
                 "  ((t += vbn_lp_rows[R * WAVE + L.lane]), ...);",
                 "  vbn_plan_step_direct<KM, I>(A, params, L, t);",
                 "}",
                 "template <unsigned KM>",
                 "__device__ __forceinline__ void vbn_plan_sweep_levels(const vbn_walk_args& A, "
                 "const float* __restrict__ params, int wave, Lane& L, float& lp) {"]

        def call(op):
            if op[0] == "run":
                return f"vbn_plan_step_direct<KM, {op[1]}>(A, params, L, lp);"
            if op[0] == "lpout":
                return f"vbn_plan_step_lpout<KM, {op[1]}, {op[2]}>(A, params, L);"
            return f"vbn_plan_step_select<KM, {op[1]}, {', '.join(map(str, op[2]))}>(A, params, L);"

        for k, waves in enumerate(phases):
            sweep.append(f"  // phase {k}")
            first = True
            for w, ops in enumerate(waves):
                if not ops:
                    continue
                body = " ".join(call(op) for op in ops)
                sweep.append(f"  {'if' if first else 'else if'} (wave == {w}) {{ {body} }}")
                first = False
            sweep.append("  __syncthreads();")
        sweep.append("}")
    # lean production walks whose wide mdn / softmax_nn heads need more than 128 VGPRs (cfg3:
    # 41 spills, ~0.8 GB of scratch traffic per launch at 4 waves per SIMD) run at 3 waves per
    # SIMD without spills -- measured equal time (1.792 vs 1.794 ms, profiles/r05_bench/
    # r05f_ab_cfg3.txt); KDE kind sets keep 4 waves (their exp stream needs the occupancy)
    wpe = (["#define VBN_WPE 3"] if (kind_set & 128) and (kind_set & 20) and not (kind_set & 8) and not schedule
           else [])
    # chain workgroups may run up to 8 waves (vbn_hip_module_chain_waves)
    bounds = max(len(schedule[0][0]), 4) if schedule else "WG_MAX_WAVES"
    return "\n".join([
        "// plan-specialised walk (vectorizedbayesiannetwork_amd/jit.py)",
        *wpe,
        '#include "vbn_walk_impl.h"',
        f"#define VBN_PLAN_N_STEPS {len(rows)}",
        *chain,
        "constexpr vbn_step VBN_PLAN_STEPS[VBN_PLAN_N_STEPS] = {",
        *rows,
        "};",
        f"__constant__ int32_t VBN_PLAN_IC[{len(ic)}] = {{{', '.join(map(str, ic))}}};",
        '#include "vbn_walk_plan.h"',
        *sweep,
        f'extern "C" __global__ void __launch_bounds__({bounds} * WAVE) '
        f"__attribute__((amdgpu_waves_per_eu(VBN_WPE))) {KERNEL}(const vbn_walk_args A, "
        f"const float* __restrict__ params) {{ if (A.run_if && *A.run_if == 0) return; "
        f"vbn_walk_plan_body<{int(kind_set)}u>(A, params); }}",
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


PACKAGE_CACHE = os.path.join(HERE, "plan_cache")


def _read_dirs():
    """Directories searched for a compiled plan: $VBN_HIP_CACHE, then the package's plan_cache
    (code objects precompiled on the build host by scripts/precompile_plans.py travel with the
    built library), then the per-user fallback -- whether or not they are writable."""
    out = []
    for d in (os.environ.get("VBN_HIP_CACHE"), PACKAGE_CACHE, _user_cache()):
        if d and d not in out:
            out.append(d)
    return out


def _user_cache() -> str:
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    return os.path.join(base, "vbn_hip_plans")


def _cache_dir() -> Optional[str]:
    """First writable directory for new code objects: $VBN_HIP_CACHE or the package's
    plan_cache, else the per-user fallback (read-only installs), else None (not persisted)."""
    for d in (os.environ.get("VBN_HIP_CACHE") or PACKAGE_CACHE, _user_cache()):
        try:
            os.makedirs(d, exist_ok=True)
            if os.access(d, os.W_OK):
                return d
        except OSError:
            continue
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


def _source_key(src: str) -> str:
    return hashlib.sha256("\n".join([src, " ".join(OPTIONS), _version_tag(), _headers_digest()]).encode()
                          ).hexdigest()[:32]


def _cached_code(key: str) -> Optional[bytes]:
    code = _codes.get(key)
    if code is not None:
        return code
    for d in _read_dirs():
        p = os.path.join(d, f"{key}.hsaco")
        if os.path.exists(p):
            with open(p, "rb") as f:
                STATS["disk_hits"] += 1
                code = f.read()
            _codes[key] = code
            return code
    return None


def _compile_store(src: str, key: str) -> bytes:
    """hiprtc compile + disk cache write (any thread: hiprtc runs without the GIL)."""
    t0 = time.perf_counter()
    code = compile_source(src)
    dt = time.perf_counter() - t0
    with _stats_lock:
        STATS["compiled"] += 1
        STATS["compile_s"] += dt
    d = _cache_dir()
    if d:
        path = os.path.join(d, f"{key}.hsaco")
        tmp = f"{path}.{os.getpid()}.{threading.get_ident()}.tmp"
        with open(tmp, "wb") as f:
            f.write(code)
        os.replace(tmp, path)
    _codes[key] = code
    return code


def code_object(steps: np.ndarray, in_cols: np.ndarray, kind_set: int, schedule=None) -> Tuple[str, bytes]:
    """(cache key, code object) of a plan, from the memory / disk cache or compiled."""
    src = plan_source(steps, in_cols, kind_set, schedule)
    key = _source_key(src)
    code = _cached_code(key)
    if code is None:
        job = _jobs.get(key)
        code = job.result() if job is not None else _compile_store(src, key)
    return key, code


class _Job:
    """One background hiprtc compile on a daemon thread (process exit does not wait for it)."""

    def __init__(self, src: str, key: str):
        self.done = threading.Event()
        self.code: Optional[bytes] = None
        self.error: Optional[BaseException] = None
        threading.Thread(target=self._run, args=(src, key), daemon=True, name=f"vbn-hiprtc-{key[:8]}").start()

    def _run(self, src, key):
        try:
            with _bg_slots:
                self.code = _compile_store(src, key)
        except BaseException as e:          # noqa: BLE001 -- reported to the launching thread
            self.error = e
        finally:
            self.done.set()

    def result(self) -> bytes:
        self.done.wait()
        if self.error is not None:
            raise RuntimeError(f"background plan compile failed: {self.error}") from self.error
        return self.code


def pending() -> int:
    """Background compiles not finished yet."""
    return sum(1 for j in _jobs.values() if not j.done.is_set())


def wait_pending(timeout: Optional[float] = None) -> bool:
    """Wait for every background compile; True if none is left running."""
    t_end = None if timeout is None else time.monotonic() + timeout
    for j in list(_jobs.values()):
        left = None if t_end is None else max(0.0, t_end - time.monotonic())
        if not j.done.wait(left):
            return False
    return True


def _split_env(chain_waves: int) -> str:
    return os.environ.get("VBN_GIBBS_SPLIT", "") if chain_waves > 0 else ""


def _split_arg(split_env: str):
    # VBN_GIBBS_SPLIT=0/1/levels/dag: whole / split / per-level choice / the step-level schedule
    # (ablation); unset: the cost model
    return {"0": False, "1": True, "dag": "dag", "levels": "levels"}.get(split_env)


LDS_BYTES = 160 * 1024         # per CU (one chain workgroup must fit)
_chain_lds: dict = {}


def chain_lds_bytes(steps: np.ndarray, in_cols: np.ndarray, plan_key: str, chain_waves: int, n_slots: int,
                    max_out: int) -> int:
    """LDS of one chain workgroup of ``chain_waves`` waves running this sweep table: the dynamic
    slots + per-wave scratch rows (vbn_hip_walk_module) plus the unit's static score rows
    (``vbn_lp_rows``, plan_source: n_rows of the schedule)."""
    split_env = _split_env(chain_waves)
    k = (plan_key, chain_waves, n_slots, max_out, split_env)
    got = _chain_lds.get(k)
    if got is None:
        from .plan import gibbs_schedule
        _, n_rows = gibbs_schedule(steps, in_cols, chain_waves, split=_split_arg(split_env))
        rows = max_out if max_out > 0 else 1
        got = (n_slots + chain_waves * rows) * 256 + max(int(n_rows), 1) * 256
        _chain_lds[k] = got
    return got


def module_for(steps: np.ndarray, in_cols: np.ndarray, kind_set: int, device_index: int,
               plan_key: str, chain_waves: int = 0, compile: str = "sync") -> Optional[int]:
    """Loaded module handle for (plan, kind set, device); None if the plan cannot be specialised
    here or is not ready (the caller runs the interpreter).  A code object in the memory or disk
    cache is loaded right away; otherwise ``compile`` says what happens: "sync" compiles in this
    call, "background" starts a hiprtc compile on a daemon thread (the module is used by the first
    launch after it finishes; jit.wait_pending() joins), "never" only uses cached code.
    ``chain_waves`` > 0: a Gibbs sweep table run on chain workgroups of that many waves
    (plan.gibbs_schedule)."""
    global _warned
    split_env = _split_env(chain_waves)
    mk = (device_index, f"{plan_key}:{kind_set}:{chain_waves}:{split_env}")
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
            schedule = None
            if chain_waves > 0:
                from .plan import gibbs_schedule
                schedule = gibbs_schedule(steps, in_cols, chain_waves, split=_split_arg(split_env))
            src = plan_source(steps, in_cols, kind_set, schedule)
            key = _source_key(src)
            code = _cached_code(key)
            if code is None:
                job = _jobs.get(key)
                if compile == "sync":
                    code = job.result() if job is not None else _compile_store(src, key)
                elif compile == "background" and job is None:
                    _jobs[key] = _Job(src, key)
                    STATS["background"] += 1
                    return None
                elif job is not None and job.done.is_set():
                    code = job.result()
                else:
                    return None
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
