"""PyTorch-ROCm custom ops over the C-ABI (``torch.ops.vbn_hip.*``).

* ``vbn_hip::walk``               -> ``vbn_hip_walk``             (particle pass)
* ``vbn_hip::walk_segment``       -> ``vbn_hip_walk``             (one segment of a split pass)
* ``vbn_hip::normalize_weights``  -> ``vbn_hip_normalize_weights`` (softmax over S + ESS)
* ``vbn_hip::rb_epilogue``        -> ``vbn_hip_rb_epilogue``       (Rao-Blackwellized target)
* ``vbn_hip::resample``           -> ``vbn_hip_resample``          (multinomial particle resampling)
* ``vbn_hip::posterior_stats``    -> ``vbn_hip_posterior_stats``   (weighted mean / std / ESS)

Both run asynchronously on the current HIP stream, allocate fresh contiguous outputs and
have fake (meta) implementations for shape inference.  Host-side checks make sure every
buffer the kernel indexes is large enough before the launch.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from .plan import MODE_GIBBS, MODE_MCM, S_WBLK_LEN, STEP_INTS

__all__ = ["walk", "walk_segment", "normalize_weights", "rb_epilogue", "resample", "posterior_stats"]


def _ptr(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None or t.numel() == 0 else t.data_ptr()


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _check_dev(name: str, t: Tensor, dtype: torch.dtype, device: torch.device) -> None:
    if t.device != device or t.dtype != dtype or not t.is_contiguous():
        raise ValueError(f"vbn_hip::walk: {name} must be a contiguous {dtype} tensor on {device} "
                         f"(got {t.dtype} on {t.device}, contiguous={t.is_contiguous()})")


@torch.library.custom_op("vbn_hip::walk", mutates_args=())
def walk(steps: Tensor, in_cols: Tensor, params: Tensor, fixed: Tensor, noise: Optional[Tensor],
         out_cols: Tensor, n_queries: int, n_samples: int, n_slots: int, max_out: int,
         fixed_ld: int, fixed_per_particle: bool, noise_b: int, n_noise: int, dmax: int,
         n_out_cols: int, mode: int, q_base: int, seed: int, offset: int,
         want_lp: bool, kind_mask: int = 63, wbuf: int = 0, plan_jit: int = 1,
         precomp: Optional[Tensor] = None, precomp_q: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """One particle walk over the whole step table (``wbuf``: floats per LDS weight buffer,
    >= every step's weight-block length).  ``plan_jit``: 0 = step-table interpreter, 1 = the
    plan-specialised walk (jit.py) for lean launches of >= jit.JIT_MIN_PARTICLES particles,
    2 = for every lean launch.  ``precomp`` / ``precomp_q``: the per-sample / per-query
    quantities of the table's VBN_F_PRECOMP steps ([S, stride] / [B, stride_q], the pre-pass
    walks' out_x; plan.precompute_plans)."""
    return walk_ex(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots, max_out,
                   fixed_ld, fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode, q_base, seed, offset,
                   want_lp, kind_mask, wbuf, plan_jit, precomp, precomp_q)


def walk_ex(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots, max_out, fixed_ld,
            fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode, q_base, seed, offset, want_lp,
            kind_mask=63, wbuf=0, plan_jit=1, precomp=None, precomp_q=None, *, run_if=None, out_x=None,
            stats_part=None):
    """:func:`walk` as a plain launch, plus ``run_if`` (device int32 [1]: the launch does
    nothing when it holds 0, vbn_walk_args.run_if), ``out_x`` (write the samples into this
    [B*S, n_out_cols] tensor; a predicated launch that does not run leaves it untouched) and
    ``stats_part`` (float64 [B * S/64, 2 + 4 n_out_cols]: the MCM walk's fused posterior-summary
    partials, vbn_walk_args.stats_part; :func:`posterior_stats_merge` finishes them)."""
    for name, t, rows, attr in (("precomp", precomp, n_samples, "_vbn_precomp_stride"),
                                ("precomp_q", precomp_q, n_queries, "_vbn_precomp_q_stride")):
        need = getattr(steps, attr, None)
        if t is None:
            if need is not None:
                raise ValueError(f"vbn_hip::walk: the step table reads {name} ({need} columns), none given")
            continue
        if noise is not None:
            raise ValueError("vbn_hip::walk: precomputed quantities need a walk without injected draws")
        if n_samples % 64 != 0:
            raise ValueError("vbn_hip::walk: precomputed quantities need a multiple of 64 samples per query")
        if t.dim() != 2 or t.shape[0] != rows:
            raise ValueError(f"vbn_hip::walk: {name} must be [{rows}, stride], got {tuple(t.shape)}")
        if need is not None and t.shape[1] != need:
            raise ValueError(f"vbn_hip::walk: {name} has {t.shape[1]} columns, the step table reads {need}")
        _check_dev(name, t, torch.float32, params.device)
    return _walk_launch(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots,
                        max_out, fixed_ld, fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode,
                        q_base, seed, offset, want_lp, kind_mask, precomp, 4 if precomp is not None else 0,
                        0, -1, wbuf, plan_jit, precomp_q, run_if=run_if, out_x=out_x, stats_part=stats_part)


@torch.library.custom_op("vbn_hip::walk_segment", mutates_args=("state",))
def walk_segment(steps: Tensor, in_cols: Tensor, params: Tensor, fixed: Tensor, noise: Optional[Tensor],
                 out_cols: Tensor, n_queries: int, n_samples: int, n_slots: int, max_out: int,
                 fixed_ld: int, fixed_per_particle: bool, noise_b: int, n_noise: int, dmax: int,
                 n_out_cols: int, mode: int, q_base: int, seed: int, offset: int,
                 want_lp: bool, kind_mask: int, state: Tensor, state_flags: int, step_begin: int,
                 step_end: int, wbuf: int = 0) -> Tuple[Tensor, Tensor]:
    """One segment steps[step_begin:step_end] of a split walk; ``state`` [n_slots + 1, B*S]
    carries node values and log-weights between segments (state_flags 1 = load, 2 = store)."""
    return _walk_launch(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots,
                        max_out, fixed_ld, fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode,
                        q_base, seed, offset, want_lp, kind_mask, state, state_flags, step_begin, step_end,
                        wbuf)


@walk_segment.register_fake
def _walk_segment_fake(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots, max_out,
                       fixed_ld, fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode, q_base, seed,
                       offset, want_lp, kind_mask, state, state_flags, step_begin, step_end, wbuf=0):
    total = n_queries * n_samples
    return params.new_empty(total if want_lp else 0), params.new_empty((total, n_out_cols) if n_out_cols > 0 else (0,))


def _check_wbuf(op: str, steps: Tensor, begin: int, end: int, wbuf: int) -> None:
    """``wbuf`` (floats per LDS weight buffer) must hold every staged weight block of the
    steps walked.  Step tables from the plan packer carry their maximum (``_vbn_wblk_max``);
    any other table costs one device read here."""
    need = getattr(steps, "_vbn_wblk_max", None)
    if need is None:
        need = int(steps[begin:end, S_WBLK_LEN].max().item()) if end > begin else 0
    if wbuf < need:
        raise ValueError(f"vbn_hip::{op}: wbuf={wbuf} floats is smaller than the largest weight block "
                         f"of the step table ({need} floats)")


def _walk_launch(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots, max_out,
                 fixed_ld, fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode, q_base, seed,
                 offset, want_lp, kind_mask, state, state_flags, step_begin, step_end, wbuf, plan_jit=0,
                 precomp_q=None, run_if=None, out_x=None, stats_part=None):
    device = params.device
    if device.type != "cuda":
        raise RuntimeError("vbn_hip::walk runs on the GPU only (no CPU fallback); "
                           f"params are on {device}")
    _check_dev("steps", steps, torch.int32, device)
    _check_dev("in_cols", in_cols, torch.int32, device)
    _check_dev("out_cols", out_cols, torch.int32, device)
    _check_dev("params", params, torch.float32, device)
    _check_dev("fixed", fixed, torch.float32, device)
    if steps.dim() != 2 or steps.shape[1] != STEP_INTS:
        raise ValueError("vbn_hip::walk: steps must be [n_steps, 32]")
    step_end = steps.shape[0] if step_end < 0 else step_end
    if not 0 <= step_begin <= step_end <= steps.shape[0]:
        raise ValueError(f"vbn_hip::walk: bad step range [{step_begin}, {step_end})")
    _check_wbuf("walk", steps, step_begin, step_end, wbuf)
    total = n_queries * n_samples
    if state_flags:
        if state is None:
            raise ValueError("vbn_hip::walk: state_flags without a state buffer")
        _check_dev("state", state, torch.float32, device)
        if state_flags & 3 and state.numel() < (n_slots + 1) * total:
            raise ValueError(f"vbn_hip::walk: state has {state.numel()} values, needs {(n_slots + 1) * total}")
    rows = total if fixed_per_particle else n_queries
    if fixed.numel() < rows * fixed_ld:
        raise ValueError(f"vbn_hip::walk: fixed buffer has {fixed.numel()} values, needs {rows}x{fixed_ld}")
    if noise is not None:
        _check_dev("noise", noise, torch.float32, device)
        need = n_noise * 2 * noise_b * n_samples * dmax
        if noise.numel() < need or noise_b not in (1, n_queries):
            raise ValueError(f"vbn_hip::walk: noise has {noise.numel()} values, needs {need}")
    lp = torch.empty(total if want_lp else 0, device=device, dtype=torch.float32)
    if out_x is None:
        x = torch.empty((total, n_out_cols) if n_out_cols > 0 else (0,), device=device, dtype=torch.float32)
    else:
        _check_dev("out_x", out_x, torch.float32, device)
        if n_out_cols <= 0 or out_x.numel() != total * n_out_cols or not out_x.is_contiguous():
            raise ValueError(f"vbn_hip::walk: out_x must be a contiguous [{total}, {n_out_cols}] float32 tensor")
        x = out_x
    if run_if is not None:
        _check_dev("run_if", run_if, torch.int32, device)
    if stats_part is not None:
        _check_dev("stats_part", stats_part, torch.float64, device)
        rows, stride = stats_part_rows(n_queries, n_samples, n_out_cols)
        if mode != MODE_MCM or n_samples % 64 or not 1 <= n_out_cols <= 15 or stats_part.numel() != rows * stride:
            raise ValueError("vbn_hip::walk: stats_part needs an MCM walk with n_samples % 64 == 0, 1..15 output "
                             f"columns and [{rows}, {stride}] float64 partials")
    a = _lib.VbnWalkArgs()
    a.steps = steps.data_ptr() + step_begin * STEP_INTS * 4 if step_end > step_begin else None
    a.in_cols = _ptr(in_cols)
    a.params = _ptr(params)
    a.fixed = _ptr(fixed)
    a.noise = _ptr(noise)
    a.out_cols = _ptr(out_cols)
    a.out_lp = _ptr(lp)
    a.out_x = _ptr(x)
    a.n_queries = n_queries
    a.n_samples = n_samples
    a.n_steps = step_end - step_begin
    a.state = _ptr(state) if state_flags else None
    a.state_flags = int(state_flags)
    a.precomp_q = _ptr(precomp_q)
    a.run_if = _ptr(run_if)
    a.stats_part = _ptr(stats_part)
    a.n_slots = n_slots
    a.max_out = max_out
    a.fixed_ld = fixed_ld
    a.fixed_per_particle = int(fixed_per_particle)
    a.noise_b = noise_b
    a.dmax = dmax
    a.n_out_cols = n_out_cols
    a.mode = mode
    a.kind_mask = kind_mask
    a.q_base = q_base
    a.seed = seed & ((1 << 64) - 1)
    a.offset = offset & ((1 << 64) - 1)
    a.wbuf_floats = int(wbuf)
    lib = _lib.load()
    with torch.cuda.device(device):
        stream = ctypes.c_void_p(_stream_handle(device))
        module = _plan_module(lib, a, steps, step_begin, step_end, total, plan_jit, device)
        if module is not None:
            _lib.check(lib.vbn_hip_walk_module(ctypes.c_void_p(module), ctypes.byref(a), stream), "vbn_hip_walk_module")
        else:
            _lib.check(lib.vbn_hip_walk(ctypes.byref(a), stream), "vbn_hip_walk")
    LAST_WALK["specialised"] = module is not None
    return lp, x


# how the last walk ran (bench.py / tests): {"specialised": bool}
LAST_WALK = {"specialised": False}


def _plan_module(lib, a, steps, step_begin, step_end, work, plan_jit, device, chain_waves=0):
    """Module handle of the plan-specialised walk for this launch, or None (interpreter).
    ``work`` = particles x sweeps; ``plan_jit`` 1 (auto: launches without injected draws whose
    plan is compiled; one of at least jit.JIT_MIN_PARTICLES particle-steps starts a missing
    compile in the background) or 2 (always, compiling in the call); ``chain_waves`` > 0: a Gibbs
    sweep on chain workgroups of that many waves (:func:`gibbs_walk`)."""
    if not plan_jit or step_begin != 0 or step_end != steps.shape[0]:
        return None
    from . import jit
    if not jit.enabled() or (plan_jit == 1 and a.noise):
        return None
    host = getattr(steps, "_vbn_host", None)
    if host is None:
        return None
    km = lib.vbn_hip_walk_kind_set(ctypes.byref(a))
    if km <= 0:
        return None
    if a.mode == MODE_GIBBS and not a.noise:
        km |= 256           # the draw-free unit at full wave too (vbn_hip_walk_module)
    # auto: a compiled plan serves every launch size (bit-identical outputs, so the choice never
    # depends on how a batch is sharded); large launches start a missing compile in the background
    compile = "sync" if plan_jit == 2 else ("background" if work >= jit.JIT_MIN_PARTICLES else "never")
    return jit.module_for(host[0], host[1], km, device.index if device.index is not None else 0, host[2],
                          chain_waves, compile=compile)


@walk.register_fake
def _walk_fake(steps, in_cols, params, fixed, noise, out_cols, n_queries, n_samples, n_slots, max_out,
               fixed_ld, fixed_per_particle, noise_b, n_noise, dmax, n_out_cols, mode, q_base, seed,
               offset, want_lp, kind_mask=63, wbuf=0, plan_jit=1, precomp=None, precomp_q=None):
    total = n_queries * n_samples
    lp = params.new_empty(total if want_lp else 0)
    x = params.new_empty((total, n_out_cols) if n_out_cols > 0 else (0,))
    return lp, x


@torch.library.custom_op("vbn_hip::gibbs_walk", mutates_args=())
def gibbs_walk(steps: Tensor, in_cols: Tensor, params: Tensor, fixed: Tensor, noise: Optional[Tensor],
               state: Tensor, n_queries: int, n_slots: int, max_out: int, fixed_ld: int, noise_b: int,
               n_noise: int, dmax: int, out_dim: int, iters: int, burn_in: int, thin: int, q_base: int,
               seed: int, offset: int, kind_mask: int, wbuf: int = 0, wave_particles: int = 0,
               plan_jit: int = 1, chain_waves: int = -1) -> Tensor:
    """``iters`` Gibbs sweeps (gibbs.py:34-87) over B chains x 8 candidate lanes, started from
    ``state`` [n_slots + 1, B*8]; returns the collected target values [B, n_collect, out_dim].
    ``wave_particles`` 32: half-wave launch (4 chains per wave64, include/vbn_hip.h); 0 = auto
    (full waves on chain workgroups; half waves for fewer than HALF_WAVE_BELOW candidate lanes
    otherwise).
    ``plan_jit`` as for :func:`walk` (0 interpreter, 1 auto, 2 always specialised).
    ``chain_waves`` (specialised sweeps only): 1..8 = chain workgroups of that many waves that
    split each sweep's node updates by level (plan.gibbs_schedule; bit-identical chains), 0 = one
    wave per chain group, -1 = auto (chain workgroups of auto_chain_waves(groups) waves)."""
    if wave_particles not in (0, 32, 64):
        raise ValueError(f"vbn_hip::gibbs_walk: wave_particles must be 0 (auto), 32 or 64, got {wave_particles}")
    if not -1 <= chain_waves <= 8:
        raise ValueError(f"vbn_hip::gibbs_walk: chain_waves must be -1 (auto) or 0..8, got {chain_waves}")
    device = params.device
    if device.type != "cuda":
        raise RuntimeError("vbn_hip::gibbs_walk runs on the GPU only (no CPU fallback); "
                           f"params are on {device}")
    for name, t, dt in (("steps", steps, torch.int32), ("in_cols", in_cols, torch.int32),
                        ("params", params, torch.float32), ("fixed", fixed, torch.float32),
                        ("state", state, torch.float32)):
        _check_dev(name, t, dt, device)
    if steps.dim() != 2 or steps.shape[1] != STEP_INTS:
        raise ValueError("vbn_hip::gibbs_walk: steps must be [n_steps, 32]")
    _check_wbuf("gibbs_walk", steps, 0, steps.shape[0], wbuf)
    if iters <= 0 or not 0 <= burn_in < iters or thin <= 0 or out_dim <= 0:
        raise ValueError("vbn_hip::gibbs_walk: need iters > burn_in >= 0, thin > 0, out_dim > 0")
    total = n_queries * 8
    if state.numel() < (n_slots + 1) * total:
        raise ValueError(f"vbn_hip::gibbs_walk: state has {state.numel()} values, needs {(n_slots + 1) * total}")
    if fixed.numel() < n_queries * fixed_ld:
        raise ValueError(f"vbn_hip::gibbs_walk: fixed buffer needs {n_queries}x{fixed_ld} values")
    if noise is not None:
        _check_dev("noise", noise, torch.float32, device)
        need = iters * n_noise * 2 * noise_b * 8 * dmax
        if noise.numel() < need or noise_b not in (1, n_queries):
            raise ValueError(f"vbn_hip::gibbs_walk: noise has {noise.numel()} values, needs {need}")
    n_collect = (iters - burn_in + thin - 1) // thin
    x = torch.empty((n_queries, n_collect, out_dim), device=device, dtype=torch.float32)
    a = _lib.VbnWalkArgs()
    a.steps = steps.data_ptr()
    a.in_cols = _ptr(in_cols)
    a.params = _ptr(params)
    a.fixed = _ptr(fixed)
    a.noise = _ptr(noise)
    a.out_cols = _ptr(in_cols)            # unused by the Gibbs walk (COLLECT reads the target slots)
    a.out_lp = None
    a.out_x = _ptr(x)
    a.n_queries = n_queries
    a.n_samples = 8
    a.n_steps = int(steps.shape[0])
    a.state = _ptr(state)
    a.state_flags = 1
    a.n_slots = n_slots
    a.max_out = max_out
    a.fixed_ld = fixed_ld
    a.fixed_per_particle = 0
    a.noise_b = noise_b
    a.dmax = dmax
    a.n_out_cols = out_dim
    a.mode = MODE_GIBBS
    a.kind_mask = kind_mask
    a.q_base = q_base
    a.seed = seed & ((1 << 64) - 1)
    a.offset = offset & ((1 << 64) - 1)
    a.gibbs_iters = iters
    a.gibbs_burn_in = burn_in
    a.gibbs_thin = thin
    a.n_noise = n_noise
    a.wbuf_floats = int(wbuf)
    auto_wp = wave_particles == 0
    cw = chain_waves
    if cw < 0:        # auto: chain workgroups whose LDS fits (fit_chain_waves), else the one-wave form
        cw = fit_chain_waves(steps, auto_chain_waves(total // (WAVE if auto_wp else wave_particles)),
                             n_slots, max_out)
    if auto_wp:       # full waves wherever a chain workgroup may run (r05k: 4096 chains, 64 x 8 waves
        # 101.6 ms, 32 x 4 117.0 ms); the one-wave forms keep half waves for small batches
        wave_particles = 64 if cw > 0 or total >= HALF_WAVE_BELOW else 32
    a.wave_particles = int(wave_particles)
    lib = _lib.load()
    with torch.cuda.device(device):
        stream = ctypes.c_void_p(_stream_handle(device))
        module = _plan_module(lib, a, steps, 0, int(steps.shape[0]), total * iters, plan_jit, device, cw)
        if module is None and auto_wp and total < HALF_WAVE_BELOW:
            a.wave_particles = 32                   # interpreter: half waves below HALF_WAVE_BELOW
        if module is not None:
            _lib.check(lib.vbn_hip_walk_module(ctypes.c_void_p(module), ctypes.byref(a), stream), "vbn_hip_walk_module")
        else:
            _lib.check(lib.vbn_hip_walk(ctypes.byref(a), stream), "vbn_hip_walk")
    LAST_WALK["specialised"] = module is not None
    LAST_WALK["chain_waves"] = cw if module is not None else 0
    LAST_WALK["wave_particles"] = int(a.wave_particles)
    return x


# Specialised Gibbs sweeps run on chain workgroups (plan.gibbs_schedule) at every batch size:
# about CHAIN_TARGET_WAVES waves in all (4 per SIMD), so more chains take fewer waves per chain
# group.  Sweep kernel ms, full wave, YAML defaults (profiles/r05_bench/r05ag_*, r05ah_*, r05w_*):
#   2048 chains: 8 waves 73.0, 4: 97.8      4096: 8 94.7, 4 110.7
#   8192: 4 157.4, 8 188.5, one-wave 318.9   16384: 2 287.6, 4 306.3, one-wave 335.3, 8 371.9
#   32768: 2 562.2, 1 568.8, 4 595.1, one-wave 625.0
CHAIN_TARGET_WAVES = 4096
CHAIN_WAVES = 8               # the most (vbn_hip_module_chain_waves); 4096 chains -- the bench


def auto_chain_waves(groups: int) -> int:
    """Waves per chain workgroup for ``groups`` chain groups (64 -- half wave: 32 -- candidate
    lanes each): the power of two nearest below CHAIN_TARGET_WAVES / groups, within [2, 8]."""
    w = CHAIN_TARGET_WAVES // max(int(groups), 1)
    cw = 2
    while cw * 2 <= min(w, CHAIN_WAVES):
        cw *= 2
    return cw
def fit_chain_waves(steps, cw: int, n_slots: int, max_out: int) -> int:
    """The largest wave count <= ``cw`` (8, 4, 2, 1) whose chain workgroup fits the CU's LDS
    with the sweep unit's static score rows (jit.chain_lds_bytes); 0 (the one-wave form) when
    none does.  Steps without a host copy (no specialised unit) keep ``cw``."""
    host = getattr(steps, "_vbn_host", None)
    if host is None or cw <= 0:
        return cw
    from . import jit
    while cw > 0 and jit.chain_lds_bytes(host[0], host[1], host[2], cw, n_slots, max_out) > jit.LDS_BYTES:
        cw //= 2
    return cw


# below this many candidate lanes (B x 8) the one-wave sweep forms run half-wave (4 chains per
# wave64): 1536 full waves = 1.5 per SIMD
HALF_WAVE_BELOW = 1536 * 64
WAVE = 64


@gibbs_walk.register_fake
def _gibbs_walk_fake(steps, in_cols, params, fixed, noise, state, n_queries, n_slots, max_out, fixed_ld,
                     noise_b, n_noise, dmax, out_dim, iters, burn_in, thin, q_base, seed, offset, kind_mask, wbuf=0,
                     wave_particles=0, plan_jit=1, chain_waves=-1):
    return params.new_empty((n_queries, (iters - burn_in + thin - 1) // thin, out_dim))


@torch.library.custom_op("vbn_hip::normalize_weights", mutates_args=())
def normalize_weights(log_w: Tensor, normalize: bool, eps: float) -> Tuple[Tensor, Tensor]:
    w, ess, _ = normalize_weights_ex(log_w, normalize, eps)
    return w, ess


# The ESS fallback flags: a zeroed device pool per GPU handed out one int32 slot per call, and
# zeroed again (one fill) after FLAG_SLOTS calls -- instead of one zero-fill launch per call
# (~5 us of GPU time each on a busy queue, r06a cfg3 trace).  Stream order keeps a slot's
# readers (the predicated fallback launches) ahead of the refill; a returned flag stays valid
# for the next FLAG_SLOTS - 1 calls on its device.
FLAG_SLOTS = 4096
_FLAG_POOLS: dict = {}
_FLAG_LOCK = threading.Lock()


def _flag_slot(device: torch.device) -> Tensor:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with _FLAG_LOCK:
        ent = _FLAG_POOLS.get(idx)
        if ent is None:
            ent = _FLAG_POOLS[idx] = [torch.zeros(FLAG_SLOTS, device=device, dtype=torch.int32), 0]
        elif ent[1] >= FLAG_SLOTS:
            ent[0].zero_()
            ent[1] = 0
        k = ent[1]
        ent[1] += 1
        return ent[0][k:k + 1]


def normalize_weights_ex(log_w: Tensor, normalize: bool, eps: float, *, ess_thr: Optional[float] = None,
                         run_if: Optional[Tensor] = None, w_out: Optional[Tensor] = None,
                         ess_out: Optional[Tensor] = None, stats: Optional[dict] = None
                         ) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
    """The normalisation kernel (vbn_hip_normalize_weights_ex) as a plain launch: ``ess_thr``
    returns a device int32 [1] flag, 1 when some query's ESS < ess_thr (importance_sampling.py
    :85-86, decided without a host sync); ``run_if`` (device int32 [1]) predicates the launch;
    ``w_out`` / ``ess_out``: write into these instead of fresh tensors (predicated launches
    leave them untouched when *run_if == 0).  ``stats``: {"x": samples [B,S,D], "eps": float,
    and optionally "mean" / "std" / "ess" output tensors}: VBN._posterior_stats of the weights
    written, fused into the same pass (vbn_hip_normalize_weights_stats, S <= 4096); the dict
    gets "mean" [B,D], "std" [B,D], "ess" [B]."""
    if log_w.device.type != "cuda" or log_w.dtype != torch.float32 or log_w.dim() != 2:
        raise ValueError("vbn_hip::normalize_weights: log_w must be a float32 [B,S] GPU tensor")
    log_w = log_w.contiguous()
    b, s = log_w.shape
    w = torch.empty_like(log_w) if w_out is None else w_out
    ess = torch.empty(b, device=log_w.device, dtype=torch.float32) if ess_out is None else ess_out
    for name, t, shape in (("w_out", w_out, (b, s)), ("ess_out", ess_out, (b,))):
        if t is not None and (t.dtype != torch.float32 or tuple(t.shape) != shape or not t.is_contiguous()
                              or t.device != log_w.device):
            raise ValueError(f"vbn_hip::normalize_weights: {name} must be a contiguous float32 {shape} tensor "
                             "on log_w's device")
    if run_if is not None:
        _check_dev("run_if", run_if, torch.int32, log_w.device)
    flag = None
    if ess_thr is not None:
        if not normalize:
            raise ValueError("vbn_hip::normalize_weights: the ESS flag needs normalize=True")
        flag = _flag_slot(log_w.device)
    lib = _lib.load()
    if stats is not None:
        x = stats["x"]
        _check_dev("stats x", x, torch.float32, log_w.device)
        if x.dim() != 3 or tuple(x.shape[:2]) != (b, s) or s > 4096:
            raise ValueError(f"vbn_hip::normalize_weights: stats x must be [{b}, {s}, D] with S <= 4096")
        d = int(x.shape[2])
        for name, shape in (("mean", (b, d)), ("std", (b, d)), ("ess", (b,))):
            t = stats.get(name)
            if t is None:
                stats[name] = torch.empty(shape, device=log_w.device, dtype=torch.float32)
            elif t.dtype != torch.float32 or tuple(t.shape) != shape or not t.is_contiguous():
                raise ValueError(f"vbn_hip::normalize_weights: stats {name} must be a contiguous float32 {shape}")
        with torch.cuda.device(log_w.device):
            _lib.check(lib.vbn_hip_normalize_weights_stats(
                _ptr(log_w), _ptr(w), _ptr(ess) if normalize else None, b, s, int(normalize), float(eps),
                _ptr(run_if), _ptr(flag), float(ess_thr or 0.0), _ptr(x), d, float(stats.get("eps", 1e-12)),
                _ptr(stats["mean"]), _ptr(stats["std"]), _ptr(stats["ess"]),
                ctypes.c_void_p(_stream_handle(log_w.device))), "vbn_hip_normalize_weights_stats")
        return w, ess, flag
    with torch.cuda.device(log_w.device):
        _lib.check(lib.vbn_hip_normalize_weights_ex(
            _ptr(log_w), _ptr(w), _ptr(ess) if normalize else None, b, s, int(normalize), float(eps),
            _ptr(run_if), _ptr(flag), float(ess_thr or 0.0),
            ctypes.c_void_p(_stream_handle(log_w.device))), "vbn_hip_normalize_weights_ex")
    return w, ess, flag


@normalize_weights.register_fake
def _normalize_fake(log_w, normalize, eps):
    return torch.empty_like(log_w), log_w.new_empty(log_w.shape[0])


@torch.library.custom_op("vbn_hip::rb_epilogue", mutates_args=())
def rb_epilogue(log_w: Tensor, params: Tensor, z: Tensor, n_out: int, mode: int, stddevs: float,
                min_scale: float, eps: float) -> Tuple[Tensor, Tensor]:
    """log_w [B,P]; params [B|1, P, 2] (mode 0: loc, scale) or [B|1, P, C] (mode 1: probs);
    z [n_out] grid fractions (mode 0).  Returns (pdf [B, n_out], grid [B, n_out])."""
    if log_w.device.type != "cuda" or log_w.dtype != torch.float32 or log_w.dim() != 2:
        raise ValueError("vbn_hip::rb_epilogue: log_w must be a float32 [B,P] GPU tensor")
    b, p = log_w.shape
    width = 2 if mode == 0 else n_out
    if params.dim() != 3 or params.shape[1] != p or params.shape[2] != width or params.shape[0] not in (1, b):
        raise ValueError(f"vbn_hip::rb_epilogue: params must be [B|1, {p}, {width}], got {tuple(params.shape)}")
    log_w = log_w.contiguous()
    params = params.to(torch.float32).contiguous()
    if mode == 0:
        z = z.to(device=log_w.device, dtype=torch.float32).contiguous()
        if z.numel() != n_out:
            raise ValueError("vbn_hip::rb_epilogue: z must have n_out values")
    pdf = torch.empty(b, n_out, device=log_w.device, dtype=torch.float32)
    grid = torch.empty(b, n_out, device=log_w.device, dtype=torch.float32) if mode == 0 else pdf.new_empty(0)
    lib = _lib.load()
    with torch.cuda.device(log_w.device):
        _lib.check(lib.vbn_hip_rb_epilogue(
            _ptr(log_w), _ptr(params), params.shape[0], _ptr(z) if mode == 0 else None, _ptr(pdf),
            _ptr(grid), b, p, n_out, mode, float(stddevs), float(min_scale), float(eps),
            ctypes.c_void_p(_stream_handle(log_w.device))), "vbn_hip_rb_epilogue")
    return pdf, grid


@rb_epilogue.register_fake
def _rb_fake(log_w, params, z, n_out, mode, stddevs, min_scale, eps):
    b = log_w.shape[0]
    return log_w.new_empty(b, n_out), log_w.new_empty((b, n_out) if mode == 0 else (0,))


@torch.library.custom_op("vbn_hip::resample", mutates_args=("state_out",))
def resample(w: Tensor, u: Optional[Tensor], seed: int, offset: int, q_base: int, state_in: Tensor,
             state_out: Tensor) -> None:
    """w [B,S] normalized weights; state_in/state_out [n_cols, B*S] (last row: log-weights,
    reset to 0); u [B,S] injected uniforms or None (Philox)."""
    if w.device.type != "cuda" or w.dtype != torch.float32 or w.dim() != 2:
        raise ValueError("vbn_hip::resample: w must be a float32 [B,S] GPU tensor")
    b, s = w.shape
    for name, t in (("state_in", state_in), ("state_out", state_out)):
        _check_dev(name, t, torch.float32, w.device)
        if t.dim() != 2 or t.shape[1] != b * s:
            raise ValueError(f"vbn_hip::resample: {name} must be [n_cols, {b * s}]")
    if state_in.shape != state_out.shape or state_in.data_ptr() == state_out.data_ptr():
        raise ValueError("vbn_hip::resample: state_in and state_out must be distinct buffers of one shape")
    w = w.contiguous()
    if u is not None:
        u = u.to(device=w.device, dtype=torch.float32).contiguous()
        if u.numel() != b * s:
            raise ValueError("vbn_hip::resample: u must be [B,S]")
    lib = _lib.load()
    with torch.cuda.device(w.device):
        _lib.check(lib.vbn_hip_resample(
            _ptr(w), _ptr(u), seed & ((1 << 64) - 1), offset & ((1 << 64) - 1), q_base, _ptr(state_in),
            _ptr(state_out), b, s, state_in.shape[0], ctypes.c_void_p(_stream_handle(w.device))),
            "vbn_hip_resample")


@resample.register_fake
def _resample_fake(w, u, seed, offset, q_base, state_in, state_out):
    return None


@torch.library.custom_op("vbn_hip::posterior_stats", mutates_args=())
def posterior_stats(pdf: Tensor, samples: Tensor, eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    """pdf [B,S], samples [B,S,D] -> (mean [B,D], std [B,D], ess [B]) (vbn.py:483-504)."""
    if pdf.device.type != "cuda" or pdf.dim() != 2 or samples.dim() != 3:
        raise ValueError("vbn_hip::posterior_stats: pdf [B,S] and samples [B,S,D] GPU tensors expected")
    b, s = pdf.shape
    d = samples.shape[2]
    pdf = pdf.to(torch.float32).contiguous()
    samples = samples.to(device=pdf.device, dtype=torch.float32).contiguous()
    mean = torch.empty(b, d, device=pdf.device, dtype=torch.float32)
    std = torch.empty_like(mean)
    ess = torch.empty(b, device=pdf.device, dtype=torch.float32)
    lib = _lib.load()
    with torch.cuda.device(pdf.device):
        _lib.check(lib.vbn_hip_posterior_stats(
            _ptr(pdf), _ptr(samples), _ptr(mean), _ptr(std), _ptr(ess), b, s, d, float(eps),
            ctypes.c_void_p(_stream_handle(pdf.device))), "vbn_hip_posterior_stats")
    return mean, std, ess


@posterior_stats.register_fake
def _posterior_stats_fake(pdf, samples, eps):
    b, d = pdf.shape[0], samples.shape[2]
    return pdf.new_empty(b, d), pdf.new_empty(b, d), pdf.new_empty(b)


def stats_part_rows(n_queries: int, n_samples: int, dim: int) -> Tuple[int, int]:
    """(rows, doubles per row) of a walk's fused posterior-summary partials
    (vbn_walk_args.stats_part): one row per 64-particle wave."""
    return n_queries * (n_samples // 64), 2 + 4 * dim


def posterior_stats_merge(part: Tensor, n_queries: int, n_samples: int, dim: int, eps: float
                          ) -> Tuple[Tensor, Tensor, Tensor]:
    """Finish VBN._posterior_stats (vbn.py:483-504) from an MCM walk's epilogue partials
    (vbn_hip_posterior_stats_merge): (mean [B,D], std [B,D], ess [B])."""
    rows, stride = stats_part_rows(n_queries, n_samples, dim)
    _check_dev("stats_part", part, torch.float64, part.device)
    if part.numel() != rows * stride:
        raise ValueError(f"vbn_hip::posterior_stats_merge: part has {part.numel()} values, needs {rows * stride}")
    mean = torch.empty(n_queries, dim, device=part.device, dtype=torch.float32)
    std = torch.empty_like(mean)
    ess = torch.empty(n_queries, device=part.device, dtype=torch.float32)
    lib = _lib.load()
    with torch.cuda.device(part.device):
        _lib.check(lib.vbn_hip_posterior_stats_merge(
            _ptr(part), n_queries, n_samples // 64, dim, float(eps), _ptr(mean), _ptr(std), _ptr(ess),
            ctypes.c_void_p(_stream_handle(part.device))), "vbn_hip_posterior_stats_merge")
    return mean, std, ess


@torch.library.custom_op("vbn_hip::discrete_posterior", mutates_args=())
def discrete_posterior(samples: Tensor, weights: Tensor, k: int) -> Tuple[Tensor, Tensor]:
    """samples [B,S] or [B,S,D] (feature 0), weights [B,S], k bins -> (probs [B,k] float64,
    bad [B] int32) (benchmarking/models/vbn.py:202-242; bad: 1 / 2 where a finite-weight sample
    is NaN / +-inf, which the reference raises on)."""
    if weights.device.type != "cuda" or weights.dim() != 2 or samples.dim() not in (2, 3):
        raise ValueError("vbn_hip::discrete_posterior: samples [B,S(,D)] and weights [B,S] GPU tensors expected")
    if tuple(samples.shape[:2]) != tuple(weights.shape) or k <= 0:
        raise ValueError("vbn_hip::discrete_posterior: samples/weights shape mismatch or k <= 0")
    b, s = weights.shape
    # float32 / float64 elements as given (the reference's float() of each); other dtypes are
    # converted to float32 (the engines' outputs are float32)
    keep = (torch.float32, torch.float64)
    weights = (weights if weights.dtype in keep else weights.to(torch.float32)).contiguous()
    samples = samples.to(device=weights.device)
    samples = (samples if samples.dtype in keep else samples.to(torch.float32)).contiguous()
    stride = samples.shape[2] if samples.dim() == 3 else 1
    probs = torch.empty(b, k, device=weights.device, dtype=torch.float64)
    bad = torch.empty(b, device=weights.device, dtype=torch.int32)
    if b == 0 or s == 0:
        probs.fill_(1.0 / k)
        bad.zero_()
        return probs, bad
    lib = _lib.load()
    with torch.cuda.device(weights.device):
        _lib.check(lib.vbn_hip_discrete_posterior_typed(
            _ptr(samples), int(samples.dtype == torch.float64), stride, _ptr(weights),
            int(weights.dtype == torch.float64), _ptr(probs), _ptr(bad), b, s, int(k),
            ctypes.c_void_p(_stream_handle(weights.device))), "vbn_hip_discrete_posterior_typed")
    return probs, bad


@discrete_posterior.register_fake
def _discrete_posterior_fake(samples, weights, k):
    b = weights.shape[0]
    return weights.new_empty(b, k, dtype=torch.float64), weights.new_empty(b, dtype=torch.int32)


# ------------------------------------------------------------------------------------------
# Query-level ops: a packed plan + evidence in, the engine's outputs out.
#
#   vbn_hip::pack_plan(steps[], in_cols[], out_cols[], meta) -> plan   (int32 host blob)
#   vbn_hip::mcm(plan, params, fixed, n_samples, seed, ...)     -> (pdf [B,S], samples [B,S,Dt])
#   vbn_hip::is_lw(plan, ..., lw_mode, normalize, eps)           -> (weights, samples, ess, fallback)
#   vbn_hip::ancestral(plan, ...)                                -> samples [B,S,n_out]
#
# They replace the engine bodies of the reference (monte_carlo_marginalization.py:18-92,
# importance_sampling.py:24-93 / likelihood_weighting.py:24-82, sampling/ancestral.py:13-65)
# for an out-of-tree caller that holds a plan from VBN.pack_query: no Python engine, one call.
# A plan blob holds up to four walk sections -- 0 the walk, 1 the same walk reading the
# precomputed per-sample / per-query quantities, 2 the per-sample pre-pass, 3 the per-query
# pre-pass (plan.precompute_plans) -- each [header 16 | steps n x 32 | in_cols | out_cols].
# ------------------------------------------------------------------------------------------

PLAN_MAGIC = 0x56424E50          # "VBNP"
PLAN_SECTIONS = 4
_SEC_META = 8                    # n_slots, max_out, fixed_ld, mode, kind_mask, wbuf, dmax, n_noise


@torch.library.custom_op("vbn_hip::pack_plan", mutates_args=())
def pack_plan(steps: list[Tensor], in_cols: list[Tensor], out_cols: list[Tensor], meta: list[int]) -> Tensor:
    """Pack up to 4 walk sections into one int32 host tensor: [4 + 4 offsets] then per section
    [magic, n_steps, n_in_cols, n_out_cols, 8 x meta, precomp stride, precomp_q stride, 0, 0 |
    steps | in_cols | out_cols] (an empty steps tensor = absent section)."""
    if not (len(steps) == len(in_cols) == len(out_cols)) or len(steps) > PLAN_SECTIONS:
        raise ValueError("vbn_hip::pack_plan: steps / in_cols / out_cols lists of equal length <= 4")
    if len(meta) != _SEC_META * len(steps):
        raise ValueError(f"vbn_hip::pack_plan: meta needs {_SEC_META} ints per section")
    from .plan import F_PRECOMP, F_PRECOMP_Q, S_AUX2, S_FLAGS
    parts = [torch.tensor([PLAN_MAGIC, 1, len(steps), 0], dtype=torch.int32), torch.zeros(PLAN_SECTIONS, dtype=torch.int32)]
    pos = 4 + PLAN_SECTIONS
    offs = [0] * PLAN_SECTIONS
    for i, (st, ic, oc) in enumerate(zip(steps, in_cols, out_cols)):
        if st.numel() == 0:
            continue
        st = st.detach().to("cpu", torch.int32).reshape(-1, STEP_INTS)
        ic = ic.detach().to("cpu", torch.int32).reshape(-1)
        oc = oc.detach().to("cpu", torch.int32).reshape(-1)
        fl, aux = st[:, S_FLAGS], st[:, S_AUX2]
        pcs = ((fl & F_PRECOMP) != 0) & ((fl & F_PRECOMP_Q) == 0)
        pcq = (fl & F_PRECOMP_Q) != 0
        stride_s = int(aux[pcs][0]) >> 16 if bool(pcs.any()) else 0
        stride_q = int(aux[pcq][0]) >> 16 if bool(pcq.any()) else 0
        hdr = torch.tensor([PLAN_MAGIC, st.shape[0], ic.numel(), oc.numel(),
                            *meta[_SEC_META * i:_SEC_META * (i + 1)], stride_s, stride_q, 0, 0], dtype=torch.int32)
        offs[i] = pos
        parts += [hdr, st.reshape(-1), ic, oc]
        pos += hdr.numel() + st.numel() + ic.numel() + oc.numel()
    parts[1] = torch.tensor(offs, dtype=torch.int32)
    return torch.cat(parts)


@pack_plan.register_fake
def _pack_plan_fake(steps, in_cols, out_cols, meta):
    n = 4 + PLAN_SECTIONS + sum(16 + s.numel() + i.numel() + o.numel()
                                for s, i, o in zip(steps, in_cols, out_cols) if s.numel())
    return torch.empty(n, dtype=torch.int32)


_PLAN_DEV = {}          # (blob content hash, device) -> unpacked sections on the device


def _unpack(plan: Tensor, device: torch.device):
    """Plan blob -> per section (steps, in_cols, out_cols, header ints) on ``device`` (cached)."""
    import hashlib
    if plan.device.type != "cpu" or plan.dtype != torch.int32 or plan.dim() != 1:
        raise ValueError("vbn_hip: plan must be the int32 host tensor of vbn_hip::pack_plan")
    raw = plan.numpy()
    key = (hashlib.sha1(raw.tobytes()).hexdigest(), str(device))
    got = _PLAN_DEV.get(key)
    if got is not None:
        return got
    if raw.size < 4 + PLAN_SECTIONS or int(raw[0]) != PLAN_MAGIC:
        raise ValueError("vbn_hip: not a packed plan (bad magic)")
    secs = []
    for i in range(PLAN_SECTIONS):
        o = int(raw[4 + i])
        if o == 0:
            secs.append(None)
            continue
        h = [int(x) for x in raw[o:o + 16]]
        if h[0] != PLAN_MAGIC:
            raise ValueError(f"vbn_hip: plan section {i} is corrupt")
        n, nic, noc = h[1], h[2], h[3]
        p = o + 16
        st_np = raw[p:p + n * STEP_INTS].reshape(n, STEP_INTS).copy()
        ic_np = raw[p + n * STEP_INTS:p + n * STEP_INTS + nic].copy()
        oc_np = raw[p + n * STEP_INTS + nic:p + n * STEP_INTS + nic + noc].copy()
        st = torch.from_numpy(st_np).to(device)
        st._vbn_wblk_max = int(st_np[:, S_WBLK_LEN].max()) if n else 0
        st._vbn_host = (st_np, ic_np, hashlib.sha1(st_np.tobytes() + b"|" + ic_np.tobytes()).hexdigest())
        if h[12]:
            st._vbn_precomp_stride = h[12]
        if h[13]:
            st._vbn_precomp_q_stride = h[13]
        ic = torch.from_numpy(ic_np if nic else raw[:1].copy()).to(device)
        oc = torch.from_numpy(oc_np if noc else raw[:1].copy()).to(device)
        secs.append((st, ic, oc, h))
    if len(_PLAN_DEV) > 256:
        _PLAN_DEV.clear()
    _PLAN_DEV[key] = secs
    return secs


def _section_walk(sec, params, fixed, b, n, seed, offset, q_base, noise, plan_jit, precomp=None, precomp_q=None):
    st, ic, oc, h = sec
    n_slots, max_out, fixed_ld, mode, kind_mask, wbuf, dmax, n_noise = h[4:12]
    noise_b = int(noise.shape[2]) if noise is not None else 1
    lp, x = walk(st, ic, params, fixed, noise, oc, b, n, n_slots, max_out, fixed_ld, False, noise_b,
                 n_noise, dmax, h[3], mode, q_base, seed, offset, mode != 2, kind_mask, wbuf, plan_jit,
                 precomp, precomp_q)
    return lp, x


def _query_walk(plan, params, fixed, n_samples, seed, offset, q_base, noise, plan_jit):
    """The walk of a packed plan with its pre-passes (engines.run_walk's precompute rule)."""
    device = params.device
    secs = _unpack(plan, device)
    if secs[0] is None:
        raise ValueError("vbn_hip: plan has no walk section")
    b = int(fixed.shape[0])
    if fixed.dim() != 2 or fixed.shape[1] < secs[0][3][6]:
        raise ValueError(f"vbn_hip: fixed must be [B, {secs[0][3][6]}] (plan fixed-buffer columns)")
    fixed = fixed.to(device=device, dtype=torch.float32).contiguous()
    if noise is not None:
        noise = noise.to(device=device, dtype=torch.float32).contiguous()
    use_pc = secs[1] is not None and noise is None and n_samples % 64 == 0
    if not use_pc:
        return _section_walk(secs[0], params, fixed, b, n_samples, seed, offset, q_base, noise, plan_jit), secs[0]
    precomp = precomp_q = None
    if secs[2] is not None:
        _, x = _section_walk(secs[2], params, fixed, 1, n_samples, seed, offset, 0, None, 0)
        precomp = x.view(n_samples, -1)
    if secs[3] is not None:
        _, x = _section_walk(secs[3], params, fixed, b, 64, seed, offset, q_base, None, 0)
        w = x.shape[-1]
        precomp_q = (x.view(b, 64 * w) if getattr(secs[1][0], "_vbn_precomp_q_stride", None) == 64 * w
                     else x.view(b, 64, w)[:, 0].contiguous())
    return _section_walk(secs[1], params, fixed, b, n_samples, seed, offset, q_base, None, plan_jit,
                         precomp, precomp_q), secs[1]


@torch.library.custom_op("vbn_hip::mcm", mutates_args=())
def mcm(plan: Tensor, params: Tensor, fixed: Tensor, n_samples: int, seed: int, offset: int = 0, q_base: int = 0,
        noise: Optional[Tensor] = None, plan_jit: int = 1) -> Tuple[Tensor, Tensor]:
    """Monte-Carlo marginalization of a packed MCM plan (VBN.pack_query): fixed [B, fixed_ld]
    evidence / do values in the plan's column order -> (pdf [B,S], samples [B,S,Dt])."""
    (lp, x), sec = _query_walk(plan, params, fixed, n_samples, seed, offset, q_base, noise, plan_jit)
    if sec[3][7] != 0:
        raise ValueError("vbn_hip::mcm: the plan is not an MCM walk")
    b = int(fixed.shape[0])
    return lp.view(b, n_samples), x.view(b, n_samples, -1)


@mcm.register_fake
def _mcm_fake(plan, params, fixed, n_samples, seed, offset=0, q_base=0, noise=None, plan_jit=1):
    b = fixed.shape[0]
    return params.new_empty(b, n_samples), params.new_empty(b, n_samples, 1)


@torch.library.custom_op("vbn_hip::is_lw", mutates_args=())
def is_lw(plan: Tensor, params: Tensor, fixed: Tensor, n_samples: int, seed: int, offset: int = 0,
          q_base: int = 0, noise: Optional[Tensor] = None, lw_mode: bool = False, normalize: bool = True,
          eps: float = 0.0, ess_threshold: float = 0.1, plan_jit: int = 1) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Importance sampling (lw_mode False: the plan's roots drawn per query, evidence raw) or
    likelihood weighting (True: shared roots; the packed LW plan clamps the evidence as it reads
    it, VBN_F_CLAMP_EV, so a caller's own clamp is harmless but not needed) of a packed
    weighted plan -> (weights [B,S], samples [B,S,Dt], ess [B], fallback flag (device bool): IS
    -- some ESS below max(1, ess_threshold S), NaN never triggers; LW -- False).  As the
    reference, the fallback re-draw with LW is the caller's (its plan is another signature)."""
    (lw, x), sec = _query_walk(plan, params, fixed, n_samples, seed, offset, q_base, noise, plan_jit)
    if sec[3][7] != 1:
        raise ValueError("vbn_hip::is_lw: the plan is not a weighted walk")
    b = int(fixed.shape[0])
    w, ess = normalize_weights(lw.view(b, n_samples), bool(normalize) or not lw_mode, float(eps))
    if lw_mode:
        flag = torch.zeros((), dtype=torch.bool, device=w.device)
    else:
        flag = (ess < max(1.0, float(ess_threshold) * n_samples)).any()
    return w, x.view(b, n_samples, -1), ess, flag


@is_lw.register_fake
def _is_lw_fake(plan, params, fixed, n_samples, seed, offset=0, q_base=0, noise=None, lw_mode=False,
                normalize=True, eps=0.0, ess_threshold=0.1, plan_jit=1):
    b = fixed.shape[0]
    return (params.new_empty(b, n_samples), params.new_empty(b, n_samples, 1), params.new_empty(b),
            torch.empty((), dtype=torch.bool, device=params.device))


@torch.library.custom_op("vbn_hip::ancestral", mutates_args=())
def ancestral(plan: Tensor, params: Tensor, fixed: Tensor, n_samples: int, seed: int, offset: int = 0,
              q_base: int = 0, noise: Optional[Tensor] = None, plan_jit: int = 1) -> Tensor:
    """Ancestral sampling of a packed sample plan -> [B, S, n_out] (the plan's output nodes'
    columns in topological order)."""
    (_, x), sec = _query_walk(plan, params, fixed, n_samples, seed, offset, q_base, noise, plan_jit)
    if sec[3][7] != 2:
        raise ValueError("vbn_hip::ancestral: the plan is not a sampling walk")
    return x.view(int(fixed.shape[0]), n_samples, -1)


@ancestral.register_fake
def _ancestral_fake(plan, params, fixed, n_samples, seed, offset=0, q_base=0, noise=None, plan_jit=1):
    return params.new_empty(fixed.shape[0], n_samples, 1)
