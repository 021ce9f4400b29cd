"""Accelerated engines with the reference's plugin protocol.

Each class follows the reference engine contract (reference ``core/base.py:94-101``):
``cls(**params)`` then ``infer_posterior(vbn, query, **kw) -> (pdf[B,S], samples[B,S,Dt])``
or ``sample(vbn, query, n_samples, **kw)``; ``vbn`` is read duck-typed (``vbn.dag``,
``vbn.nodes``, ``vbn.device``), so the classes work with this package's :class:`VBN` and
can be registered into the reference's own ``INFERENCE_REGISTRY``.

Semantics mirror the reference branch by branch:

* MCM (monte_carlo_marginalization.py:18-92): do-target -> pdf = 1; all target parents
  observed -> only the target is walked (root target gives ``(1,S)``); otherwise the full
  walk, pdf = p(target | sampled parents), evidence not weighted; root draws shared by
  all queries.
* IS (importance_sampling.py:24-93): per-query root draws, evidence log-weights, softmax
  over S, ESS, batch-global fallback to LW when any ESS < max(1, 0.1*S) (NaN never triggers).
* LW (likelihood_weighting.py:24-82): evidence clamped (nan->0, +-1e6), shared root draws,
  softmax or max-shifted exp.
* ancestral (sampling/ancestral.py:13-65): the walk without weights; target slice or all nodes.
* RB (rao_blackwellized_marginalization.py:196-324): LW-style walk over the target's
  non-descendants with the target written as its conditional parameters, then one epilogue
  launch (weights, mixture moments, grid density / categorical marginal); fallback engine for
  observed descendants and unsupported target CPDs.
* RIS (resampled_importance_sampling.py:43-105): the LW walk split after every evidence node;
  between segments the particle state stays in HBM, per-query softmax + ESS, and when any
  query's ESS is below the threshold (batch-global, host sync as the reference) one
  multinomial resampling launch for the whole batch.

RNG: counter-based Philox keyed by ``(seed, offset, node, query, sample)``.  The seed of a
call is taken from the global torch generator (so ``torch.manual_seed`` makes runs
repeatable, and the reference's "batch row 0 == single query" property holds for IS).
For parity tests the draws can be injected (``_noise=``).
"""
from __future__ import annotations

import contextlib
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import ops
from .model import BNModel, model_from_vbn
from .plan import (F_PRE_OUT, KIND_ID, MODE_MCM, MODE_SAMPLE, MODE_WEIGHTED, S_FLAGS, S_KIND, GibbsPlan, PackedModel,
                   QueryPlan, barren_pruned,
                   liveness_order, precompute_plans,
                   build_gibbs_plan, build_plan)
from .registry import register_inference, register_sampling

__all__ = [
    "Query",
    "MonteCarloMarginalization",
    "ImportanceSampling",
    "LikelihoodWeighting",
    "AncestralSampler",
    "RaoBlackwellizedMarginalization",
    "ResampledImportanceSampling",
    "infer_batch_size",
]


@dataclass
class Query:
    """Inference/sampling query (reference core/base.py:18-25)."""

    target: Optional[str]
    evidence: Dict[str, torch.Tensor]
    do: Dict[str, torch.Tensor] = field(default_factory=dict)


def infer_batch_size(evidence: Dict, do: Optional[Dict] = None) -> int:
    """reference utils/__init__.py:46-61"""
    evidence = evidence or {}
    do = do or {}
    if evidence:
        b = int(next(iter(evidence.values())).shape[0])
        if do and int(next(iter(do.values())).shape[0]) != b:
            raise ValueError("Evidence and do batch sizes must match.")
        return b
    if do:
        return int(next(iter(do.values())).shape[0])
    return 1


def _as2d(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 1:
        return x.unsqueeze(-1)
    if x.dim() == 2:
        return x
    raise ValueError(f"Expected 1D or 2D tensor, got shape {tuple(x.shape)}")


def _device_of(vbn) -> torch.device:
    dev = torch.device(getattr(vbn, "device", "cuda"))
    if dev.type != "cuda":
        raise RuntimeError(
            f"the accelerated engines run on an MI355X; vbn.device is {dev} "
            "(construct the model with device='cuda' or call vbn.to_device('cuda'))")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def packed_model(vbn, device: torch.device) -> PackedModel:
    model: BNModel = model_from_vbn(vbn)
    key = ("packed", str(device), model.version)
    pk = model._cache.get(key)
    if pk is None:
        pk = PackedModel(model, device)
        model._cache[key] = pk
    return pk


def _plan(pk: PackedModel, key, **kw) -> QueryPlan:
    ck = ("plan",) + key
    p = pk.model._cache.get(ck)
    if p is None:
        p = build_plan(pk, **kw)
        if LIVENESS_ORDER and key[0] in _ORDERED and not kw.get("params") and _lds_bound(p):
            # the wave's LDS (value slots + scratch rows) limits the waves per CU: walk the DAG
            # in an order that keeps fewer values live (same draws, keyed by node; plan.py
            # liveness_order) when that frees slots
            # the greedy, then seeded restarts with other tie orders until the plan no longer
            # bounds the occupancy (cfg5: 32 -> 25 greedy -> 24 at the tenth restart)
            for seed in (None,) + tuple(range(ORDER_RESTARTS)):
                q = build_plan(pk, order=liveness_order(pk.model, fixed=kw.get("fixed", ()), logp=kw.get("logp", ()),
                                                        out_nodes=kw.get("out_nodes", ()), skip=kw.get("skip", ()),
                                                        seed=seed), **kw)
                if q.n_slots < p.n_slots:
                    p = q
                if not _lds_bound(p):
                    break
        if not kw.get("params"):
            # nodes whose parents are all shared root draws (once per sample) or all evidence
            # (once per query)
            pc = precompute_plans(pk, p, skip=kw.get("skip", ()), exact_f32=kw.get("exact_f32", False),
                                  kde_valu=kw.get("kde_valu", False), per_query=PRECOMPUTE_Q)
            if pc is not None:
                p.pc, p.pre, p.pre_q = pc
        pk.model._cache[ck] = p
    return p


# walk orders other than the model's (plan.liveness_order) for these plan kinds when LDS bounds
# the occupancy; RIS keeps the topological segments, Gibbs its level schedule
LIVENESS_ORDER = os.environ.get("VBN_LIVENESS_ORDER", "1") != "0"
_ORDERED = ("mcm", "mcm-short", "weighted", "ancestral")
WAVES_PER_CU = 16                    # 4 waves per SIMD at the walk's 128-VGPR budget
ORDER_RESTARTS = 64                  # seeded restarts of the liveness greedy (<= ~0.4 s per plan build)


def _resident_waves(p: QueryPlan) -> int:
    """Waves per CU the walk's launch shape gives a full-size launch of plan ``p`` (walk_shape in
    csrc/vbn_walk.hip): per-wave LDS vbn_hip_lds_bytes(n_slots, max_out), plus, for the kind sets
    that stage MLP weights in LDS (only gaussian_nn / linear_gaussian, no generic MLP shapes:
    staged_kinds), two weight buffers of ``wbuf`` floats per workgroup of 4, 2 or 1 waves."""
    per_wave = (p.n_slots + max(p.max_out, 1)) * 64 * 4
    staged = (p.kind_mask & 28) == 0 and not (p.kind_mask & 512)
    best = 0
    for w in ((4, 2, 1) if staged else (1,)):
        lds = w * per_wave + (2 * p.wbuf * 4 if staged else 0)
        if lds <= 160 * 1024:
            best = max(best, min(WAVES_PER_CU, (160 * 1024 // lds) * w))
    if staged and best == 0:                     # walk_shape falls back to an unstaged kind set
        best = min(WAVES_PER_CU, 160 * 1024 // per_wave)
    return best


def _lds_bound(p: QueryPlan) -> bool:
    """LDS (value slots, scratch rows and staged weight buffers) holds fewer than WAVES_PER_CU
    waves of the plan per CU"""
    return _resident_waves(p) < WAVES_PER_CU


# per-sample / per-query precompute (plan.precompute_plans) in production walks; False: every
# node per particle (A/B, tests).  PRECOMPUTE_Q (env VBN_PRECOMP_Q=0: off) applies to plans
# built afterwards
PRECOMPUTE = True
PRECOMPUTE_Q = os.environ.get("VBN_PRECOMP_Q", "1") != "0"


def _fixed_values(query, device, clamp: bool = False) -> Dict[str, torch.Tensor]:
    """prepare_fixed_values (reference inference/_core.py:117-135)."""
    vals: Dict[str, torch.Tensor] = {}
    for k, v in (query.do or {}).items():
        vals[k] = _as2d(torch.as_tensor(v)).to(device=device, dtype=torch.float32)
    for k, v in (query.evidence or {}).items():
        v = _as2d(torch.as_tensor(v)).to(device=device, dtype=torch.float32)
        if clamp:                                             # clamp_evidence (_core.py:112-114)
            v = torch.nan_to_num(v, nan=0.0, posinf=1e6, neginf=-1e6).clamp(min=-1e6, max=1e6)
        vals[k] = v
    return vals


def _fixed_buffer(plan: QueryPlan, vals: Dict[str, torch.Tensor], rows: int, device) -> torch.Tensor:
    if not plan.fixed_nodes:
        return torch.zeros(rows, 1, device=device, dtype=torch.float32)
    cols = []
    for n in plan.fixed_nodes:
        v = vals[n]
        if v.shape[0] != rows:
            v = v.expand(rows, -1)
        cols.append(v)
    return torch.cat(cols, dim=1).contiguous()


def _has_discrete(pk: PackedModel, nodes: Sequence[str]) -> bool:
    """some node of ``nodes`` is a softmax_nn with discrete dims (its evidence is checked)"""
    for n in nodes:
        rec = pk.model.cpds[n]
        if rec.kind == "softmax_nn" and bool(rec.state["_is_discrete"].bool().any()):
            return True
    return False


def _check_discrete(pk: PackedModel, vals: Dict[str, torch.Tensor], nodes: Sequence[str]) -> None:
    """softmax_nn discrete dims reject values outside the class set (softmax_nn.py:622-625)."""
    for n in nodes:
        rec = pk.model.cpds[n]
        if rec.kind != "softmax_nn" or n not in vals:
            continue
        disc = rec.state["_is_discrete"].bool()
        if not disc.any():
            continue
        cv = rec.state["_class_values"].to(vals[n].device)
        v = vals[n]
        match = (v.unsqueeze(-1) == cv.unsqueeze(0)).any(-1)
        if bool(((~match) & disc.to(v.device).unsqueeze(0)).any()):
            raise ValueError("Found values outside discrete class set.")


def _next_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


# last walk launched (introspection for bench.py's per-kernel timing)
LAST_LAUNCH: Dict[str, object] = {}

# VBN.precompile: engines build their plans and compile the specialised walks without launching.
# Per thread: a precompile in one thread must not turn another thread's launches into no-ops.
_PC_LOCAL = threading.local()


def _pc_state() -> Dict[str, object]:
    st = getattr(_PC_LOCAL, "state", None)
    if st is None:
        st = _PC_LOCAL.state = {"on": False, "compile": "sync", "plans": 0, "ready": 0}
    return st


@contextlib.contextmanager
def precompile_mode(compile: str = "sync"):
    """Inside, run_walk compiles (``compile`` "sync" or "background", jit.module_for; "none":
    nothing) the walk each engine call would launch, records its plan and returns zero outputs
    instead of launching it.  Yields a dict that holds, after the block, "plans" (walks seen),
    "ready" (their specialised modules loaded) and "seen" (the plans)."""
    pc = _pc_state()
    prev = dict(pc)
    res: Dict[str, object] = {}
    pc.update(on=True, compile=compile, plans=0, ready=0, seen=[])
    try:
        yield res
    finally:
        res.update(plans=pc["plans"], ready=pc["ready"], seen=list(pc["seen"]))
        pc.clear()
        pc.update(prev)


def noise_tensor(pk: PackedModel, plan: QueryPlan, noise: Dict[str, Tuple], b: int, n: int) -> torch.Tensor:
    """Injected draws by node name -> kernel layout [n_latent, 2, b, n, Dmax].

    ``noise[node] = (slot0, slot1)``: slot0 = uniforms of categorical/index choices
    ([B|1, S] or [B|1, S, D]), slot1 = normals / within-bin uniforms ([B|1, S, D]).
    """
    out = torch.zeros(max(len(plan.noise_nodes), 1), 2, b, n, pk.dmax, dtype=torch.float32)
    for i, node in enumerate(plan.noise_nodes):
        if node not in noise:
            continue
        for slot, v in enumerate(noise[node]):
            if v is None:
                continue
            v = torch.as_tensor(v, dtype=torch.float32).cpu()
            if v.dim() == 2:
                v = v.unsqueeze(-1)
            out[i, slot, :, :, :v.shape[-1]] = v.expand(b, n, v.shape[-1])
    return out.to(pk.device)


# KDE walks launched in generations of about GEN_WAVES waves (0: one launch; env VBN_GEN_WAVES)
GEN_WAVES = int(os.environ.get("VBN_GEN_WAVES", "0"))


def _generations(plan: QueryPlan, b: int, n: int) -> int:
    if GEN_WAVES <= 0 or not (plan.kind_mask & (1 << KIND_ID["kde"])) or n % 64:
        return 1
    waves = b * n // 64
    return max(1, min(b, round(waves / GEN_WAVES)))


def _query_rows(pq: torch.Tensor, b: int, steps: torch.Tensor) -> torch.Tensor:
    """The per-query pre-pass's out_x [b * 64, w] as the walk's precomp_q: read in place as
    [b, 64 w] when the step table's stride is 64 w (plan.precompute_plans), else row 64 b
    gathered into [b, w]."""
    w = pq.shape[-1]
    if getattr(steps, "_vbn_precomp_q_stride", None) == 64 * w:
        return pq.view(b, 64 * w)
    return pq.view(b, 64, w)[:, 0].contiguous()


# the per-sample pre-pass on a side stream next to the per-query one: on when the per-sample
# pre-pass has KDE nodes (a few waves streaming whole point packs, latency-bound: cfg4 0.3 %
# shorter steps, profiles/r05_bench/r05ae_*), off for NN-only ones (cfg2 / anchor64 2-3 % slower
# steps, profiles/r04_bench/r04j_ab_*); env VBN_PRE_STREAM=1 / 0 forces it on / off
PRE_SIDE_STREAM = {"1": True, "0": False}.get(os.environ.get("VBN_PRE_STREAM", ""))


def _pre_side(plan) -> bool:
    if PRE_SIDE_STREAM is not None:
        return PRE_SIDE_STREAM
    v = getattr(plan, "_pre_has_kde", None)
    if v is None:
        host = getattr(plan.pre.steps, "_vbn_host", None)
        rows = host[0] if host is not None else plan.pre.steps.cpu().numpy()
        v = bool(((rows[:, S_KIND] == KIND_ID["kde"]) & ((rows[:, S_FLAGS] & F_PRE_OUT) != 0)).any())
        plan._pre_has_kde = v
    return v
_SIDE_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def _side_stream(device: torch.device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get(idx)
    if s is None:
        s = _SIDE_STREAMS[idx] = torch.cuda.Stream(device=torch.device("cuda", idx))
    return s


def run_walk(pk: PackedModel, plan: QueryPlan, fixed: torch.Tensor, b: int, n: int, *,
             seed: int, offset: int = 0, q_base: int = 0, noise=None,
             fixed_per_particle: bool = False, state: Optional[torch.Tensor] = None, state_flags: int = 0,
             step_begin: int = 0, step_end: int = -1, plan_jit: int = 1, run_if: Optional[torch.Tensor] = None,
             out_x: Optional[torch.Tensor] = None, stats_part: Optional[torch.Tensor] = None
             ) -> Tuple[torch.Tensor, torch.Tensor]:
    """One launch of the particle walk; returns (lp [b,n] or empty, x [b,n,n_out_cols]).
    ``state``/``state_flags``/``step_begin``/``step_end``: one segment of a split walk;
    ``plan_jit``: ops.walk (0 interpreter, 1 plan-specialised for large lean launches, 2 always);
    ``run_if``: device int32 [1] predicating the launch (the plain plan, no pre-passes: their
    outputs are bit-identical; nothing runs and nothing is written when it holds 0); ``out_x``: samples written into this [b, n, n_out_cols]
    tensor (a predicated launch that does not run leaves it as it was); ``stats_part``: an MCM
    walk's fused posterior-summary partials (float64 [b * n/64, 2 + 4 n_out_cols],
    ops.posterior_stats_merge)."""
    n_out_cols = int(plan.out_cols.numel()) if plan.out_nodes else 0
    noise_b = 1
    if isinstance(noise, dict):
        noise = noise_tensor(pk, plan, noise, b, n)
    if noise is not None:
        noise = noise.to(device=pk.device, dtype=torch.float32).contiguous()
        if noise.dim() != 5 or noise.shape[0] < len(plan.noise_nodes) or noise.shape[1] != 2:
            raise ValueError("noise must be [n_latent, 2, B|1, S, Dmax]")
        noise_b = int(noise.shape[2])
        if noise.shape[3] != n or noise.shape[4] != pk.dmax:
            raise ValueError(f"noise must be [n_latent, 2, B|1, {n}, {pk.dmax}]")
    precomp = precomp_q = None
    walk_plan = plan
    pre_ran = False
    # a predicated launch (run_if: importance sampling's fallback, which rarely runs) walks the
    # plain plan: its pre-passes would be two more launches of no-op waves on every call
    use_pc = (PRECOMPUTE and plan.pc is not None and noise is None and state is None and step_begin == 0
              and step_end < 0 and n % 64 == 0 and not fixed_per_particle and run_if is None)
    pcs = _pc_state()
    if pcs["on"]:
        # VBN.precompile / pack_query: compile (or load) the specialised walk this launch would
        # run, record its plan, no launch
        pcs.setdefault("seen", []).append(plan)
        if state is None and noise is None and plan_jit and pcs["compile"] != "none":
            from . import jit
            wp = plan.pc if use_pc else plan
            km = jit.walk_kind_set(wp, b, n, precomp=use_pc and plan.pre is not None)
            host = wp.steps._vbn_host
            dev = pk.device.index if pk.device.index is not None else 0
            if jit.module_for(host[0], host[1], km, dev, host[2], compile=pcs["compile"]) is not None:
                pcs["ready"] += 1
            pcs["plans"] += 1
        lp = torch.zeros(b, n, device=pk.device) if plan.mode != MODE_SAMPLE else torch.empty(0, device=pk.device)
        return lp, torch.zeros(b, n, n_out_cols, device=pk.device)
    if use_pc:
        # the per-sample quantities of nodes with shared-root parents, once per sample (same
        # seed / offset: the pre-pass draws the main walk's root values), the per-query ones of
        # nodes with evidence parents, once per query (one wave of identical lanes), then the
        # main walk
        # with both, the per-sample one (a few waves walking the root nodes, latency-bound) runs
        # on a side stream next to the per-query one
        side = (_side_stream(pk.device) if (plan.pre is not None and plan.pre_q is not None and _pre_side(plan))
                else None)
        if side is not None:
            main = torch.cuda.current_stream(pk.device)
            side.wait_stream(main)
        if plan.pre is not None:
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                _, precomp = run_walk(pk, plan.pre, fixed, 1, n, seed=seed, offset=offset, plan_jit=0,
                                      run_if=run_if)
            precomp = precomp.view(n, -1)
        if plan.pre_q is not None:
            _, pq = run_walk(pk, plan.pre_q, fixed, b, 64, seed=seed, offset=offset, q_base=q_base, plan_jit=0,
                             run_if=run_if)
            precomp_q = _query_rows(pq, b, plan.pc.steps)
        if side is not None:
            main.wait_stream(side)
            precomp.record_stream(main)
        walk_plan = plan.pc
        pre_ran = True
    # (the plan as given: a re-run of this launch repeats the pre-passes; a predicated launch --
    # importance sampling's fallback re-draw -- is not recorded, so LAST_LAUNCH stays the walk
    # whose outputs the call returns unless the fallback fired)
    if run_if is None:
        LAST_LAUNCH.update(pk=pk, plan=plan, fixed=fixed, b=b, n=n, fixed_per_particle=fixed_per_particle,
                           noise=noise, state=state, seed=seed, offset=offset, plan_jit=plan_jit,
                           precomputed=pre_ran, q_base=q_base)
    plan = walk_plan
    args = (plan.steps, plan.in_cols, pk.params, fixed, noise, plan.out_cols, b, n,
            plan.n_slots, plan.max_out, plan.fixed_ld, fixed_per_particle, noise_b,
            len(plan.noise_nodes), pk.dmax, n_out_cols, plan.mode, q_base, seed, offset,
            plan.mode != MODE_SAMPLE, plan.kind_mask)
    gens = (_generations(plan, b, n) if (state is None and noise is None and not fixed_per_particle
                                          and run_if is None and out_x is None) else 1)
    if gens > 1:
        # KDE walks in launches of about one resident wave per slot (GEN_WAVES): all waves of a
        # launch start at the first node together and stay near each other in the node
        # sequence, so the point packs they stream stay in L2 (scripts/gen_ab.py); per-query
        # draws are keyed by q_base + query, so the outputs are the single launch's
        step = -(-b // gens)
        lps, xss = [], []
        for b0 in range(0, b, step):
            b1 = min(b, b0 + step)
            fx = fixed[b0:b1] if fixed.shape[0] == b else fixed
            a = args[:3] + (fx,) + args[4:6] + (b1 - b0,) + args[7:17] + (q_base + b0,) + args[18:]
            pq = precomp_q[b0:b1] if precomp_q is not None else None
            if stats_part is None:
                l, x = ops.walk(*a, plan.wbuf, plan_jit, precomp, pq)
            else:
                rows = stats_part.shape[0] // b
                l, x = ops.walk_ex(*a, plan.wbuf, plan_jit, precomp, pq,
                                   stats_part=stats_part[b0 * rows:b1 * rows])
            lps.append(l.view(b1 - b0, n) if plan.mode != MODE_SAMPLE else l)
            xss.append(x.view(b1 - b0, n, -1) if n_out_cols else x)
        lp = torch.cat(lps) if plan.mode != MODE_SAMPLE else lps[0]
        x = torch.cat(xss) if n_out_cols else xss[0]
    elif state is None and run_if is None and out_x is None and stats_part is None:
        lp, x = ops.walk(*args, plan.wbuf, plan_jit, precomp, precomp_q)
    elif state is None and run_if is None and out_x is None:
        lp, x = ops.walk_ex(*args, plan.wbuf, plan_jit, precomp, precomp_q, stats_part=stats_part)
    elif state is None:
        lp, x = ops.walk_ex(*args, plan.wbuf, plan_jit, precomp, precomp_q, run_if=run_if,
                            out_x=None if out_x is None else out_x.view(b * n, n_out_cols))
    else:
        lp, x = ops.walk_segment(*args, state, state_flags, step_begin, step_end, plan.wbuf)
    if plan.mode != MODE_SAMPLE:
        lp = lp.view(b, n)
    if n_out_cols:
        x = x.view(b, n, n_out_cols)
    return lp, x


def _stats_request(kwargs, xs: torch.Tensor) -> Optional[dict]:
    """The caller's fused posterior-summary request (``_stats``: a dict with "eps", filled with
    "mean" / "std" / "ess"; VBN.infer_relative) as normalize_weights_ex's ``stats`` argument, or
    None when the normalisation cannot fuse it (S > 4096: the caller runs the separate pass)."""
    stats = kwargs.get("_stats")
    if stats is None or xs.dim() != 3 or xs.shape[1] > 4096 or xs.shape[2] < 1:
        return None
    stats["x"] = xs
    stats.setdefault("eps", 1e-12)
    return stats


class _EngineBase:
    def __init__(self, n_samples: int = 200, seed: Optional[int] = None, prune_barren: bool = False,
                 q_base: int = 0, exact_f32: bool = False, kde_valu: bool = False, plan_jit="auto", **kwargs):
        self.n_samples = int(n_samples)
        # plan-specialised walks (jit.py): "auto" = large lean launches, True = every lean launch
        self.plan_jit = 2 if plan_jit is True else (0 if plan_jit is False else 1)
        self.seed = seed
        self.prune_barren = bool(prune_barren)
        self.q_base = int(q_base)
        self.exact_f32 = bool(exact_f32)     # hidden layer on the exact f32 MFMA chain
        self.kde_valu = bool(kde_valu)       # KDE distances on packed VALU (else the MFMA tile)
        self._calls = 0

    def _plan(self, pk, key, **kw):
        return _plan(pk, key + (self.exact_f32, self.kde_valu), exact_f32=self.exact_f32,
                     kde_valu=self.kde_valu, **kw)

    def _seed(self, kwargs) -> int:
        if "seed" in kwargs and kwargs["seed"] is not None:
            return int(kwargs["seed"])
        if self.seed is not None:
            s = int(self.seed) + self._calls
            self._calls += 1
            return s
        return _next_seed()

    @staticmethod
    def _query(query):
        ev = dict(getattr(query, "evidence", None) or {})
        do = dict(getattr(query, "do", None) or {})
        return query.target, ev, do


@register_inference("monte_carlo_marginalization")
class MonteCarloMarginalization(_EngineBase):
    """monte_carlo_marginalization.py:12-92 on the GPU."""

    def infer_posterior(self, vbn, query, **kwargs):
        n = int(kwargs.get("n_samples", self.n_samples))
        target, ev, do = self._query(query)
        b = infer_batch_size(ev, do)
        dev = _device_of(vbn)
        pk = packed_model(vbn, dev)
        model = pk.model
        vals = _fixed_values(query, dev)
        if target in do:                                                    # Q3
            return (torch.ones(b, n, device=dev, dtype=torch.float32),
                    vals[target].unsqueeze(1).expand(b, n, -1))
        parents = model.parents[target]
        fixed = [x for x in model.topo if x in vals]
        _check_discrete(pk, vals, [target] if target in vals else [])
        prune = self.prune_barren
        if all(p in vals for p in parents):                                 # Q2 shortcut
            t_fixed = target in vals
            nodes = set(parents) | {target}
            key = ("mcm-short", target, t_fixed)
            plan = self._plan(pk, key, latent=[] if t_fixed else [target],
                         fixed=[x for x in model.topo if x in nodes and x != target] + ([target] if t_fixed else []),
                         logp=[target], out_nodes=[target], shared_roots=True, mode=MODE_MCM,
                         skip=[x for x in model.topo if x not in nodes])
            b_eff = b if (parents or t_fixed) else 1                        # Q4: root -> (1,S)
        else:
            keep = barren_pruned(model, [target]) if prune else set(model.topo)
            key = ("mcm", target, tuple(sorted(vals)), prune)
            plan = self._plan(pk, key, latent=[x for x in model.topo if x in keep and x not in vals],
                         fixed=[x for x in fixed if x in keep], logp=[target], out_nodes=[target],
                         shared_roots=True, mode=MODE_MCM, skip=[x for x in model.topo if x not in keep])
            b_eff = b
        fx = _fixed_buffer(plan, vals, b_eff, dev)
        stats = kwargs.get("_stats")
        d = int(plan.out_cols.numel())
        part = None
        if stats is not None and n % 64 == 0 and 1 <= d <= 15:
            # VBN._posterior_stats fused into the walk's epilogue (vbn_walk_args.stats_part)
            rows, stride = ops.stats_part_rows(b_eff, n, d)
            part = torch.empty(rows, stride, device=dev, dtype=torch.float64)
        pdf, xs = run_walk(pk, plan, fx, b_eff, n, seed=self._seed(kwargs), q_base=self.q_base,
                           noise=kwargs.get("_noise"), plan_jit=self.plan_jit, stats_part=part)
        if part is not None:
            stats["mean"], stats["std"], stats["ess"] = ops.posterior_stats_merge(part, b_eff, n, d,
                                                                                   stats.get("eps", 1e-12))
        return pdf, xs


@register_inference("likelihood_weighting")
class LikelihoodWeighting(_EngineBase):
    """likelihood_weighting.py:11-82 on the GPU."""

    def __init__(self, n_samples: int = 512, eps: float = 1e-12, normalize: bool = True, **kwargs):
        super().__init__(n_samples=n_samples, **kwargs)
        self.eps = float(eps)
        self.normalize = bool(normalize)

    def _walk(self, vbn, query, n, *, clamp, shared_roots, kwargs, offset=0, noise=None, run_if=None, out_x=None,
              fixed_from=None):
        """``clamp``: the evidence is clamped as clamp_evidence does (_core.py:112-114) -- by the
        kernel as it reads the fixed buffer (VBN_F_CLAMP_EV), so no clamp kernels run; the host
        clamps too only where the discrete-class check needs the clamped values.
        ``fixed_from``: (fixed nodes, [B, fixed_ld] buffer) of an unclamped walk of the same query
        (importance sampling's): with no do-values this walk reads that buffer as it is."""
        target, ev, do = self._query(query)
        b = infer_batch_size(ev, do)
        dev = _device_of(vbn)
        pk = packed_model(vbn, dev)
        model = pk.model
        host_clamp = clamp and _has_discrete(pk, list(ev))
        reuse = fixed_from is not None and not do and not host_clamp
        vals = _fixed_values(query, dev, clamp=host_clamp)
        _check_discrete(pk, vals, list(ev))
        keep = barren_pruned(model, [target] + list(ev)) if self.prune_barren else set(model.topo)
        key = ("weighted", target, tuple(sorted(ev)), tuple(sorted(do)), shared_roots, bool(clamp), self.prune_barren)
        plan = self._plan(pk, key, latent=[x for x in model.topo if x in keep and x not in vals],
                     fixed=[x for x in model.topo if x in keep and x in vals],
                     logp=[x for x in model.topo if x in ev and x in keep], out_nodes=[target],
                     shared_roots=shared_roots, mode=MODE_WEIGHTED,
                     skip=[x for x in model.topo if x not in keep],
                     clamp=[x for x in ev if x in keep] if clamp else ())
        if reuse and tuple(fixed_from[0]) == tuple(plan.fixed_nodes):
            fx = fixed_from[1]
        else:
            fx = _fixed_buffer(plan, vals, b, dev)
        self._last_fixed = (tuple(plan.fixed_nodes), fx)
        seed = kwargs.get("_seed_value")
        if seed is None:
            seed = self._seed(kwargs)
        log_w, xs = run_walk(pk, plan, fx, b, n, seed=seed, offset=offset, q_base=self.q_base, noise=noise,
                             plan_jit=self.plan_jit, run_if=run_if, out_x=out_x)
        return log_w, xs

    def infer_posterior(self, vbn, query, **kwargs):
        n = int(kwargs.get("n_samples", self.n_samples))
        normalize = bool(kwargs.get("normalize", self.normalize))
        eps = float(kwargs.get("eps", self.eps))
        log_w, xs = self._walk(vbn, query, n, clamp=True, shared_roots=True, kwargs=kwargs,
                               offset=int(kwargs.get("_offset", 0)), noise=kwargs.get("_noise"))
        stats = _stats_request(kwargs, xs)
        if stats is not None:
            # VBN._posterior_stats fused into the normalisation (vbn_hip_normalize_weights_stats)
            w, _, _ = ops.normalize_weights_ex(log_w, normalize, eps, stats=stats)
            return w, xs
        w, _ = ops.normalize_weights(log_w, normalize, eps)
        return w, xs

    def infer_into(self, vbn, query, n: int, *, seed: int, offset: int, run_if: torch.Tensor,
                   w_out: torch.Tensor, x_out: torch.Tensor, noise=None, fixed_from=None, stats=None) -> None:
        """The whole LW call predicated on the device flag ``run_if``: walk and normalisation
        write their weights / samples into ``w_out`` / ``x_out`` when it holds 1 and launch as
        no-ops otherwise (importance sampling's fallback without a host sync); ``stats``: the
        fused posterior summary's outputs, overwritten likewise."""
        log_w, _ = self._walk(vbn, query, n, clamp=True, shared_roots=True, kwargs={"_seed_value": seed},
                              offset=offset, noise=noise, run_if=run_if, out_x=x_out, fixed_from=fixed_from)
        ops.normalize_weights_ex(log_w, self.normalize, self.eps, run_if=run_if, w_out=w_out,
                                 stats=None if stats is None else dict(stats, x=x_out))


@register_inference("importance_sampling")
class ImportanceSampling(LikelihoodWeighting):
    """importance_sampling.py:14-93 on the GPU (walk + wave-reduced softmax/ESS + fallback)."""

    def __init__(self, n_samples: int = 200, **kwargs):
        kwargs.pop("normalize", None)
        super().__init__(n_samples=n_samples, **kwargs)
        self.ess_threshold = 0.1
        self._fallback_flag: Optional[torch.Tensor] = None    # device int32 [1] of the last call
        self._fallback_bool: Optional[bool] = False
        self._last_ess: Optional[torch.Tensor] = None
        self._lw = LikelihoodWeighting(n_samples=self.n_samples, q_base=self.q_base,
                                       exact_f32=self.exact_f32, kde_valu=self.kde_valu,
                                       plan_jit={0: False, 1: "auto", 2: True}[self.plan_jit])

    def fallback_needed(self, ess: torch.Tensor, n: int) -> torch.Tensor:
        """Device-side flag (NaN ESS never triggers; importance_sampling.py:85-86)."""
        thr = max(1.0, self.ess_threshold * float(n))
        return (ess < thr).any()

    @property
    def _last_fallback(self) -> bool:
        """Whether the last call fell back to likelihood weighting (the reference's attribute).
        The decision stays on the device until this is read (one host sync, then cached)."""
        if self._fallback_bool is None:
            self._fallback_bool = bool(self._fallback_flag.item())
        return self._fallback_bool

    @_last_fallback.setter
    def _last_fallback(self, value: bool) -> None:
        self._fallback_flag, self._fallback_bool = None, bool(value)

    def fallback_flag(self) -> Optional[torch.Tensor]:
        """The last call's fallback decision as a device int32 [1] tensor (no host sync)."""
        return self._fallback_flag

    def infer_posterior(self, vbn, query, **kwargs):
        n = int(kwargs.get("n_samples", self.n_samples))
        seed = self._seed(kwargs)
        log_w, xs = self._walk(vbn, query, n, clamp=False, shared_roots=False,
                               kwargs={**kwargs, "_seed_value": seed}, noise=kwargs.get("_noise"))
        # softmax + ESS, and the fallback decision (any ESS < threshold) on the device
        thr = max(1.0, self.ess_threshold * float(n))
        stats = _stats_request(kwargs, xs)
        w, ess, flag = ops.normalize_weights_ex(log_w, True, 0.0, ess_thr=thr, stats=stats)
        self._last_ess = ess
        reduce = kwargs.get("_reduce_flag")          # multi-GPU: batch-global decision
        if reduce is not None:
            flag = reduce(flag).to(device=w.device, dtype=torch.int32).reshape(1)
        # importance_sampling.py:85-88: the likelihood-weighting re-draw replaces the outputs when
        # the flag is set -- launched predicated on it and written into w / xs in place, so the
        # host never waits for the decision (the reference syncs here)
        self._lw.q_base = self.q_base
        self._lw.infer_into(vbn, query, n, seed=seed, offset=1, run_if=flag, w_out=w, x_out=xs,
                            noise=kwargs.get("_noise_fallback"), fixed_from=self._last_fixed,
                            stats=None if stats is None else {k: stats[k] for k in ("mean", "std", "ess", "eps")})
        self._fallback_flag, self._fallback_bool = flag, None
        return w, xs


def _descendants(model: BNModel, node: str) -> set:
    ch = model.children()
    out, stack = set(), [node]
    while stack:
        for c in ch[stack.pop()]:
            if c not in out:
                out.add(c)
                stack.append(c)
    return out


@register_inference("rao_blackwellized_marginalization")
class RaoBlackwellizedMarginalization(_EngineBase):
    """rao_blackwellized_marginalization.py:15-324 on the GPU."""

    _BASE_KW = ("seed", "prune_barren", "q_base", "exact_f32", "kde_valu", "plan_jit")

    def __init__(self, n_samples: int = 200, n_particles: Optional[int] = None, stddevs: float = 4.0,
                 min_scale: float = 1e-6, fallback: Optional[str] = "likelihood_weighting", **kwargs):
        super().__init__(n_samples=n_samples, **{k: kwargs[k] for k in self._BASE_KW if k in kwargs})
        self.n_particles = int(n_particles) if n_particles is not None else self.n_samples
        self.stddevs = float(stddevs)
        self.min_scale = float(min_scale)
        self.fallback = str(fallback).strip().lower() if fallback is not None else "none"
        self._fallback = None
        self._last_fallback = False
        self._last_reason: Optional[str] = None
        if self.fallback != "none":
            from .registry import INFERENCE_REGISTRY
            if self.fallback not in INFERENCE_REGISTRY:
                raise ValueError(
                    f"Unknown fallback inference '{fallback}'. Available: {list(INFERENCE_REGISTRY.keys())}")
            if self.fallback == "rao_blackwellized_marginalization":
                raise ValueError("fallback cannot be 'rao_blackwellized_marginalization'")
            fk = dict(kwargs)
            fk.setdefault("n_samples", self.n_samples)
            self._fallback = INFERENCE_REGISTRY[self.fallback](**fk)

    def _fallback_infer(self, vbn, query, *, reason: str, **kwargs):
        self._last_fallback = True
        self._last_reason = reason
        if self._fallback is None:
            raise RuntimeError("rao_blackwellized_marginalization cannot handle this query and has no fallback")
        kw = {k: v for k, v in kwargs.items() if k not in ("n_particles", "_noise")}
        if "_noise_fallback" in kw:
            kw["_noise"] = kw.pop("_noise_fallback")
        return self._fallback.infer_posterior(vbn, query, **kw)

    def infer_posterior(self, vbn, query, **kwargs):
        self._last_fallback = False
        self._last_reason = None
        n = max(1, int(kwargs.get("n_samples", self.n_samples)))
        n_part = max(1, int(kwargs.get("n_particles", self.n_particles)))
        target, ev, do = self._query(query)
        b = infer_batch_size(ev, do)
        dev = _device_of(vbn)
        pk = packed_model(vbn, dev)
        model = pk.model
        desc = _descendants(model, target)
        if any(x in ev or x in do for x in desc):                                   # 209-217
            return self._fallback_infer(vbn, query, reason="target has observed/intervened descendants", **kwargs)
        vals = _fixed_values(query, dev, clamp=True)                                 # 219
        if target in vals:                                                           # 220-224
            return (torch.ones(b, 1, device=dev, dtype=torch.float32),
                    vals[target].unsqueeze(1).expand(b, 1, -1))
        rec = model.cpds[target]
        if rec.kind == "softmax_nn" and model.out_dim(target) == 1:
            mode = 1
        elif rec.kind in ("gaussian_nn", "linear_gaussian") and model.out_dim(target) == 1:
            mode = 0
        else:
            return self._fallback_infer(vbn, query, reason="unsupported target CPD for RB marginalization",
                                        **kwargs)
        _check_discrete(pk, vals, list(ev))
        keep = [x for x in model.topo if x not in desc]
        key = ("rb", target, tuple(sorted(ev)), tuple(sorted(do)))
        plan = self._plan(pk, key, latent=[x for x in keep if x not in vals and x != target],
                          fixed=[x for x in keep if x in vals], logp=[x for x in keep if x in ev],
                          out_nodes=[target], params=[target], shared_roots=True, mode=MODE_WEIGHTED,
                          skip=sorted(desc))
        fx = _fixed_buffer(plan, vals, b, dev)
        log_w, prm = run_walk(pk, plan, fx, b, n_part, seed=self._seed(kwargs), q_base=self.q_base,
                              noise=kwargs.get("_noise"), plan_jit=self.plan_jit)
        if mode == 0:
            z = torch.linspace(0.0, 1.0, n).to(dev)                                   # 304
            pdf, grid = ops.rb_epilogue(log_w, prm, z, n, 0, self.stddevs, self.min_scale, 1e-12)
            return pdf, grid.unsqueeze(-1)
        c = int(rec.hp("n_classes"))
        pdf, _ = ops.rb_epilogue(log_w, prm, log_w.new_empty(0), c, 1, self.stddevs, self.min_scale, 1e-12)
        support = rec.state["_sample_values"][0].to(device=dev, dtype=torch.float32)
        return pdf, support.view(1, -1, 1).expand(b, -1, 1)


@register_inference("resampled_importance_sampling")
class ResampledImportanceSampling(_EngineBase):
    """resampled_importance_sampling.py:13-105 on the GPU (segmented walk + resampling)."""

    def __init__(self, n_samples: int = 512, ess_threshold: float = 0.5, resample: bool = True,
                 clamp_obs: bool = True, **kwargs):
        super().__init__(n_samples=n_samples, **kwargs)
        self.ess_threshold = float(ess_threshold)
        self.resample = bool(resample)
        self.clamp_obs = bool(clamp_obs)
        self._last_ess: Optional[torch.Tensor] = None
        self._last_resampled = False

    def infer_posterior(self, vbn, query, **kwargs):
        n = int(kwargs.get("n_samples", self.n_samples))
        thr_in = float(kwargs.get("ess_threshold", self.ess_threshold))
        resample = bool(kwargs.get("resample", self.resample))
        clamp = bool(kwargs.get("clamp_obs", self.clamp_obs))
        target, ev, do = self._query(query)
        b = infer_batch_size(ev, do)
        dev = _device_of(vbn)
        pk = packed_model(vbn, dev)
        model = pk.model
        vals = _fixed_values(query, dev, clamp=clamp)
        _check_discrete(pk, vals, list(ev))
        key = ("ris", target, tuple(sorted(ev)), tuple(sorted(do)), clamp)
        plan = self._plan(pk, key, latent=[x for x in model.topo if x not in vals],
                          fixed=[x for x in model.topo if x in vals], logp=[x for x in model.topo if x in ev],
                          out_nodes=[target], shared_roots=True, mode=MODE_WEIGHTED)
        fx = _fixed_buffer(plan, vals, b, dev)
        seed = self._seed(kwargs)
        noise = kwargs.get("_noise")
        if isinstance(noise, dict):
            noise = noise_tensor(pk, plan, noise, b, n)
        u_list = list(kwargs.get("_resample_u") or [])
        threshold = max(1.0, thr_in * float(n)) if thr_in <= 1.0 else thr_in            # 62-65
        self._last_resampled = False
        order = [x for x in model.topo]                                                 # plan order
        # a segment ends after every evidence node (ESS check, 75-90); the last segment may be
        # empty when the last node is evidence (it only reloads the state and writes outputs)
        cuts = ([i + 1 for i, x in enumerate(order) if x in ev] if resample else []) + [len(order)]
        if len(cuts) == 1:
            log_w, xs = run_walk(pk, plan, fx, b, n, seed=seed, q_base=self.q_base, noise=noise,
                                 plan_jit=self.plan_jit)
        else:
            total = b * n
            st_a = torch.empty(plan.n_slots + 1, total, device=dev, dtype=torch.float32)
            st_b = torch.empty_like(st_a)
            begin, events = 0, 0
            for k, end in enumerate(cuts):
                last = k == len(cuts) - 1
                flags = (1 if k > 0 else 0) | (0 if last else 2)
                log_w, xs = run_walk(pk, plan, fx, b, n, seed=seed, q_base=self.q_base, noise=noise,
                                     state=st_a, state_flags=flags, step_begin=begin, step_end=end)
                begin = end
                if last:
                    break
                w, ess = ops.normalize_weights(st_a[plan.n_slots].view(b, n), True, 0.0)     # 85-87
                self._last_ess = ess
                flag = (ess < threshold).any()
                reduce = kwargs.get("_reduce_flag")          # multi-GPU: batch-global decision
                if reduce is not None:
                    flag = reduce(flag)
                if bool(flag):                                                               # 88-90
                    u = u_list.pop(0) if u_list else None
                    ops.resample(w, u, seed, events + 1, self.q_base, st_a, st_b)
                    st_a, st_b = st_b, st_a
                    events += 1
                    self._last_resampled = True
        w, _ = ops.normalize_weights(log_w, True, 0.0)                                     # 102
        return w, xs


@register_sampling("ancestral")
class AncestralSampler(_EngineBase):
    """sampling/ancestral.py:57-65 on the GPU."""

    def sample(self, vbn, query, n_samples: Optional[int] = None, **kwargs):
        n = int(n_samples or self.n_samples)
        target, ev, do = self._query(query)
        b = infer_batch_size(ev, do)
        dev = _device_of(vbn)
        pk = packed_model(vbn, dev)
        model = pk.model
        vals = _fixed_values(query, dev)
        outs = [target] if target else list(model.topo)
        keep = barren_pruned(model, outs) if (self.prune_barren and target) else set(model.topo)
        key = ("ancestral", target, tuple(sorted(vals)), self.prune_barren and bool(target))
        plan = self._plan(pk, key, latent=[x for x in model.topo if x in keep and x not in vals],
                     fixed=[x for x in model.topo if x in keep and x in vals], logp=[],
                     out_nodes=outs, shared_roots=True, mode=MODE_SAMPLE,
                     skip=[x for x in model.topo if x not in keep])
        fx = _fixed_buffer(plan, vals, b, dev)
        _, xs = run_walk(pk, plan, fx, b, n, seed=self._seed(kwargs), q_base=self.q_base,
                         noise=kwargs.get("_noise"), plan_jit=self.plan_jit)
        if target:
            return xs
        out, c = {}, 0
        for node in model.topo:
            d = model.out_dim(node)
            out[node] = xs[..., c:c + d]
            c += d
        return out


@register_sampling("gibbs")
class GibbsSampler(_EngineBase):
    """sampling/gibbs.py:12-92 on the GPU: one ancestral walk for the start state (29), then
    every sweep of every chain in one launch (lanes = chain x 8 candidates, gibbs.py:36-87).

    ``collect="reference"`` (default) returns what the reference returns: its ``collected``
    list holds views of the chain state (gibbs.py:86), so every entry is the state after the
    LAST sweep; the walk then writes only that sweep.  ``collect="chain"`` writes the target
    at every collected sweep instead (burn-in, thinning by ``n_steps``) -- the Markov chain.
    """

    HALF_WAVE_BELOW = ops.HALF_WAVE_BELOW   # ops.gibbs_walk's automatic half-wave threshold

    def __init__(self, n_samples: int = 200, burn_in: int = 10, n_steps: int = 1, collect: str = "reference",
                 wave_particles: Optional[int] = None, chain_waves: Optional[int] = None, **kwargs):
        super().__init__(n_samples=n_samples, **kwargs)
        if wave_particles not in (None, 32, 64):
            raise ValueError(f"wave_particles must be None (auto), 32 or 64, got {wave_particles!r}")
        if chain_waves not in (None, *range(9)):
            raise ValueError(f"chain_waves must be None (auto) or 0..8, got {chain_waves!r}")
        self.wave_particles = wave_particles
        self.chain_waves = chain_waves    # specialised sweeps: waves splitting a chain group's updates
        self.burn_in = int(burn_in)
        self.n_steps = int(n_steps)
        self.n_candidates = 8
        if collect not in ("reference", "chain"):
            raise ValueError(f"collect must be 'reference' or 'chain', got {collect!r}")
        self.collect = collect

    def _wave_particles(self, b: int) -> int:
        """32 / 64, or 0: ops.gibbs_walk chooses (full waves on chain workgroups, half waves
        for small batches otherwise; ops.LAST_WALK["wave_particles"] says which ran)."""
        return 0 if self.wave_particles is None else self.wave_particles

    def _gibbs_plan(self, pk: PackedModel, target: str, vals) -> GibbsPlan:
        model = pk.model
        ck = ("gibbs", target, tuple(sorted(vals)), self.exact_f32, self.kde_valu)
        gp = model._cache.get(ck)
        if gp is None:
            gp = build_gibbs_plan(pk, latent=[x for x in model.topo if x not in vals],
                                  fixed=[x for x in model.topo if x in vals], target=target,
                                  exact_f32=self.exact_f32, kde_valu=self.kde_valu)
            model._cache[ck] = gp
        return gp

    def sample(self, vbn, query, n_samples: Optional[int] = None, **kwargs):
        n = int(n_samples or self.n_samples)
        target, ev, do = self._query(query)
        if not target:
            raise ValueError("Gibbs sampling needs a query target")
        b = infer_batch_size(ev, do)
        dev = _device_of(vbn)
        pk = packed_model(vbn, dev)
        model = pk.model
        if target not in model.cpds:
            raise ValueError(f"Unknown target node: {target}")
        vals = _fixed_values(query, dev)
        thin = max(self.n_steps, 1)
        iters = self.burn_in + n * thin                                                 # 37
        if iters > 0:
            # every sweep scores the observed children of latent nodes, evidence and do nodes
            # alike (gibbs.py:56-78), so out-of-class values raise as in softmax_nn._x_to_bin
            _check_discrete(pk, vals, [x for x in model.topo if x in vals
                                       and any(p not in vals for p in model.parents[x])])
        gp = self._gibbs_plan(pk, target, vals)
        init = gp.init
        fx = _fixed_buffer(init, vals, b, dev)
        seed = self._seed(kwargs)
        init_noise, sweep_noise = kwargs.get("_noise") or (None, None)
        state = torch.empty(init.n_slots + 1, b, device=dev, dtype=torch.float32)
        _, x0 = run_walk(pk, init, fx, b, 1, seed=seed, q_base=self.q_base, noise=init_noise,
                         state=state, state_flags=2)                                    # gibbs.py:29
        slot, dt = init.slot_of[target], model.out_dim(target)
        if iters == 0:
            return x0[..., slot:slot + dt].contiguous()                                 # 89-91
        if self.collect == "chain" and n > 0:
            burn, th = self.burn_in, thin
        else:
            burn, th = iters - 1, 1                       # the final sweep (every collected view)
        chains = state.view(init.n_slots + 1, b, 1).expand(-1, -1, 8).reshape(init.n_slots + 1, b * 8)
        noise_b = b
        if sweep_noise is not None:
            sweep_noise = sweep_noise.to(device=dev, dtype=torch.float32).contiguous()
            if sweep_noise.shape != (iters, gp.n_noise, 2, b, 8, pk.dmax):
                raise ValueError(f"sweep noise must be [{iters}, {gp.n_noise}, 2, {b}, 8, {pk.dmax}]")
        out = ops.gibbs_walk(gp.steps, gp.in_cols, pk.params, fx,
                             sweep_noise, chains.contiguous(), b, init.n_slots, init.max_out, init.fixed_ld,
                             noise_b, gp.n_noise, pk.dmax, dt, iters, burn, th, self.q_base, seed, 1,
                             gp.kind_mask, gp.wbuf, self._wave_particles(b), self.plan_jit,
                             -1 if self.chain_waves is None else self.chain_waves)
        if self.collect == "chain" and n > 0:
            return out
        return out.expand(b, max(n, 1), dt).contiguous()
