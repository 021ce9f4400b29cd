"""VBN-compatible facade over the accelerated path.

Mirrors the reference's public surface for this path (reference ``vbn/vbn.py``):

* ``VBN.set_inference_method(method, **kw)`` / ``set_sampling_method`` accept a registry
  name, a ``{"name": ...}`` dict, a :class:`ConfigItem` (``vbn.config.inference.<name>``)
  or a callable, and merge YAML defaults with keyword overrides (vbn.py:257-335);
* ``VBN.infer_posterior(query, **kw) -> (pdf[B,S], samples[B,S,Dt])`` (vbn.py:474-481);
* ``VBN.sample(query, n_samples, **kw)`` (vbn.py:570-577);
* query normalisation and its errors (vbn.py:579-618).

Models come from the reference checkpoint format (``VBN.load``), a live fitted reference
object (``VBN.from_reference``) or an in-memory :class:`BNModel` (``VBN.from_model``).
Training (``fit``/``update``) stays with the reference; this package consumes its output.
"""
from __future__ import annotations

import os

from dataclasses import dataclass
from types import SimpleNamespace
from typing import Any, Dict, List, Optional

import networkx as nx
import torch

from .engines import Query, infer_batch_size
from .handle import CPDHandle
from .model import BNModel, checkpoint_from_model, load_checkpoint, model_from_checkpoint, model_from_vbn
from .registry import INFERENCE_REGISTRY, SAMPLING_REGISTRY

__all__ = ["VBN", "ConfigItem", "defaults"]


# Packaged defaults of the in-scope engines (reference vbn/configs/inference/*.yaml,
# vbn/configs/sampling/{ancestral,gibbs}.yaml).
_ENGINE_DEFAULTS = {
    "inference": {
        "monte_carlo_marginalization": {"n_samples": 1024},
        "importance_sampling": {"n_samples": 1024},
        "likelihood_weighting": {"n_samples": 1024, "eps": 1e-12, "normalize": True},
        "rao_blackwellized_marginalization": {"n_samples": 256, "n_particles": 256, "stddevs": 4.0,
                                              "min_scale": 1e-6, "fallback": "likelihood_weighting"},
        "resampled_importance_sampling": {"n_samples": 1024, "ess_threshold": 0.5, "resample": True,
                                          "clamp_obs": True},
    },
    "sampling": {"ancestral": {"n_samples": 512},
                 "gibbs": {"n_samples": 512, "burn_in": 50, "n_steps": 5}},
}


@dataclass
class ConfigItem:
    """reference vbn.py:37-51"""

    name: str
    params: Dict
    kind: Optional[str] = None

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, **self.params}

    def as_dict(self) -> Dict[str, Any]:
        return self.to_dict()


class ConfigNamespace(SimpleNamespace):
    def __getitem__(self, item):
        return getattr(self, item)


def _load_configs() -> ConfigNamespace:
    cats = {}
    for cat, items in _ENGINE_DEFAULTS.items():
        cats[cat] = ConfigNamespace(**{k: ConfigItem(name=k, params=dict(v), kind=cat) for k, v in items.items()})
    return ConfigNamespace(**cats)


class _Defaults:
    def inference(self, name) -> Dict:
        name = getattr(name, "name", name)
        return {"name": name, **dict(_ENGINE_DEFAULTS["inference"][name])}

    def sampling(self, name) -> Dict:
        name = getattr(name, "name", name)
        return {"name": name, **dict(_ENGINE_DEFAULTS["sampling"][name])}


defaults = _Defaults()


class _DAG:
    """Topology view with the reference StaticDAG interface (core/dags.py:23-45)."""

    def __init__(self, model: BNModel):
        self._m = model

    def nodes(self) -> List[str]:
        return list(self._m.nodes)

    def edges(self):
        return list(self._m.edges)

    def parents(self, node: str) -> List[str]:
        return list(self._m.parents.get(node, []))

    def topological_order(self) -> List[str]:
        return list(self._m.topo)


def _resolve(method, registry, kind: str, kwargs):
    if isinstance(method, dict):
        name = method.get("name") or method.get("method")
        if name is None:
            raise TypeError("method dict must include a 'name' field")
        if not isinstance(name, str):
            raise TypeError("method name must be a string")
        key = name.lower().strip()
        if key not in registry:
            raise ValueError(f"Unknown {kind} method '{name}'. Available: {list(registry.keys())}")
        base = {k: v for k, v in method.items() if k not in {"name", "method"}}
        return key, {**base, **kwargs}
    if isinstance(method, ConfigItem) or (hasattr(method, "name") and hasattr(method, "params")):
        return method.name, {**dict(method.params), **kwargs}
    if isinstance(method, str):
        key = method.lower().strip()
        if key not in registry:
            raise ValueError(f"Unknown {kind} method '{method}'. Available: {list(registry.keys())}")
        return key, dict(kwargs)
    if callable(method):
        return method, {}
    raise TypeError("method must be a string, ConfigItem, or callable")


def _local_engine(engine):
    """The engine a ShardedEngine wraps (distributed.py), else the engine itself."""
    from .distributed import ShardedEngine
    return engine.engine if isinstance(engine, ShardedEngine) else engine


class VBN:
    """Accelerated VBN: same inference/sampling surface, GPU execution."""

    def __init__(self, model: BNModel, seed: Optional[int] = None, device: Optional[str] = None):
        if device is None or str(device) == "auto":
            device = "cuda"
        self.device = torch.device(device)
        self.seed = seed
        if seed is not None:
            torch.manual_seed(seed)
        self.model = model
        self.dag = _DAG(model)
        self.nodes = model.cpds
        self.config = _load_configs()
        self._inference = None
        self._sampling = None
        self._inference_config = None
        self._sampling_config = None

    # ---- construction -------------------------------------------------------------------
    @classmethod
    def from_model(cls, model: BNModel, device: Optional[str] = None, seed: Optional[int] = None) -> "VBN":
        return cls(model, seed=seed, device=device)

    @classmethod
    def load(cls, path_or_ckpt, *, map_location: str = "cuda") -> "VBN":
        """Load a reference ``VBN.save`` checkpoint (weights_only; reference vbn.py:736-824)."""
        ckpt = load_checkpoint(path_or_ckpt) if isinstance(path_or_ckpt, str) else path_or_ckpt
        model = model_from_checkpoint(ckpt)
        seed = (ckpt.get("meta") or {}).get("seed")
        vbn = cls(model, seed=seed, device=map_location)
        cfg = ckpt.get("config") or {}
        inf = cfg.get("inference") or {}
        if inf.get("name") in INFERENCE_REGISTRY:
            vbn.set_inference_method(inf["name"], **(inf.get("params") or {}))
        smp = cfg.get("sampling") or {}
        if smp.get("name") in SAMPLING_REGISTRY:
            vbn.set_sampling_method(smp["name"], **(smp.get("params") or {}))
        return vbn

    @classmethod
    def from_reference(cls, ref_vbn, device: str = "cuda") -> "VBN":
        """Snapshot a fitted reference VBN (duck-typed; the reference is not imported)."""
        return cls(model_from_vbn(ref_vbn), seed=getattr(ref_vbn, "seed", None), device=device)

    def to_device(self, device) -> None:
        self.device = torch.device(device)

    # ---- persistence (reference vbn.py:644-734) ------------------------------------------
    def save(self, path: str, *, include_configs: bool = True, extra: Optional[dict] = None) -> None:
        """Write the reference checkpoint format: ``path`` ending in .pt/.pth/.ckpt is the
        file; otherwise a directory gets ``checkpoint.pt`` + ``meta.json``.  The reference's
        ``VBN.load`` reads it back (tests/test_model.py checks the round trip)."""
        import json
        import os
        config = None
        if include_configs:
            for label, cfg in (("inference", self._inference_config), ("sampling", self._sampling_config)):
                if cfg and cfg.get("callable"):
                    raise ValueError(f"Cannot serialize callable {label} method: {cfg.get('name')}")
            config = {"learning": None, "inference": self._inference_config,
                      "sampling": self._sampling_config, "update": None}
        ck = checkpoint_from_model(self.model, seed=self.seed, device=str(self.device), config=config, extra=extra)
        _, ext = os.path.splitext(path)
        meta_path = None
        if ext in {".pt", ".pth", ".ckpt"}:
            ck_path = path
        else:
            os.makedirs(path, exist_ok=True)
            ck_path, meta_path = os.path.join(path, "checkpoint.pt"), os.path.join(path, "meta.json")
        torch.save(ck, ck_path)
        if meta_path is not None:
            summary = {"meta": ck["meta"], "dag": ck["dag"],
                       "nodes": {k: {"cpd_key": v["cpd_key"]} for k, v in ck["nodes"].items()},
                       "config": ck.get("config")}
            with open(meta_path, "w", encoding="utf-8") as f:
                json.dump(summary, f, indent=2, default=str)

    # ---- CPD access (reference vbn.py:634-641) -------------------------------------------
    def cpd(self, node: str) -> CPDHandle:
        return CPDHandle(self, node)

    def get_cpd(self, node: str) -> CPDHandle:
        return CPDHandle(self, node)

    def get_cpds(self) -> Dict[str, CPDHandle]:
        return {node: CPDHandle(self, node) for node in self.dag.nodes()}

    # ---- configuration ------------------------------------------------------------------
    def set_inference_method(self, method, **kwargs):
        name, params = _resolve(method, INFERENCE_REGISTRY, "inference", kwargs)
        if callable(name) and not isinstance(name, str):
            self._inference = name
            self._inference_config = {"callable": True, "name": getattr(name, "__qualname__", str(name))}
            return
        self._inference = INFERENCE_REGISTRY[name](**params)
        self._inference_config = {"name": name, "params": params}

    def set_sampling_method(self, method, **kwargs):
        name, params = _resolve(method, SAMPLING_REGISTRY, "sampling", kwargs)
        if callable(name) and not isinstance(name, str):
            self._sampling = name
            self._sampling_config = {"callable": True, "name": getattr(name, "__qualname__", str(name))}
            return
        self._sampling = SAMPLING_REGISTRY[name](**params)
        self._sampling_config = {"name": name, "params": params}

    # ---- inference / sampling -----------------------------------------------------------
    def infer_posterior(self, query, **kwargs):
        if self._inference is None:
            raise RuntimeError("Call set_inference_method(...) before infer_posterior().")
        q = self._normalize_query(query)
        pdf, samples = self._inference.infer_posterior(self, q, **kwargs)
        if pdf is None:                     # ShardedEngine(gather=True) on a rank other than dst
            return None, None
        return pdf.detach(), samples.detach()

    def sample(self, query, n_samples: int = 200, **kwargs):
        if self._sampling is None:
            raise RuntimeError("Call set_sampling_method(...) before sample().")
        q = self._normalize_query(query)
        out = self._sampling.sample(self, q, n_samples=n_samples, **kwargs)
        if isinstance(out, dict):
            return {k: v.detach() for k, v in out.items()}
        return out.detach()

    def precompile(self, signatures, *, n_samples: Optional[int] = None, background: bool = False) -> Dict[str, int]:
        """Compile the plan-specialised walks (jit.py) of query signatures ahead of time, so no
        later ``infer_posterior`` / ``sample`` call of those signatures runs the interpreter or
        waits for hiprtc.  ``signatures``: iterable of dicts ``{"target": name, "evidence": names,
        "do": names}`` (names as a list or the keys of a dict; the benchmark adapter's batches
        share one signature per evidence skeleton, benchmarking/models/vbn.py:678-693).  The
        configured inference method (and, when set, the sampling method: ancestral only) builds
        each plan exactly as a call would; nothing is launched.  ``background``: start the
        compiles on background threads and return at once (jit.wait_pending() joins).
        Returns {"plans": n, "ready": n already loadable}."""
        from . import engines as E
        out = {"plans": 0, "ready": 0}
        methods = []
        if self._inference is not None:
            methods.append("infer")
        if self._sampling is not None and type(self._sampling).__name__ == "AncestralSampler":
            methods.append("sample")
        if not methods:
            raise RuntimeError("Call set_inference_method(...) or set_sampling_method(...) before precompile().")
        # the local engines build the plans: a ShardedEngine's collectives (seed broadcast,
        # gathers) and its call counter stay untouched, and an explicit seed keeps a seeded
        # engine's sequence and the global torch RNG where they were
        infer, samp = _local_engine(self._inference), _local_engine(self._sampling)
        for sig in signatures:
            names = {k: list(sig.get(k) or []) for k in ("evidence", "do")}
            q = self._normalize_query({"target": sig.get("target") or sig.get("target_feature"),
                                       "evidence": {n: torch.zeros(1, self.model.out_dim(n)) for n in names["evidence"]},
                                       "do": {n: torch.zeros(1, self.model.out_dim(n)) for n in names["do"]}})
            kw = {} if n_samples is None else {"n_samples": int(n_samples)}
            with E.precompile_mode("background" if background else "sync") as st:
                if "infer" in methods:
                    infer.infer_posterior(self, q, seed=0, **kw)
                if "sample" in methods:
                    samp.sample(self, q, n_samples=200 if n_samples is None else int(n_samples), seed=0)
            out["plans"] += st["plans"]
            out["ready"] += st["ready"]
        return out

    def pack_query(self, signature, method: str = "monte_carlo_marginalization", *, n_samples: int = 1024,
                   **method_kwargs) -> Dict[str, Any]:
        """The packed plan of one query signature for the query-level custom ops
        (``torch.ops.vbn_hip.mcm`` / ``is_lw`` / ``ancestral``, ops.py): the walk the engine
        ``method`` would launch, with its precompute variant and pre-passes.  Returns
        {"plan": int32 host tensor (vbn_hip::pack_plan), "params": the device parameter blob,
        "fixed_nodes": evidence / do node names in the order of the ``fixed`` [B, fixed_ld]
        buffer's columns, "fixed_cols": their first columns, "out_nodes": the output nodes,
        "op": the op to call}.  ``signature``: {"target": name, "evidence": names, "do": names}."""
        from . import engines as E
        from . import ops
        from .registry import INFERENCE_REGISTRY, SAMPLING_REGISTRY
        ops_of = {"monte_carlo_marginalization": "mcm", "importance_sampling": "is_lw",
                  "likelihood_weighting": "is_lw", "ancestral": "ancestral"}
        if method not in ops_of:
            raise ValueError(f"pack_query: method must be one of {sorted(ops_of)}")
        names = {k: list(signature.get(k) or []) for k in ("evidence", "do")}
        q = self._normalize_query({"target": signature.get("target"),
                                   "evidence": {n: torch.zeros(1, self.model.out_dim(n)) for n in names["evidence"]},
                                   "do": {n: torch.zeros(1, self.model.out_dim(n)) for n in names["do"]}})
        with E.precompile_mode("none") as st:
            if method == "ancestral":
                SAMPLING_REGISTRY[method](n_samples=n_samples, **method_kwargs).sample(self, q, n_samples, seed=0)
            else:
                INFERENCE_REGISTRY[method](n_samples=n_samples, **method_kwargs).infer_posterior(self, q, seed=0)
        seen = st["seen"]
        if not seen:
            raise RuntimeError("pack_query: the engine launched no walk for this signature")
        plan = seen[0]
        pk = E.packed_model(self, E._device_of(self))
        secs = [plan, plan.pc, plan.pre, plan.pre_q]
        empty = torch.zeros(0, dtype=torch.int32)
        steps, ics, ocs, meta = [], [], [], []
        for p in secs:
            if p is None:
                steps.append(empty), ics.append(empty), ocs.append(empty)
                meta += [0] * 8
                continue
            steps.append(torch.from_numpy(p.steps._vbn_host[0]))
            ics.append(torch.from_numpy(p.steps._vbn_host[1]))
            ocs.append(p.out_cols.cpu())
            meta += [p.n_slots, p.max_out, p.fixed_ld, p.mode, p.kind_mask, p.wbuf, pk.dmax, len(p.noise_nodes)]
        cols, c = [], 0
        for n in plan.fixed_nodes:
            cols.append(c)
            c += self.model.out_dim(n)
        return {"plan": ops.pack_plan(steps, ics, ocs, meta), "params": pk.params,
                "fixed_nodes": list(plan.fixed_nodes), "fixed_cols": cols, "out_nodes": list(plan.out_nodes),
                "op": ops_of[method]}

    # ---- posterior summaries (vbn.py:483-568) ---------------------------------------------
    def _posterior_stats(self, pdf: torch.Tensor, samples: torch.Tensor, *, eps: float = 1e-12
                         ) -> Dict[str, torch.Tensor]:
        """reference vbn.py:483-504, one HIP launch (vbn_hip_posterior_stats)."""
        from . import ops
        if pdf.dim() != 2:
            raise ValueError(f"Expected pdf with shape [B,S], got {tuple(pdf.shape)}")
        if samples.dim() != 3:
            raise ValueError(f"Expected samples with shape [B,S,D], got {tuple(samples.shape)}")
        if pdf.shape[0] != samples.shape[0] or pdf.shape[1] != samples.shape[1]:
            raise ValueError("pdf and samples shapes are incompatible.")
        mean, std, ess = ops.posterior_stats(pdf, samples, float(eps))
        return {"mean": mean, "std": std, "ess": ess}

    def _infer_stats(self, q, eps: float, kwargs) -> Dict[str, torch.Tensor]:
        """infer_posterior + _posterior_stats (vbn.py:536-539) with the summary fused into the
        engine's reduction where it has one: the MCM walk's epilogue partials
        (vbn_walk_args.stats_part + vbn_hip_posterior_stats_merge) or the IS / LW normalisation
        (vbn_hip_normalize_weights_stats).  Other engines, sharded engines and shapes the fused
        forms do not take (S % 64 != 0 for MCM, S > 4096 for IS / LW) run the separate pass."""
        from .engines import ImportanceSampling, LikelihoodWeighting, MonteCarloMarginalization
        if self._inference is None:
            raise RuntimeError("Call set_inference_method(...) before infer_posterior().")
        fused = (type(self._inference) in (MonteCarloMarginalization, LikelihoodWeighting, ImportanceSampling)
                 and os.environ.get("VBN_FUSED_STATS", "1") != "0")        # 0: A/B against the separate pass
        st = {"eps": float(eps)} if fused else None
        pdf, samples = self.infer_posterior(q, **kwargs, **({"_stats": st} if fused else {}))
        if st is not None and "mean" in st:
            return {"mean": st["mean"], "std": st["std"], "ess": st["ess"]}
        return self._posterior_stats(pdf, samples, eps=eps)

    @staticmethod
    def _broadcast_batch(a: torch.Tensor, b: torch.Tensor):
        """reference vbn.py:506-517"""
        if a.shape[0] == b.shape[0]:
            return a, b
        if a.shape[0] == 1:
            return a.expand(b.shape[0], *a.shape[1:]), b
        if b.shape[0] == 1:
            return a, b.expand(a.shape[0], *b.shape[1:])
        raise ValueError("Query and reference batch sizes must match, unless one of them is 1.")

    def infer_relative(self, query, reference_query=None, *, eps: float = 1e-12, **kwargs):
        """reference vbn.py:519-568: posterior of ``query`` relative to ``reference_query``
        (default: the same target without evidence)."""
        q = self._normalize_query(query)
        if reference_query is None:
            reference_query = Query(target=q.target, evidence={}, do={})
        rq = self._normalize_query(reference_query)
        if rq.target != q.target:
            raise ValueError("query and reference_query must have the same target node.")
        qst = self._infer_stats(q, eps, kwargs)
        rst = self._infer_stats(rq, eps, kwargs)
        q_mean, r_mean = self._broadcast_batch(qst["mean"], rst["mean"])
        q_std, r_std = self._broadcast_batch(qst["std"], rst["std"])
        q_ess, r_ess = self._broadcast_batch(qst["ess"], rst["ess"])
        d_mean = q_mean - r_mean
        d_std = q_std - r_std
        return {
            "target": q.target,
            "query_stats": {"mean": q_mean, "std": q_std, "effective_sample_size": q_ess},
            "reference_stats": {"mean": r_mean, "std": r_std, "effective_sample_size": r_ess},
            "delta_mean": d_mean,
            "delta_std": d_std,
            "relative_mean_change": d_mean / r_mean.abs().clamp_min(eps),
            "relative_std_change": d_std / r_std.abs().clamp_min(eps),
        }

    def _tensor(self, v) -> torch.Tensor:
        t = v.to(device=self.device, dtype=torch.float32) if isinstance(v, torch.Tensor) else \
            torch.tensor(v, device=self.device, dtype=torch.float32)
        if t.dim() == 1:
            return t.unsqueeze(-1)
        if t.dim() == 2:
            return t
        raise ValueError(f"Expected 1D or 2D tensor, got shape {tuple(t.shape)}")

    def _normalize_query(self, query) -> Query:
        """reference vbn.py:579-618 (same checks, same messages)."""
        if isinstance(query, dict):
            target = query.get("target") or query.get("target_feature")
            if target is None:
                raise ValueError("query must contain 'target'")
            ev_src = query.get("evidence") or {}
            do_src = query.get("do") or {}
        elif hasattr(query, "target") and hasattr(query, "evidence"):
            target, ev_src, do_src = query.target, query.evidence or {}, getattr(query, "do", None) or {}
        else:
            raise TypeError("query must be a dict or Query")
        evidence = {k: self._tensor(v) for k, v in ev_src.items()}
        do = {k: self._tensor(v) for k, v in do_src.items()}
        nodes = set(self.model.nodes)
        if target not in nodes:
            raise ValueError(f"Unknown target node '{target}'.")
        unknown = (set(evidence) | set(do)) - nodes
        if unknown:
            raise ValueError(f"Unknown query nodes: {sorted(unknown)}")
        overlap = set(evidence) & set(do)
        if overlap:
            raise ValueError(f"Nodes cannot be in both evidence and do: {sorted(overlap)}")
        infer_batch_size(evidence, do)
        return Query(target=target, evidence=evidence, do=do)
