"""Model records: the reference's per-node CPD state in a plain, tensor-only form.

The accelerated path never imports the reference. It consumes either

* a reference checkpoint written by ``VBN.save`` (reference ``vbn/vbn.py:644-734``; one
  ``{dag, nodes, meta, ...}`` dict whose per-node entries carry ``cpd_key, input_dim,
  output_dim, init_kwargs, state_dict, extra_state``), loaded with
  ``torch.load(weights_only=True)`` so nothing in the file executes; or
* a live fitted reference ``VBN`` object, read duck-typed through ``vbn.dag`` and each
  CPD's ``state_dict()`` / ``get_init_kwargs()`` / ``get_extra_state()``
  (reference ``core/base.py:66-81``); or
* :func:`random_init_model`, which builds random-init weights of the reference
  architectures (the bench's synthetic models).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Mapping, Optional, Sequence, Tuple

import networkx as nx
import torch

__all__ = [
    "CPD_KINDS",
    "CPDRecord",
    "BNModel",
    "load_checkpoint",
    "model_from_checkpoint",
    "model_from_vbn",
    "record_from_cpd",
    "random_init_model",
    "checkpoint_from_model",
    "KIND_DEFAULTS",
]

# Registry keys of the reference CPDs on the hot path (reference core/registry.py + cpds/*).
CPD_KINDS = ("gaussian_nn", "linear_gaussian", "mdn", "kde", "softmax_nn")

_CLASS_TO_KIND = {
    "GaussianNNCPD": "gaussian_nn",
    "LinearGaussianCPD": "linear_gaussian",
    "MDNCPD": "mdn",
    "KDECPD": "kde",
    "SoftmaxNNCPD": "softmax_nn",
}

# Constructor defaults of the reference classes (gaussian_nn.py:41-50, linear_gaussian.py:14-22,
# mdn.py:41-51, kde.py:17-27, softmax_nn.py:52-71).  Values that a checkpoint carries in
# ``init_kwargs`` override these.
KIND_DEFAULTS: Dict[str, Dict[str, Any]] = {
    "gaussian_nn": dict(hidden_dims=(32, 32), activation="relu", min_scale=1e-3),
    "linear_gaussian": dict(ridge=1e-6, min_scale=1e-3),
    "mdn": dict(n_components=5, hidden_dims=(32, 32), activation="relu", min_scale=1e-3),
    "kde": dict(bandwidth=1.0, parent_bandwidth=None, max_points=1000, min_scale=1e-3),
    "softmax_nn": dict(n_classes=8, hidden_dims=(32, 32), activation="relu",
                       min_bin_width=1e-12, binning="uniform", within_bin="uniform",
                       within_bin_scale=0.25, within_bin_clip=False,
                       mode_when_not_discrete="binned"),
}

# The packaged YAML defaults the reference's ``defaults.cpd(kind)`` returns
# (reference vbn/configs/cpds/*.yaml); used by :func:`random_init_model`.
YAML_DEFAULTS: Dict[str, Dict[str, Any]] = {
    "gaussian_nn": dict(hidden_dims=(32, 32), activation="relu", min_scale=1e-4),
    "linear_gaussian": dict(ridge=1e-6, min_scale=1e-4),
    "mdn": dict(n_components=5, hidden_dims=(32, 32), activation="relu", min_scale=1e-4),
    "kde": dict(bandwidth=0.5, parent_bandwidth=0.5, max_points=4096, min_scale=1e-4),
    "softmax_nn": dict(n_classes=8, hidden_dims=(32, 32), activation="relu",
                       min_bin_width=1e-12, binning="quantile", within_bin="triangular"),
}


def _as_float(v: Any) -> Any:
    # YAML loads "1e-4" as a string; coerce like reference config_cast.py:28-42.
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return v
    return v


@dataclass
class CPDRecord:
    """One node's CPD: registry key, dims, hyper-parameters and tensors (CPU, as saved)."""

    kind: str
    input_dim: int
    output_dim: int
    hparams: Dict[str, Any]
    state: Dict[str, torch.Tensor]
    extra: Optional[Dict[str, Any]] = None

    def hp(self, name: str) -> Any:
        if name in self.hparams:
            return _as_float(self.hparams[name])
        return KIND_DEFAULTS[self.kind].get(name)

    def mlp_layers(self) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        """(weight [out,in], bias [out]) of ``net`` in order (reference gaussian_nn.py:16-34)."""
        idx = sorted({int(k.split(".")[1]) for k in self.state if k.startswith("net.")})
        return [(self.state[f"net.{i}.weight"], self.state[f"net.{i}.bias"]) for i in idx]

    @property
    def is_root(self) -> bool:
        return self.input_dim == 0


@dataclass
class BNModel:
    """DAG + CPD records.  ``topo`` and ``parents`` fix RNG order and parent-concat order
    (reference core/dags.py:30-33, vbn.py:670-675)."""

    nodes: List[str]
    edges: List[Tuple[str, str]]
    topo: List[str]
    parents: Dict[str, List[str]]
    cpds: Dict[str, CPDRecord]
    version: int = 0
    _cache: Dict[Any, Any] = field(default_factory=dict, repr=False)

    def out_dim(self, node: str) -> int:
        return int(self.cpds[node].output_dim)

    def children(self) -> Dict[str, List[str]]:
        ch: Dict[str, List[str]] = {n: [] for n in self.topo}
        for p, c in self.edges:
            ch[p].append(c)
        return ch

    def bump(self) -> None:
        """Invalidate packed device plans after an in-place parameter change."""
        self.version += 1
        self._cache.clear()


def load_checkpoint(path: str, map_location: str = "cpu") -> Dict[str, Any]:
    """Load a reference ``VBN.save`` checkpoint safely (no pickled code is executed)."""
    import os

    _, ext = os.path.splitext(path)
    if ext not in {".pt", ".pth", ".ckpt"}:
        path = os.path.join(path, "checkpoint.pt")
    return torch.load(path, map_location=map_location, weights_only=True)


def _state_to_cpu(state: Mapping[str, Any]) -> Dict[str, torch.Tensor]:
    out: Dict[str, torch.Tensor] = {}
    for k, v in state.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.detach().to("cpu")
    return out


def _extra_to_cpu(extra: Any) -> Optional[Dict[str, Any]]:
    if not isinstance(extra, Mapping):
        return None
    return {k: (v.detach().to("cpu") if isinstance(v, torch.Tensor) else v)
            for k, v in extra.items()}


def model_from_checkpoint(ckpt: Mapping[str, Any] | str) -> BNModel:
    """Build a :class:`BNModel` from a reference checkpoint dict (reference vbn.py:664-712)."""
    if isinstance(ckpt, str):
        ckpt = load_checkpoint(ckpt)
    dag = ckpt["dag"]
    nodes_state = ckpt["nodes"]
    cpds: Dict[str, CPDRecord] = {}
    for node, info in nodes_state.items():
        kind = str(info["cpd_key"]).lower().strip()
        if kind not in CPD_KINDS:
            raise ValueError(
                f"CPD '{kind}' of node '{node}' is not on the accelerated path "
                f"(supported: {list(CPD_KINDS)})")
        state = dict(info.get("state_dict") or {})
        extra = info.get("extra_state")
        if extra is None:
            extra = state.get("_extra_state")
        cpds[node] = CPDRecord(
            kind=kind,
            input_dim=int(info.get("input_dim", 0)),
            output_dim=int(info.get("output_dim", 1)),
            hparams=dict(info.get("init_kwargs") or {}),
            state=_state_to_cpu(state),
            extra=_extra_to_cpu(extra),
        )
    parents = {n: list(p) for n, p in dag["parents"].items()}
    return BNModel(
        nodes=list(dag["nodes"]),
        edges=[tuple(e) for e in dag["edges"]],
        topo=list(dag["topological_order"]),
        parents=parents,
        cpds=cpds,
    )


CLASS_NAME = {v: k for k, v in _CLASS_TO_KIND.items()}


def checkpoint_from_model(model: BNModel, *, seed: Optional[int] = None, device: str = "cpu",
                          config: Optional[Dict[str, Any]] = None, extra: Optional[dict] = None,
                          version: str = "0.3.0") -> Dict[str, Any]:
    """The reference ``VBN.save`` checkpoint dict (reference vbn/vbn.py:644-734) of ``model``:
    ``{dag, nodes, meta, extra[, config]}`` with per-node ``cpd_key, class_name, input_dim,
    output_dim, seed, init_kwargs, state_dict, extra_state`` in topological order; every
    ``state_dict`` carries the ``_extra_state`` entry BaseCPD adds (core/base.py:75-81), so the
    reference's strict ``load_state_dict`` accepts it.  Tensors and builtins only."""
    nodes_state: Dict[str, Dict[str, Any]] = {}
    dtype = "torch.float32"
    for node in model.topo:
        rec = model.cpds[node]
        extra_state = None
        if rec.kind == "kde":
            extra_state = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in (rec.extra or {}).items()}
        sd = {k: v.clone() for k, v in rec.state.items()}
        sd["_extra_state"] = extra_state
        nodes_state[node] = {
            "cpd_key": rec.kind,
            "class_name": CLASS_NAME[rec.kind],
            "input_dim": int(rec.input_dim),
            "output_dim": int(rec.output_dim),
            "seed": seed,
            "init_kwargs": {k: (tuple(v) if isinstance(v, list) else v) for k, v in rec.hparams.items()},
            "state_dict": sd,
            "extra_state": extra_state,
        }
    ck: Dict[str, Any] = {
        "dag": {"nodes": list(model.nodes), "edges": [tuple(e) for e in model.edges],
                "topological_order": list(model.topo),
                "parents": {n: list(model.parents.get(n, [])) for n in model.nodes}},
        "nodes": nodes_state,
        "meta": {"vbn_version": version, "torch_version": str(torch.__version__), "dtype": dtype,
                 "device": str(device), "seed": seed},
        "extra": extra,
    }
    if config is not None:
        ck["config"] = config
    return ck


def record_from_cpd(cpd: Any, kind: Optional[str] = None) -> CPDRecord:
    """Read a live reference CPD module duck-typed (no reference import)."""
    if kind is None:
        kind = _CLASS_TO_KIND.get(type(cpd).__name__)
    if kind is None:
        raise ValueError(f"CPD class '{type(cpd).__name__}' is not on the accelerated path")
    init_kwargs = cpd.get_init_kwargs() if hasattr(cpd, "get_init_kwargs") else {}
    extra = _extra_of(cpd)
    return CPDRecord(
        kind=kind,
        input_dim=int(cpd.input_dim),
        output_dim=int(cpd.output_dim),
        hparams=dict(init_kwargs or {}),
        state=_state_to_cpu(cpd.state_dict()),
        extra=_extra_to_cpu(extra),
    )


def _extra_of(cpd: Any) -> Any:
    """BaseCPD.get_extra_state (core/base.py:75-77); a bare nn.Module's default raises."""
    fn = getattr(cpd, "get_extra_state", None)
    if fn is None:
        return None
    try:
        return fn()
    except RuntimeError:
        return None


def _tensor_fingerprint(cpd: Any) -> Tuple:
    fp = []
    for t in cpd.state_dict(keep_vars=True).values():
        if isinstance(t, torch.Tensor):
            fp.append((t.data_ptr(), t._version))
    extra = _extra_of(cpd)
    if isinstance(extra, Mapping):
        for v in extra.values():
            if isinstance(v, torch.Tensor):
                fp.append((v.data_ptr(), v._version))
    return tuple(fp)


def model_from_vbn(vbn: Any) -> BNModel:
    """Snapshot a live VBN object (reference or ours) into a :class:`BNModel`.

    The snapshot is cached on the object and keyed by a fingerprint of every CPD tensor
    (data pointer + in-place version counter) so that ``fit``/``update`` invalidate it,
    which the reference's own topology cache does not do (reference inference/_core.py:27-33).
    """
    if isinstance(getattr(vbn, "model", None), BNModel):
        return vbn.model
    dag = vbn.dag
    topo = list(dag.topological_order())
    key = tuple((n, id(vbn.nodes[n]), _tensor_fingerprint(vbn.nodes[n])) for n in topo)
    cached = getattr(vbn, "_vbn_amd_model", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    model = BNModel(
        nodes=list(dag.nodes()),
        edges=[tuple(e) for e in dag.edges()],
        topo=topo,
        parents={n: list(dag.parents(n)) for n in dag.nodes()},
        cpds={n: record_from_cpd(vbn.nodes[n]) for n in topo},
    )
    try:
        vbn._vbn_amd_model = (key, model)
    except AttributeError:
        pass
    return model


# ----------------------------------------------------------------------------------------
# Random-init models of the reference architectures (bench / synthetic workloads).
# ----------------------------------------------------------------------------------------

def _linear(in_dim: int, out_dim: int, gen: torch.Generator) -> Tuple[torch.Tensor, torch.Tensor]:
    # nn.Linear default init: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias.
    bound = 1.0 / math.sqrt(in_dim) if in_dim > 0 else 0.0
    w = (torch.rand(out_dim, in_dim, generator=gen) * 2 - 1) * bound
    b = (torch.rand(out_dim, generator=gen) * 2 - 1) * bound
    return w, b


def _mlp_state(in_dim: int, hidden: Sequence[int], out_dim: int,
               gen: torch.Generator) -> Dict[str, torch.Tensor]:
    state: Dict[str, torch.Tensor] = {}
    last = in_dim
    for i, h in enumerate(list(hidden) + [out_dim]):
        w, b = _linear(last, h, gen)
        state[f"net.{2 * i}.weight"] = w
        state[f"net.{2 * i}.bias"] = b
        last = h
    return state


def _std(x: torch.Tensor) -> torch.Tensor:
    return x.std(dim=0, unbiased=False).clamp_min(1e-6)


def random_init_model(g: nx.DiGraph, kinds: Mapping[str, str], data: Mapping[str, torch.Tensor],
                      seed: int = 0, overrides: Optional[Mapping[str, Dict[str, Any]]] = None
                      ) -> BNModel:
    """Random-init CPDs of the reference architectures with data-derived buffers.

    Weights are random (nn.Linear init); the data-dependent buffers the reference derives in
    ``fit`` (standardisation stats, bin edges, KDE point sets, ridge solution) are derived from
    ``data`` the same way, so shapes, value ranges and sampling behaviour match a fitted model.
    """
    gen = torch.Generator().manual_seed(seed)
    topo = list(nx.topological_sort(g))
    parents = {n: list(g.predecessors(n)) for n in g.nodes}
    cpds: Dict[str, CPDRecord] = {}
    for node in topo:
        kind = kinds[node]
        hp = dict(YAML_DEFAULTS[kind])
        if overrides and node in overrides:
            hp.update(overrides[node])
        elif overrides and kind in overrides:
            hp.update(overrides[kind])
        x = data[node].float()
        par = torch.cat([data[p].float() for p in parents[node]], dim=-1) if parents[node] else None
        d_in = 0 if par is None else par.shape[1]
        d_out = x.shape[1]
        state: Dict[str, torch.Tensor] = {}
        extra = None
        if kind == "gaussian_nn":
            state["mean_x"] = par.mean(0) if par is not None else torch.zeros(0)
            state["std_x"] = _std(par) if par is not None else torch.ones(0)
            state["mean_y"] = x.mean(0)
            state["std_y"] = _std(x)
            state["_stats_ready"] = torch.tensor(True)
            if d_in == 0:
                state["_loc"] = torch.randn(d_out, generator=gen) * 0.1
                state["_log_scale"] = torch.randn(d_out, generator=gen) * 0.1
            else:
                state.update(_mlp_state(d_in, hp["hidden_dims"], 2 * d_out, gen))
        elif kind == "linear_gaussian":
            if d_in == 0:
                state["_weight"] = torch.zeros(0, d_out)
                state["_bias"] = x.mean(0)
                state["_var"] = _std(x) ** 2
            else:
                xa = torch.cat([par, torch.ones(par.shape[0], 1)], dim=1)
                theta = torch.linalg.lstsq(xa, x).solution
                state["_weight"] = theta[:-1].contiguous()
                state["_bias"] = theta[-1].contiguous()
                state["_var"] = (x - xa @ theta).var(dim=0).clamp_min(1e-6)
        elif kind == "mdn":
            k = int(hp["n_components"])
            if d_in == 0:
                state["_logits"] = torch.randn(k, generator=gen) * 0.1
                state["_loc"] = torch.randn(k, d_out, generator=gen)
                state["_log_scale"] = torch.randn(k, d_out, generator=gen) * 0.1
            else:
                state.update(_mlp_state(d_in, hp["hidden_dims"], k * (2 * d_out) + k, gen))
        elif kind == "kde":
            m = int(hp["max_points"])
            n = x.shape[0]
            idx = torch.randperm(n, generator=gen)[:m] if n > m else torch.arange(n)
            extra = {
                "parents": (par[idx] if par is not None else torch.zeros(len(idx), 0)).contiguous(),
                "targets": x[idx].contiguous(),
            }
        elif kind == "softmax_nn":
            c = int(hp["n_classes"])
            q = torch.linspace(0.0, 1.0, c + 1)
            vmin, vmax = x.amin(0), x.amax(0)
            if hp.get("binning", "quantile") == "quantile":
                edges = torch.quantile(x, q, dim=0).transpose(0, 1).contiguous()
            else:
                width = (vmax - vmin) / float(c)
                edges = vmin[:, None] + width[:, None] * q[None, :]
            edges[:, 0] = vmin
            edges[:, -1] = vmax
            centers = 0.5 * (edges[:, :-1] + edges[:, 1:])
            state.update({
                "_vmin": vmin, "_vmax": vmax, "_bin_edges": edges, "_bin_centers": centers,
                "_class_values": torch.zeros(d_out, c), "_sample_values": centers.clone(),
                "_is_discrete": torch.zeros(d_out, dtype=torch.bool),
                "_n_classes": torch.tensor(c), "_binning_id": torch.tensor(2),
                "_bins_ready": torch.tensor(True),
            })
            if d_in == 0:
                bins = ((x.unsqueeze(-1) >= edges.unsqueeze(0)).sum(-1) - 1).clamp(0, c - 1)
                counts = torch.nn.functional.one_hot(bins[:, 0], c).float().sum(0)
                probs = counts / counts.sum().clamp_min(1.0)
                state["_logits"] = torch.zeros(d_out, c)
                state["_root_log_probs"] = torch.log(probs.clamp_min(1e-12)).view(1, c).repeat(d_out, 1)
                state["_root_ready"] = torch.tensor(True)
            else:
                state["_root_log_probs"] = torch.zeros(d_out, c)
                state["_root_ready"] = torch.tensor(False)
                state.update(_mlp_state(d_in, hp["hidden_dims"], d_out * c, gen))
        else:
            raise ValueError(kind)
        cpds[node] = CPDRecord(kind=kind, input_dim=d_in, output_dim=d_out, hparams=hp,
                               state=state, extra=extra)
    return BNModel(nodes=list(g.nodes), edges=list(g.edges), topo=topo, parents=parents, cpds=cpds)
