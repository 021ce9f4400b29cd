"""Per-node CPD ``sample`` / ``log_prob`` / ``forward`` / conditional parameters on the GPU
(reference ``BaseCPD`` contract, ``core/base.py:45-59``; ``CPDHandle``,
``core/cpd_handle.py:40-118``), implemented as single-node walks: the node's parents are
fixed inputs, the node is sampled (``sample``), scored (``log_prob``), both in one launch
(``forward``), or writes its conditional parameters (``params``, the walk's PARAMS role);
everything else is skipped.

Shapes follow the reference: ``sample(parents [B,d] | None, S) -> [B|1, S, D]``,
``log_prob(x [B,D] | [B,S,D], parents [B,d] | [B,S,d] | None) -> [B, S]``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from .engines import _device_of, _next_seed, packed_model, run_walk
from .plan import MODE_SAMPLE, MODE_WEIGHTED, build_plan

__all__ = ["CPDOutput", "cpd_sample", "cpd_log_prob", "cpd_forward", "cpd_params"]


@dataclass
class CPDOutput:
    """reference core/base.py:11-15"""

    samples: torch.Tensor
    log_prob: torch.Tensor
    pdf: torch.Tensor


def _split_parents(model, node: str, parents: torch.Tensor) -> Dict[str, torch.Tensor]:
    out, c = {}, 0
    for p in model.parents[node]:
        d = model.out_dim(p)
        out[p] = parents[..., c:c + d]
        c += d
    if c != parents.shape[-1]:
        raise ValueError(f"Expected parents_dim {c}, got {parents.shape[-1]}")
    return out


def _parent_inputs(pk, node: str, parents: Optional[torch.Tensor], plan, n: int, dev
                   ) -> Tuple[int, torch.Tensor, bool]:
    """(batch, fixed buffer, per-particle?) of a single-node walk over ``parents``."""
    model = pk.model
    pa = model.parents[node]
    if not pa:
        b = 1 if parents is None else int(parents.shape[0])
        return b, torch.zeros(b, 1, device=dev), False
    parents = parents.to(dev, torch.float32)
    b = int(parents.shape[0])
    per_particle = parents.dim() == 3
    if per_particle and parents.shape[1] != n:
        raise ValueError("3-D parents must have n_samples rows per query")
    vals = _split_parents(model, node, parents.reshape(-1, parents.shape[-1]))
    return b, torch.cat([vals[p] for p in plan.fixed_nodes], dim=1).contiguous(), per_particle


def _node_plan(pk, node: str, key: str, **kw):
    ck = ("cpd-plan", node, key)
    plan = pk.model._cache.get(ck)
    if plan is None:
        model = pk.model
        pa = model.parents[node]
        plan = build_plan(pk, fixed=[p for p in model.topo if p in pa], shared_roots=False,
                          skip=[x for x in model.topo if x != node and x not in pa], **kw)
        pk.model._cache[ck] = plan
    return plan


def cpd_forward(vbn, node: str, parents: Optional[torch.Tensor], n_samples: int, *,
                seed: Optional[int] = None, _noise=None) -> CPDOutput:
    """BaseCPD.forward (core/base.py:55-59): sample, log_prob of the sample, pdf -- one walk
    that draws the node and scores the draw in the same step."""
    dev = _device_of(vbn)
    pk = packed_model(vbn, dev)
    pa = pk.model.parents[node]
    if pa and parents is None:
        raise ValueError("parents cannot be None when input_dim > 0")
    n = int(n_samples)
    plan = _node_plan(pk, node, "forward", latent=[node], logp=[node], out_nodes=[node], mode=MODE_WEIGHTED)
    b, fx, per_particle = _parent_inputs(pk, node, parents, plan, n, dev)
    lp, xs = run_walk(pk, plan, fx, b, n, seed=_next_seed() if seed is None else seed, noise=_noise,
                      fixed_per_particle=per_particle)
    return CPDOutput(samples=xs, log_prob=lp, pdf=torch.exp(lp))


def cpd_params(vbn, node: str, parents: Optional[torch.Tensor], n_rows: int = 1) -> torch.Tensor:
    """The node's conditional parameters per parent row (walk role PARAMS): ``[B, n_rows, W]``
    with gaussian_nn / linear_gaussian ``loc[D] ++ scale[D]``, softmax_nn class
    probabilities ``[D][C]``, mdn ``softmax(logits)[K] ++ loc[K][D] ++ scale[K][D]``.
    ``parents``: [B, d] (n_rows = 1), [B, n_rows, d], or None for a root (B = 1)."""
    dev = _device_of(vbn)
    pk = packed_model(vbn, dev)
    pa = pk.model.parents[node]
    if pa and parents is None:
        raise ValueError("parents cannot be None when input_dim > 0")
    n = int(parents.shape[1]) if (parents is not None and parents.dim() == 3) else int(n_rows)
    plan = _node_plan(pk, node, "params", latent=[], logp=[], params=[node], out_nodes=[node], mode=MODE_SAMPLE)
    b, fx, per_particle = _parent_inputs(pk, node, parents, plan, n, dev)
    _, out = run_walk(pk, plan, fx, b, n, seed=0, fixed_per_particle=per_particle)
    return out


def cpd_sample(vbn, node: str, parents: Optional[torch.Tensor], n_samples: int, *,
               seed: Optional[int] = None, _noise=None) -> torch.Tensor:
    dev = _device_of(vbn)
    pk = packed_model(vbn, dev)
    model = pk.model
    pa = model.parents[node]
    if pa and parents is None:
        raise ValueError("parents cannot be None when input_dim > 0")
    n = int(n_samples)
    plan = build_plan(pk, latent=[node], fixed=[p for p in model.topo if p in pa], logp=[],
                      out_nodes=[node], shared_roots=False, mode=MODE_SAMPLE,
                      skip=[x for x in model.topo if x != node and x not in pa])
    if not pa:
        b = 1 if parents is None else int(parents.shape[0])
        fx = torch.zeros(b, 1, device=dev)
        per_particle = False
    else:
        parents = parents.to(dev, torch.float32)
        b = int(parents.shape[0])
        per_particle = parents.dim() == 3
        if per_particle and parents.shape[1] != n:
            raise ValueError("3-D parents must have n_samples rows per query")
        vals = _split_parents(model, node, parents.reshape(-1, parents.shape[-1]))
        fx = torch.cat([vals[p] for p in plan.fixed_nodes], dim=1).contiguous()
    _, xs = run_walk(pk, plan, fx, b, n, seed=_next_seed() if seed is None else seed, noise=_noise,
                     fixed_per_particle=per_particle)
    return xs


def cpd_log_prob(vbn, node: str, x: torch.Tensor, parents: Optional[torch.Tensor]) -> torch.Tensor:
    dev = _device_of(vbn)
    pk = packed_model(vbn, dev)
    model = pk.model
    pa = model.parents[node]
    if pa and parents is None:
        raise ValueError("parents cannot be None when input_dim > 0")
    x = x.to(dev, torch.float32)
    if x.dim() == 1:
        x = x.unsqueeze(-1)
    if x.dim() == 2:
        x = x.unsqueeze(1)
    b, s, d = x.shape
    vals = {node: x.reshape(b * s, d)}
    if pa:
        parents = parents.to(dev, torch.float32)
        if parents.dim() == 2:
            parents = parents.unsqueeze(1).expand(-1, s, -1)
        vals.update(_split_parents(model, node, parents.reshape(b * s, -1)))
    plan = build_plan(pk, latent=[], fixed=[p for p in model.topo if p in pa or p == node], logp=[node],
                      out_nodes=[], shared_roots=False, mode=MODE_WEIGHTED,
                      skip=[q for q in model.topo if q != node and q not in pa])
    fx = torch.cat([vals[p] for p in plan.fixed_nodes], dim=1).contiguous()
    lp, _ = run_walk(pk, plan, fx, b, s, seed=0, fixed_per_particle=True)
    return lp
