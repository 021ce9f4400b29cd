"""Per-node CPD ``sample`` / ``log_prob`` on the GPU (reference ``BaseCPD`` contract,
``core/base.py:45-59``), implemented as single-node walks: the node's parents are fixed
inputs, the node is sampled (``sample``) or scored (``log_prob``), everything else skipped.

Shapes follow the reference: ``sample(parents [B,d] | None, S) -> [B|1, S, D]``,
``log_prob(x [B,D] | [B,S,D], parents [B,d] | [B,S,d] | None) -> [B, S]``.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .engines import _device_of, _next_seed, packed_model, run_walk
from .plan import MODE_SAMPLE, MODE_WEIGHTED, build_plan

__all__ = ["cpd_sample", "cpd_log_prob"]


def _split_parents(model, node: str, parents: torch.Tensor) -> Dict[str, torch.Tensor]:
    out, c = {}, 0
    for p in model.parents[node]:
        d = model.out_dim(p)
        out[p] = parents[..., c:c + d]
        c += d
    if c != parents.shape[-1]:
        raise ValueError(f"Expected parents_dim {c}, got {parents.shape[-1]}")
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
