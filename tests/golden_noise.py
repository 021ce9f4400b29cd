"""Turn a golden fixture's recorded reference draws into the kernel's injected-noise input.

Each recorded draw carries the node that made it and its phase (0 = main pass, 1 = the IS
-> LW fallback pass).  Per node, index/categorical uniforms go to slot 0 and normal /
within-bin uniform draws to slot 1, in call order (per-query calls of IS and KDE's 512-row
chunks concatenate in particle order).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch


def noise_dict(case: dict, model, phase: int = 0) -> Dict[str, Tuple[torch.Tensor, torch.Tensor]]:
    S = int(case["n_samples"])
    if case["engine"] == "rao_blackwellized_marginalization" and phase == 0:
        S = int(case["params"]["n_particles"])        # the RB walk runs over the particles
    slots: Dict[str, Dict[int, list]] = {}
    for r in case["draws"]:
        if r["phase"] != phase or r["node"] is None:       # node None: engine-level draws
            continue
        slot = 0 if r["kind"] in ("cat", "randint") else 1
        slots.setdefault(r["node"], {0: [], 1: []})[slot].append(r["value"].float())
    out = {}
    for node, sl in slots.items():
        D = model.out_dim(node)
        per_dim0 = model.cpds[node].kind == "softmax_nn"
        s0 = s1 = None
        if sl[1]:
            v = torch.cat(sl[1])
            s1 = v.view(v.numel() // (S * D), S, D)
        if sl[0]:
            v = torch.cat(sl[0])
            s0 = v.view(v.numel() // (S * D), S, D) if per_dim0 else v.view(v.numel() // S, S)
        out[node] = (s0, s1)
    return out


def resample_uniforms(case: dict):
    """The engine-level multinomial resampling draws (node None), in order: list of [B, S]."""
    S = int(case["n_samples"])
    return [r["value"].float().view(-1, S) for r in case["draws"] if r["node"] is None and r["kind"] == "cat"]
