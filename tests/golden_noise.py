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


def gibbs_noise(case: dict, model, latent, dmax: int):
    """Recorded draws of a Gibbs fixture -> (initial-walk noise dict, sweep noise tensor).

    Phase 0 is the initial ancestral draw (S = 1); phase 1 holds, per sweep and latent node,
    the node's 8-candidate draws then the chain choice (a ``cat`` record with node None,
    whose CDF midpoint is the injected uniform).  Sweep layout [iters, 2L, 2, B, 8, dmax]:
    candidate draws at index 2j, the choice uniform at 2j + 1 (slot 0, candidate 0, dim 0).
    """
    init = noise_dict({**case, "n_samples": 1, "draws": [r for r in case["draws"] if r["phase"] == 0]}, model, 0)
    B = int(next(iter(case["query"]["evidence"].values())).shape[0]) if case["query"]["evidence"] else 1
    if case["query"]["do"]:
        B = int(next(iter(case["query"]["do"].values())).shape[0])
    thin = max(int(case["params"]["n_steps"]), 1)
    iters = int(case["params"]["burn_in"]) + int(case["n_samples"]) * thin
    L = len(latent)
    out = torch.zeros(iters, max(2 * L, 1), 2, B, 8, dmax)
    recs = [r for r in case["draws"] if r["phase"] == 1]
    pos = 0
    for it in range(iters):
        for j, node in enumerate(latent):
            D = model.out_dim(node)
            per_dim0 = model.cpds[node].kind == "softmax_nn"
            while recs[pos]["node"] == node:
                r = recs[pos]
                pos += 1
                v = r["value"].float()
                bq = v.numel() // (8 * D) if (r["kind"] not in ("cat", "randint") or per_dim0) else v.numel() // 8
                if r["kind"] in ("cat", "randint"):
                    vv = v.view(bq, 8, D) if per_dim0 else v.view(bq, 8, 1)
                    out[it, 2 * j, 0, :, :, :vv.shape[-1]] = vv.expand(B, 8, vv.shape[-1])
                else:
                    out[it, 2 * j, 1, :, :, :D] = v.view(bq, 8, D).expand(B, 8, D)
            r = recs[pos]
            pos += 1
            assert r["node"] is None and r["kind"] == "cat", r["kind"]
            out[it, 2 * j + 1, 0, :, 0, 0] = r["value"].float().view(-1).expand(B)
    assert pos == len(recs)
    return init, out


def tie_mask(case: dict, model, b: int, s: int, width_tol: float, phase: int = 0):
    """[b, s] particles whose recorded categorical choice (mdn component, softmax_nn class, KDE
    point) had a CDF interval narrower than ``width_tol`` (make_golden_large.py records the
    width): fp32 probabilities may legitimately pick a neighbour there.  None if the fixture
    records no widths."""
    per_node: Dict[str, list] = {}
    for r in case["draws"]:
        if r["phase"] != phase or r["node"] is None or r["kind"] != "cat" or "width" not in r:
            continue
        per_node.setdefault(r["node"], []).append(r["width"].float())
    if not per_node:
        return None
    mask = torch.zeros(b, s, dtype=torch.bool)
    for node, ws in per_node.items():
        w = torch.cat(ws)
        dc = model.out_dim(node) if model.cpds[node].kind == "softmax_nn" else 1
        narrow = (w < width_tol).view(-1, s, dc).any(-1)          # [b | 1, s]
        mask |= narrow.expand(b, s) if narrow.shape[0] == 1 else narrow
    return mask
