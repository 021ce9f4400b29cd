#!/usr/bin/env python3
"""Diagnostic (GPU box): interpreter vs plan-specialised walk on cfg3 IS, with and without the
split-f16 MFMA head (VBN_F_HEAD_MFMA cleared on the host for every step), and per kind which
steps differ (single-step plans)."""
from __future__ import annotations

import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from workloads import synthetic_workload
    from vectorizedbayesiannetwork_amd import engines as E, plan as P
    from vectorizedbayesiannetwork_amd.engines import Query
    model, vbn, target, ev = synthetic_workload("cfg3", 8, "cuda")
    q = Query(target, {k: v.cuda() for k, v in ev.items()})

    def run(pj, seed=4242):
        eng = E.ImportanceSampling(n_samples=1024, plan_jit=pj)
        out = eng.infer_posterior(vbn, q, seed=seed)
        torch.cuda.synchronize()
        return [o.clone() for o in out]

    def cmp(tag, a, b):
        for i, (x, y) in enumerate(zip(a, b)):
            d = (x - y).abs()
            nd = int((x != y).sum())
            print(f"{tag} out{i}: differing {nd}/{x.numel()} max|d| {float(d.max()):.3e} "
                  f"max rel {float((d / y.abs().clamp_min(1e-30)).max()):.3e}", flush=True)

    a, b = run(False), run(True)
    cmp("with MFMA head", a, b)
    # clear VBN_F_HEAD_MFMA in every cached plan (both forms then run the VALU head)
    import dataclasses
    import hashlib
    pk = E.packed_model(vbn, torch.device("cuda", 0))
    n = 0
    for key, pl in list(pk.model._cache.items()):
        if isinstance(pl, P.QueryPlan):
            rows = pl.steps._vbn_host[0].copy()
            rows[:, P.S_FLAGS] &= ~P.F_HEAD_MFMA
            st = torch.from_numpy(rows).to(pk.device)
            st._vbn_wblk_max = pl.steps._vbn_wblk_max
            ic = pl.steps._vbn_host[1]
            st._vbn_host = (rows, ic, hashlib.sha1(rows.tobytes() + b"|" + ic.tobytes()).hexdigest())
            pk.model._cache[key] = dataclasses.replace(pl, steps=st)
            n += 1
    print("plans patched", n, flush=True)
    c, d = run(False), run(True)
    cmp("VALU head", c, d)
    cmp("interp MFMA vs VALU head", a, c)


if __name__ == "__main__":
    main()
