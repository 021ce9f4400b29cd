#!/usr/bin/env python3
"""KDE point-pack locality A/B (GPU box): the bench walk of a config as one launch vs the same
queries in G launches of B/G queries each (q_base offsets, so every particle's draws and
outputs are the same; checked bitwise).  A launch of about one resident wave per SIMD slot
starts every wave at the first node together, so the waves stay near each other in the node
sequence and the point packs they stream stay in the XCD's L2; one big launch lets them drift
over the whole DAG.

    python scripts/gen_ab.py --config cfg4 --gens 1 4 8 16 32
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--gens", type=int, nargs="+", default=[1, 4, 8, 16, 32])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from bench import build_workload
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd import jit

    torch.cuda.set_device(0)
    cfg, model, vbn, query = build_workload(a.config, "cuda:0", 1)
    B, S = cfg["B"], cfg["S"]
    vbn.set_inference_method(cfg["engine"], n_samples=S)
    vbn.infer_posterior(query)
    jit.wait_pending()
    vbn.infer_posterior(query)
    torch.cuda.synchronize()
    last = dict(E.LAST_LAUNCH)
    pk, plan, fixed = last["pk"], last["plan"], last["fixed"]

    def run(g, seed):
        outs = []
        step = B // g
        for i in range(g):
            b0 = i * step
            outs.append(E.run_walk(pk, plan, fixed[b0:b0 + step], step, S, seed=seed, q_base=b0,
                                   plan_jit=last["plan_jit"]))
        return outs

    ref = run(1, 7)
    for g in a.gens:
        assert B % g == 0
        out = run(g, 7)
        torch.cuda.synchronize()
        same = all(torch.equal(torch.cat([o[k] for o in out]), ref[0][k]) for k in range(2))
        stream = torch.cuda.current_stream()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run(g, 100)
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(json.dumps({"config": a.config, "launches": g, "queries_per_launch": B // g,
                          "waves_per_launch": B // g * S // 64, "ms": round(statistics.median(ts), 3),
                          "all_ms": [round(t, 3) for t in ts], "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
