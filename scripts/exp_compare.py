#!/usr/bin/env python3
"""Kernel A/B harness for experiment libraries (make exp KM=... EXP=...).

    python scripts/exp_compare.py --config cfg2 base.so variant1.so ...

For each library (own subprocess, VBN_HIP_LIB): builds the bench workload, times the walk
kernel with HIP events (median of 5 x 10 launches) and saves one fixed-seed walk's outputs;
then reports each variant's kernel ms and its max deviation from the first library.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg_name: str, out_path: str, engine_kw: str):
    sys.path.insert(0, REPO)
    import torch
    from bench import build_workload
    from vectorizedbayesiannetwork_amd import engines as E

    torch.cuda.set_device(0)
    cfg, model, vbn, query = build_workload(cfg_name, "cuda:0", 1)
    B, S = cfg["B"], cfg["S"]
    kw = json.loads(engine_kw)
    vbn.set_inference_method(cfg["engine"], n_samples=S, **kw)
    vbn.infer_posterior(query)
    torch.cuda.synchronize()
    last = dict(E.LAST_LAUNCH)
    pk, plan, fixed = last["pk"], last["plan"], last["fixed"]
    stream = torch.cuda.current_stream()
    times = []
    for rep in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(10):
            E.run_walk(pk, plan, fixed, B, S, seed=100 + i)
        e1.record(stream)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / 10)
    lp, x = E.run_walk(pk, plan, fixed, B, S, seed=7)
    torch.cuda.synchronize()
    nq = min(B, 256)                                   # a bounded sample of the outputs
    torch.save({"lp": lp[:nq].cpu().clone(), "x": x[:nq].cpu().clone(), "ms": statistics.median(times),
                "all_ms": times}, out_path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--engine-kw", default="{}")
    ap.add_argument("--child", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a.config, a.out, a.engine_kw)
        return
    import torch
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    res = []
    for i, lib in enumerate(a.libs):
        out = os.path.join(REPO, "gpurun_out", f"exp_{i}.pt")
        env = dict(os.environ, VBN_HIP_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__, "--child", lib, "--config", a.config, "--out", out,
                            "--engine-kw", a.engine_kw], env=env, timeout=150)
        if r.returncode != 0:
            print(json.dumps({"lib": lib, "error": r.returncode}), flush=True)
            sys.exit(r.returncode)
        res.append(torch.load(out, weights_only=True))
        d = {"lib": os.path.basename(lib), "kernel_ms": round(res[-1]["ms"], 4),
             "all_ms": [round(t, 4) for t in res[-1]["all_ms"]]}
        if i > 0:
            b, v = res[0], res[-1]
            for k in ("lp", "x"):
                if b[k].numel():
                    fin = torch.isfinite(b[k]) & torch.isfinite(v[k])
                    diff = (b[k][fin] - v[k][fin]).abs()
                    rel = diff / (1e-6 + b[k][fin].abs())
                    d[f"{k}_max_abs"] = float(diff.max()) if diff.numel() else 0.0
                    d[f"{k}_max_rel"] = float(rel.max()) if rel.numel() else 0.0
                    d[f"{k}_nonfinite_mismatch"] = int((torch.isfinite(b[k]) != torch.isfinite(v[k])).sum())
            d["speedup"] = round(res[0]["ms"] / res[-1]["ms"], 4)
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
