#!/usr/bin/env python3
"""A/B of plan-specialised walk code objects against the step-table interpreter (GPU box).

    python scripts/jit_ab.py --config cfg2 exp/plan_cfg2_hipcc.hsaco exp/plan_cfg2_rtc.hsaco

Per variant: walk kernel ms (HIP events, median of 5 x 10 launches, ABAB order) and whether
its outputs are bit-identical to the interpreter's.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("objects", nargs="*")
    a = ap.parse_args()
    import torch
    from bench import build_workload
    from vectorizedbayesiannetwork_amd import _lib, ops
    from vectorizedbayesiannetwork_amd import engines as E

    torch.cuda.set_device(0)
    E.PRECOMPUTE = False             # the variants are compiled from the plain plan (jit_variants.py),
    E.LIVENESS_ORDER = False         # in the model's order: the launch must carry the same table
    cfg, model, vbn, query = build_workload(a.config, "cuda:0", 1)
    B, S = cfg["B"], cfg["S"]
    vbn.set_inference_method(cfg["engine"], n_samples=S, plan_jit=False)
    vbn.infer_posterior(query)
    torch.cuda.synchronize()
    last = dict(E.LAST_LAUNCH)
    pk, plan, fixed = last["pk"], last["plan"], last["fixed"]
    lib = _lib.load()
    mods = {}
    for path in a.objects:
        code = open(path, "rb").read()
        h = ctypes.c_void_p()
        # the kind set the interpreter picks for this launch: build a throwaway args struct
        mods[path] = (code, h)

    def run(variant, seed):
        if variant == "interp":
            return E.run_walk(pk, plan, fixed, B, S, seed=seed, plan_jit=0)
        import vectorizedbayesiannetwork_amd.jit as J
        orig = J.module_for
        J.module_for = lambda *args, **kw: mods[variant][1].value
        try:
            return E.run_walk(pk, plan, fixed, B, S, seed=seed, plan_jit=2)
        finally:
            J.module_for = orig

    # load modules with the interpreter's kind set for this launch
    a0 = _lib.VbnWalkArgs()
    E.run_walk(pk, plan, fixed, B, S, seed=1, plan_jit=0)
    import vectorizedbayesiannetwork_amd.jit as J
    captured = {}
    orig = J.module_for

    def capture(steps, in_cols, kind_set, dev, key, *rest, **kw):
        captured["km"] = kind_set
        return None
    J.module_for = capture
    E.run_walk(pk, plan, fixed, B, S, seed=1, plan_jit=2)
    J.module_for = orig
    km = captured["km"]
    for path, (code, h) in mods.items():
        buf = ctypes.create_string_buffer(code, len(code))
        _lib.check(lib.vbn_hip_module_load(buf, b"vbn_walk_plan", km, plan.n_steps, ctypes.byref(h)), "load")
    ref = run("interp", 7)
    torch.cuda.synchronize()
    variants = ["interp"] + list(mods)
    res = {v: [] for v in variants}
    for rnd in range(2):
        print(f"round {rnd}", file=sys.stderr, flush=True)
        for v in variants:
            stream = torch.cuda.current_stream()
            for rep in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(10):
                    run(v, 100 + i)
                e1.record(stream)
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / 10)
    for v in variants:
        out = run(v, 7)
        torch.cuda.synchronize()
        same = all(torch.equal(x, y) for x, y in zip(out, ref))
        print(json.dumps({"variant": os.path.basename(v), "kind_set": km, "kernel_ms": round(statistics.median(res[v][5:]), 4),
                          "all_ms": [round(t, 4) for t in res[v]], "bit_identical": same,
                          "specialised_flag": ops.LAST_WALK["specialised"]}), flush=True)


if __name__ == "__main__":
    main()
