#!/usr/bin/env python3
"""A/B of plan-specialised Gibbs sweep code objects (GPU box), like scripts/jit_ab.py:

    python scripts/jit_variants.py --gibbs base= noexact=-DVBN_ABL_NOEXACT     (CPU)
    python scripts/jit_ab_gibbs.py exp/gibbs_base.hsaco exp/gibbs_noexact.hsaco (GPU)

Workload: profiles/bench_gibbs.py's (cfg2 DAG, 4096 chains, YAML defaults -> 2610 sweeps).
Per variant: sweep kernel ms (HIP events, median of 3 rounds x 2 launches) and bit identity
with the interpreter.
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def gibbs_setup(device, chains=4096, n_samples=512, burn_in=50, thin=5):
    import torch
    import bench as Bm
    from vectorizedbayesiannetwork_amd import engines as E
    cfg, model, vbn, query = Bm.build_workload("cfg2", device, 1)
    reps = -(-chains // cfg["B"])
    query = {"target": query["target"],
             "evidence": {k: v.repeat(reps, 1)[:chains].contiguous() for k, v in query["evidence"].items()}}
    vbn.set_sampling_method("gibbs", n_samples=n_samples, burn_in=burn_in, n_steps=thin, seed=1, plan_jit=False)
    eng = vbn._sampling
    q = vbn._normalize_query(query)
    pk = E.packed_model(vbn, torch.device(device))
    vals = E._fixed_values(q, pk.device)
    gp = eng._gibbs_plan(pk, q.target, vals)
    fx = E._fixed_buffer(gp.init, vals, chains, pk.device)
    iters = burn_in + n_samples * thin
    return eng, pk, gp, fx, iters, chains


def main():
    import torch
    from vectorizedbayesiannetwork_amd import _lib, ops
    import vectorizedbayesiannetwork_amd.jit as J
    torch.cuda.set_device(0)
    eng, pk, gp, fx, iters, B = gibbs_setup("cuda:0")
    state = torch.randn(gp.init.n_slots + 1, B * 8, device=pk.device)
    wp = eng._wave_particles(B)
    current = {"h": None}
    orig = J.module_for
    J.module_for = lambda *a, **k: current["h"]

    def launch(seed, pj):
        return ops.gibbs_walk(gp.steps, gp.in_cols, pk.params, fx, None, state, B, gp.init.n_slots,
                              gp.init.max_out, gp.init.fixed_ld, B, gp.n_noise, pk.dmax, 1, iters, iters - 1, 1,
                              0, seed, 1, gp.kind_mask, gp.wbuf, wp, pj)
    # kind set of this launch
    cap = {}

    def capture(steps, in_cols, kind_set, dev, key, *rest, **kw):
        cap["km"] = kind_set
        cap["cw"] = rest[0] if rest else kw.get("chain_waves", 0)
        return None
    J.module_for = capture
    launch(1, 2)
    J.module_for = lambda *a, **k: current["h"]
    km = cap["km"]
    lib = _lib.load()
    mods = {}
    for path in sys.argv[1:]:
        code = open(path, "rb").read()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(code, len(code))
        _lib.check(lib.vbn_hip_module_load(buf, b"vbn_walk_plan", km, gp.n_steps, ctypes.byref(h)), "load")
        if cap["cw"] > 0:                                   # chain workgroups (jit_variants --gibbs)
            _lib.check(lib.vbn_hip_module_chain_waves(h, cap["cw"]), "chain waves")
        mods[path] = h.value
    ref = launch(7, 0)
    torch.cuda.synchronize()
    variants = ["interp"] + list(mods)
    res = {v: [] for v in variants}
    stream = torch.cuda.current_stream()
    for rnd in range(3):
        for v in variants:
            current["h"] = mods.get(v)
            pj = 0 if v == "interp" else 2
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(2):
                launch(100 + i, pj)
            e1.record(stream)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 2)
    for v in variants:
        current["h"] = mods.get(v)
        out = launch(7, 0 if v == "interp" else 2)
        torch.cuda.synchronize()
        print(json.dumps({"variant": os.path.basename(v), "kind_set": km, "chain_waves": cap["cw"], "sweep_ms": round(statistics.median(res[v]), 2),
                          "all_ms": [round(t, 2) for t in res[v]], "bit_identical": bool(torch.equal(out, ref)),
                          "specialised_flag": ops.LAST_WALK["specialised"]}), flush=True)
    J.module_for = orig


if __name__ == "__main__":
    main()
