#!/usr/bin/env python3
"""Precompile the plan-specialised walks of the benchmark workloads on the build host (CPU,
hiprtc) into the package's plan cache (vectorizedbayesiannetwork_amd/plan_cache), so a fresh
GPU box loads them instead of compiling inside the first call.

    python scripts/precompile_plans.py [cfg2 cfg3 ...]        (default: every bench config)

Per config: the bench engine's production plan (MCM / IS / LW) and, for shared-root engines,
its shared-sample precompute variant (plan.precompute_plans) -- the same step tables the
engines build, so the cache keys match.
"""
from __future__ import annotations

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


ENGINES = {"mcm": "monte_carlo_marginalization", "is": "importance_sampling", "lw": "likelihood_weighting",
           "ancestral": "ancestral"}


def plans_for(name):
    """``cfg`` (the bench engine) or ``cfg:engine`` (mcm / is / lw / ancestral: the engines'
    plans for the GPU tests' workloads, which share the bench configs' DAGs).  Built through
    the engines' own ``engines._plan`` with their arguments (walk order and precompute
    included), so the step tables and cache keys are the engines'."""
    import bench
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd import plan as P
    cfg_name, _, eng_name = name.partition(":")
    cfg, model, target, ev = bench.build_model(cfg_name)
    pk = P.PackedModel(model, "cpu")
    vals = set(ev)
    fixed = [x for x in model.topo if x in vals]
    latent = [x for x in model.topo if x not in vals]
    logp_ev = [x for x in model.topo if x in ev]
    eng = ENGINES[eng_name] if eng_name else cfg["engine"]
    common = dict(latent=latent, fixed=fixed, out_nodes=[target], skip=[], exact_f32=False, kde_valu=False)
    if eng in ("likelihood_weighting", "importance_sampling"):
        lw = eng == "likelihood_weighting"
        key = ("weighted", target, tuple(sorted(ev)), (), lw, lw, False, False, False)
        plan = E._plan(pk, key, logp=logp_ev, shared_roots=lw, mode=P.MODE_WEIGHTED,
                       clamp=list(ev) if lw else (), **common)
    elif eng == "ancestral":
        key = ("ancestral", target, tuple(sorted(vals)), False, False, False)
        plan = E._plan(pk, key, logp=[], shared_roots=True, mode=P.MODE_SAMPLE, **common)
    elif eng == "monte_carlo_marginalization":
        key = ("mcm", target, tuple(sorted(vals)), False, False, False)
        plan = E._plan(pk, key, logp=[target], shared_roots=True, mode=P.MODE_MCM, **common)
    else:
        return cfg, []
    out = [("plain", plan, False)]
    if plan.pc is not None:
        out.append(("precompute", plan.pc, plan.pre is not None))
    return cfg, out


def _one(name):
    from vectorizedbayesiannetwork_amd import jit
    cfg, plans = plans_for(name)
    lines = []
    for tag, plan, pre in plans:
        t0 = time.perf_counter()
        key, comp = jit.precompile(plan, cfg["B"], cfg["S"], precomp=pre)
        lines.append(f"{name} {tag}: {key} ({'compiled' if comp else 'cached'} in {time.perf_counter() - t0:.1f} s)")
    return lines


def main(names):
    from concurrent.futures import ProcessPoolExecutor
    from vectorizedbayesiannetwork_amd import synthetic
    names = names or ["cfg2", "cfg3", "cfg4", "cfg5", "anchor64"]
    if names == ["--tests"]:                 # the extra plans of the GPU tests' workloads
        names = ["cfg2:is", "cfg2:lw", "cfg3:lw", "cfg3:mcm", "cfg3:ancestral", "cfg4:lw", "cfg4:ancestral",
                 "cfg5:lw", "cfg5:ancestral"]
    for name in names:
        if name.partition(":")[0] not in synthetic.CONFIGS or name.partition(":")[2] not in ("", *ENGINES):
            raise SystemExit(f"unknown config {name}")
    # one hiprtc compile per process at a time (single-threaded, ~1-2 GB each)
    workers = max(1, min(len(names), (os.cpu_count() or 1), 8))
    with ProcessPoolExecutor(workers) as ex:
        for lines in ex.map(_one, names):
            for ln in lines:
                print(ln, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
