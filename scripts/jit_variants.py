#!/usr/bin/env python3
"""Compile plan-specialised code objects of a bench workload's walk with extra options (A/B
experiments for scripts/jit_ab.py; CPU only, hiprtc).

    python scripts/jit_variants.py --config cfg3 base= wpe3=-DVBN_WPE=3 sb=-DVBN_PLAN_SCHED_BARRIER
writes exp/plan_<config>_<name>.hsaco and prints the register usage of each.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--gibbs", action="store_true",
                    help="the Gibbs sweep table of scripts/jit_ab_gibbs.py (half-wave kind set 321)")
    ap.add_argument("--outdir", default="exp", help="directory (under the repo) for the code objects")
    ap.add_argument("variants", nargs="+", help="name=space-separated extra options")
    a = ap.parse_args()
    if a.gibbs:
        return gibbs_variants(a.variants)
    import bench
    from vectorizedbayesiannetwork_amd import jit
    from vectorizedbayesiannetwork_amd.plan import MODE_MCM, MODE_WEIGHTED, PackedModel, build_plan
    cfg, model, target, ev = bench.build_model(a.config)
    pk = PackedModel(model, "cpu")
    vals = set(ev)
    lat = [x for x in model.topo if x not in vals]
    fix = [x for x in model.topo if x in vals]
    if cfg["engine"] == "importance_sampling":
        plan = build_plan(pk, latent=lat, fixed=fix, logp=fix, out_nodes=[target], shared_roots=False,
                          mode=MODE_WEIGHTED)
    else:
        plan = build_plan(pk, latent=lat, fixed=fix, logp=[target], out_nodes=[target], shared_roots=True,
                          mode=MODE_MCM)
    km = plan.kind_mask | 128
    steps, ic, _ = plan.steps._vbn_host
    src = jit.plan_source(steps, ic, km)
    os.makedirs(os.path.join(REPO, a.outdir), exist_ok=True)
    base = jit.OPTIONS
    for v in a.variants:
        name, _, opts = v.partition("=")
        jit.OPTIONS = tuple(base) + tuple(opts.split())
        t0 = time.perf_counter()
        code = jit.compile_source(src)
        out = os.path.join(REPO, a.outdir, f"plan_{a.config}_{name}.hsaco")
        with open(out, "wb") as f:
            f.write(code)
        print(f"{out}: kind set {km}, {len(code)} B, {time.perf_counter() - t0:.1f} s")
    jit.OPTIONS = base


def gibbs_variants(variants):
    import bench
    from vectorizedbayesiannetwork_amd import jit
    from vectorizedbayesiannetwork_amd.plan import PackedModel, build_gibbs_plan
    cfg, model, target, ev = bench.build_model("cfg2")
    pk = PackedModel(model, "cpu")
    vals = set(ev)
    gp = build_gibbs_plan(pk, latent=[x for x in model.topo if x not in vals],
                          fixed=[x for x in model.topo if x in vals], target=target)
    steps, ic, _ = gp.steps._vbn_host
    # the production form at 4096 chains (ops.gibbs_walk auto): full wave, no injected draws,
    # chain workgroups of ops.CHAIN_WAVES waves on the cost model's schedule
    from vectorizedbayesiannetwork_amd import ops
    from vectorizedbayesiannetwork_amd.plan import gibbs_schedule
    km = gp.kind_mask | 256
    src = jit.plan_source(steps, ic, km, gibbs_schedule(steps, ic, ops.CHAIN_WAVES))
    base = jit.OPTIONS
    for v in variants:
        name, _, opts = v.partition("=")
        jit.OPTIONS = tuple(base) + tuple(opts.split())
        t0 = time.perf_counter()
        code = jit.compile_source(src)
        os.makedirs(os.path.join(REPO, "exp"), exist_ok=True)
        out = os.path.join(REPO, "exp", f"gibbs_{name}.hsaco")
        with open(out, "wb") as f:
            f.write(code)
        print(f"{out}: kind set {km}, {len(code)} B, {time.perf_counter() - t0:.1f} s")
    jit.OPTIONS = base


if __name__ == "__main__":
    main()
