#!/usr/bin/env python3
"""Gibbs sampler measurement on the cfg2 DAG: one JSON line like bench.py's.

Workload ``gibbs32``: the cfg2 32-node gaussian_nn model and query generator, B = 4096 chains,
the reference YAML defaults (vbn/configs/sampling/gibbs.yaml: n_samples 512, burn_in 50,
n_steps 5 -> 2610 sweeps), 8 candidates per chain per latent node (gibbs.py:20).  A step is
one ``VBN.sample`` (initial ancestral walk + the one-launch sweep walk).  The roofline prices
the sweep kernel's MLP FLOPs (candidate draws + children log-probs) like bench.py.
CPU baseline: the oracle restatement (reference op sequence, vectorised over the chains like
the reference's sweep) on a bounded batch of chains for a bounded number of sweeps, scaled to
the full sweep count.

Usage: python profiles/bench_gibbs.py [--steps K] [--warmup W] [--chains B]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench as Bm  # noqa: E402
from vectorizedbayesiannetwork_amd import engines as E  # noqa: E402
from vectorizedbayesiannetwork_amd.plan import KIND_ID  # noqa: E402


def sweep_flops_per_lane(plan):
    f32, hid = 0.0, 0.0
    for i in range(plan.n_steps):
        row = plan.steps[i].tolist()
        kind, role, flags, nin, n_out = row[0], row[1], row[2], row[4], row[10]
        if role not in (1, 2) or not (flags & 1):
            continue
        if kind in (KIND_ID["gaussian_nn"], KIND_ID["mdn"], KIND_ID["softmax_nn"]) and not (flags & 2):
            f32 += 2.0 * (32 * nin + 32 * n_out)
            hid += 2.0 * 32 * 32
        elif kind == KIND_ID["linear_gaussian"]:
            f32 += 2.0 * nin * row[7]
    return f32, hid


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chains", type=int, default=4096)
    ap.add_argument("--n-samples", type=int, default=512)
    ap.add_argument("--burn-in", type=int, default=50)
    ap.add_argument("--thin", type=int, default=5)
    ap.add_argument("--cpu-sweeps", type=int, default=4)
    ap.add_argument("--cpu-chains", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--wave-particles", type=int, default=None, help="32 / 64 (default: the engine's choice)")
    ap.add_argument("--chain-waves", type=int, default=None,
                    help="0..8: waves per chain workgroup of the specialised sweep (default: the engine's choice)")
    ap.add_argument("--plan-jit", choices=("auto", "on", "off"), default="auto",
                    help="plan-specialised sweep kernel (vectorizedbayesiannetwork_amd/jit.py) or the interpreter")
    args = ap.parse_args()
    pj = {"auto": "auto", "on": True, "off": False}[args.plan_jit]
    torch.cuda.set_device(0)
    cfg, model, vbn, query = Bm.build_workload("cfg2", "cuda:0", 1)
    B = args.chains
    reps_ev = -(-B // cfg["B"])                      # more chains than cfg2 queries: tile the evidence rows
    query = {"target": query["target"],
             "evidence": {k: v.repeat(reps_ev, 1)[:B].contiguous() for k, v in query["evidence"].items()}}
    vbn.set_sampling_method("gibbs", n_samples=args.n_samples, burn_in=args.burn_in, n_steps=args.thin, seed=1,
                            wave_particles=args.wave_particles, plan_jit=pj, chain_waves=args.chain_waves)
    for _ in range(args.warmup):
        vbn.sample(query, n_samples=args.n_samples)
    torch.cuda.synchronize()
    # a sweep plan missing from the code-object cache compiles in the background while the
    # first calls run the interpreter: wait for it, so the timed steps run one walk form
    from vectorizedbayesiannetwork_amd import jit
    jit.wait_pending()
    vbn.sample(query, n_samples=args.n_samples)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        xs = vbn.sample(query, n_samples=args.n_samples)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert xs.shape == (B, args.n_samples, 1) and bool(torch.isfinite(xs).all())
    iters = args.burn_in + args.n_samples * args.thin

    # sweep kernel alone, HIP events on the stream it is launched on
    eng = vbn._sampling
    q = vbn._normalize_query(query)
    pk = E.packed_model(vbn, torch.device("cuda", 0))
    vals = E._fixed_values(q, pk.device)
    gp = eng._gibbs_plan(pk, q.target, vals)
    fx = E._fixed_buffer(gp.init, vals, B, pk.device)
    state = torch.randn(gp.init.n_slots + 1, B * 8, device=pk.device)
    from vectorizedbayesiannetwork_amd import ops
    wp = eng._wave_particles(B)

    def launch(seed):
        return ops.gibbs_walk(gp.steps, gp.in_cols, pk.params, fx, None, state, B, gp.init.n_slots,
                              gp.init.max_out, gp.init.fixed_ld, B, gp.n_noise, pk.dmax, 1, iters, iters - 1, 1,
                              0, seed, 1, gp.kind_mask, gp.wbuf, wp, eng.plan_jit,
                              -1 if eng.chain_waves is None else eng.chain_waves)
    launch(0)
    specialised = bool(ops.LAST_WALK.get("specialised"))
    chain_waves = int(ops.LAST_WALK.get("chain_waves") or 0)
    wp = int(ops.LAST_WALK.get("wave_particles") or wp)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record(stream)
    for i in range(reps):
        launch(i + 1)
    e1.record(stream)
    torch.cuda.synchronize()
    kern_ms = e0.elapsed_time(e1) / reps
    f32, hid = sweep_flops_per_lane(gp)
    lanes = B * 8 * iters
    f32, hid = f32 * lanes, hid * lanes
    t_min = f32 / (Bm.FP32_PEAK_TFLOPS * 1e12) + hid / (Bm.F16_PEAK_TFLOPS / Bm.SPLIT_PASSES * 1e12)
    peak = (f32 + hid) / t_min / 1e12
    ach = (f32 + hid) / (kern_ms * 1e-3) / 1e12
    out = {
        "metric": "Gibbs posterior queries/sec (VBN.sample, gibbs YAML defaults) on 1 MI355X",
        "value": round(B * args.steps / el, 2), "unit": "queries/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic (cfg2 DAG/SEM/query generator; {cfg.get('model_origin', 'random-init')} CPDs)",
        "config": {"workload": "gibbs32: 32node-gaussian_nn-gibbs", "chains": B, "n_samples": args.n_samples,
                   "burn_in": args.burn_in, "n_steps": args.thin, "sweeps": iters, "candidates": 8,
                   "wave_particles": wp, "chain_waves": chain_waves,
                   "walk": "plan-specialised" if specialised else "step-table interpreter"},
        "roofline": {"bound": "mfma", "achieved": round(ach, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
                     "frac": round(ach / peak, 4), "traffic": None, "kernel": ("vbn_walk_plan" if specialised else "vbn_walk_kernel") + " (GIBBS)",
                     "kernel_ms": round(kern_ms, 3), "flops_per_launch": f32 + hid,
                     "sweep_lane_evals_per_s": round(lanes / (kern_ms * 1e-3), 1), "launches_timed": reps},
    }
    if not args.no_cpu_baseline:
        from oracle import vbn_oracle as O
        bc = min(args.cpu_chains, B)
        ev1 = {k: v[:bc].cpu() for k, v in query["evidence"].items()}
        n_cpu = args.cpu_sweeps
        with torch.no_grad():
            O.gibbs(model, query["target"], ev1, {}, 1, O.TorchDraws(), burn_in=0, n_steps=1, root_expand=True)
            t0 = time.perf_counter()
            O.gibbs(model, query["target"], ev1, {}, n_cpu, O.TorchDraws(), burn_in=0, n_steps=1,
                    root_expand=True)
            t = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(bc / (t / n_cpu * iters), 6), "unit": "queries/s",
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"{bc} chains (one batched call, as the reference vectorises each "
                                         f"sweep over the chains; latent-root candidates broadcast, "
                                         f"since the reference indexes them only at b = 1) x {n_cpu} "
                                         f"sweeps of the oracle, "
                                         f"scaled to {iters} sweeps per query"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
