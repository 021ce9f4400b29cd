#!/usr/bin/env python3
"""Throughput of ``VBN.infer_posterior`` on MI355X (BASELINE.json metric).

A step = one ``infer_posterior`` call over one batch of synthetic queries:
default workload cfg4 = 64-node random DAG, kde CPDs with 10,000 stored points each (the
reference-fitted model: KDE fitting keeps the training rows), 4096 queries x 1024 samples per
GPU, monte_carlo_marginalization -- BASELINE.json's largest single-GPU config and the
north-star's 64-node target; ``--config cfg2`` etc. select the other workloads.  Every N
runs the same path: the global batch (4096 x N queries) goes through ``ShardedEngine(engine, gather=True, overlap=True)`` -- each rank walks
its contiguous 4096-query shard (weak scaling; the global query index keys the RNG) and the
pdf / samples are gathered on rank 0 with one RCCL gather over xGMI per step, issued
asynchronously so it overlaps the next step's walk (N = 1: no collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5|anchor64|...]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Rank 0 prints one JSON line.  ``roofline`` prices the dominant kernel (vbn_walk_kernel) with
HIP events on the stream it runs on; ``cpu_baseline`` times the CPU oracle (the reference's
torch op sequence, oracle/vbn_oracle.py) on a bounded sample on this host's cores, in a
fresh child process with the tuned glibc allocator settings of BASELINE.md.
"""
from __future__ import annotations

import argparse
import gc
import glob
import json
import math
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from vectorizedbayesiannetwork_amd import VBN, synthetic  # noqa: E402
from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query  # noqa: E402
from vectorizedbayesiannetwork_amd.model import random_init_model  # noqa: E402
from vectorizedbayesiannetwork_amd.plan import KIND_ID  # noqa: E402

FP32_PEAK_TFLOPS = 157.3     # MI355X FP32 dense (vector = f32-input MFMA), MI355X_MICROARCH.md
F16_PEAK_TFLOPS = 2516.6     # f16 MFMA dense: 32x32x16 = 32768 FLOP / 32 cyc / SIMD x 1024 SIMD x 2.4 GHz
SPLIT_PASSES = 3             # split-f16 hidden layer: A_lo.B_hi + A_hi.B_lo + A_hi.B_hi
HBM_PEAK_GBS = 8000.0
# v_exp_f32: 8 issue cycles per wave64 instruction per SIMD (MI355X_MICROARCH.md constants)
# -> 8 exp/clk/SIMD x 1024 SIMDs x 2.4 GHz
EXP_PEAK_T = 8 * 1024 * 2.4e9 / 1e12
MODELS_DIR = os.path.join(REPO, "tests", "golden", "models")


def build_model(cfg_name: str):
    """The synthetic model of ``cfg_name``: random DAG, SEM data and the CPDs
    the reference fitted on it (``tests/golden/models``, make_golden_models.py: YAML
    hyper-parameters, one epoch of batch 4096); configs without a fitted fixture get random-init
    CPDs of the reference architectures (``cfg["model_origin"]`` says which).  Returns (cfg,
    model, target, evidence nodes)."""
    cfg = dict(synthetic.CONFIGS[cfg_name])
    g = synthetic.random_dag(cfg["n_nodes"], seed=0)
    model = synthetic.fitted_model(cfg_name, MODELS_DIR)
    origin = "reference-fitted"
    if model is None:
        data = synthetic.sem_data(g, cfg.get("rows", 2048), seed=0)
        kinds = synthetic.round_robin_kinds(g, cfg["kinds"])
        overrides = {"kde": {"max_points": cfg["kde_max_points"]}} if "kde_max_points" in cfg else None
        model = random_init_model(g, kinds, data, seed=0, overrides=overrides)
        origin = "random-init"
    cfg["model_origin"] = origin
    target, ev_nodes = synthetic.default_query_nodes(g, seed=1)
    return cfg, model, target, ev_nodes


def build_workload(cfg_name: str, device: str, world: int = 1):
    """Model on ``device`` + the global query of ``world`` x B queries (identical on every
    rank): on-manifold evidence = B rows of the model's own ancestral draw (seed 2)."""
    cfg, model, target, ev_nodes = build_model(cfg_name)
    vbn = VBN.from_model(model, device=device)
    B = cfg["B"] * world
    torch.manual_seed(2)
    joint = AncestralSampler(n_samples=B).sample(vbn, Query(target=None, evidence={}, do={}), n_samples=B)
    evidence = {n: joint[n][0].contiguous() for n in ev_nodes}
    return cfg, model, vbn, {"target": target, "evidence": evidence}


def mlp_flops_per_particle(model, plan):
    """Algorithmic FLOPs of one particle in one walk, by the unit that executes them:
    (f32 FLOPs: layer 1, head, linear_gaussian means; FLOPs of the 32x32 hidden layer).
    MLP = in -> 32 -> 32 -> out, 2 x MACs (bias adds not counted)."""
    f32, hidden = 0.0, 0.0
    for i in range(plan.n_steps):
        row = plan.steps[i].tolist()
        kind, role, flags, nin, n_out = row[0], row[1], row[2], row[4], row[10]
        if role == 0 or (role == 2 and not (flags & 1)):
            continue
        if kind in (KIND_ID["gaussian_nn"], KIND_ID["mdn"], KIND_ID["softmax_nn"]) and not (flags & 2):
            f32 += 2.0 * (32 * nin + 32 * n_out)
            hidden += 2.0 * 32 * 32
        elif kind == KIND_ID["linear_gaussian"]:
            f32 += 2.0 * nin * row[7]
    return f32, hidden


def executed_work(model, plan, B: int, S: int, precomputed: bool):
    """(f32 FLOPs, hidden-layer FLOPs, KDE exps) the launch actually executes: with the
    precompute, a VBN_F_PRECOMP node's MLP / KDE pass 1 runs once per sample (per-sample
    pre-pass, S particles) or once per query (per-query pre-pass, B waves of 64 lanes) instead of
    once per particle (plan.precompute_plans)."""
    if not precomputed or plan.pc is None:
        f, h = mlp_flops_per_particle(model, plan)
        return f * B * S, h * B * S, kde_exps_per_particle(model, plan, executed=True) * B * S
    f32 = hid = exps = 0.0
    rows = plan.pc.steps.cpu().tolist()
    for i, row in enumerate(rows):
        one = _RowPlan([row])
        f, h = mlp_flops_per_particle(model, one)
        e = kde_exps_per_particle(model, one, executed=True)
        fl = row[2]
        if fl & 8192:                                 # precomputed: pre-pass particles only
            n = B * 64 if fl & 32768 else S
            kde_p1 = (float(row[9]) if row[0] == KIND_ID["kde"] and row[1] == 1 and row[31] < 0
                      else 0.0)
            f32, hid, exps = f32 + f * n, hid + h * n, exps + kde_p1 * n + (e - kde_p1) * B * S
        else:
            f32, hid, exps = f32 + f * B * S, hid + h * B * S, exps + e * B * S
    return f32, hid, exps


class _RowPlan:
    """one step row as a plan (mlp_flops_per_particle / kde_exps_per_particle)"""

    def __init__(self, rows):
        self.steps = torch.tensor(rows, dtype=torch.int32)
        self.n_steps = len(rows)


def kde_exps_per_particle(model, plan, executed: bool = False) -> float:
    """Algorithmic kernel-weight evaluations (one exp each) of one particle in one walk:
    M for a sampled non-root KDE node (the CDF pass; the chunk rescan is not counted),
    2M for a non-root log-prob (LSE over K_p and over K_p K_y), M for a root log-prob.
    ``executed``: without the CDF pass of nodes whose pass 1 comes from a moment table
    (plan.kde_moment_table: no exps; a wave with a particle off the table's grid falls back to
    the exp pass, which on-manifold workloads do not do), and with M instead of 2M for the
    log-prob of a node that is also sampled (its denominator is the sampling pass's total,
    csrc kde_index_mfma lsp)."""
    exps = 0.0
    for i in range(plan.n_steps):
        row = plan.steps[i].tolist()
        if row[0] != KIND_ID["kde"] or row[1] == 0:
            continue
        m, root = row[9], bool(row[2] & 2)
        sampled = row[1] == 1 and not root
        if sampled and not (executed and row[31] >= 0):
            exps += m
        if row[2] & 1:
            exps += m if (root or (executed and sampled)) else 2 * m
    return exps


CPU_ENV = {"MALLOC_MMAP_MAX_": "0", "MALLOC_TRIM_THRESHOLD_": "1000000000000"}


def cpu_threads() -> int:
    """Host cores this process may use: the CPU affinity set, capped by OMP_NUM_THREADS when
    the launcher sets it (the GPU box grants one GPU's share of a larger host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else max(1, n)


def cpu_baseline_child(cfg_name: str, n_queries: int, reps: int):
    """Runs in a fresh child process (tuned glibc env, every granted core): the oracle (the
    reference's op sequence and RNG calls, TorchDraws) on ``n_queries`` queries of the same
    workload; 1 warm-up, median of ``reps``."""
    from oracle import vbn_oracle as O
    threads = cpu_threads()
    torch.set_num_threads(threads)
    cfg, model, target, ev_nodes = build_model(cfg_name)
    torch.manual_seed(2)                          # on-manifold evidence, as the GPU leg
    joint = O.ancestral(model, None, {}, {}, n_queries, O.TorchDraws())
    ev = {n: joint[n][0].contiguous() for n in ev_nodes}
    query = {"target": target}
    S, eng = cfg["S"], cfg["engine"]
    fallbacks = []

    def one():
        with torch.no_grad():
            if eng == "monte_carlo_marginalization":
                O.monte_carlo_marginalization(model, query["target"], ev, {}, S, O.TorchDraws())
            else:
                fallbacks.append(bool(O.importance_sampling(model, query["target"], ev, {}, S, O.TorchDraws())[3]))

    one()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    env = " ".join(f"{k}={os.environ.get(k, '')}" for k in CPU_ENV)
    out = {"value": n_queries / med, "unit": "queries/s", "cores": threads, "kind": "port",
           "sample": f"{n_queries} queries x {S} samples of {cfg_name}, median of {reps} after 1 warm-up, "
                     f"torch CPU {threads} threads (affinity {len(os.sched_getaffinity(0))}, "
                     f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}), no_grad, fresh process, {env}",
           "seconds": [round(t, 4) for t in ts]}
    if fallbacks:
        out["is_fallback"] = any(fallbacks)
    print(json.dumps(out), flush=True)


def cpu_baseline(cfg_name: str, n_queries: int, reps: int = 5):
    """Start :func:`cpu_baseline_child` as a fresh process (never an exec of this one)."""
    import subprocess
    env = dict(os.environ, **CPU_ENV)
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--config", cfg_name,
           "--cpu-queries", str(n_queries), "--cpu-reps", str(reps)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def load_traffic(cfg_name: str):
    """Per-launch HBM bytes of vbn_walk_kernel from the newest committed rocprofv3 PMC summary
    of this workload (profiles/r*_<cfg>_pmc.json; PMC counters cannot be read from inside the
    timed process).  Returns (bytes or None, source path)."""
    paths = glob.glob(os.path.join(REPO, "profiles", f"r*_{cfg_name}_pmc.json"))
    paths.sort(key=lambda p: os.path.basename(p))
    if not paths:
        return None, None
    try:
        with open(paths[-1]) as f:
            return json.load(f).get("hbm_bytes_per_launch"), os.path.relpath(paths[-1], REPO)
    except Exception:
        return None, None


KT_UNTIMED, KT_TIMED = 64, 20     # roofline kernel timing: untimed launches, then timed ones
_T0 = time.perf_counter()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """``bench.py --gpus N`` started without a launcher: run N rank processes on this node as
    fresh children (``torch.distributed.run``, rendezvous on 127.0.0.1) and return their exit
    code.  This process has not touched the GPU (the package import does not) and is never
    replaced by another program; rank 0's JSON line reaches stdout through the child."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def init_ranks(args):
    """(world, rank, local, device) of this process; the process group when world > 1.
    Exits non-zero when the launcher's WORLD_SIZE disagrees with ``--gpus``."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch with --nproc-per-node "
              f"{args.gpus}, or run `python bench.py --gpus {args.gpus}` without a launcher", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:                                     # CPU rehearsal of the launch path only
        if world > 1:
            import torch.distributed as tdist
            tdist.init_process_group("gloo")
        return world, rank, local, "cpu"
    if world > 1:
        import torch.distributed as tdist
        if args.dist_backend == "nccl":
            if torch.cuda.device_count() < world:
                print(f"bench.py: {world} ranks over RCCL need {world} GPUs, "
                      f"{torch.cuda.device_count()} visible (--dist-backend gloo rehearses several "
                      f"ranks on one GPU)", file=sys.stderr)
                sys.exit(2)
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:                                         # rehearsal: ranks share the visible GPUs
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            tdist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, local, f"cuda:{local}"


def ranks_seen(world: int, backend: str, device) -> list:
    """Every rank's global rank as the process group sees it (an all-gather), so the JSON line
    proves that N ranks took part."""
    if world == 1:
        return [0]
    import torch.distributed as tdist
    dev = device if backend == "nccl" else "cpu"
    mine = torch.tensor([tdist.get_rank()], dtype=torch.int64, device=dev)
    outs = [torch.zeros_like(mine) for _ in range(tdist.get_world_size())]
    tdist.all_gather(outs, mine)
    return sorted(int(t.item()) for t in outs)


def stub_main(args) -> None:
    """``--stub``: the launch / rank / reporting path with no GPU work (CPU tests)."""
    world, rank, local, device = init_ranks(args)
    seen = ranks_seen(world, "gloo", device)
    n_gpus = world
    if world > 1:
        import torch.distributed as tdist
        n_gpus = tdist.get_world_size()
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": 0.0, "unit": "queries/s", "n_gpus": n_gpus,
                          "ranks_seen": seen, "steps": args.steps, "warmup": args.warmup,
                          "stub": True}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def log(msg: str) -> None:
    """progress on stderr (the JSON line is the only stdout output)"""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s rank {os.environ.get('RANK', '0')}] {msg}",
          file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg4",
                    help="workload (vectorizedbayesiannetwork_amd/synthetic.py CONFIGS); default cfg4, the "
                         "largest single-GPU config of BASELINE.json (64-node KDE DAG, M = 10k, 4096 x 1024)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-queries", type=int, default=0)
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-gather", action="store_true", help="shards only (no RCCL gather of the outputs)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, one GPU per rank); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--prune-barren", action="store_true")
    ap.add_argument("--no-precompute", action="store_true",
                    help="recompute nodes with shared-root parents per query (A/B of plan.precompute_plans)")
    ap.add_argument("--exact-f32", action="store_true", help="hidden layer on the exact f32 MFMA chain")
    ap.add_argument("--kde-valu", action="store_true", help="KDE distances on packed VALU (default: 16x16x4 f32 MFMA tile)")
    ap.add_argument("--plan-jit", choices=("auto", "on", "off"), default="auto",
                    help="plan-specialised walk kernel (hiprtc, vectorizedbayesiannetwork_amd/jit.py) or the "
                         "step-table interpreter")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.no_precompute:
        from vectorizedbayesiannetwork_amd import engines as _E
        _E.PRECOMPUTE = False
    if args.cpu_baseline_child:                       # fresh process, never touches the GPU
        cpu_baseline_child(args.config, args.cpu_queries, args.cpu_reps)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks as children (before anything touches the GPU)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.stub:
        stub_main(args)
        return

    from vectorizedbayesiannetwork_amd.distributed import ShardedEngine
    world, rank, local, device = init_ranks(args)
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        if tdist.get_world_size() != args.gpus:
            print(f"bench.py: process group has {tdist.get_world_size()} ranks, --gpus {args.gpus}",
                  file=sys.stderr)
            sys.exit(2)
    seen = ranks_seen(world, args.dist_backend, device)

    log(f"world {world}, backend {args.dist_backend if dist else '-'}, device {device}: building {args.config}")
    cfg, model, vbn, query = build_workload(args.config, device, world)
    B, S = cfg["B"], cfg["S"]                         # B = queries per GPU
    extra = {"n_particles": S} if cfg["engine"] == "rao_blackwellized_marginalization" else {}
    vbn.set_inference_method(cfg["engine"], n_samples=S, prune_barren=args.prune_barren,
                             exact_f32=args.exact_f32, kde_valu=args.kde_valu,
                             plan_jit={"auto": "auto", "on": True, "off": False}[args.plan_jit], **extra)
    engine = vbn._inference
    gather = not args.no_gather
    # every N the same path: shard the global batch, gather pdf / samples on rank 0 (async,
    # overlapping the next step's walk); N = 1 is the trivial shard with no collective
    # verify: every untimed call first checks that all ranks issue the same call (a 32-byte
    # all-gather); off for the timed steps and the gather accounting
    sharded = ShardedEngine(engine, gather=gather, overlap=True, verify=dist)
    vbn._inference = sharded

    def barrier():
        if dist:
            tdist.barrier()

    # dominant kernel: walk launch duration with HIP events on its stream, measured before the
    # warmup and timed steps (KT_UNTIMED untimed launches, then KT_TIMED timed), so the kernel
    # time is a steady-state figure and the chip's clocks have left their idle state before
    # the timed region (the first ~25 walks after idle run up to 17 % slower)
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd import jit, ops
    log("first call")
    t_first = time.perf_counter()
    vbn.infer_posterior(query)                # builds the plan of the timed steps
    sharded.wait()
    torch.cuda.synchronize()
    t_first = time.perf_counter() - t_first
    # a plan missing from the code-object cache compiles in the background (jit.py) while the
    # first call runs the interpreter: wait for it, so every later step runs the same form
    t_wait = time.perf_counter()
    jit.wait_pending()
    t_wait = time.perf_counter() - t_wait
    vbn.infer_posterior(query)
    sharded.wait()
    torch.cuda.synchronize()
    specialised = bool(ops.LAST_WALK.get("specialised"))
    last = dict(E.LAST_LAUNCH)
    pk, plan, fixed = last["pk"], last["plan"], last["fixed"]
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    log("kernel timing")
    ev0.record(stream)
    E.run_walk(pk, plan, fixed, B, S, seed=1000)
    ev1.record(stream)
    torch.cuda.synchronize()
    first_ms = max(ev0.elapsed_time(ev1), 1e-3)
    # ~60 ms of untimed walks (the clock ramp: a 0.9-ms walk needs ~35 launches to reach its
    # steady clock, profiles/r03_cfg2_kernel_trace), then >= 3 timed (~20 ms, at most 20)
    untimed = max(2, min(KT_UNTIMED, math.ceil(60.0 / first_ms)))
    reps = max(3, min(KT_TIMED, math.ceil(20.0 / first_ms)))
    for i in range(untimed):
        E.run_walk(pk, plan, fixed, B, S, seed=1001 + i)
    ev0.record(stream)
    for i in range(reps):
        E.run_walk(pk, plan, fixed, B, S, seed=i + 2)
    ev1.record(stream)
    torch.cuda.synchronize()
    kern_ms = ev0.elapsed_time(ev1) / reps
    assert bool(ops.LAST_WALK.get("specialised")) == specialised, "kernel timing ran another walk form"
    kernel_name = "vbn_walk_plan" if specialised else "vbn_walk_kernel"
    precomputed = bool(E.LAST_LAUNCH.get("precomputed"))
    n_pre_s = n_pre_q = 0
    if precomputed:
        # nodes with shared-root parents computed once per sample, nodes with evidence parents
        # once per query: the HIP-event interval holds both pre-pass launches as well as the
        # walk (plan.precompute_plans)
        fl = plan.pc.steps[:, 2]
        n_pre_q = int(((fl & 32768) != 0).sum().item())
        n_pre_s = int(((fl & 8192) != 0).sum().item()) - n_pre_q
        kernel_name += (" + pre-passes (vbn_walk_kernel: " + ", ".join(
            t for t, n in (("per-sample, 1 query", n_pre_s), ("per-query, B x 64", n_pre_q)) if n) + ")")

    # the host path's own settling (caching allocator, Python-side caches) before the W warmup
    # steps: ~50 ms of untimed infer_posterior calls, like the walks of the kernel timing above
    # (a 20-step window right after a handful of calls measured 0.92 vs 0.82 ms per step in
    # steady state, profiles/r03_bench/r03t_blocks.txt)
    log(f"kernel {kern_ms:.4f} ms; settling calls")
    n_settle = max(5, min(200, math.ceil(50.0 / kern_ms)))
    if dist:
        # every call gathers (a collective): all ranks must make the same number of calls, and
        # their kernel times differ (the max keeps the slowest rank's ~50 ms)
        t = torch.tensor([n_settle], dtype=torch.int64, device=device if args.dist_backend == "nccl" else "cpu")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        n_settle = int(t.item())
    for _ in range(n_settle):
        vbn.infer_posterior(query)
    sharded.wait()
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        vbn.infer_posterior(query)
    sharded.wait()
    torch.cuda.synchronize()

    # timed region: exactly K steps, barrier + synchronize on both sides (the synchronize
    # also waits for the last step's gather on RCCL's stream)
    fallbacks = []
    # Python's cyclic GC off inside the timed region (as timeit does): a collection pause early
    # in a short timed loop, while the host is only a step or two ahead, idles the GPU.  No
    # gc.collect() here: a full collection right before t0 idles the GPU for long enough that
    # its clocks drop (0.976 vs 0.813 ms per step over the driver's 20 steps)
    log("timed region")
    sharded.verify = False
    gc.disable()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pdf, samples = vbn.infer_posterior(query)
        if hasattr(engine, "fallback_flag"):        # IS: the device flag, read after the timing
            fallbacks.append(engine.fallback_flag())
    sharded.wait()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    fallbacks = [bool(f.item()) for f in fallbacks if f is not None]
    if dist:
        t = torch.tensor([elapsed], device=device if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = world * B * args.steps / elapsed
    if rank == 0 and gather:
        assert pdf is not None and pdf.shape[0] == world * B, "rank 0 must hold the gathered batch"

    # the gather's cost, outside the timed region: the same steps with no gather and with a
    # synchronous (not overlapped) gather, max over ranks; rank 0's received bytes per step
    gather_info = None
    if dist and gather:
        def window(n, on, overlap):
            sharded.gather, sharded.overlap = on, overlap
            barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(n):
                vbn.infer_posterior(query)
            sharded.wait()
            torch.cuda.synchronize()
            barrier()
            dt = torch.tensor([time.perf_counter() - t], dtype=torch.float64,
                              device=device if args.dist_backend == "nccl" else "cpu")
            tdist.all_reduce(dt, op=tdist.ReduceOp.MAX)
            return 1e3 * float(dt.item()) / n
        log("gather accounting")
        n_g = max(5, min(args.steps, 20))
        b0 = sharded.gather_bytes
        walk_only = window(n_g, False, False)
        sync_gather = window(n_g, True, False)
        per_step = (sharded.gather_bytes - b0) / n_g
        sharded.gather, sharded.overlap = True, True
        gather_info = {"bytes_to_rank0_per_step": int(per_step) if rank == 0 else None,
                       "walk_only_ms_per_step": round(walk_only, 4),
                       "sync_gather_ms_per_step": round(sync_gather, 4),
                       "gather_ms_per_step_unoverlapped": round(sync_gather - walk_only, 4),
                       "overlapped_ms_per_step": round(ms_per_step, 4),
                       "steps_each": n_g}

    f32_fl, hid_fl = mlp_flops_per_particle(model, plan)
    f32_fl, hid_fl = f32_fl * B * S, hid_fl * B * S
    flops = f32_fl + hid_fl
    exact = bool(getattr(engine, "exact_f32", False))
    hid_peak = FP32_PEAK_TFLOPS if exact else F16_PEAK_TFLOPS / SPLIT_PASSES
    exps = kde_exps_per_particle(model, plan) * B * S
    traffic, traffic_src = load_traffic(args.config)
    kern_s = kern_ms * 1e-3
    ex_f32, ex_hid, ex_exps = executed_work(model, plan, B, S, precomputed)
    ex_flops = ex_f32 + ex_hid
    if exps > 0.1 * flops / 64:
        # KDE: one exp per (particle, point) kernel weight; the bound is the v_exp_f32 issue rate
        ach = exps / kern_s / 1e12
        roof = {"bound": "exp", "achieved": round(ach, 4), "peak": round(EXP_PEAK_T, 2), "unit": "Texp/s",
                "frac": round(ach / EXP_PEAK_T, 4), "traffic": traffic, "kernel": kernel_name,
                "kernel_ms": round(kern_ms, 4), "exps_per_launch": exps,
                "peak_basis": "v_exp_f32 issue: 8 cyc per wave64 per SIMD, 1024 SIMDs, 2.4 GHz",
                "executed_exps_per_launch": ex_exps,
                "executed_frac": round(ex_exps / kern_s / 1e12 / EXP_PEAK_T, 4),
                "launches_timed": reps, "launches_untimed_before": untimed + 1}
    else:
        # blended peak: each FLOP class at the dense peak of the unit that runs it
        t_min = f32_fl / (FP32_PEAK_TFLOPS * 1e12) + hid_fl / (hid_peak * 1e12)
        peak = flops / t_min / 1e12
        achieved = flops / kern_s / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "kernel": kernel_name, "kernel_ms": round(kern_ms, 4), "flops_per_launch": flops,
                "hidden_layer": "f32 MFMA" if exact else "split-f16 MFMA (3 pass, f32 accumulate)",
                "peak_basis": f"f32 FLOPs at {FP32_PEAK_TFLOPS} TF, hidden-layer FLOPs at {hid_peak:.1f} TF",
                "f32_equiv_frac_of_fp32_peak": round(achieved / FP32_PEAK_TFLOPS, 4),
                "executed_flops_per_launch": ex_flops,
                "executed_frac": round(ex_flops / kern_s / 1e12 /
                                       (ex_flops / (ex_f32 / (FP32_PEAK_TFLOPS * 1e12) + ex_hid / (hid_peak * 1e12)) / 1e12), 4),
                "launches_timed": reps, "launches_untimed_before": untimed + 1}
    roof["traffic_source"] = traffic_src

    par = f"query-sharded dp{world}" + (" + one RCCL gather of pdf/samples to rank 0 per step (async, "
                                        "overlapping the next walk)" if gather and dist else "")
    out = {
        "metric": "posterior queries/sec (infer_posterior, n_samples=1024) at 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "queries/s",
        "n_gpus": tdist.get_world_size() if dist else 1,
        "ranks_seen": seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (SURVEY §8d DAG/SEM/query generator; {cfg['model_origin']} CPDs)",
        "config": {"workload": f"{args.config}: {cfg['name']}", "queries_per_gpu": B, "global_batch": B * world,
                   "n_samples": S, "n_nodes": cfg["n_nodes"], "engine": cfg["engine"],
                   "parallelism": par, "gather": gather and dist, "prune_barren": args.prune_barren,
                   "exact_f32": args.exact_f32, "kde_distances": "valu" if args.kde_valu else "mfma",
                   "walk": ("plan-specialised (step table compiled in with hiprtc)" if specialised
                            else "step-table interpreter"),
                   "plan_compile_s": round(jit.STATS["compile_s"], 2), "plan_cache_hits": jit.STATS["disk_hits"],
                   "first_call_s": round(t_first, 2), "background_compile_wait_s": round(t_wait, 2),
                   "precompute_nodes": {"per_sample": n_pre_s, "per_query": n_pre_q},
                   "kde_moment_nodes": int(sum(1 for r in plan.steps.tolist()
                                               if r[0] == KIND_ID["kde"] and r[1] == 1 and r[31] >= 0))},
        "roofline": roof,
    }
    if fallbacks:
        out["config"]["is_fallback_steps"] = sum(fallbacks)
    if gather_info is not None:
        out["gather"] = gather_info
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # a bounded sample of ~10-30 s of CPU work (the oracle's q/s is linear in B): cfg2 /
        # anchor64 1024 queries, cfg3 (IS, ~100 q/s) 256, cfg5 (~0.7 q/s) 4, cfg4 (~0.2 q/s) 1;
        # KDE configs time 3 repetitions after the warm-up (~5 s each), the others 5
        kde = "kde" in cfg["kinds"]
        if args.cpu_queries:
            nq = args.cpu_queries
        elif kde:
            nq = 1 if cfg["kinds"] == ("kde",) else 4
        else:
            nq = 1024 if cfg["engine"] == "monte_carlo_marginalization" else 256
        reps_cpu = min(3, args.cpu_reps) if kde else args.cpu_reps
        print(f"cpu baseline: {nq} queries in a child process ...", file=sys.stderr, flush=True)
        out["cpu_baseline"] = cpu_baseline(args.config, nq, reps_cpu)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
