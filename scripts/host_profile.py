#!/usr/bin/env python3
"""Host-side cost of one bench step (GPU box): cProfile over K infer_posterior calls of a bench
workload through the bench's ShardedEngine wrapper, with the GPU kept busy as in the timed
loop; prints the top functions by own time and the per-call wall time."""
from __future__ import annotations

import cProfile
import os
import pstats
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from vectorizedbayesiannetwork_amd.distributed import ShardedEngine
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    torch.cuda.set_device(0)
    cfg, model, vbn, query = bench.build_workload(cfg_name, "cuda:0", 1)
    vbn.set_inference_method(cfg["engine"], n_samples=cfg["S"])
    sh = ShardedEngine(vbn._inference, gather=True, overlap=True)
    vbn._inference = sh
    for _ in range(20):
        vbn.infer_posterior(query)
    sh.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        vbn.infer_posterior(query)
    t_cpu = time.perf_counter() - t0
    sh.wait()
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"{cfg_name}: host issue {1e3 * t_cpu / k:.3f} ms/call, wall {1e3 * t_all / k:.3f} ms/call", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(k):
        vbn.infer_posterior(query)
    pr.disable()
    sh.wait()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
