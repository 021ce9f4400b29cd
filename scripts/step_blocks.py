#!/usr/bin/env python3
"""Per-block step time of a bench workload (GPU box): blocks of K infer_posterior calls, each
bracketed by synchronize, with and without the shared-sample precompute."""
from __future__ import annotations

import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.distributed import ShardedEngine
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    torch.cuda.set_device(0)
    cfg, model, vbn, query = bench.build_workload(cfg_name, "cuda:0", 1)
    vbn.set_inference_method(cfg["engine"], n_samples=cfg["S"])
    sh = ShardedEngine(vbn._inference, gather=True, overlap=True)
    vbn._inference = sh
    for pc in (True, False, True, False):
        E.PRECOMPUTE = pc
        for _ in range(5):
            vbn.infer_posterior(query)
        torch.cuda.synchronize()
        out = []
        for blk in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                vbn.infer_posterior(query)
            sh.wait()
            torch.cuda.synchronize()
            out.append(1e3 * (time.perf_counter() - t0) / 20)
        print(f"precompute={pc}: ms/step per 20-step block " + " ".join(f"{x:.3f}" for x in out), flush=True)


if __name__ == "__main__":
    main()
