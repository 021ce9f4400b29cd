"""The one rank of tests/test_gpu_rccl_world1.py (not a test module).

A process group of ONE rank on the nccl backend (RCCL) with ``ShardedEngine(...,
force_collectives=True)``: the seed broadcast, the IS fallback flag's MAX all-reduce and the
gathers of pdf / samples (async, into the [world, shard, ...] buffer) all run as RCCL
collectives on the box's GPU -- the multi-GPU bench's code path, at the world size a one-GPU box
allows.  Saves what it saw for the test to compare with unsharded engines.
"""
from __future__ import annotations

import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B, S = 64, 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=a.init, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from _sharded_worker import cases
        from workloads import synthetic_workload
        from vectorizedbayesiannetwork_amd.distributed import ShardedEngine
        from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query
        model, vbn, target, ev = synthetic_workload("cfg2", B, "cuda")
        res = {"backend": dist.get_backend()}
        for name, make, query, overlap in cases(vbn, target, ev):
            torch.manual_seed(4242)
            sh = ShardedEngine(make(), gather=True, overlap=overlap, force_collectives=True)
            seeds = []
            for _ in range(2):
                pdf, xs = sh.infer_posterior(vbn, query)
                seeds.append(sh.last_seed)
            sh.wait()
            torch.cuda.synchronize()
            res[name] = {"seeds": seeds, "fallback": bool(getattr(sh.engine, "_last_fallback", False)),
                         "pdf": pdf.cpu(), "xs": xs.cpu(), "pending": len(sh._pending)}
        torch.manual_seed(4242)
        sh = ShardedEngine(AncestralSampler(n_samples=S), gather=True, force_collectives=True)
        xs = sh.sample(vbn, Query(target, {k: v.cuda() for k, v in ev.items()}), S)
        torch.cuda.synchronize()
        res["ancestral"] = {"seeds": [sh.last_seed], "fallback": False, "pdf": None, "xs": xs.cpu()}
        torch.save(res, a.out)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
