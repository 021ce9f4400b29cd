"""One rank of tests/test_gpu_0_sharded_ranks.py (not a test module).

Runs the real engines behind ``ShardedEngine(..., gather=True)`` on this rank's query shard
(all ranks on cuda:0 of the box, collectives over gloo: RCCL refuses two ranks on one GPU)
and saves what it saw: rank 0 the gathered batch, every rank its seeds and fallback flags.
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
B_BIG = 1536                 # cfg3 IS: 1.5 M particles in one process (>= jit.JIT_MIN_PARTICLES), 0.75 M per rank
HOT_NODE_VALUE = 50.0        # off-manifold evidence in the last query (rank 1's shard): ESS ~ 1


def cases(vbn, target, ev):
    from vectorizedbayesiannetwork_amd.engines import ImportanceSampling, MonteCarloMarginalization, Query
    hot = {k: v.clone() for k, v in ev.items()}
    # an evidence node with latent parents: its log-weight varies across the particles, so an
    # off-manifold value collapses that query's ESS (a root's would shift every weight alike)
    par = vbn.model.parents
    k0 = next(k for k in sorted(hot) if par[k] and not any(p in hot for p in par[k]))
    hot[k0][B - 1, 0] = HOT_NODE_VALUE
    q = Query(target, {k: v.cuda() for k, v in ev.items()})
    qh = Query(target, {k: v.cuda() for k, v in hot.items()})
    return [
        ("mcm", lambda: MonteCarloMarginalization(n_samples=S), q, False),
        ("mcm_overlap", lambda: MonteCarloMarginalization(n_samples=S), q, True),
        ("is", lambda: ImportanceSampling(n_samples=S), q, False),
        ("is_hot", lambda: ImportanceSampling(n_samples=S), qh, False),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--init", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dist.init_process_group("gloo", init_method=a.init, rank=a.rank, world_size=a.world)
    try:
        torch.cuda.set_device(0)
        from workloads import synthetic_workload
        from vectorizedbayesiannetwork_amd.distributed import ShardedEngine
        from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query
        model, vbn, target, ev = synthetic_workload("cfg2", B, "cuda")
        res = {}
        for name, make, query, overlap in cases(vbn, target, ev):
            torch.manual_seed(1000 + a.rank)          # ranks disagree: the seed is broadcast
            sh = ShardedEngine(make(), gather=True, overlap=overlap)
            seeds, outs = [], None
            for _ in range(2):                          # call 2: seed from the replicated stream
                outs = sh.infer_posterior(vbn, query)
                seeds.append(sh.last_seed)
            sh.wait()
            torch.cuda.synchronize()
            pdf, xs = outs
            res[name] = {"seeds": seeds, "fallback": bool(getattr(sh.engine, "_last_fallback", False)),
                         "pdf": None if pdf is None else pdf.cpu(), "xs": None if xs is None else xs.cpu()}
        # VBN.precompile behind a ShardedEngine: builds the local plan with no
        # collective and leaves the sharded call counter and the torch RNG alone, so the two
        # calls after it see the seeds of the "mcm" case above
        from vectorizedbayesiannetwork_amd.engines import MonteCarloMarginalization
        torch.manual_seed(1000 + a.rank)
        sh = ShardedEngine(MonteCarloMarginalization(n_samples=S), gather=True)
        vbn._inference = sh
        st = vbn.precompile([{"target": target, "evidence": sorted(ev)}])
        seeds = []
        for _ in range(2):
            pdf, xs = vbn.infer_posterior(Query(target, {k: v.cuda() for k, v in ev.items()}))
            seeds.append(sh.last_seed)
        torch.cuda.synchronize()
        vbn._inference = None
        res["mcm_precompiled"] = {"seeds": seeds, "fallback": False, "plans": st["plans"],
                                  "pdf": None if pdf is None else pdf.cpu(), "xs": None if xs is None else xs.cpu()}
        torch.manual_seed(1000 + a.rank)
        sh = ShardedEngine(AncestralSampler(n_samples=S), gather=True)
        xs = sh.sample(vbn, Query(target, {k: v.cuda() for k, v in ev.items()}), S)
        torch.cuda.synchronize()
        res["ancestral"] = {"seeds": [sh.last_seed], "fallback": False, "pdf": None,
                            "xs": None if xs is None else xs.cpu()}
        # a batch whose single-process launch runs the plan-specialised walk while each rank's
        # half runs the step-table interpreter (forced): the gathered result must not depend on it
        from vectorizedbayesiannetwork_amd.engines import ImportanceSampling
        model3, vbn3, target3, ev3 = synthetic_workload("cfg3", B_BIG, "cuda")
        torch.manual_seed(1000 + a.rank)
        sh = ShardedEngine(ImportanceSampling(n_samples=S, plan_jit=False), gather=True)
        pdf, xs = sh.infer_posterior(vbn3, Query(target3, {k: v.cuda() for k, v in ev3.items()}))
        torch.cuda.synchronize()
        res["is_big_cfg3"] = {"seeds": [sh.last_seed], "fallback": bool(sh.engine._last_fallback),
                              "pdf": None if pdf is None else pdf.cpu(), "xs": None if xs is None else xs.cpu()}
        torch.save(res, a.out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
