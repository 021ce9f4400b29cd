"""VBN.infer_relative per call (vbn.py:519-568: two posteriors + two summaries) with the summary
fused into the engines' reductions (default) against the separate vbn_hip_posterior_stats pass
(VBN_FUSED_STATS=0), same process, alternating ABAB, on a bench workload.

    python scripts/bench_relative.py [--config cfg3] [--reps 20]

Prints one JSON line: per-call milliseconds (median over reps) of each form and the maximum
difference of their outputs (same seeds, so the same draws)."""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    cfg, model, vbn, query = bench.build_workload(a.config, "cuda:0")
    vbn.set_inference_method(cfg["engine"], n_samples=cfg["S"], seed=1)
    ref_query = {"target": query["target"]}
    times = {"fused": [], "separate": []}
    outs = {}
    for rep in range(a.reps + 2):
        for mode in ("fused", "separate"):
            os.environ["VBN_FUSED_STATS"] = "1" if mode == "fused" else "0"
            vbn._inference.seed = 1                  # same draws in both forms
            vbn._inference._calls = 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = vbn.infer_relative(query, ref_query)
            torch.cuda.synchronize()
            if rep >= 2:
                times[mode].append((time.perf_counter() - t0) * 1e3)
            outs[mode] = out
    diff = max(float((outs["fused"][k][s] - outs["separate"][k][s]).abs().max())
               for k in ("query_stats", "reference_stats") for s in ("mean", "std", "effective_sample_size"))
    print(json.dumps({"config": a.config, "engine": cfg["engine"], "B": cfg["B"], "S": cfg["S"],
                      "fused_ms": statistics.median(times["fused"]),
                      "separate_ms": statistics.median(times["separate"]),
                      "max_abs_diff": diff, "reps": a.reps}))


if __name__ == "__main__":
    main()
