#!/bin/bash
# GPU iteration loop: parity tests, then short benches of the given configs (no CPU baseline).
#   bash scripts/gpu_check.sh [config ...]      (default: cfg2 anchor64 cfg3)
set -o pipefail
mkdir -p gpurun_out
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=(cfg2 anchor64 cfg3)
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "max scaled|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -5
[ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for c in "${cfgs[@]}"; do
  timeout -k 10 300 python bench.py --config "$c" --steps 20 --warmup 5 --no-cpu-baseline > "gpurun_out/bench_$c.log" 2>&1
  rc=$?; echo "$c exit $rc"; tail -1 "gpurun_out/bench_$c.log" | python3 -c '
import sys, json
try:
    d = json.loads(sys.stdin.read()); r = d["roofline"]
    print(d["config"]["workload"], round(d["value"]), round(d["ms_per_step"], 4), "kernel_ms", r.get("kernel_ms"), "frac", round(r["frac"], 4))
except Exception as e:
    print("unparsed", e)'
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/bench_$c.log"; exit $rc; }
done
exit 0
