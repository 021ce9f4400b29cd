#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03u_bench_$i.json 2>/dev/null || exit 1
  cat gpurun_out/r03u_bench_$i.json
done
