#!/bin/bash
# round 4: every config's bench with the CPU baseline, rocprofv3 kernel stats + PMC per config
# (profiles/r04_<cfg>_*), and a 2-rank gather rehearsal (gloo, one GPU)
set -o pipefail
mkdir -p gpurun_out
for c in cfg2 cfg3 anchor64 cfg4 cfg5; do
  timeout -k 10 500 python -u bench.py --config $c > gpurun_out/r04c_bench_$c.json 2>gpurun_out/r04c_bench_$c.err || exit 1
  cat gpurun_out/r04c_bench_$c.json
done
