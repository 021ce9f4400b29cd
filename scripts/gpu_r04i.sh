#!/bin/bash
# round 4 i: rocprofv3 kernel stats + PMC passes of the bf16x3 KDE kernels (cfg4, cfg5), then
# their benches with the CPU baseline
set -o pipefail
mkdir -p gpurun_out
bash scripts/profile_configs.sh r04 cfg4 cfg5 || exit 1
for c in cfg4 cfg5; do
  timeout -k 10 500 python -u bench.py --config $c > gpurun_out/r04i_bench_$c.json 2>gpurun_out/r04i_bench_$c.err || exit 1
  cat gpurun_out/r04i_bench_$c.json
done
