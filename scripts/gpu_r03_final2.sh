#!/bin/bash
# round 3 final evidence, part 2: the other configs with the CPU baseline, Gibbs (auto form)
set -o pipefail
mkdir -p gpurun_out
for c in cfg3 anchor64 cfg4 cfg5; do
  timeout -k 10 500 python -u bench.py --config $c > gpurun_out/r03f_bench_$c.json 2>gpurun_out/r03f_bench_$c.err || exit 1
  cat gpurun_out/r03f_bench_$c.json
done
timeout -k 10 400 python -u profiles/bench_gibbs.py > gpurun_out/r03f_gibbs_4096.json 2>gpurun_out/r03f_gibbs_4096.err || exit 1
cat gpurun_out/r03f_gibbs_4096.json
