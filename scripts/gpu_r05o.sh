#!/bin/bash
# round 5 o: after the plan-cache regeneration: the default (cfg4) bench, then cfg3 / cfg5 / cfg2
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05o}
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
for c in cfg3 cfg5 cfg2; do
  timeout -k 10 400 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/${T}_bench_$c.json 2>gpurun_out/${T}_bench_$c.err || { tail -30 gpurun_out/${T}_bench_$c.err; exit 1; }
  cat gpurun_out/${T}_bench_$c.json; echo
done
# KDE pass-1 microbenchmark with the pipelined variants (profiles/microbench/kde_pass1.hip, built on the host)
timeout -k 10 300 profiles/microbench/kde_pass1_bin > gpurun_out/${T}_kde_pass1.json 2>&1 || { tail -20 gpurun_out/${T}_kde_pass1.json; exit 1; }
cat gpurun_out/${T}_kde_pass1.json
