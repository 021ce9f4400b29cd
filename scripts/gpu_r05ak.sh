#!/bin/bash
# round 5 ak: final same-box bench lines on the final tree: cfg4 (default),
# cfg5, cfg3, cfg2, anchor64, then the Gibbs bench
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ak}
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
for c in cfg5 cfg3 cfg2 anchor64; do
  timeout -k 10 400 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/${T}_bench_$c.json 2>gpurun_out/${T}_bench_$c.err || { tail -30 gpurun_out/${T}_bench_$c.err; exit 1; }
  cat gpurun_out/${T}_bench_$c.json; echo
done
timeout -k 10 500 python -u profiles/bench_gibbs.py > gpurun_out/${T}_gibbs_4096.json 2>gpurun_out/${T}_gibbs.err || { tail -30 gpurun_out/${T}_gibbs.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096.json
