#!/bin/bash
# round 5 f: the other workloads' benches (driver form: 20 steps, 5 warmup) with CPU baselines,
# and the Gibbs sampler bench
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05f}
for c in cfg2 cfg3 anchor64 cfg5; do
  timeout -k 10 600 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/${T}_bench_$c.json 2>gpurun_out/${T}_bench_$c.err || { tail -30 gpurun_out/${T}_bench_$c.err; exit 1; }
  cat gpurun_out/${T}_bench_$c.json
done
timeout -k 10 400 python -u profiles/bench_gibbs.py > gpurun_out/${T}_gibbs_4096.json 2>gpurun_out/${T}_gibbs.err || { tail -30 gpurun_out/${T}_gibbs.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096.json
# 2-rank rehearsal of the multi-GPU bench path (default workload cfg4) on one GPU over gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.err || { tail -20 gpurun_out/${T}_gloo2.err; exit 1; }
cat gpurun_out/${T}_gloo2.json
