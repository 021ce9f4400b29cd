#!/bin/bash
# round 5 f: the other workloads' benches (driver form: 20 steps, 5 warmup) with CPU baselines,
# the cfg3 occupancy and cfg5 ablation A/Bs, and the 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05f}
for c in cfg2 cfg3 anchor64 cfg5; do
  timeout -k 10 600 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/${T}_bench_$c.json 2>gpurun_out/${T}_bench_$c.err || { tail -30 gpurun_out/${T}_bench_$c.err; exit 1; }
  cat gpurun_out/${T}_bench_$c.json
done
# 2-rank rehearsal of the multi-GPU bench path (default workload cfg4) on one GPU over gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.err || { tail -20 gpurun_out/${T}_gloo2.err; exit 1; }
cat gpurun_out/${T}_gloo2.json
# cfg3 at 3 waves per SIMD (no spills) against 4 (A/B code objects, ABAB)
VBN_LIVENESS_ORDER=0 timeout -k 10 400 python -u scripts/jit_ab.py --config cfg3 abx5/plan_cfg3_base.hsaco abx5/plan_cfg3_wpe3.hsaco \
  abx5/plan_cfg3_base.hsaco abx5/plan_cfg3_wpe3.hsaco > gpurun_out/${T}_ab_cfg3.txt 2>&1 || { tail -20 gpurun_out/${T}_ab_cfg3.txt; exit 1; }
grep variant gpurun_out/${T}_ab_cfg3.txt
# cfg5 per-kind ablations (model-order plan without precompute)
if [ -f abx5/plan_cfg5_nol2.hsaco ]; then
  VBN_LIVENESS_ORDER=0 timeout -k 10 600 python -u scripts/jit_ab.py --config cfg5 abx5/plan_cfg5_base.hsaco abx5/plan_cfg5_nop1.hsaco \
    abx5/plan_cfg5_noscan.hsaco abx5/plan_cfg5_norng.hsaco abx5/plan_cfg5_nohead.hsaco abx5/plan_cfg5_nol2.hsaco \
    > gpurun_out/${T}_ab_cfg5.txt 2>&1 || { tail -20 gpurun_out/${T}_ab_cfg5.txt; exit 1; }
  grep variant gpurun_out/${T}_ab_cfg5.txt
fi
