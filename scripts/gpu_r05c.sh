#!/bin/bash
# round 5 c: cfg4 with the factored 32x32x16 KDE pass (bench + rocprof), and the cfg4
# ablations (A/B code objects from the model-order plan without precompute)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05c_bench_cfg4.json 2>gpurun_out/r05c_bench_cfg4.err || { tail -30 gpurun_out/r05c_bench_cfg4.err; exit 1; }
cat gpurun_out/r05c_bench_cfg4.json
VBN_LIVENESS_ORDER=0 timeout -k 10 400 python -u scripts/jit_ab.py --config cfg4 abx5/plan_cfg4_base.hsaco \
  abx5/plan_cfg4_noscan.hsaco abx5/plan_cfg4_nop1.hsaco abx5/plan_cfg4_norng.hsaco > gpurun_out/r05c_ab_cfg4.txt 2>&1 || { tail -20 gpurun_out/r05c_ab_cfg4.txt; exit 1; }
grep variant gpurun_out/r05c_ab_cfg4.txt
bash scripts/profile_configs.sh r05c cfg4 || exit 1
