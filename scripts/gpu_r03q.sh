#!/bin/bash
# round 3: specialised-vs-interpreter identity with the MFMA head off; MFMA-head A/B on cfg3;
# shared-sample precompute A/B benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_jit.py -q -rs -x --timeout 600 --timeout-method thread -k "specialised_walk" > gpurun_out/r03q_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r03q_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 exp/plan_cfg3_base.hsaco exp/plan_cfg3_nohm.hsaco > gpurun_out/r03q_ab_cfg3.txt 2>&1 || { tail -5 gpurun_out/r03q_ab_cfg3.txt; exit 1; }
grep variant gpurun_out/r03q_ab_cfg3.txt
for c in cfg2 anchor64 cfg4 cfg5; do
  for pc in pc nopc; do
    extra=""; [ $pc = nopc ] && extra="--no-precompute"
    timeout -k 10 500 python -u bench.py --config $c --no-cpu-baseline $extra > gpurun_out/r03q_bench_${c}_$pc.json 2>gpurun_out/r03q_bench_${c}_$pc.err || exit 1
    cat gpurun_out/r03q_bench_${c}_$pc.json
  done
done
