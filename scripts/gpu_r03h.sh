#!/bin/bash
# round 3: layer-1 operand bound instead of the activation range check -- full GPU suite,
# A/B against the previous plan kernels, default bench
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 300 --timeout-method thread > gpurun_out/r03h_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r03h_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg2 exp/plan_cfg2_base.hsaco exp/plan_cfg2_zb.hsaco > gpurun_out/r03h_ab_cfg2.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 exp/plan_cfg3_base.hsaco exp/plan_cfg3_zb.hsaco exp/plan_cfg3_zbrcp.hsaco exp/plan_cfg3_sel.hsaco exp/plan_cfg3_selrcp.hsaco > gpurun_out/r03h_ab_cfg3.txt 2>&1 || exit 1
grep variant gpurun_out/r03h_ab_cfg2.txt gpurun_out/r03h_ab_cfg3.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03h_bench_cfg2.json 2>gpurun_out/r03h_bench_cfg2.err || exit 1
cat gpurun_out/r03h_bench_cfg2.json
