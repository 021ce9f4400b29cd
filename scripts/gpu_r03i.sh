#!/bin/bash
# round 3: reciprocal probabilities (suite), Gibbs sweep variants A/B, cfg3 bench
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 300 --timeout-method thread > gpurun_out/r03i_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r03i_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/jit_ab_gibbs.py exp/gibbs_base.hsaco exp/gibbs_noexact.hsaco > gpurun_out/r03i_ab_gibbs.txt 2>&1 || exit 1
grep variant gpurun_out/r03i_ab_gibbs.txt
timeout -k 10 400 python -u bench.py --config cfg3 --no-cpu-baseline > gpurun_out/r03i_bench_cfg3.json 2>gpurun_out/r03i_bench_cfg3.err || exit 1
cat gpurun_out/r03i_bench_cfg3.json
