#!/bin/bash
# round 3: split-f16 MFMA head for mdn / softmax_nn -- suite on HEAD, cfg3 A/B (MFMA head vs the
# VALU head, same plan), cfg2 / cfg3 / cfg5 benches
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 300 --timeout-method thread > gpurun_out/r03k_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r03k_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 exp/plan_cfg3_base.hsaco exp/plan_cfg3_nohm.hsaco > gpurun_out/r03k_ab_cfg3.txt 2>&1 || exit 1
grep variant gpurun_out/r03k_ab_cfg3.txt
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r03k_bench_$c.json 2>gpurun_out/r03k_bench_$c.err || exit 1
  cat gpurun_out/r03k_bench_$c.json
done
