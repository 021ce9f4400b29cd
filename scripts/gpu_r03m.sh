#!/bin/bash
# round 3: suite on the ABI-v8 build (split-f16 MFMA heads, chain-workgroup Gibbs sweeps);
# Gibbs benches (4096 / 8192 chains, chain waves 0 / 4); cfg3 A/B (MFMA head vs VALU head);
# cfg2 / cfg3 / cfg5 benches
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 300 --timeout-method thread > gpurun_out/r03m_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r03m_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for c in 4096 8192; do
  for w in 0 4; do
    timeout -k 10 300 python -u profiles/bench_gibbs.py --chains $c --chain-waves $w --no-cpu-baseline > gpurun_out/r03m_gibbs_${c}_cw$w.json 2>gpurun_out/r03m_gibbs_${c}_cw$w.err || exit 1
    cat gpurun_out/r03m_gibbs_${c}_cw$w.json
  done
done
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 exp/plan_cfg3_base.hsaco exp/plan_cfg3_nohm.hsaco > gpurun_out/r03m_ab_cfg3.txt 2>&1 || exit 1
grep variant gpurun_out/r03m_ab_cfg3.txt
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r03m_bench_$c.json 2>gpurun_out/r03m_bench_$c.err || exit 1
  cat gpurun_out/r03m_bench_$c.json
done
