#!/bin/bash
# round 3: Gibbs sweeps on chain workgroups (plan.gibbs_levels) -- suite on the ABI-v8 build,
# chain-form parity, Gibbs benches (4096 / 8192 chains, chain waves 0 / 2 / 4)
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 300 --timeout-method thread > gpurun_out/r03l_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r03l_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for c in 4096 8192; do
  for w in 0 2 4; do
    timeout -k 10 300 python -u profiles/bench_gibbs.py --chains $c --chain-waves $w --no-cpu-baseline > gpurun_out/r03l_gibbs_${c}_cw$w.json 2>gpurun_out/r03l_gibbs_${c}_cw$w.err || exit 1
    cat gpurun_out/r03l_gibbs_${c}_cw$w.json
  done
done
