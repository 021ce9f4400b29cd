#!/bin/bash
# round 3: cfg3 interpreter vs specialised with / without the MFMA head (diagnostic), then the
# rest of the suite past test_gpu_jit, Gibbs chain-workgroup benches
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 300 python -u scripts/diag_headmfma.py > gpurun_out/r03n_diag.txt 2>&1; rc=$?
cat gpurun_out/r03n_diag.txt | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread --deselect "tests/test_gpu_jit.py::test_specialised_walk_bit_identical[cfg3-is]" > gpurun_out/r03n_pytest_gpu.txt 2>&1; rc=$?
tail -8 gpurun_out/r03n_pytest_gpu.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in 4096 8192; do
  for w in 0 4; do
    timeout -k 10 300 python -u profiles/bench_gibbs.py --chains $c --chain-waves $w --no-cpu-baseline > gpurun_out/r03n_gibbs_${c}_cw$w.json 2>gpurun_out/r03n_gibbs_${c}_cw$w.err || exit 1
    cat gpurun_out/r03n_gibbs_${c}_cw$w.json
  done
done
