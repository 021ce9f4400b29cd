#!/bin/bash
# round 3: plan-specialised walks on the box -- JIT bit-identity, full GPU suite, smoke,
# cfg2 / cfg3 bench (specialised), rocprofv3 trace + PMC of the cfg2 bench
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -m gpu -v -rs --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest_jit.txt 2>&1; rc=$?
tail -15 gpurun_out/r03d_pytest_jit.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r03d_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03d_smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r03d_bench_cfg2.json 2>gpurun_out/r03d_bench_cfg2.err || exit 1
cat gpurun_out/r03d_bench_cfg2.json
timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline > gpurun_out/r03d_bench_cfg3.json 2>gpurun_out/r03d_bench_cfg3.err || exit 1
cat gpurun_out/r03d_bench_cfg3.json
bash scripts/profile_configs.sh r03 cfg2 || exit 1
