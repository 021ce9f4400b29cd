#!/bin/bash
# round 3: full GPU suite (generic MLP / shapes / handles), cfg2 bench, stall PMC on cfg2 and cfg3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > gpurun_out/r03c_pytest_gpu.txt 2>&1; rc=$?
tail -25 gpurun_out/r03c_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03c_bench_cfg2.json 2>gpurun_out/r03c_bench.err || exit 1
cat gpurun_out/r03c_bench_cfg2.json
timeout -k 10 30 rocprofv3 -L > gpurun_out/r03c_counters.txt 2>&1 || true
bash scripts/pmc_stalls.sh r03c_cfg2 "" cfg2 || exit 1
bash scripts/pmc_stalls.sh r03c_cfg3 "" cfg3 || exit 1
