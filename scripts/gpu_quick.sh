#!/bin/bash
# GPU tests, default bench, cfg2 A/B of experiment libraries given as arguments.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("default", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])'
if [ $# -gt 0 ]; then timeout -k 10 500 python scripts/exp_compare.py --config cfg2 "$@" || exit $?; fi
exit 0
