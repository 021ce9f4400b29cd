#!/bin/bash
# One GPU call: parity tests, smoke, default bench (with CPU baseline), short benches of other configs.
#   bash scripts/gpu_round.sh [config ...]
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; tail -1 gpurun_out/bench_default.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_default.log; exit $rc; }
for c in "$@"; do
  timeout -k 10 300 python bench.py --config "$c" --steps 10 --warmup 2 --no-cpu-baseline > "gpurun_out/bench_$c.log" 2>&1
  rc=$?; echo "$c exit $rc"; tail -1 "gpurun_out/bench_$c.log"
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/bench_$c.log"; exit $rc; }
done
exit 0
