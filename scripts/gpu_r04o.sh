#!/bin/bash
# round 4 o: cfg5 plans from the restarted liveness greedy (24 LDS slots, 16 waves per CU):
# the cfg5 GPU tests, then the cfg5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "cfg5" -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04o_pytest_cfg5.txt 2>&1
rc=$?
tail -3 gpurun_out/r04o_pytest_cfg5.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > gpurun_out/r04o_bench_cfg5.json 2>gpurun_out/r04o_bench_cfg5.err || exit 1
cat gpurun_out/r04o_bench_cfg5.json
