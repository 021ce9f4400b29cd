#!/bin/bash
# round 4 second pass: library with the per-query precompute (ABI v9) and hardware
# transcendentals; smoke, the GPU suite, the driver-form default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04b_smoke.txt 2>&1 || { cat gpurun_out/r04b_smoke.txt; exit 1; }
tail -1 gpurun_out/r04b_smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04b_pytest_gpu.txt 2>&1
rc=$?
tail -4 gpurun_out/r04b_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04b_bench_$i.json 2>gpurun_out/r04b_bench_$i.err || exit 1
  cat gpurun_out/r04b_bench_$i.json
done
