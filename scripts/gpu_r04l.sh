#!/bin/bash
# round 4 l: relu folded into the f16 split, side-stream pre-pass off (final kernels of the
# round): smoke, GPU suite, benches of every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04l_smoke.txt 2>&1 || { cat gpurun_out/r04l_smoke.txt; exit 1; }
tail -1 gpurun_out/r04l_smoke.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04l_bench_$i.json 2>gpurun_out/r04l_bench_$i.err || exit 1
  cat gpurun_out/r04l_bench_$i.json
done
timeout -k 10 800 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04l_pytest_gpu.txt 2>&1
rc=$?
tail -3 gpurun_out/r04l_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for c in cfg3 anchor64 cfg4 cfg5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r04l_bench_$c.json 2>gpurun_out/r04l_bench_$c.err || exit 1
  cat gpurun_out/r04l_bench_$c.json
done
