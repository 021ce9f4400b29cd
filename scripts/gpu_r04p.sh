#!/bin/bash
# round 4 p: the final tree as the driver runs it -- smoke, GPU suite, the default bench (with
# its CPU baseline), and the 2-rank gather rehearsal (gloo, one GPU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04p_smoke.txt 2>&1 || { cat gpurun_out/r04p_smoke.txt; exit 1; }
tail -1 gpurun_out/r04p_smoke.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04p_pytest_gpu.txt 2>&1
rc=$?
tail -3 gpurun_out/r04p_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/r04p_bench_default.json 2>gpurun_out/r04p_bench_default.err || exit 1
cat gpurun_out/r04p_bench_default.json
bash scripts/gpu_r04e.sh || exit 1
