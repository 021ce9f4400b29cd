#!/bin/bash
# round 5 b: KDE pass-1 microbenchmark (walk-form variants) and the GPU test suite
set -o pipefail
mkdir -p gpurun_out
hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 profiles/microbench/kde_pass1.hip -o gpurun_out/kde_pass1 2>/dev/null || exit 1
timeout -k 10 180 gpurun_out/kde_pass1 > gpurun_out/r05b_kde_pass1.json 2>&1 || exit 1
cat gpurun_out/r05b_kde_pass1.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r05b_pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/r05b_pytest_gpu.txt
exit $rc
