#!/bin/bash
# round 5 e: smoke, the GPU suite and the default (cfg4) bench on the final KDE kernels
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05e}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json
