#!/bin/bash
# round 3: full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > gpurun_out/r03b_pytest_gpu.txt 2>&1; rc=$?
tail -15 gpurun_out/r03b_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03b_smoke.txt 2>&1 || { tail -20 gpurun_out/r03b_smoke.txt; exit 1; }
cat gpurun_out/r03b_smoke.txt
