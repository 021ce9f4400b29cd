#!/bin/bash
# round 5 aj: final check on the final tree:
# smoke and the GPU suite (scripts/gpu_r05q.sh: benches + profiles)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05aj}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
tail -22 gpurun_out/${T}_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
