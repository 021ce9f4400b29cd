#!/bin/bash
# round 6 l: half sums kept to long chunks (KDE_HALF_MIN): smoke, GPU suite, cfg4 / cfg5 benches,
# cfg4 / cfg5 profiles (kernel trace + PMC)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r06l}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
tail -8 gpurun_out/${T}_pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
head -c 700 gpurun_out/${T}_bench_cfg4.json; echo
timeout -k 10 400 python -u bench.py --config cfg5 > gpurun_out/${T}_bench_cfg5.json 2>gpurun_out/${T}_bench_cfg5.err || { tail -30 gpurun_out/${T}_bench_cfg5.err; exit 1; }
head -c 700 gpurun_out/${T}_bench_cfg5.json; echo
timeout -k 10 900 bash scripts/profile_configs.sh ${T} cfg4 cfg5 > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
tail -3 gpurun_out/${T}_prof.log
exit $rc
