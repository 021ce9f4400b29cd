#!/bin/bash
# round 6 b: smoke + GPU suite (regenerated fixtures, in-kernel LW clamp, register-resident
# normalisation, tighter lean-parity margin), the cfg3 IS bench + kernel trace (the step's
# small kernels), the cfg4 bench, then cfg4's profile (trace + PMC passes) for the roofline's
# traffic figure
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r06b}
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
tail -8 gpurun_out/${T}_pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config cfg3 --steps 20 --warmup 5 > gpurun_out/${T}_bench_cfg3.json 2>gpurun_out/${T}_bench_cfg3.err || { tail -30 gpurun_out/${T}_bench_cfg3.err; exit 1; }
cat gpurun_out/${T}_bench_cfg3.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_cfg3_trace -o run -- python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_cfg3_trace.log 2>&1 || { tail -20 gpurun_out/${T}_cfg3_trace.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
timeout -k 10 900 bash scripts/profile_configs.sh ${T} cfg4 > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
tail -3 gpurun_out/${T}_prof.log
exit $rc
