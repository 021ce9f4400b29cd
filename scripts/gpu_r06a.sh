#!/bin/bash
# round 6 a: smoke + GPU suite on the round-6 tree (moment tables, bench rank launch, Gibbs LDS
# fit), then the cfg4 bench with and without the KDE moment tables (same box), the 2-rank
# launch rehearsal (gloo, both ranks on the one GPU), cfg5 and a cfg3 kernel trace
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r06a}
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
tail -8 gpurun_out/${T}_pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
VBN_KDE_MOMENTS=0 timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_cfg4_nomt.json 2>gpurun_out/${T}_bench_cfg4_nomt.err || { tail -30 gpurun_out/${T}_bench_cfg4_nomt.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4_nomt.json; echo
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1 > gpurun_out/${T}_bench_cfg4_gloo2.json 2>gpurun_out/${T}_bench_cfg4_gloo2.err || { tail -30 gpurun_out/${T}_bench_cfg4_gloo2.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4_gloo2.json; echo
timeout -k 10 400 python -u bench.py --config cfg5 > gpurun_out/${T}_bench_cfg5.json 2>gpurun_out/${T}_bench_cfg5.err || { tail -30 gpurun_out/${T}_bench_cfg5.err; exit 1; }
cat gpurun_out/${T}_bench_cfg5.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_cfg3_trace -o run -- python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_cfg3_trace.log 2>&1 || { tail -20 gpurun_out/${T}_cfg3_trace.log; exit 1; }
ls gpurun_out/${T}_cfg3_trace
exit $rc
