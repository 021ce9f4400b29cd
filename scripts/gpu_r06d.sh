#!/bin/bash
# round 6 d: the fused posterior summary (ABI v13): its GPU tests first, then smoke + the whole GPU
# suite, the cfg4 / cfg3 bench lines, infer_relative fused vs separate (cfg3 IS, cfg4 MCM), and a
# kernel trace of the cfg3 infer_relative calls
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r06d}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_stats.py -v -rA --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest_stats.txt 2>&1
rc=$?
tail -25 gpurun_out/${T}_pytest_stats.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc2=$?
tail -8 gpurun_out/${T}_pytest_gpu.txt
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
timeout -k 10 400 python -u bench.py --config cfg3 > gpurun_out/${T}_bench_cfg3.json 2>gpurun_out/${T}_bench_cfg3.err || { tail -30 gpurun_out/${T}_bench_cfg3.err; exit 1; }
cat gpurun_out/${T}_bench_cfg3.json; echo
timeout -k 10 300 python -u scripts/bench_relative.py --config cfg3 --reps 20 > gpurun_out/${T}_relative_cfg3.json 2>gpurun_out/${T}_relative_cfg3.err || { tail -30 gpurun_out/${T}_relative_cfg3.err; exit 1; }
cat gpurun_out/${T}_relative_cfg3.json
timeout -k 10 300 python -u scripts/bench_relative.py --config cfg4 --reps 6 > gpurun_out/${T}_relative_cfg4.json 2>gpurun_out/${T}_relative_cfg4.err || { tail -30 gpurun_out/${T}_relative_cfg4.err; exit 1; }
cat gpurun_out/${T}_relative_cfg4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_relprof -o rel -- python3 scripts/bench_relative.py --config cfg3 --reps 5 > gpurun_out/${T}_relprof.log 2>&1 || { tail -20 gpurun_out/${T}_relprof.log; exit 1; }
find gpurun_out/${T}_relprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_relative_cfg3_kernel_stats.csv \;
[ $rc -eq 0 ] && exit $rc2
exit $rc
