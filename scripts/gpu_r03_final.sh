#!/bin/bash
# round 3 final evidence: suite, smoke, default bench (as the driver runs it), rocprofv3 kernel
# stats + PMC passes of the default bench (profiles/profile_round.sh), cfg3/cfg4/cfg5/anchor64
# benches with the CPU baseline
set -o pipefail
mkdir -p gpurun_out
# heartbeat: plan compiles inside a test (hiprtc, up to ~4 min for the 128-node plans) print nothing
(while true; do date >> gpurun_out/r03f_heartbeat.txt; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs -x --timeout 600 --timeout-method thread > gpurun_out/r03f_pytest_gpu.txt 2>&1 || { tail -20 gpurun_out/r03f_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/r03f_pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/r03f_smoke.txt 2>&1 || { tail -20 gpurun_out/r03f_smoke.txt; exit 1; }
tail -1 gpurun_out/r03f_smoke.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03f_bench_default.json 2>gpurun_out/r03f_bench_default.err || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03f_bench_default2.json 2>/dev/null || exit 1
cat gpurun_out/r03f_bench_default2.json
cat gpurun_out/r03f_bench_default.json
bash profiles/profile_round.sh gpurun_out/r03f_prof cfg2 > gpurun_out/r03f_prof.log 2>&1 || { tail -5 gpurun_out/r03f_prof.log; exit 1; }
echo profiled
