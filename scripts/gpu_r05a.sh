#!/bin/bash
# round 5 a: KDE pass-1 microbenchmark, smoke, the default (cfg4) bench with its CPU baseline,
# and the cfg4 rocprofv3 kernel stats + PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 profiles/microbench/kde_pass1.hip -o gpurun_out/kde_pass1 || exit 1
timeout -k 10 120 gpurun_out/kde_pass1 > gpurun_out/r05a_kde_pass1.json 2>&1 || exit 1
cat gpurun_out/r05a_kde_pass1.json
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a_smoke.txt 2>&1 || { tail -30 gpurun_out/r05a_smoke.txt; exit 1; }
tail -1 gpurun_out/r05a_smoke.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05a_bench_cfg4.json 2>gpurun_out/r05a_bench_cfg4.err || { tail -30 gpurun_out/r05a_bench_cfg4.err; exit 1; }
cat gpurun_out/r05a_bench_cfg4.json
bash scripts/profile_configs.sh r05a cfg4 || exit 1
