#!/bin/bash
# round 5 i: rocprofv3 kernel stats + PMC of cfg2 / cfg3 (3 waves per SIMD) / cfg5 / anchor64,
# and the cfg3 bench on the 3-wave plan kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config cfg3 --steps 20 --warmup 5 > gpurun_out/r05i_bench_cfg3.json 2>gpurun_out/r05i_bench_cfg3.err || { tail -20 gpurun_out/r05i_bench_cfg3.err; exit 1; }
cat gpurun_out/r05i_bench_cfg3.json
bash scripts/profile_configs.sh r05i cfg3 cfg2 cfg5 anchor64 || exit 1
