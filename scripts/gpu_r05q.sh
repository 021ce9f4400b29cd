#!/bin/bash
# round 5 q: the tile-pipelined KDE pass 1: default (cfg4) bench, cfg5 bench, then rocprofv3
# kernel stats + PMC of cfg4 and cfg5 (the bench's roofline traffic source)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05q}
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
timeout -k 10 400 python -u bench.py --config cfg5 --steps 20 --warmup 5 > gpurun_out/${T}_bench_cfg5.json 2>gpurun_out/${T}_bench_cfg5.err || { tail -30 gpurun_out/${T}_bench_cfg5.err; exit 1; }
cat gpurun_out/${T}_bench_cfg5.json; echo
bash scripts/profile_configs.sh r05p cfg4 cfg5 || exit 1
