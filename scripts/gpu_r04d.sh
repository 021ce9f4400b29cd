#!/bin/bash
# round 4: rocprofv3 kernel stats + PMC per config, then the 2-rank gather rehearsal
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/profile_configs.sh r04 cfg2 cfg3 cfg4 cfg5 anchor64 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r04d_gloo2.json 2> gpurun_out/r04d_gloo2.err || exit 1
cat gpurun_out/r04d_gloo2.json
