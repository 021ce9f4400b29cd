#!/bin/bash
# round 5 ab: 2-rank rehearsal of the multi-GPU bench path (default workload cfg4) on one GPU over
# gloo, on the final tree
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ab}
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.err || { tail -20 gpurun_out/${T}_gloo2.err; exit 1; }
cat gpurun_out/${T}_gloo2.json
