#!/bin/bash
# round 4: 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo collectives; both
# ranks started by torch.distributed.run before any GPU call): gather accounting fields
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r04e_gloo2.json 2> gpurun_out/r04e_gloo2.err || { tail -20 gpurun_out/r04e_gloo2.err; exit 1; }
cat gpurun_out/r04e_gloo2.json
