#!/bin/bash
# round 3: sharded-ranks test, lean parity, bench N=1 (+CPU baseline), 2-rank gloo rehearsal of the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_0_sharded_ranks.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03a_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { echo "bench failed"; tail -30 gpurun_out/r03a_bench.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/r03a_bench2.json 2> gpurun_out/r03a_bench2.err || { echo "bench2 failed"; tail -30 gpurun_out/r03a_bench2.err; exit 1; }
cat gpurun_out/r03a_bench.json gpurun_out/r03a_bench2.json
