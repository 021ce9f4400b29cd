#!/bin/bash
# round 4 n: the Gibbs sampler bench on the final kernels (cfg2 DAG, 4096 chains, YAML defaults)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/r04n_gibbs_4096.json 2>gpurun_out/r04n_gibbs_4096.err || { tail -20 gpurun_out/r04n_gibbs_4096.err; exit 1; }
cat gpurun_out/r04n_gibbs_4096.json
