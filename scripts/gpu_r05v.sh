#!/bin/bash
# round 5 v: Gibbs step-level (DAG) schedule: bitwise chain tests, then the bench with the cost
# model's pick (the step-level form) and with the per-level choice (the r05m form)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05v}
timeout -k 10 900 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 400 --timeout-method thread -k "chain or gibbs" > gpurun_out/${T}_pytest_chain.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_chain.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest_chain.txt
timeout -k 10 500 python -u profiles/bench_gibbs.py > gpurun_out/${T}_gibbs_4096.json 2>gpurun_out/${T}_gibbs.err || { tail -30 gpurun_out/${T}_gibbs.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096.json; echo
VBN_GIBBS_SPLIT=levels timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_levels.json 2>gpurun_out/${T}_gibbs_levels.err || { tail -30 gpurun_out/${T}_gibbs_levels.err; exit 1; }
cat gpurun_out/${T}_gibbs_levels.json; echo
timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_4096b.json 2>gpurun_out/${T}_gibbs_b.err || { tail -30 gpurun_out/${T}_gibbs_b.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096b.json
