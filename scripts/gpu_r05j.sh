#!/bin/bash
# round 5 j: Gibbs split levels (plan.gibbs_schedule): bitwise chain tests, then the Gibbs bench
# with the cost-model schedule and with whole levels only (VBN_GIBBS_SPLIT=0, the r05h form)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05j}
timeout -k 10 900 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 400 --timeout-method thread -k "chain or gibbs" > gpurun_out/${T}_pytest_chain.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_chain.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest_chain.txt
timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_split.json 2>gpurun_out/${T}_gibbs_split.err || { tail -30 gpurun_out/${T}_gibbs_split.err; exit 1; }
cat gpurun_out/${T}_gibbs_split.json
VBN_GIBBS_SPLIT=0 timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_whole.json 2>gpurun_out/${T}_gibbs_whole.err || { tail -30 gpurun_out/${T}_gibbs_whole.err; exit 1; }
cat gpurun_out/${T}_gibbs_whole.json
