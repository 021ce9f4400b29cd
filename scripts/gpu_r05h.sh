#!/bin/bash
# round 5 g: the Gibbs sampler bench (4096 chains, YAML defaults) and its rocprofv3 stats + PMC
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05h}
timeout -k 10 400 python -u profiles/bench_gibbs.py > gpurun_out/${T}_gibbs_4096.json 2>gpurun_out/${T}_gibbs.err || { tail -30 gpurun_out/${T}_gibbs.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096.json
# Gibbs sweep kernel: rocprofv3 stats + PMC
bash profiles/profile_gibbs.sh gpurun_out/prof_gibbs || exit 1
python3 profiles/summarize.py gpurun_out/prof_gibbs gpurun_out/${T}_gibbs_pmc.json vbn_walk_plan 1 > /dev/null || exit 1
cp gpurun_out/prof_gibbs/trace/run_kernel_stats.csv gpurun_out/${T}_gibbs_kernel_stats.csv
cat gpurun_out/${T}_gibbs_pmc.json
