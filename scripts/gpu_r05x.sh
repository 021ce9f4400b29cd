#!/bin/bash
# round 5 x: rocprofv3 kernel stats + PMC of the Gibbs sweep on the step-level schedule
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05x}
bash profiles/profile_gibbs.sh gpurun_out/prof_gibbs || exit 1
python3 profiles/summarize.py gpurun_out/prof_gibbs gpurun_out/${T}_gibbs_pmc.json vbn_walk_plan 1 > /dev/null || exit 1
cp gpurun_out/prof_gibbs/trace/run_kernel_stats.csv gpurun_out/${T}_gibbs_kernel_stats.csv
cat gpurun_out/${T}_gibbs_pmc.json
