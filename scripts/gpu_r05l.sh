#!/bin/bash
# round 5 l: Gibbs on auto (full waves, 8-wave chain workgroups): GPU Gibbs tests, the bench with
# its CPU baseline, the split-level ablation at 64 x 8, then rocprofv3 stats + PMC
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "gibbs or Gibbs" > gpurun_out/${T}_pytest_gibbs.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gibbs.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest_gibbs.txt
timeout -k 10 500 python -u profiles/bench_gibbs.py > gpurun_out/${T}_gibbs_4096.json 2>gpurun_out/${T}_gibbs.err || { tail -30 gpurun_out/${T}_gibbs.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096.json; echo
for sp in 0 1; do
  VBN_GIBBS_SPLIT=$sp timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_split$sp.json 2>gpurun_out/${T}_gibbs_split$sp.err || { tail -30 gpurun_out/${T}_gibbs_split$sp.err; exit 1; }
  cat gpurun_out/${T}_gibbs_split$sp.json; echo
done
bash profiles/profile_gibbs.sh gpurun_out/prof_gibbs || exit 1
python3 profiles/summarize.py gpurun_out/prof_gibbs gpurun_out/${T}_gibbs_pmc.json vbn_walk_plan 1 > /dev/null || exit 1
cp gpurun_out/prof_gibbs/trace/run_kernel_stats.csv gpurun_out/${T}_gibbs_kernel_stats.csv
cat gpurun_out/${T}_gibbs_pmc.json
