#!/bin/bash
# rocprofv3 kernel-trace/stats + separate PMC passes per config, summarised to JSON.
#   bash scripts/profile_configs.sh <round-tag> cfg2 [cfg3 ...]
set -o pipefail
tag=$1; shift
for c in "$@"; do
  bash profiles/profile_round.sh gpurun_out/prof_$c $c || exit $?
  python3 profiles/summarize.py gpurun_out/prof_$c gpurun_out/${tag}_${c}_pmc.json > /dev/null || exit $?
  cp gpurun_out/prof_$c/trace/run_kernel_stats.csv gpurun_out/${tag}_${c}_kernel_stats.csv
  echo "$c: $(python3 -c "import json;d=json.load(open('gpurun_out/${tag}_${c}_pmc.json'));print(d.get('avg_ns_full_size'), d.get('hbm_bytes_per_launch'), d.get('mfma_busy_frac'))")"
done
