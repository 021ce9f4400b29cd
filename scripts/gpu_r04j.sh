#!/bin/bash
# round 4 j: side-stream pre-pass A/B on one box (cfg2, anchor64), then rocprofv3 kernel stats +
# PMC passes of the current kernels (cfg4, cfg5, cfg2) -> gpurun_out/r04_<cfg>_*
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for ps in 1 0; do
    for c in cfg2 anchor64; do
      VBN_PRE_STREAM=$ps timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/r04j_ab_${c}_ps${ps}_$rep.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('gpurun_out/r04j_ab_${c}_ps${ps}_$rep.json'));print('$c ps=$ps rep $rep', d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
bash scripts/profile_configs.sh r04 cfg4 cfg5 || exit 1
