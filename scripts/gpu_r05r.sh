#!/bin/bash
# round 5 r: same-box A/B of the tile-pipelined KDE pass 1 (abx6/plan_<cfg>_pipe) against the
# previous loop (abx6/plan_<cfg>_nopipe: the header of commit 0b35465), plain plans
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05r}
for c in ${CFGS:-cfg4}; do
  timeout -k 10 500 python -u scripts/jit_ab.py --config $c abx6/plan_${c}_pipe.hsaco abx6/plan_${c}_nopipe.hsaco abx6/plan_${c}_pipe.hsaco > gpurun_out/${T}_ab_$c.txt 2>&1 || { tail -20 gpurun_out/${T}_ab_$c.txt; exit 1; }
  cat gpurun_out/${T}_ab_$c.txt
done
