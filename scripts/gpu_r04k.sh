#!/bin/bash
# round 4 k: A/Bs on one box -- cfg2 plan kernels: before / relu folded into the f16 split /
# not folded (same source); cfg4 bf16x3 KDE kernel vs its L2-resident-pack ablation
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg2 abx/plan_cfg2_prev.hsaco abx/plan_cfg2_nofuse.hsaco \
  abx/plan_cfg2_fz.hsaco > gpurun_out/r04k_ab_cfg2.txt 2>&1 || { tail -20 gpurun_out/r04k_ab_cfg2.txt; exit 1; }
grep variant gpurun_out/r04k_ab_cfg2.txt
timeout -k 10 400 python -u scripts/jit_ab.py --config cfg4 abx/plan_cfg4_kb.hsaco abx/plan_cfg4_kbl2.hsaco \
  > gpurun_out/r04k_ab_cfg4.txt 2>&1 || { tail -20 gpurun_out/r04k_ab_cfg4.txt; exit 1; }
grep variant gpurun_out/r04k_ab_cfg4.txt
