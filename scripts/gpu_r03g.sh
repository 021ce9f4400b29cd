#!/bin/bash
# round 3: upper bound of dropping the per-node exact-path branch (measurement only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg2 exp/plan_cfg2_base.hsaco exp/plan_cfg2_noexact.hsaco exp/plan_cfg2_noexact_sgb4.hsaco exp/plan_cfg2_sgb4.hsaco > gpurun_out/r03g_ab_cfg2.txt 2>&1 || exit 1
cat gpurun_out/r03g_ab_cfg2.txt
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 exp/plan_cfg3_base.hsaco exp/plan_cfg3_noexact.hsaco > gpurun_out/r03g_ab_cfg3.txt 2>&1 || exit 1
cat gpurun_out/r03g_ab_cfg3.txt
