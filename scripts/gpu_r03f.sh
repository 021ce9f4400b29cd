#!/bin/bash
# round 3: plan-kernel variants A/B (waves per SIMD, step-boundary scheduling barrier)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg2 exp/plan_cfg2_base.hsaco exp/plan_cfg2_sb.hsaco exp/plan_cfg2_wpe3.hsaco exp/plan_cfg2_wpe5.hsaco > gpurun_out/r03f_ab_cfg2.txt 2>&1 || exit 1
cat gpurun_out/r03f_ab_cfg2.txt
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 exp/plan_cfg3_base.hsaco exp/plan_cfg3_sb.hsaco exp/plan_cfg3_wpe3.hsaco > gpurun_out/r03f_ab_cfg3.txt 2>&1 || exit 1
cat gpurun_out/r03f_ab_cfg3.txt
