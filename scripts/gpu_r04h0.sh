#!/bin/bash
# round 4 h0: A/B of the bf16x3 KDE kernels (plan-specialised, no precompute) vs the interpreter
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/jit_ab.py --config cfg4 abx/plan_cfg4_kb.hsaco > gpurun_out/r04h0_ab_cfg4.txt 2>&1 || { tail -20 gpurun_out/r04h0_ab_cfg4.txt; exit 1; }
grep variant gpurun_out/r04h0_ab_cfg4.txt
timeout -k 10 400 python -u scripts/jit_ab.py --config cfg5 abx/plan_cfg5_kb.hsaco > gpurun_out/r04h0_ab_cfg5.txt 2>&1 || { tail -20 gpurun_out/r04h0_ab_cfg5.txt; exit 1; }
grep variant gpurun_out/r04h0_ab_cfg5.txt
