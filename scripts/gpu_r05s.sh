#!/bin/bash
# round 5 s: cfg3 per-stage ablations of the current lean plan kernel (scripts/jit_variants.py
# -DVBN_ABL_*: no Philox, no head, no softplus, no layer 2, no exact-path branch)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05s}
timeout -k 10 600 python -u scripts/jit_ab.py --config cfg3 abx6/plan_cfg3_base.hsaco abx6/plan_cfg3_norng.hsaco abx6/plan_cfg3_nohead.hsaco abx6/plan_cfg3_nosp.hsaco abx6/plan_cfg3_nol2.hsaco abx6/plan_cfg3_noexact.hsaco > gpurun_out/${T}_ab_cfg3.txt 2>&1 || { tail -20 gpurun_out/${T}_ab_cfg3.txt; exit 1; }
cat gpurun_out/${T}_ab_cfg3.txt
