#!/bin/bash
# round 5 z: Gibbs sweep ablations on the production chain form (scripts/jit_variants.py --gibbs,
# abx7/): no Philox, no softplus, no exact-path branch, no head
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05z}
timeout -k 10 900 python -u scripts/jit_ab_gibbs.py abx7/gibbs_base.hsaco abx7/gibbs_norng.hsaco abx7/gibbs_nosp.hsaco abx7/gibbs_noexact.hsaco abx7/gibbs_nohead.hsaco > gpurun_out/${T}_ab_gibbs.txt 2>&1 || { tail -20 gpurun_out/${T}_ab_gibbs.txt; exit 1; }
cat gpurun_out/${T}_ab_gibbs.txt
