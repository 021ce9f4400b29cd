#!/bin/bash
# round 4 m: rocprofv3 kernel stats + PMC passes of the final kernels -> gpurun_out/r04_<cfg>_*
set -o pipefail
mkdir -p gpurun_out
bash scripts/profile_configs.sh r04 cfg2 cfg5 cfg3 || exit 1
