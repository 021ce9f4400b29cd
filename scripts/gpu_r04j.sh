#!/bin/bash
# round 4 j: rocprofv3 kernel stats + PMC passes of the current kernels (cfg4, cfg5 bf16x3 KDE;
# cfg2 with the side-stream pre-pass), summaries -> gpurun_out/r04_<cfg>_*
set -o pipefail
mkdir -p gpurun_out
bash scripts/profile_configs.sh r04 cfg4 cfg5 cfg2 || exit 1
