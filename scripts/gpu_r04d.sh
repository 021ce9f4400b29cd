#!/bin/bash
# round 4: rocprofv3 kernel stats + PMC per config (profiles/r04_<cfg>_*): usage gpu_r04d.sh cfg...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/profile_configs.sh r04 "$@" || exit 1
