#!/bin/bash
# A/B of experiment libraries: bash scripts/gpu_ab.sh <config> <lib...>   (ABAB order recommended)
set -o pipefail
mkdir -p gpurun_out
cfg=$1; shift
timeout -k 10 600 python -u scripts/exp_compare.py --config $cfg "$@"
