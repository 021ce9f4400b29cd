#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/step_blocks.py cfg2 > gpurun_out/r03t_blocks.txt 2>&1 || { tail -5 gpurun_out/r03t_blocks.txt; exit 1; }
grep precompute gpurun_out/r03t_blocks.txt
