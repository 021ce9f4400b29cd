#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/host_profile.py cfg2 200 > gpurun_out/r03r_host_cfg2.txt 2>&1 || { tail -20 gpurun_out/r03r_host_cfg2.txt; exit 1; }
head -3 gpurun_out/r03r_host_cfg2.txt
