#!/bin/bash
# cfg2 step time with / without the shared-sample precompute, driver-default steps and 100 steps
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for pc in pc nopc; do
    extra=""; [ $pc = nopc ] && extra="--no-precompute"
    timeout -k 10 300 python -u bench.py --config cfg2 --no-cpu-baseline $extra > gpurun_out/r03s_${pc}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python -u bench.py --config cfg2 --no-cpu-baseline --steps 100 $extra > gpurun_out/r03s_${pc}_${rep}_100.json 2>/dev/null || exit 1
  done
done
for f in gpurun_out/r03s_*.json; do python -c "
import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; done
