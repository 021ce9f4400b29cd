#!/bin/bash
# round 5 ae: cfg4 with the per-sample pre-pass on a side stream beside the per-query one
# (VBN_PRE_STREAM=1) against the default, ABAB on one box
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ae}
for r in 1 2; do
  for s in 0 1; do
    VBN_PRE_STREAM=$s timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_cfg4_s${s}_$r.json 2>gpurun_out/${T}_cfg4_s${s}_$r.err || { tail -20 gpurun_out/${T}_cfg4_s${s}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${T}_cfg4_s${s}_$r.json'));print('stream $s rep $r', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
