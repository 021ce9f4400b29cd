#!/bin/bash
# round 5 af: the side-stream per-sample pre-pass on by default for KDE pre-passes: precompute
# bit-identity tests, then cfg5 / cfg4 auto against VBN_PRE_STREAM=0, ABAB on one box
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05af}
timeout -k 10 600 python -u -m pytest tests/test_gpu_precompute.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_pre.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_pre.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_pre.txt
for c in cfg5 cfg4; do
  for r in 1 2; do
    for s in "" 0; do
      VBN_PRE_STREAM=$s timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_${c}_s${s}_$r.json 2>gpurun_out/${T}_${c}_s${s}_$r.err || { tail -20 gpurun_out/${T}_${c}_s${s}_$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/${T}_${c}_s${s}_$r.json'));print('$c stream[${s:-auto}] rep $r', d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
