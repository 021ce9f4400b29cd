#!/bin/bash
# round 5 aa: kernel traces of the cfg2 / cfg3 benches (timed steps), for the host-side gaps
# between ms_per_step and the kernel time
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in cfg2 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05aa_$c.json 2>gpurun_out/r05aa_$c.err || { tail -20 gpurun_out/r05aa_$c.err; exit 1; }
  cat gpurun_out/r05aa_$c.json; echo
done
