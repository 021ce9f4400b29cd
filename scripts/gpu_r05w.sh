#!/bin/bash
# round 5 w: Gibbs step-level schedule variants: per-wave budget 1.2 and unbounded (all ready
# steps per phase) on 8 waves, and the default on 4-wave chain workgroups
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05w}
VBN_GIBBS_DAG_BUDGET=1.2 timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_b12.json 2>gpurun_out/${T}_b12.err || { tail -30 gpurun_out/${T}_b12.err; exit 1; }
cat gpurun_out/${T}_gibbs_b12.json; echo
VBN_GIBBS_DAG_BUDGET=inf timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_binf.json 2>gpurun_out/${T}_binf.err || { tail -30 gpurun_out/${T}_binf.err; exit 1; }
cat gpurun_out/${T}_gibbs_binf.json; echo
timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline --wave-particles 64 --chain-waves 4 > gpurun_out/${T}_gibbs_cw4.json 2>gpurun_out/${T}_cw4.err || { tail -30 gpurun_out/${T}_cw4.err; exit 1; }
cat gpurun_out/${T}_gibbs_cw4.json; echo
timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_def.json 2>gpurun_out/${T}_def.err || { tail -30 gpurun_out/${T}_def.err; exit 1; }
cat gpurun_out/${T}_gibbs_def.json
