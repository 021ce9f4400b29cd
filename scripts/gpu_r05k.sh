#!/bin/bash
# round 5 k: chain workgroups of 8 waves (full-wave chains, no mirrored half-wave lanes):
# bitwise chain tests for 8 waves, then the Gibbs bench over (wave_particles, chain_waves)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 400 --timeout-method thread -k "chain_workgroup_gibbs_bit_identical and (64-8 or 32-8)" > gpurun_out/${T}_pytest_chain8.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_chain8.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest_chain8.txt
for v in "64 8" "64 4" "32 8"; do
  set -- $v
  timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline --wave-particles $1 --chain-waves $2 > gpurun_out/${T}_gibbs_$1_$2.json 2>gpurun_out/${T}_gibbs_$1_$2.err || { tail -30 gpurun_out/${T}_gibbs_$1_$2.err; exit 1; }
  cat gpurun_out/${T}_gibbs_$1_$2.json; echo
done
