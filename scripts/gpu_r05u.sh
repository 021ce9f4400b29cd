#!/bin/bash
# round 5 u: the specialised one-wave Gibbs sweep (chain_waves 0) at full and half wave, bitwise
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05u}
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 400 --timeout-method thread -k "chain_workgroup_gibbs_bit_identical and (64-0 or 32-0)" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -4 gpurun_out/${T}_pytest.txt
