#!/bin/bash
# round 5 ac: the Gibbs GPU tests on the precompiled sweep units (scripts/precompile_gibbs_tests.py)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ac}
timeout -k 10 900 python -u -m pytest tests/test_gpu_jit.py -x -v --durations=8 --timeout 400 --timeout-method thread -k "chain or gibbs" > gpurun_out/${T}_pytest_chain.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_chain.txt; exit 1; }
tail -14 gpurun_out/${T}_pytest_chain.txt
