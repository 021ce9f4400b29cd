#!/bin/bash
# round 4, first GPU pass (library with the MFMA-head hazard fix, per-query precompute off):
# MFMA-head bit identity (diag), then the whole GPU suite at the SURVEY §8(c) tolerances with
# the new cfg4 / cfg5 lean parity cases
set -o pipefail
mkdir -p gpurun_out
export VBN_PRECOMP_Q=0
timeout -k 10 300 python -u scripts/diag_headmfma.py > gpurun_out/r04a_headmfma_diag.txt 2>&1 || exit 1
cat gpurun_out/r04a_headmfma_diag.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04a_pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/r04a_pytest_gpu.txt
exit $rc
