#!/bin/bash
# round 4 g: the discrete-histogram kernel's GPU tests, the 2-rank gather rehearsal (settling
# calls agreed across ranks), cfg5 with and without the liveness walk order, and the KDE
# ablations of cfg5 and cfg4 (A/B code objects compiled from the default-order plans)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_histogram.py tests/test_abi.py tests/test_gpu_generations.py -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04g_hist.txt 2>&1 || { tail -30 gpurun_out/r04g_hist.txt; exit 1; }
tail -2 gpurun_out/r04g_hist.txt
bash scripts/gpu_r04e.sh || exit 1
for lo in 1 0; do
  VBN_LIVENESS_ORDER=$lo timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline \
    > gpurun_out/r04g_bench_cfg5_lo$lo.json 2> gpurun_out/r04g_bench_cfg5_lo$lo.err || exit 1
  cat gpurun_out/r04g_bench_cfg5_lo$lo.json
done
VBN_LIVENESS_ORDER=0 timeout -k 10 300 python -u scripts/jit_ab.py --config cfg5 abx/plan_cfg5_base.hsaco abx/plan_cfg5_nop1.hsaco \
  abx/plan_cfg5_noscan.hsaco abx/plan_cfg5_norng.hsaco > gpurun_out/r04g_ab_cfg5.txt 2>&1 || exit 1
grep variant gpurun_out/r04g_ab_cfg5.txt
VBN_LIVENESS_ORDER=0 timeout -k 10 400 python -u scripts/jit_ab.py --config cfg4 abx/plan_cfg4_base.hsaco abx/plan_cfg4_l2fit.hsaco \
  abx/plan_cfg4_noscan.hsaco abx/plan_cfg4_nop1.hsaco > gpurun_out/r04g_ab_cfg4.txt 2>&1 || exit 1
grep variant gpurun_out/r04g_ab_cfg4.txt
VBN_LIVENESS_ORDER=0 timeout -k 10 300 python -u scripts/jit_ab.py --config cfg3 abx/plan_cfg3_base.hsaco abx/plan_cfg3_wpe3.hsaco \
  > gpurun_out/r04g_ab_cfg3.txt 2>&1 || exit 1
grep variant gpurun_out/r04g_ab_cfg3.txt
timeout -k 10 300 python -u scripts/gen_ab.py --config cfg4 --gens 1 4 8 16 32 > gpurun_out/r04g_gen_cfg4.txt 2>&1 || exit 1
cat gpurun_out/r04g_gen_cfg4.txt
timeout -k 10 300 python -u scripts/gen_ab.py --config cfg5 --gens 1 4 8 16 32 > gpurun_out/r04g_gen_cfg5.txt 2>&1 || exit 1
cat gpurun_out/r04g_gen_cfg5.txt
