#!/bin/bash
# round 4, build 5 (KDE operand prefetch across chunks, branch-free categorical inverse CDF,
# three-input XOR Philox): smoke, GPU suite, benches, 2-rank gather rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.txt 2>&1 || { cat gpurun_out/r04f_smoke.txt; exit 1; }
tail -1 gpurun_out/r04f_smoke.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04f_pytest_gpu.txt 2>&1
rc=$?
tail -3 gpurun_out/r04f_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04f_bench_$i.json 2>gpurun_out/r04f_bench_$i.err || exit 1
  cat gpurun_out/r04f_bench_$i.json
done
for c in cfg3 anchor64 cfg4 cfg5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r04f_bench_$c.json 2>gpurun_out/r04f_bench_$c.err || exit 1
  cat gpurun_out/r04f_bench_$c.json
done
bash scripts/gpu_r04e.sh
timeout -k 10 300 python -u scripts/jit_ab.py --config cfg5 abx/plan_cfg5_base.hsaco abx/plan_cfg5_nop1.hsaco \
  abx/plan_cfg5_noscan.hsaco abx/plan_cfg5_norng.hsaco > gpurun_out/r04f_ab_cfg5.txt 2>&1 || exit 1
cat gpurun_out/r04f_ab_cfg5.txt | grep variant
