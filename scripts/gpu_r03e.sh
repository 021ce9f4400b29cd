#!/bin/bash
# round 3: plan-specialised Gibbs sweeps (bit identity + A/B), co-issue microbenchmark with
# hand-placed fillers, cfg2/cfg4/cfg5 benches with the specialised walk
set -o pipefail
mkdir -p gpurun_out
export VBN_HIP_CACHE=/tmp/vbn_hip_cache
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -m gpu -v -rs --timeout 300 --timeout-method thread > gpurun_out/r03e_pytest_jit.txt 2>&1; rc=$?
tail -15 gpurun_out/r03e_pytest_jit.txt
[ $rc -eq 0 ] || exit $rc
hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize profiles/microbench/coissue_sgb.hip -o /tmp/coissue_sgb || exit 1
timeout -k 10 120 /tmp/coissue_sgb > gpurun_out/r03e_coissue_sgb.json || exit 1
timeout -k 10 400 python -u profiles/bench_gibbs.py --plan-jit off --no-cpu-baseline > gpurun_out/r03e_gibbs_interp.json 2>gpurun_out/r03e_gibbs_interp.err || exit 1
cat gpurun_out/r03e_gibbs_interp.json
timeout -k 10 400 python -u profiles/bench_gibbs.py --plan-jit on --no-cpu-baseline > gpurun_out/r03e_gibbs_plan.json 2>gpurun_out/r03e_gibbs_plan.err || exit 1
cat gpurun_out/r03e_gibbs_plan.json
for c in cfg2 cfg4 cfg5 anchor64; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r03e_bench_$c.json 2>gpurun_out/r03e_bench_$c.err || exit 1
  cat gpurun_out/r03e_bench_$c.json
done
