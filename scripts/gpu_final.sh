#!/bin/bash
# Round-end evidence on one GPU: parity tests, smoke, the default bench (CPU baseline included),
# the driver's 20/5 bench, then rocprofv3 kernel stats + PMC passes per config.
#   bash scripts/gpu_final.sh <round-tag> [config ...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1
rc=$?; tail -1 gpurun_out/${tag}_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || exit $?
tail -2 gpurun_out/${tag}_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench_default.log > gpurun_out/${tag}_bench_default.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_steps20.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench_steps20.log > gpurun_out/${tag}_bench_default_steps20_warmup5.json
python3 -c "import json;d=json.load(open('gpurun_out/${tag}_bench_default.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['cpu_baseline']['value'])"
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_bench_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/${tag}_bench_$c.log > gpurun_out/${tag}_bench_$c.json
done
STEPS=20 WARMUP=5 bash scripts/profile_configs.sh $tag "$@" || exit $?
exit 0
