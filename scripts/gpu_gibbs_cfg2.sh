set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for B in 4096 8192; do
  timeout -k 10 200 python profiles/bench_gibbs.py --chains $B --wave-particles 32 --no-cpu-baseline > gpurun_out/gibbs_${B}_32.json || exit $?
  python -c "import json;d=json.load(open('gpurun_out/gibbs_${B}_32.json'));print($B,d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --config cfg2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cfg2.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("cfg2", d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])'
