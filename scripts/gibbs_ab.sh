set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for wp in 32 64; do for B in 4096 8192; do
  timeout -k 10 200 python profiles/bench_gibbs.py --chains $B --wave-particles $wp --no-cpu-baseline > gpurun_out/gibbs_${B}_${wp}.json || exit $?
  python -c "import json;d=json.load(open('gpurun_out/gibbs_${B}_${wp}.json'));print($B,$wp,d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done; done
