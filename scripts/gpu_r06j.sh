#!/bin/bash
# round 6 j: the half-chunk KDE scan on the final tree: smoke, the whole GPU suite, the default
# (cfg4) bench with its CPU baseline, the other configs' bench lines, the Gibbs bench, then the
# cfg4 and cfg5 profiles (kernel trace + PMC passes: the roofline's traffic figures)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r06j}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -30 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --maxfail=40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
tail -8 gpurun_out/${T}_pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench_cfg4.json 2>gpurun_out/${T}_bench_cfg4.err || { tail -30 gpurun_out/${T}_bench_cfg4.err; exit 1; }
cat gpurun_out/${T}_bench_cfg4.json; echo
for c in cfg5 cfg3 cfg2 anchor64; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/${T}_bench_$c.json 2>gpurun_out/${T}_bench_$c.err || { tail -30 gpurun_out/${T}_bench_$c.err; exit 1; }
  head -c 600 gpurun_out/${T}_bench_$c.json; echo
done
timeout -k 10 400 python -u profiles/bench_gibbs.py > gpurun_out/${T}_bench_gibbs.json 2>gpurun_out/${T}_bench_gibbs.err || { tail -30 gpurun_out/${T}_bench_gibbs.err; exit 1; }
head -c 600 gpurun_out/${T}_bench_gibbs.json; echo
timeout -k 10 900 bash scripts/profile_configs.sh ${T} cfg4 cfg5 > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
tail -3 gpurun_out/${T}_prof.log
exit $rc
