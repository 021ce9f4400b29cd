#!/bin/bash
# round 5 ai: the auto chain-wave rule: Gibbs GPU tests, then the bench at 4096 (auto: 8 waves)
# and 8192 / 16384 chains (auto: 4 / 2 waves)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ai}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gibbs or Gibbs or chain" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for ch in 4096 8192 16384; do
  timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline --chains $ch > gpurun_out/${T}_$ch.json 2>gpurun_out/${T}_$ch.err || { tail -20 gpurun_out/${T}_$ch.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_$ch.json'));r=d['roofline'];print('$ch chains auto:', d['value'], r['kernel_ms'], r['frac'], d['config']['wave_particles'], d['config']['chain_waves'])"
done
