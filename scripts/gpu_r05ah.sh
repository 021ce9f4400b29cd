#!/bin/bash
# round 5 ah: Gibbs chain-wave choice at 16384 / 32768 / 2048 chains (the auto rule's data)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ah}
for v in "16384 2" "32768 0" "32768 1" "32768 2" "32768 4" "2048 8" "2048 4"; do
  set -- $v
  timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline --steps 2 --chains $1 --wave-particles 64 --chain-waves $2 > gpurun_out/${T}_$1_$2.json 2>gpurun_out/${T}_$1_$2.err || { tail -20 gpurun_out/${T}_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_$1_$2.json'));r=d['roofline'];print('$1 chains cw $2:', d['value'], r['kernel_ms'], r['frac'], d['config']['chain_waves'])"
done
