#!/bin/bash
# round 5 ag: Gibbs at 16384 and 8192 chains: the auto form against chain workgroups of 8 / 4
# waves and the one-wave form (where the auto threshold ops.CHAIN_WAVES_BELOW should sit)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05ag}
for ch in 16384 8192; do
  for cw in auto 8 4 0; do
    a=""; [ "$cw" != auto ] && a="--wave-particles 64 --chain-waves $cw"
    timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline --steps 2 --chains $ch $a > gpurun_out/${T}_${ch}_$cw.json 2>gpurun_out/${T}_${ch}_$cw.err || { tail -20 gpurun_out/${T}_${ch}_$cw.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${T}_${ch}_$cw.json'));r=d['roofline'];print('$ch chains cw $cw:', d['value'], r['kernel_ms'], r['frac'], d['config']['wave_particles'], d['config']['chain_waves'])"
  done
done
