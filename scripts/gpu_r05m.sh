#!/bin/bash
# round 5 m: full-wave Gibbs sweeps on the draw-free (| 256) plan unit (no VGPR spills): bitwise
# chain tests, the bench (auto = 64 x 8, with its CPU baseline), 64 x 4, whole levels at 64 x 8,
# then rocprofv3 stats + PMC of the auto form
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r05m}
timeout -k 10 900 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 400 --timeout-method thread -k "chain or gibbs" > gpurun_out/${T}_pytest_chain.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_chain.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest_chain.txt
timeout -k 10 500 python -u profiles/bench_gibbs.py > gpurun_out/${T}_gibbs_4096.json 2>gpurun_out/${T}_gibbs.err || { tail -30 gpurun_out/${T}_gibbs.err; exit 1; }
cat gpurun_out/${T}_gibbs_4096.json; echo
timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline --wave-particles 64 --chain-waves 4 > gpurun_out/${T}_gibbs_64_4.json 2>gpurun_out/${T}_gibbs_64_4.err || { tail -30 gpurun_out/${T}_gibbs_64_4.err; exit 1; }
cat gpurun_out/${T}_gibbs_64_4.json; echo
VBN_GIBBS_SPLIT=0 timeout -k 10 400 python -u profiles/bench_gibbs.py --no-cpu-baseline > gpurun_out/${T}_gibbs_split0.json 2>gpurun_out/${T}_gibbs_split0.err || { tail -30 gpurun_out/${T}_gibbs_split0.err; exit 1; }
cat gpurun_out/${T}_gibbs_split0.json; echo
bash profiles/profile_gibbs.sh gpurun_out/prof_gibbs || exit 1
python3 profiles/summarize.py gpurun_out/prof_gibbs gpurun_out/${T}_gibbs_pmc.json vbn_walk_plan 1 > /dev/null || exit 1
cp gpurun_out/prof_gibbs/trace/run_kernel_stats.csv gpurun_out/${T}_gibbs_kernel_stats.csv
cat gpurun_out/${T}_gibbs_pmc.json
