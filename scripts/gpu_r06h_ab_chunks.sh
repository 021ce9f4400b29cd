set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python -u scripts/jit_ab.py --config cfg4 abx_r06/plan_cfg4_c16.hsaco > gpurun_out/r06h_ab_c16_$r.txt 2>&1 || exit 1
  VBN_KDE_CHUNKS=32 timeout -k 10 200 python -u scripts/jit_ab.py --config cfg4 abx_r06/plan_cfg4_c32.hsaco > gpurun_out/r06h_ab_c32_$r.txt 2>&1 || exit 1
done
grep -h variant gpurun_out/r06h_ab_*.txt
