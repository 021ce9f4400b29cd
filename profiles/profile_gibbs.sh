#!/bin/bash
# rocprofv3 kernel trace + stats and separate PMC passes of the Gibbs sweep bench
# (profiles/bench_gibbs.py, 4096 chains, YAML defaults); summarised like profile_round.sh.
#   bash profiles/profile_gibbs.sh gpurun_out/prof_gibbs
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_gibbs}
mkdir -p $OUT
B="profiles/bench_gibbs.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $B > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $B > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 $B > $OUT/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY --output-format csv -d $OUT/pmc_sq2 -o run -- python3 $B > $OUT/pmc_sq2.log 2>&1
echo done
