#!/bin/bash
# VALU instruction mix + per-unit issue cycles of the walk (two PMC passes per config).
#   bash scripts/pmc_valu_mix.sh cfg2 [cfg3 ...]
set -o pipefail
export TMPDIR=/tmp
for c in "$@"; do
  B="bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d gpurun_out/mix_$c/p1 -o run -- python3 $B > gpurun_out/mix_$c.p1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/mix_$c/p2 -o run -- python3 $B > gpurun_out/mix_$c.p2.log 2>&1 || exit $?
  python3 - "$c" <<'PY'
import csv, glob, sys, collections
c = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"gpurun_out/mix_{c}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "vbn_walk" not in r["Kernel_Name"] or int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) < 4096 * 64:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
w = tot["SQ_WAVES"] / max(n["SQ_WAVES"], 1)
print(c, {k: round(v / max(n[k], 1) / w, 1) for k, v in sorted(tot.items())})
PY
done
