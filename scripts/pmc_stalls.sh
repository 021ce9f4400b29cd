#!/bin/bash
# Stall-breakdown PMC passes of vbn_walk_kernel for one library (run on the GPU box):
#   bash scripts/pmc_stalls.sh <tag> [lib.so] [config]
# Writes gpurun_out/stalls_<tag>/pass*/ and gpurun_out/stalls_<tag>.json (per-wave averages,
# average in-flight latency of VMEM / SMEM / LDS instructions from SQ_INST_LEVEL_* / SQ_INSTS_*).
set -o pipefail
export TMPDIR=/tmp
tag=$1; lib=${2:-}; cfg=${3:-cfg2}
out=gpurun_out/stalls_$tag
mkdir -p $out
[ -n "$lib" ] && export VBN_HIP_LIB=$(readlink -f $lib)
B="bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
  "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_SMEM SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $out/pass$i -o run -- python3 $B > $out/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/pass$i.log; exit 1; }
  i=$((i+1))
done
python3 - "$out" "$tag" <<'EOF'
import collections, csv, glob, json, sys
d, tag = sys.argv[1], sys.argv[2]
pmc = collections.defaultdict(list)
for f in glob.glob(f"{d}/pass*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "vbn_walk_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) >= 4096 * 64:
            pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(v) / len(v) for k, v in pmc.items()}
w = a.get("SQ_WAVES", 1.0)
res = {"tag": tag, "per_wave": {k: round(v / w, 1) for k, v in a.items() if k != "SQ_WAVES"}, "waves": w}
for lvl, n in (("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD"), ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM"),
               ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS")):
    if lvl in a and a.get(n):
        res[f"avg_latency_{n[9:].lower()}_cycles"] = round(a[lvl] / a[n], 1)
wc = a.get("SQ_WAVE_CYCLES")
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS"):
        if k in a:
            res[f"frac_{k[3:].lower()}"] = round(a[k] / wc, 4)
if "GRBM_GUI_ACTIVE" in a:
    res["gui_active_cycles_per_xcd"] = a["GRBM_GUI_ACTIVE"] / 8
json.dump(res, open(f"gpurun_out/stalls_{tag}.json", "w"), indent=1)
print(json.dumps(res))
EOF
