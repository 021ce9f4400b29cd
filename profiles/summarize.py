#!/usr/bin/env python3
"""Summarise a profiles/profile_round.sh output dir into a JSON (kernel time + PMC per launch).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reads half the bytes of wide coalesced streaming reads (doubled here,
flagged as an upper estimate for other access widths); WRITE_SIZE is exact for 16-B
streaming stores and uncalibrated for the walk's 4-B-per-lane stores (reported as is).
Usage: summarize.py <prof_dir> <out.json> [kernel_substring] [min_grid]
(min_grid: launches with fewer threads are ignored, default 4096 * 64: the full-size walks;
the Gibbs sweep passes 1)
(default: the plan-specialised walk vbn_walk_plan when the trace has it, else vbn_walk_kernel)
"""
import collections
import csv
import json
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_stats.csv")))
    min_grid = int(sys.argv[4]) if len(sys.argv) > 4 else 4096 * 64
    if len(sys.argv) > 3 and sys.argv[3] != "-":
        kname = sys.argv[3]
    else:
        kname = "vbn_walk_plan" if any("vbn_walk_plan" in r["Name"] for r in rows) else "vbn_walk_kernel"
    res = {"kernel": kname}
    for r in rows:
        if kname in r["Name"]:
            res.update(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), min_ns=float(r["MinNs"]),
                       max_ns=float(r["MaxNs"]), pct=float(r["Percentage"]))
    trace = list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")))
    big = [int(t["End_Timestamp"]) - int(t["Start_Timestamp"]) for t in trace
           if kname in t["Kernel_Name"] and int(t.get("Grid_Size_X", 0) or 0) >= min_grid]
    # launches that did no work: importance sampling's likelihood-weighting fallback walk is
    # enqueued predicated on the device flag every call (engines.ImportanceSampling) and exits at
    # once when the flag is 0 -- same kernel name and grid, ~15 us; left out of the averages
    if big:
        keep = [t for t in big if t >= 0.1 * max(big)]
        res["avg_ns_full_size"] = sum(keep) / len(keep)
        res["noop_launches_dropped"] = len(big) - len(keep)
    pmc = collections.defaultdict(list)
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
        try:
            for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
                if kname in r["Kernel_Name"] and int(r["Grid_Size"]) >= min_grid:
                    pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        except FileNotFoundError:
            pass
    avg = {}
    for k, v in pmc.items():                  # the same no-op launches, by a vanishing count
        keep = [x for x in v if x >= 0.02 * max(v)] if max(v) > 0 else v
        avg[k] = sum(keep) / len(keep)
    res["pmc_per_launch"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        res["hbm_bytes_per_launch"] = int((2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024)
        res["hbm_read_bytes_per_launch"] = int(2 * avg["FETCH_SIZE"] * 1024)
        res["hbm_write_bytes_per_launch"] = int(avg["WRITE_SIZE"] * 1024)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        cycles = avg["GRBM_GUI_ACTIVE"] / 8
        res["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cycles)
        res["clock_ghz"] = cycles / (res.get("avg_ns_full_size", res.get("avg_ns", 1)) )
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        res["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
        res["mfma_insts_per_wave"] = avg.get("SQ_INSTS_MFMA", 0) / avg["SQ_WAVES"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
