#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes (one directory per pass, tools/gpu_job.sh
pmc_a/pmc_b/pmc_c/...) into one per-launch summary of the dominant kernel:
each counter summed over XCDs/SEs per dispatch, averaged over dispatches
(the first, cold dispatch dropped when there are several).

  python tools/pmc_summary.py OUT.json KERNEL_SUBSTR DIR [DIR ...]
"""
import csv
import json
import os
import sys


def main():
    out, kname, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    counters = {}
    for d in dirs:
        per = {}
        with open(os.path.join(d, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if kname not in r["Kernel_Name"]:
                    continue
                key = (r["Counter_Name"], int(r["Dispatch_Id"]))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        names = sorted({k[0] for k in per})
        for n in names:
            vals = [v for (c, _), v in sorted(per.items(), key=lambda kv: kv[0][1]) if c == n]
            vals = vals[1:] if len(vals) > 1 else vals
            counters[n] = {"per_launch_mean": sum(vals) / len(vals), "launches": len(vals), "pass": os.path.basename(d)}
    c = {k: v["per_launch_mean"] for k, v in counters.items()}
    derived = {}
    if "SQ_INSTS_VALU" in c and "SQ_THREAD_CYCLES_VALU" in c:
        derived["lanes_active_per_valu"] = c["SQ_THREAD_CYCLES_VALU"] / c["SQ_INSTS_VALU"]
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        derived["wait_any_frac_of_wave_cycles"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
        derived["wait_inst_any_frac_of_wave_cycles"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        derived["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCP_TCC_READ_REQ_sum" in c and "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        derived["l1_hit_rate"] = 1.0 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_VALU" in c:
        # per SIMD (1024 of them) over the per-XCD active cycles (GRBM sums the 8 XCDs)
        derived["valu_per_simd_cycle"] = (c["SQ_INSTS_VALU"] / 1024.0) / (c["GRBM_GUI_ACTIVE"] / 8.0)
        derived["valu_issue_frac_of_peak_0.5_per_cycle"] = derived["valu_per_simd_cycle"] / 0.5
    json.dump({"kernel": kname, "method": "rocprofv3 --pmc <group> --kernel-trace, one pass per group; summed over "
               "XCDs/SEs per dispatch; SQ_* cycle counters in quad-cycles", "counters": counters,
               "derived": derived}, open(out, "w"), indent=1)
    print(json.dumps(derived, indent=1))


if __name__ == "__main__":
    main()
