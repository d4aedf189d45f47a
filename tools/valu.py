#!/usr/bin/env python3
"""Per-launch VALU issue of the dominant kernel from one rocprofv3 --pmc pass
(SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE), stamped with the sha256
of the libcvr.so it ran (bench.py reports it as roofline.valu only for that
build, as it does profiles/traffic.json).  Writes profiles/valu.json.

  python tools/valu.py gpurun_out/pmcv_manix KEY [KERNEL_SUBSTR]

gfx950 (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs; a SIMD issues one wave64
VALU instruction per 2 cycles.  SQ_INSTS_VALU counts wave-level
instructions; SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU is the lanes active per
instruction; GRBM_GUI_ACTIVE is summed over the 8 XCDs (per-XCD busy cycles
of the dispatch = value / 8).
"""
import csv
import json
import os
import sys

N_SIMD = 1024
ISSUE_PER_CYCLE = 0.5


def per_dispatch(d, kname):
    vals = {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kname in r["Kernel_Name"]:
                k = (r["Counter_Name"], int(r["Dispatch_Id"]))
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    out = {}
    for (c, did), v in vals.items():
        out.setdefault(c, {})[did] = v
    return {c: [m[k] for k in sorted(m)] for c, m in out.items()}


def mean_warm(v):
    v = v[1:] if len(v) > 1 else v  # the first (cold) dispatch dropped when there are several
    return sum(v) / len(v)


def main():
    d, key = sys.argv[1:3]
    kname = sys.argv[3] if len(sys.argv) > 3 else "k_wpool"
    c = per_dispatch(d, kname)
    need = ("SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "GRBM_GUI_ACTIVE")
    miss = [n for n in need if n not in c]
    if miss:
        sys.exit(f"{d}: counters {miss} missing")
    insts = mean_warm(c["SQ_INSTS_VALU"])
    lanes = mean_warm(c["SQ_THREAD_CYCLES_VALU"]) / insts
    cycles = mean_warm(c["GRBM_GUI_ACTIVE"]) / 8.0
    issue = insts / N_SIMD / cycles / ISSUE_PER_CYCLE
    p = os.path.join(d, "libcvr.sha256")
    if not os.path.exists(p):
        sys.exit(f"{p} missing")
    sha = open(p).read().split()[0]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles", "valu.json")
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[key] = {"valu_insts_per_launch": insts, "lanes_per_inst": lanes, "busy_cycles_per_xcd": cycles,
                 "issue_frac": issue, "lane_frac": issue * lanes / 64.0,
                 "dispatches": len(c["SQ_INSTS_VALU"]), "kernel": kname, "libcvr_sha256": sha,
                 "method": "rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE, one pass; "
                           "summed over XCDs/SEs per dispatch, first dispatch dropped; issue_frac = "
                           "SQ_INSTS_VALU / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8) / 0.5; lane_frac = issue_frac x "
                           "lanes / 64"}
    json.dump(data, open(out, "w"), indent=1)
    print(key, json.dumps(data[key]))


if __name__ == "__main__":
    main()
