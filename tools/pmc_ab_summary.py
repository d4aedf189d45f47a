#!/usr/bin/env python3
"""Summarise tools/pmc_ab.sh output: per directory, each counter's per-dispatch
sum over XCDs / SEs for the k_wpool dispatches (first, cold dispatch dropped),
FETCH_SIZE x2 KB (gfx950 counts 128-B requests as 64 B) and WRITE_SIZE KB as bytes."""
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcab"
for d in sorted(glob.glob(os.path.join(root, "*"))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if "k_wpool" not in r["Kernel_Name"] and "k_wpair" not in r["Kernel_Name"]:
                continue
            k = (r["Counter_Name"], int(r["Dispatch_Id"]))
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    out = []
    for ctr in sorted({c for c, _ in vals}):
        ds = sorted(i for c, i in vals if c == ctr)
        ds = ds[1:] if len(ds) > 1 else ds
        v = sum(vals[(ctr, i)] for i in ds) / len(ds)
        if ctr == "FETCH_SIZE":
            v = v * 2 * 1024 / 1e9
            out.append(f"{ctr} {v:.3f} GB")
        elif ctr == "WRITE_SIZE":
            v = v * 1024 / 1e9
            out.append(f"{ctr} {v:.3f} GB")
        else:
            out.append(f"{ctr} {v:.4g}")
    vals2 = {c: sum(vals[(c, i)] for i in sorted(i for cc, i in vals if cc == c)[1:] or
                    sorted(i for cc, i in vals if cc == c)) for c in {c for c, _ in vals}}
    if "SQ_INSTS_VALU" in vals2 and "SQ_THREAD_CYCLES_VALU" in vals2:
        out.append(f"lanes/VALU {vals2['SQ_THREAD_CYCLES_VALU'] / vals2['SQ_INSTS_VALU']:.2f}")
    print(os.path.basename(d), " | ".join(out))
