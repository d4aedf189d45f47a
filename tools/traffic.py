#!/usr/bin/env python3
"""Per-launch HBM traffic of the dominant kernel from separate rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md §HBM says
(stamped with the sha256 of the libcvr.so the passes ran, which bench.py
checks before it reports the traffic):
FETCH_SIZE (KB) counts 128-B requests as 64 B on gfx950 -> x2; WRITE_SIZE (KB)
is exact for 16-B stores / f32 atomics.  Writes profiles/traffic.json.

  python tools/traffic.py gpurun_out/pmc_f gpurun_out/pmc_w KEY [KERNEL_SUBSTR]
"""
import csv
import json
import os
import sys


def per_dispatch(d, counter, kname):
    vals = {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals, key=int)]


def main():
    fdir, wdir, key = sys.argv[1:4]
    kname = sys.argv[4] if len(sys.argv) > 4 else "k_wpool"
    fetch = per_dispatch(fdir, "FETCH_SIZE", kname)
    write = per_dispatch(wdir, "WRITE_SIZE", kname)
    # drop the first (cold) dispatch when there are several
    f = fetch[1:] if len(fetch) > 1 else fetch
    w = write[1:] if len(write) > 1 else write
    fb = 2.0 * 1024.0 * sum(f) / len(f)
    wb = 1024.0 * sum(w) / len(w)
    shas = set()
    for d in (fdir, wdir):
        p = os.path.join(d, "libcvr.sha256")
        shas.add(open(p).read().split()[0] if os.path.exists(p) else None)
    if len(shas) != 1 or None in shas:
        sys.exit(f"libcvr.sha256 missing or different in {fdir} / {wdir}: {shas}")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles", "traffic.json")
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[key] = {"fetch_bytes": fb, "write_bytes": wb, "bytes_per_launch": fb + wb,
                 "dispatches": len(f), "kernel": kname, "libcvr_sha256": shas.pop(),
                 "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; "
                           "FETCH_SIZE x2 (gfx950 counts 128-B requests as 64 B), KB x1024; "
                           "includes Infinity-Cache hits (memory-side of L2)"}
    json.dump(data, open(out, "w"), indent=1)
    print(key, json.dumps(data[key]))


if __name__ == "__main__":
    main()
