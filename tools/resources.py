#!/usr/bin/env python3
"""Register / spill / occupancy table of every kernel in a HIP source, compiled with the
Makefile's flags:  python3 tools/resources.py cudavolumerenderer_amd/csrc/cvr_wpool.hip [hipcc flags]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-Iinclude", "-Icudavolumerenderer_amd/csrc",
       "-Wno-unused-function", *sys.argv[2:], "-Rpass-analysis=kernel-resource-usage", "-c", sys.argv[1],
       "-o", "/dev/null"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for ln in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|TotalSGPRs|VGPRs|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]):\s*(\S+)",
                  ln)
    if not m:
        if "error" in ln:
            print(ln)
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    g = r.get
    print(f"{g('VGPRs', '?'):>4} v {g('VGPRs Spill', '?'):>3} vsp {g('TotalSGPRs', '?'):>4} s "
          f"{g('SGPRs Spill', '?'):>3} ssp occ {g('Occupancy [waves/SIMD]', '?')}  {r['name']}")
