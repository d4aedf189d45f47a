#!/bin/bash
# In-launch output, attribution: frame probe (flush vs copy) per experiment build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/flush4
mkdir -p "$OUT"
for L in "$@"; do
  if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
  timeout -k 10 200 python3 tools/frame_probe.py $LA --variants flush,copy --rounds 2 --reps 10 > "$OUT/probe_$L.log" 2>&1 || { tail -20 "$OUT/probe_$L.log"; exit 1; }
  grep round "$OUT/probe_$L.log" | sed "s/^/$L /" | cut -c1-120
done
