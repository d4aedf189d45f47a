#!/bin/bash
# In-launch output diagnostics: per library (default, experiment builds), one synchronous
# C2 render per call with and without it.  gpurun_out/flush2/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/flush2
mkdir -p "$OUT"
for L in default "$@"; do
  if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
  timeout -k 10 200 python3 tools/frame_probe.py $LA --variants flush,copy --rounds 2 --reps 10 > "$OUT/probe_$L.log" 2>&1 || { tail -20 "$OUT/probe_$L.log"; exit 1; }
  grep round "$OUT/probe_$L.log" | sed "s/^/$L /" | cut -c1-150
done
