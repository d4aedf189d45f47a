#!/bin/bash
# Re-tune the wave-pool knobs at the current build (one-launch kernel, variants interleaved
# in one process per scene).  gpurun_out/retune2/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/retune2
mkdir -p "$OUT"
V='"regenerationSK:" "regenerationSK:batch=4" "regenerationSK:batch=12" "regenerationSK:chunk=128" "regenerationSK:chunk=512" "regenerationSK:drain=2" "regenerationSK:drain=0" "regenerationSK:sub=4" "regenerationSK:sub=1"'
for sc in manix hetvol; do
  eval timeout -k 10 400 python3 tools/tune.py --scene $sc --rounds 5 --variants $V > "$OUT/$sc.log" 2>&1 || { tail -20 "$OUT/$sc.log"; exit 1; }
  grep regen "$OUT/$sc.log" | cut -c1-90 | sed "s/^/$sc /"
done
