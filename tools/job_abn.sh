#!/bin/bash
# A/B of experiment builds vs the in-tree build, one-launch kernel, C2 and C3, interleaved:
#   bash tools/job_abn.sh ROUNDS LIB...   (gpurun_out/abn/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abn
mkdir -p "$OUT"
R=$1; shift
for sc in manix hetvol; do
  for r in $(seq 1 $R); do
    for L in default "$@"; do
      if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
      timeout -k 10 200 python3 tools/tune.py $LA --scene $sc --rounds 3 --variants "regenerationSK:" > "$OUT/${sc}_${L}_$r.log" 2>&1 || { tail -20 "$OUT/${sc}_${L}_$r.log"; exit 1; }
      grep regen "$OUT/${sc}_${L}_$r.log" | cut -c1-90 | sed "s/^/$sc $L $r /"
    done
  done
done
