#!/bin/bash
# Sparse instances specialised on their medium layout: sparse GPU parity tests,
# then C5 (cloud 4096^2, 20 it) one-launch kernel vs HEAD, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c5spec
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -k "sparse or cloud or vdb or records or production" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for L in default head; do
    if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
    timeout -k 10 300 python3 tools/tune.py $LA --scene cloud --res 4096 --rounds 2 --variants "regenerationSK:" > "$OUT/c5_${L}_$r.log" 2>&1 || { tail -20 "$OUT/c5_${L}_$r.log"; exit 1; }
    grep regen "$OUT/c5_${L}_$r.log" | cut -c1-90 | sed "s/^/$L $r /"
  done
done
