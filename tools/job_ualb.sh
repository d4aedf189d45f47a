#!/bin/bash
# Uniform albedo read as a constant: GPU tests of the affected paths, then C3 (uniform)
# and C2 (not uniform) one-launch kernels: in-tree build with the option on / off, and HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ualb
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for sc in hetvol manix; do
  for r in 1 2 3; do
    timeout -k 10 200 python3 tools/tune.py --scene $sc --rounds 3 --variants "regenerationSK:" "regenerationSK:ualb=0" > "$OUT/${sc}_default_$r.log" 2>&1 || exit 1
    timeout -k 10 200 python3 tools/tune.py --lib build/variants/head/libcvr.so --scene $sc --rounds 3 --variants "regenerationSK:" > "$OUT/${sc}_head_$r.log" 2>&1 || exit 1
    grep regen "$OUT/${sc}_default_$r.log" "$OUT/${sc}_head_$r.log" | cut -c1-120
  done
done
