#!/bin/bash
# In-launch output, round 2: GPU tests of the current build, the frame probe for the
# current build and experiment builds, then the one-launch kernel (no in-launch
# output) A/B against HEAD.  gpurun_out/flush3/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/flush3
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_flush.py tests/test_gpu_inflight.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for L in default "$@"; do
  if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
  timeout -k 10 200 python3 tools/frame_probe.py $LA --variants flush,copy --rounds 2 --reps 10 > "$OUT/probe_$L.log" 2>&1 || { tail -20 "$OUT/probe_$L.log"; exit 1; }
  grep round "$OUT/probe_$L.log" | sed "s/^/$L /" | cut -c1-150
done
for sc in manix hetvol; do
  for r in 1 2 3; do
    for L in default head; do
      if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
      timeout -k 10 200 python3 tools/tune.py $LA --scene $sc --rounds 3 --variants "regenerationSK:" > "$OUT/ab_${sc}_${L}_$r.log" 2>&1 || { tail -20 "$OUT/ab_${sc}_${L}_$r.log"; exit 1; }
      grep regen "$OUT/ab_${sc}_${L}_$r.log" | cut -c1-90 | sed "s/^/$sc $L $r /"
    done
  done
done
