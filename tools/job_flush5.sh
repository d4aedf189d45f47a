#!/bin/bash
# In-launch output tests, then flush/copy probes (C2, C1) for the in-tree build and experiment builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/flush5
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_flush.py tests/test_gpu_inflight.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
for L in default "$@"; do
  if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
  timeout -k 10 200 python3 tools/frame_probe.py $LA --variants flush,copy --rounds 1 --reps 20 > "$OUT/probe_${L}_$r.log" 2>&1 || { tail -20 "$OUT/probe_${L}_$r.log"; exit 1; }
  grep round "$OUT/probe_${L}_$r.log" | sed "s/^/$L $r /" | cut -c1-110
  timeout -k 10 200 python3 tools/frame_probe.py $LA --scene bucky --res 256 --iters 4 --variants flush,copy --rounds 1 --reps 50 > "$OUT/probe1_${L}_$r.log" 2>&1 || { tail -20 "$OUT/probe1_${L}_$r.log"; exit 1; }
  grep round "$OUT/probe1_${L}_$r.log" | sed "s/^/C1 $L $r /" | cut -c1-110
done
done
