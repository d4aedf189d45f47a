#!/bin/bash
# In-launch output (CVR_OPT_FRAME_FLUSH): its GPU tests, then one synchronous
# render per call with and without it (C2, C3, C1 sizes).  gpurun_out/flush/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/flush
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_flush.py tests/test_gpu_inflight.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python3 tools/frame_probe.py --variants flush,copy --rounds 4 > "$OUT/probe_c2.log" 2>&1 || { tail -20 "$OUT/probe_c2.log"; exit 1; }
cat "$OUT/probe_c2.log"
timeout -k 10 300 python3 tools/frame_probe.py --scene hetvol --variants flush,copy --rounds 3 > "$OUT/probe_c3.log" 2>&1 || { tail -20 "$OUT/probe_c3.log"; exit 1; }
cat "$OUT/probe_c3.log"
timeout -k 10 300 python3 tools/frame_probe.py --scene bucky --res 256 --iters 4 --variants flush,copy --rounds 3 > "$OUT/probe_c1.log" 2>&1 || { tail -20 "$OUT/probe_c1.log"; exit 1; }
cat "$OUT/probe_c1.log"
