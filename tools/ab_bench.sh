#!/bin/bash
# Driver-style bench lines of experiment builds, interleaved, one process per run:
#   tools/ab_bench.sh ROUNDS "BENCH ARGS" VARIANT [VARIANT ...]
# VARIANT: "default" (in-tree libcvr.so) or a name under build/variants/ (CVR_LIB).
# Prints value / serial / kernel_ms / shard-emulation speed-ups per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1 args=$2
shift 2
for r in $(seq "$rounds"); do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="build/variants/$v/libcvr.so"; fi
    CVR_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > /tmp/abb_$$.json 2>/tmp/abb_$$.err \
      || { echo "== $v FAILED"; tail -20 /tmp/abb_$$.err; exit 1; }
    python3 - "$v" "$r" /tmp/abb_$$.json <<'PY'
import json, sys
v, r, p = sys.argv[1:]
d = json.loads([l for l in open(p) if l.startswith("{")][-1])
se = d.get("shard_emulation") or {}
s = d.get("serial") or {}
sh = " ".join(f"n{n} {se[f'n{n}']['implied_speedup']:.3f}" for n in (2, 4, 8) if f"n{n}" in se)
print(f"[{r}] {v:12s} value {d['value']:9.1f} serial {s.get('value', 0):9.1f} ({s.get('value', 0) / d['value']:.3f}) "
      f"kernel {d['roofline']['kernel_ms']:.4f} ms  {sh}", flush=True)
PY
  done
done
