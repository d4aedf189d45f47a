#!/bin/bash
# Run-to-run spread of the driver's default bench line: N fresh `python bench.py`
# processes on one box (default 5), each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-5}
OUT=gpurun_out/repeat
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 "$N"); do
  timeout -k 10 200 python3 bench.py --no-shard-emulation > "$OUT/run$i.log" 2>&1 || { echo "run $i rc=$?"; tail -5 "$OUT/run$i.log"; exit 1; }
  grep '^{' "$OUT/run$i.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('run $i', d['value'], d['serial']['value'], r['kernel_ms'], r['frac'])"
done
