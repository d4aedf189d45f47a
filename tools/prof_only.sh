#!/bin/bash
# The kernel-trace passes of tools/final_profile.sh alone (C2, C3, C5), into gpurun_out/final.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p "$OUT"
export TMPDIR=/tmp
for sc in manix hetvol cloud; do
  if [ $sc = cloud ]; then S="--steps 3 --warmup 1"; else S="--steps 10 --warmup 2"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$sc" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-shard-emulation --scene $sc $S > "$OUT/prof_$sc.log" 2>&1 || { echo "prof_$sc failed"; tail -5 "$OUT/prof_$sc.log"; exit 1; }
  echo "prof_$sc ok"
done
