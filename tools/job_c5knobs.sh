# C5 (cloud 4096^2, 20 it): run-time knobs and Woodcock unroll builds vs the default, interleaved
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/c5knobs
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 400 python3 tools/tune.py --scene cloud --res 4096 --rounds 1 --variants "regenerationSK:" "regenerationSK:batch=4" "regenerationSK:batch=12" "regenerationSK:batch=16" "regenerationSK:ev=16" "regenerationSK:ev=32" "regenerationSK:drain=2" "regenerationSK:sub=1" "regenerationSK:sub=4" > "$OUT/knobs_$r.log" 2>&1 || { tail -20 "$OUT/knobs_$r.log"; exit 1; }
  grep regen "$OUT/knobs_$r.log" | sed 's/  */ /g' | cut -c1-90 | sed "s/^/knobs $r /"
  for L in default u2 u3 u6; do
    if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
    timeout -k 10 300 python3 tools/tune.py $LA --scene cloud --res 4096 --rounds 2 --variants "regenerationSK:" > "$OUT/c5_${L}_$r.log" 2>&1 || { tail -20 "$OUT/c5_${L}_$r.log"; exit 1; }
    grep regen "$OUT/c5_${L}_$r.log" | sed 's/  */ /g' | cut -c1-90 | sed "s/^/$L $r /"
  done
done
