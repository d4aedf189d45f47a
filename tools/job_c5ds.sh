set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/c5ds
mkdir -p "$OUT"
for r in 1 2; do
  for L in default ds1 ds2; do
    if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
    timeout -k 10 300 python3 tools/tune.py $LA --scene cloud --res 4096 --rounds 2 --variants "regenerationSK:" > "$OUT/c5_${L}_$r.log" 2>&1 || { tail -20 "$OUT/c5_${L}_$r.log"; exit 1; }
    grep regen "$OUT/c5_${L}_$r.log" | sed 's/  */ /g' | cut -c1-100 | sed "s/^/$L $r /"
  done
done
