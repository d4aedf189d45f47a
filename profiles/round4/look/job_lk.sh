# C5: K-point lookahead with the deferred fetch (sparse), K = 3 / 4, and 4 waves per SIMD.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default lk3 lk4 lk4u4 default; do
  if [ $v = default ]; then L=""; else L="--lib build/variants/$v/libcvr.so"; fi
  timeout -k 10 200 python3 tools/tune.py $L --scene cloud --res 4096 --rounds 1 --variants "regenerationSK:" "regenerationSK:waves=4" > gpurun_out/lk_$v.log 2>&1
  grep regen gpurun_out/lk_$v.log | cut -c1-100 | sed "s/^/$v /"
done
