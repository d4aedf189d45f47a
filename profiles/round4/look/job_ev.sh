# A/B: event batch trigger at 48 / 56 waiting items instead of 64 (the drain stand-in scaled to match).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for sc in manix hetvol; do
  for v in default ev48 ev56 default; do
    if [ $v = default ]; then L=""; else L="--lib build/variants/$v/libcvr.so"; fi
    timeout -k 10 100 python3 tools/tune.py $L --scene $sc --rounds 3 --variants "regenerationSK:" > gpurun_out/ev_${sc}_$v.log 2>&1
    grep regen gpurun_out/ev_${sc}_$v.log | cut -c1-110 | sed "s/^/$sc $v /"
  done
done
