# A/B of experiment builds vs HEAD: bash tools/ab_scenes.sh ROUNDS "VARIANTS" LIB...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$1; V=$2; shift 2
for sc in manix hetvol; do
  for L in "$@"; do
    if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
    if [ $L = head ]; then VV='"regenerationSK:" "regenerationSK:shard=8"'; else VV="$V"; fi
    eval timeout -k 10 200 python3 tools/tune.py $LA --scene $sc --rounds $R --variants $VV > gpurun_out/ab2_${sc}_$L.log 2>&1
    grep regen gpurun_out/ab2_${sc}_$L.log | cut -c1-80 | sed "s/^/$sc $L /"
  done
done
