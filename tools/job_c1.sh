# C1-size launches (bucky 256^2, 4 it) and C2: HEAD build vs the in-tree build, drain on/off
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for L in head default head default; do
  if [ $L = default ]; then LA=""; V='"regenerationSK:grid=2560" "regenerationSK:grid=2560,drain=0" "regenerationSK:grid=1280" "regenerationSK:grid=1280,drain=0"'; else LA="--lib build/variants/$L/libcvr.so"; V='"regenerationSK:grid=2560" "regenerationSK:grid=1280"'; fi
  eval timeout -k 10 200 python3 tools/tune.py $LA --scene bucky --res 256 --iters 4 --rounds 10 --variants $V > gpurun_out/c1ab_$L.log 2>&1
  grep regen gpurun_out/c1ab_$L.log | cut -c1-80 | sed "s/^/c1 $L /"
done
