# Brick size sweep on the final build (dense: 2^1, 2^2 default, 2^3 cells per brick edge), interleaved per process.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for sc in manix hetvol; do
  timeout -k 10 300 python3 tools/tune.py --scene $sc --rounds 4 --variants "regenerationSK:" "regenerationSK:bounds=1" "regenerationSK:bounds=3" > gpurun_out/bounds_$sc.log 2>&1
  grep regen gpurun_out/bounds_$sc.log | cut -c1-200 | sed "s/^/$sc /"
done
