# 4 vs 5 waves per SIMD on the final build (runtime CVR_OPT_WAVES), interleaved per process.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for sc in manix hetvol; do
  timeout -k 10 150 python3 tools/tune.py --scene $sc --rounds 4 --variants "regenerationSK:" "regenerationSK:waves=4" > gpurun_out/waves_$sc.log 2>&1
  grep regen gpurun_out/waves_$sc.log | cut -c1-110 | sed "s/^/$sc /"
done
