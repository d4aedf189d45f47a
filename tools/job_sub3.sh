set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sc in manix hetvol; do
  timeout -k 10 300 python3 tools/tune.py --scene $sc --rounds 10 --variants "regenerationSK:sub=1" "regenerationSK:sub=8" > gpurun_out/sub3_$sc.log 2>&1
  grep regen gpurun_out/sub3_$sc.log | cut -c1-80 | sed "s/^/$sc /"
done
