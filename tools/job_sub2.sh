set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sc in manix hetvol; do
  timeout -k 10 250 python3 tools/tune.py --scene $sc --rounds 6 --variants "regenerationSK:" "regenerationSK:sub=8" "regenerationSK:shard=8" "regenerationSK:shard=8,sub=1" "regenerationSK:shard=4" "regenerationSK:shard=4,sub=1" > gpurun_out/retune_sub2_$sc.log 2>&1
  grep regen gpurun_out/retune_sub2_$sc.log | cut -c1-80 | sed "s/^/$sc /"
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_records.py -x -q --timeout 300 -p no:cacheprovider > gpurun_out/pytest_sub2.log 2>&1; tail -1 gpurun_out/pytest_sub2.log
