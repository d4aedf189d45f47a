set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_records.py tests/test_gpu_inflight.py -x -q --timeout 240 > gpurun_out/pytest_sub.log 2>&1 || { tail -30 gpurun_out/pytest_sub.log; exit 1; }
tail -1 gpurun_out/pytest_sub.log
for sc in manix hetvol; do
timeout -k 10 250 python3 tools/tune.py --scene $sc --rounds 5 --variants "regenerationSK:sub=1" "regenerationSK:" "regenerationSK:chunk=128" "regenerationSK:chunk=64" "regenerationSK:sub=1,shard=8" "regenerationSK:shard=8" "regenerationSK:shard=8,chunk=32" > gpurun_out/tune_sub_$sc.log 2>&1
grep regen gpurun_out/tune_sub_$sc.log | cut -c1-100
done
timeout -k 10 200 python3 tools/tailstamps.py --opt OPT_CHUNK=64 > gpurun_out/tail_c2_sub.log 2>&1
timeout -k 10 200 python3 tools/tailstamps.py --shard 8 > gpurun_out/tail_c2s8_sub.log 2>&1
grep -v "^  xcc\|^    " gpurun_out/tail_c2_sub.log gpurun_out/tail_c2s8_sub.log
