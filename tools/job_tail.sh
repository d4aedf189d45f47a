set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_records.py -x -q --timeout 240 > gpurun_out/pytest_records.log 2>&1 || { tail -30 gpurun_out/pytest_records.log; exit 1; }
tail -2 gpurun_out/pytest_records.log
timeout -k 10 200 python3 tools/tune.py --rounds 6 --variants "regenerationSK:" "regenerationSK:tailu=0" "regenerationSK:tailc=16" "regenerationSK:tailc=64" "regenerationSK:shard=8" "regenerationSK:shard=8,tailu=0" > gpurun_out/tune_tail.log 2>&1
cat gpurun_out/tune_tail.log
timeout -k 10 200 python3 tools/tailstamps.py > gpurun_out/tail_c2.log 2>&1
timeout -k 10 200 python3 tools/tailstamps.py --shard 8 > gpurun_out/tail_c2s8.log 2>&1
timeout -k 10 200 python3 tools/tailstamps.py --opt OPT_TAIL_UNITS=0 > gpurun_out/tail_c2_notail.log 2>&1
cat gpurun_out/tail_c2.log gpurun_out/tail_c2s8.log gpurun_out/tail_c2_notail.log
