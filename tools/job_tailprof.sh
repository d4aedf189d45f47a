# Ramp/drain profile of one wave-pool launch (tail-stamps build): C2 whole, 1/8 shard, C3
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/tailstamps.py > gpurun_out/tail_c2.log 2>&1
timeout -k 10 200 python3 tools/tailstamps.py --shard 8 > gpurun_out/tail_c2s8.log 2>&1
timeout -k 10 200 python3 tools/tailstamps.py --scene hetvol > gpurun_out/tail_c3.log 2>&1
timeout -k 10 200 python3 tools/tune.py --rounds 4 --variants "regenerationSK:" "regenerationSK:shard=8" "regenerationSK:sub=1" "regenerationSK:sub=1,shard=8" > gpurun_out/tune_base.log 2>&1
cat gpurun_out/tail_c2.log gpurun_out/tail_c2s8.log gpurun_out/tune_base.log
