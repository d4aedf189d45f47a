# Sub-queues on large launches (C4-like: 2048^2 manix, many paths per wave): 1 vs 8 per band
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/tune.py --scene manix --res 2048 --iters 32 --rounds 4 --variants "regenerationSK:" "regenerationSK:sub=8" "regenerationSK:sub=4" > gpurun_out/c4sub.log 2>&1
grep regen gpurun_out/c4sub.log | cut -c1-80
