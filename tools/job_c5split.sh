# C5: sparse pool with the event part in global memory (split) at 4 / 5 waves vs the default (4 waves, T in LDS)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/tune.py --scene cloud --res 4096 --rounds 2 --variants "regenerationSK:" "regenerationSK:waves=5" > gpurun_out/c5split_default.log 2>&1
grep regen gpurun_out/c5split_default.log | cut -c1-80 | sed "s/^/default /"
timeout -k 10 400 python3 tools/tune.py --lib build/variants/splitsp/libcvr.so --scene cloud --res 4096 --rounds 2 --variants "regenerationSK:" "regenerationSK:waves=5" > gpurun_out/c5split_split.log 2>&1
grep regen gpurun_out/c5split_split.log | cut -c1-80 | sed "s/^/split /"
