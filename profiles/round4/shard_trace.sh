# Kernel trace of one rank's step of an 8-GPU block-shard run (bench.py --emulate-only), and timings at N=4/8
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/shardprof
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/n8r3 -o run --output-format csv -- python3 bench.py --emulate-only 8 3 --steps 30 --warmup 5 > $OUT/n8r3.log 2>&1
for c in 2 3 4 6; do timeout -k 10 60 python3 bench.py --emulate-only 8 3 --contexts $c --steps 30 --warmup 5 2>/dev/null | tail -1; done
for c in 3; do timeout -k 10 60 python3 bench.py --emulate-only 4 0 --contexts $c --steps 30 --warmup 5 2>/dev/null | tail -1; done
