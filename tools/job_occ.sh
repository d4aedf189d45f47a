set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 bash tools/ab.sh manix 6 default g1 default g1 > gpurun_out/ab_occ_manix.log 2>&1
timeout -k 10 200 bash tools/ab.sh hetvol 6 default g1 > gpurun_out/ab_occ_hetvol.log 2>&1
for L in "" "--lib build/variants/g1/libcvr.so"; do
  timeout -k 10 120 python3 tools/tune.py $L --rounds 6 --variants "regenerationSK:shard=8" "regenerationSK:shard=4" >> gpurun_out/ab_occ_shard.log 2>&1
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_occ.log 2>&1
cat gpurun_out/ab_occ_manix.log gpurun_out/ab_occ_hetvol.log gpurun_out/ab_occ_shard.log; tail -1 gpurun_out/bench_occ.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['serial'], d['roofline']['kernel_ms'])"
