# Drain migration (CVR_OPT_MIGRATE) and drain batches (CVR_OPT_DRAIN): parity, then A/B vs HEAD
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_records.py tests/test_gpu_inflight.py tests/test_gpu_production.py -x -q --timeout 300 > gpurun_out/pytest_mig.log 2>&1 || { tail -30 gpurun_out/pytest_mig.log; exit 1; }
tail -1 gpurun_out/pytest_mig.log
for sc in manix hetvol; do
  for L in head default noC; do
    if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
    if [ $L = head ]; then V='"regenerationSK:" "regenerationSK:shard=8"'; else V='"regenerationSK:" "regenerationSK:migrate=0" "regenerationSK:drain=0,migrate=0" "regenerationSK:migrate=12" "regenerationSK:migrate=40" "regenerationSK:shard=8" "regenerationSK:shard=8,migrate=0" "regenerationSK:shard=8,migrate=40"'; fi
    eval timeout -k 10 200 python3 tools/tune.py $LA --scene $sc --rounds 4 --variants $V > gpurun_out/tune_mig_${sc}_$L.log 2>&1
    grep regen gpurun_out/tune_mig_${sc}_$L.log | cut -c1-80 | sed "s/^/$sc $L /"
  done
done
timeout -k 10 200 python3 tools/tailstamps.py > gpurun_out/tail_c2_m.log 2>&1
timeout -k 10 200 python3 tools/tailstamps.py --shard 8 > gpurun_out/tail_c2s8_m.log 2>&1
grep -v "^  wave\|^    \|xcc" gpurun_out/tail_c2_m.log gpurun_out/tail_c2s8_m.log
