# Re-tune after the round-3 changes: sub-queues per XCD band, renders in flight
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sc in manix hetvol; do
  timeout -k 10 250 python3 tools/tune.py --scene $sc --rounds 5 --variants "regenerationSK:" "regenerationSK:sub=1" "regenerationSK:sub=2" "regenerationSK:sub=4" "regenerationSK:shard=8" "regenerationSK:shard=8,sub=1" "regenerationSK:shard=8,sub=4" > gpurun_out/retune_sub_$sc.log 2>&1
  grep regen gpurun_out/retune_sub_$sc.log | cut -c1-80 | sed "s/^/$sc /"
done
for n in 2 3 4; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --contexts $n --no-cpu-baseline > gpurun_out/retune_ctx$n.log 2>&1
  tail -1 gpurun_out/retune_ctx$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('contexts $n', d['value'], d['ms_per_step'])"
done
