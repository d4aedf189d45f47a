# Per-rank step of N-GPU block-shard runs vs wave-pool grid and dequeue chunk (bench.py --emulate-only)
cd $GRAFT_REPO_ROOT
for spec in "4 0 0 0" "4 0 2560 0" "4 0 3840 0" "4 0 2560 128" "8 3 0 0" "8 3 1920 0" "8 3 3840 0" "8 3 2560 32" "8 3 2560 128" "2 0 0 0" "2 0 3840 0"; do
  set -- $spec
  timeout -k 10 60 python3 bench.py --emulate-only $1 $2 --grid $3 --chunk $4 --steps 40 --warmup 5 2>/dev/null | tail -1 | sed "s/^/grid=$3 chunk=$4 /" || exit 1
done
