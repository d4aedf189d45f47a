# Runtime-knob sweep on the kept build (wave-pool refill batch, drain rule), interleaved per process.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for sc in manix hetvol; do
  timeout -k 10 300 python3 tools/tune.py --scene $sc --rounds 4 --variants "regenerationSK:" "regenerationSK:batch=4" "regenerationSK:batch=6" "regenerationSK:batch=12" "regenerationSK:batch=16" "regenerationSK:drain=2" "regenerationSK:drain=0" > gpurun_out/sweep_$sc.log 2>&1
  grep regen gpurun_out/sweep_$sc.log | cut -c1-110
done
timeout -k 10 300 python3 tools/tune.py --scene cloud --res 4096 --rounds 2 --variants "regenerationSK:" "regenerationSK:batch=4" "regenerationSK:batch=12" "regenerationSK:batch=16" > gpurun_out/sweep_cloud.log 2>&1
grep regen gpurun_out/sweep_cloud.log | cut -c1-110
