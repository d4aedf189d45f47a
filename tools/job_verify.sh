# Full GPU verification of the in-tree build: smoke, every GPU test, bench, A/B vs HEAD
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['serial']['value'], d['roofline']['kernel_ms'])"
bash tools/job_ab2.sh 4 '"regenerationSK:" "regenerationSK:shard=8"' head default head default
