# cvr_render_frame + block output step: tests, then C2 / C3 bench lines
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_inflight.py tests/test_multiprocess_gpu.py -x -q --timeout 300 -p no:cacheprovider > gpurun_out/pytest_frame.log 2>&1 || { tail -40 gpurun_out/pytest_frame.log; exit 1; }
tail -1 gpurun_out/pytest_frame.log
for p in 3 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --frame-parts $p --no-cpu-baseline > gpurun_out/bench_frame$p.log 2>&1 || { tail -20 gpurun_out/bench_frame$p.log; exit 1; }
tail -1 gpurun_out/bench_frame$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 parts $p', d['value'], d['serial']['value'], d['serial']['one_launch']['value'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --scene hetvol --no-cpu-baseline > gpurun_out/bench_frame_c3.log 2>&1 || { tail -20 gpurun_out/bench_frame_c3.log; exit 1; }
tail -1 gpurun_out/bench_frame_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['serial']['value'], d['serial']['one_launch']['value'], d['roofline']['kernel_ms'])"
