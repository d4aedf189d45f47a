# A/B: survivors' (T, image_id) stored before their AABB test (CVR_WPOOL_TSTORE_EARLY=1), then the repeat bench.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default ts default ts 2>&1 | tee gpurun_out/ts_scenes.log
bash tools/repeat_bench.sh 5
