# A/B: deferred cell fetch inside the two-point lookahead (CVR_WPOOL_LOOKDEFER: 2 sparse only, 14 all).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default ld default ld 2>&1 | tee gpurun_out/ld_cloud.log
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default ld14 default ld14 2>&1 | tee gpurun_out/ld_scenes.log
