set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--res 4096" bash tools/ab.sh cloud 2 default defer look default defer look 2>&1 | tee gpurun_out/defer_cloud.log
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default defer look default defer look 2>&1 | tee gpurun_out/defer_scenes.log
