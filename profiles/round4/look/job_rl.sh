# A/B: one roulette call for boundary and collision lanes (working tree) vs the in-tree build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default rl default rl 2>&1 | tee gpurun_out/rl_scenes.log
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default rl 2>&1 | tee gpurun_out/rl_cloud.log
