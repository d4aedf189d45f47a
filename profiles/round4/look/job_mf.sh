# A/B: one merged cell-fetch block per two-point group (CVR_WPOOL_MERGEFETCH=1) vs the in-tree build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default mf default mf 2>&1 | tee gpurun_out/mf_scenes.log
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default mf default mf 2>&1 | tee gpurun_out/mf_cloud.log
