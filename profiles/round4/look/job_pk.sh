# A/B: packed two-lane log in the Woodcock group (CVR_WPOOL_PK=1) vs the in-tree build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default pk default pk 2>&1 | tee gpurun_out/pk_scenes.log
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default pk default pk 2>&1 | tee gpurun_out/pk_cloud.log
