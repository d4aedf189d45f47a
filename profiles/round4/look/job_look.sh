# A/B of the Woodcock lookahead variants (round 4): C5 cloud at 4096^2, then manix / hetvol.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default look look2s look3 look3s look4 default look 2>&1 | tee gpurun_out/look_cloud.log
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default look look2u8 look2u2 look2s look3 look3s look4 2>&1 | tee gpurun_out/look_scenes.log
