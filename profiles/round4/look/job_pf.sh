# A/B on C5: the parked lane's cell loaded when it parks (CVR_WPOOL_PREFETCH=1) vs the in-tree build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default pf default pf 2>&1 | tee gpurun_out/pf_cloud.log
