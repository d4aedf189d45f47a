# A/B: sparse bound codes as a separate u8 table (CVR_SPARSE_CODES=1) vs the in-tree build, C5.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default codes default codes 2>&1 | tee gpurun_out/codes_cloud.log
