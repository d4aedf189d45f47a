# A/B on C5: deferred fetch inside the lookahead (sparse) with 1, 2, 3, 4 groups per swap check.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default ld ldu2 ldu6 ldu8 default ld 2>&1 | tee gpurun_out/ldu_cloud.log
