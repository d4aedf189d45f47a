# A/B: kind-major batch thresholds (boundary 40/56, collision 16/32) on the lookahead build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_scenes.sh 3 '"regenerationSK:"' default km40 km56 kc16 kc32 u6 default 2>&1 | tee gpurun_out/kind_scenes.log
