# event-batch policy variants vs the in-tree build (C2, C3, 1/8 shard)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/job_ab2.sh 4 '"regenerationSK:" "regenerationSK:shard=8"' default major km32 default major km32
