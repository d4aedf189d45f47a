# A/B of experiment builds: C2, C3 and the C2 1/8 shard, one process per build,
#   bash tools/job_ab.sh ROUNDS VARIANT...   ("default" = in-tree libcvr.so)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$1; shift
for sc in manix hetvol; do
  for v in "$@"; do
    if [ "$v" = default ]; then L=""; else L="--lib build/variants/$v/libcvr.so"; fi
    timeout -k 10 150 python3 tools/tune.py $L --scene $sc --rounds $R --variants "regenerationSK:" "regenerationSK:shard=8" > /tmp/ab.log 2>&1 || { cat /tmp/ab.log; exit 1; }
    grep regen /tmp/ab.log | sed "s/^/$sc $v /"
  done
done
