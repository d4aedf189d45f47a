#!/bin/bash
# A/B timing of experiment builds on the GPU box (one process per build,
# interleaved, each under its own time limit):
#   tools/ab.sh SCENE ROUNDS VARIANT [VARIANT ...]
# VARIANT is "default" (the in-tree libcvr.so) or a name under build/variants/
# (make variant NAME=... DEFS=...).  Stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scene=$1 rounds=$2
shift 2
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L="--lib build/variants/$v/libcvr.so"; fi
  echo "== $v ($scene)"
  timeout -k 10 150 python3 tools/tune.py $L --scene "$scene" ${AB_ARGS:-} --rounds "$rounds" --variants "regenerationSK:" \
    > /tmp/ab_$$.log 2>&1 || { cat /tmp/ab_$$.log; exit 1; }
  grep regen /tmp/ab_$$.log
done
