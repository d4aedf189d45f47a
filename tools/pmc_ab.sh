#!/bin/bash
# PMC of experiment builds on the GPU box: one rocprofv3 pass per (counter set,
# variant, scene) over tools/tune.py (2 launches of the C2-style workload).
#   tools/pmc_ab.sh "CTR1 CTR2" SCENES VARIANT [VARIANT ...]
# Output: gpurun_out/pmcab/<variant>_<scene>_<ctrs>/ ; summary: tools/pmc_ab_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ctrs=$1 scenes=$2
shift 2
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L="--lib build/variants/$v/libcvr.so"; fi
  for sc in ${scenes//,/ }; do
    d=gpurun_out/pmcab/${v}_${sc}_${ctrs// /_}
    mkdir -p "$d"
    timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-trace -d "$d" -o run --output-format csv -- \
      python3 tools/tune.py $L --scene "$sc" --rounds 1 --variants "regenerationSK:" > "$d/log" 2>&1
    rc=$?
    echo "== $v $sc ($ctrs) rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$d/log"; exit $rc; }
  done
done
