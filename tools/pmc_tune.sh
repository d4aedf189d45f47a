#!/bin/bash
# PMC of run-time option variants on the GPU box: one rocprofv3 pass per
# (counter set, scene, variant) over tools/tune.py (2 launches each).
#   tools/pmc_tune.sh "CTR1 CTR2" SCENES NAME=TUNE_VARIANT [NAME=TUNE_VARIANT ...]
#   e.g. tools/pmc_tune.sh "SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" manix,hetvol \
#          one=regenerationSK: pair=regenerationSK:pair=1
# Output: gpurun_out/pmcab/<name>_<scene>_<ctrs>/ ; summary: tools/pmc_ab_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ctrs=$1 scenes=$2
shift 2
for nv in "$@"; do
  name=${nv%%=*} v=${nv#*=}
  for sc in ${scenes//,/ }; do
    d=gpurun_out/pmcab/${name}_${sc}_${ctrs// /_}
    mkdir -p "$d"
    timeout -k 10 150 rocprofv3 --pmc $ctrs --kernel-trace -d "$d" -o run --output-format csv -- \
      python3 tools/tune.py --scene "$sc" --rounds 1 --variants "$v" > "$d/log" 2>&1
    rc=$?
    echo "== $name $sc ($ctrs) rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$d/log"; exit $rc; }
  done
done
