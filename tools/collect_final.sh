#!/bin/bash
# Fold a tools/final_profile.sh run (gpurun_out/final) into profiles/round2 and
# profiles/traffic.json, and print the numbers DESIGN.md quotes.
set -eu
cd "$(dirname "$0")/.."
F=gpurun_out/final
P=${1:-profiles/round6}
for sc in manix hetvol cloud; do
  case $sc in manix) key=k_wpool_1024x1024_20it; c=c2;; hetvol) key=hetvol_k_wpool_1024x1024_20it; c=c3;;
                     cloud) key=cloud_k_wpool_4096x4096_20it; c=c5;; esac
  case $sc in manix) inst="k_wpool<false, 5, 2, false, false>";; hetvol) inst="k_wpool<false, 5, 3, false, false>";;
              cloud) inst="k_wpool<false, 5, 1, false, false>";; esac
  python3 tools/traffic.py $F/pmcf_$sc $F/pmcw_$sc $key "$inst" | cut -c1-140
  python3 tools/valu.py $F/pmcv_$sc $key "$inst" | cut -c1-140
  cp $F/prof_$sc/run_kernel_stats.csv $P/${c}_kernel_stats.csv
  if [ $sc = cloud ]; then sw="3 1"; else sw="20 5"; fi
  python3 tools/kernel_phases.py $F/prof_$sc/run_kernel_trace.csv "$inst" $sw $P/${c}_kernel_phases.json $F/prof_$sc.log | grep "_ms\|_over_"
done
if [ -d $F/pmc_d ]; then  # final_profile.sh part 2
  python3 tools/pmc_summary.py $P/pmc_k_wpool.json k_wpool $F/pmc_a $F/pmc_b $F/pmc_c $F/pmc_d
  python3 tools/pmc_summary.py $P/pmc_k_wpool_cloud.json k_wpool $F/pmc5_a $F/pmc5_b $F/pmc5_c
fi
for c in c1 c2 c3 c4 c5; do
  [ -f $F/${c}_bench.log ] || continue
  cp $F/${c}_bench.log $P/${c}_bench.log
  grep '^{' $F/${c}_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; cb=d.get('cpu_baseline') or {}
print('$c value', d['value'], 'ms', d['ms_per_step'], 'kernel', r['kernel_ms'], 'frac', r['frac'], 'achieved', r['achieved'],
      'serial', d.get('serial',{}).get('value'), 'cpu', cb.get('value'), 'traffic', r['traffic'], 'hbm_frac', r['hbm_frac_measured'])"
done
cp $F/pytest_gpu.log $P/pytest_gpu.log; cp $F/smoke.log $P/smoke.log; cp $F/libcvr.sha256 $P/libcvr.sha256
for f in $F/k_*.log $F/pair_*.log; do [ -f "$f" ] && cp "$f" $P/; done
tail -1 $P/pytest_gpu.log; tail -1 $P/smoke.log; cat $P/libcvr.sha256; sha256sum cudavolumerenderer_amd/libcvr.so
