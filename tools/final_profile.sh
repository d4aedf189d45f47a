#!/bin/bash
# One measurement pass of the committed build on the GPU box (gpurun):
# GPU tests, bench lines for C1-C5, rocprofv3 kernel stats (C2, C3, C5), PMC
# traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs), the VALU issue pass
# (tools/valu.py) and the SQ counter groups for C2 and C5.  Every step under its own time limit; stops at the first
# failure.  Output: gpurun_out/final/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p "$OUT"
export TMPDIR=/tmp
sha256sum cudavolumerenderer_amd/libcvr.so > "$OUT/libcvr.sha256"
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - t0 ))s"
  [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
}
B="python3 bench.py --no-cpu-baseline"
PART=${1:-all}  # 1: tests, traces, traffic / VALU passes, bench lines; 2: SQ groups, kernel ids, pair
if [ "$PART" != 2 ]; then
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python3 -u -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider
for sc in manix hetvol cloud; do
  # the driver's own bench settings (--steps 20 --warmup 5) for C2/C3, so the traced pipelined
  # phase is the headline step; no shard emulation in the traced run: tools/kernel_phases.py
  # reads the bench's own launches and compares their span with the run's ms_per_step
  if [ $sc = cloud ]; then S="--steps 3 --warmup 1"; else S="--steps 20 --warmup 5"; fi
  step prof_$sc 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$sc" -o run --output-format csv -- $B --no-shard-emulation --scene $sc $S
  if [ $sc = cloud ]; then S="--steps 2 --warmup 1"; else S="--steps 3 --warmup 1"; fi
  # (--no-count-words: no counting launch of a sparse medium, so only the benchmarked instance runs)
  step pmcf_$sc 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_$sc" -o run --output-format csv -- $B --scene $sc --serial --no-count-words $S
  step pmcw_$sc 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_$sc" -o run --output-format csv -- $B --scene $sc --serial --no-count-words $S
  step pmcv_$sc 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmcv_$sc" -o run --output-format csv -- $B --scene $sc --serial --no-count-words $S
  cp "$OUT/libcvr.sha256" "$OUT/pmcf_$sc/"; cp "$OUT/libcvr.sha256" "$OUT/pmcw_$sc/"; cp "$OUT/libcvr.sha256" "$OUT/pmcv_$sc/"
done
# fold the traffic passes into profiles/traffic.json here too, so the bench lines
# below (same libcvr.so) carry their measured traffic
python3 tools/traffic.py "$OUT/pmcf_manix" "$OUT/pmcw_manix" k_wpool_1024x1024_20it "k_wpool<false, 5, 2, false, false>" > /dev/null &&
  python3 tools/traffic.py "$OUT/pmcf_hetvol" "$OUT/pmcw_hetvol" hetvol_k_wpool_1024x1024_20it "k_wpool<false, 5, 3, false, false>" > /dev/null &&
  python3 tools/traffic.py "$OUT/pmcf_cloud" "$OUT/pmcw_cloud" cloud_k_wpool_4096x4096_20it "k_wpool<false, 5, 1, false, false>" > /dev/null || exit 1
# and the VALU issue (roofline.valu) of each benchmark kernel instance
python3 tools/valu.py "$OUT/pmcv_manix" k_wpool_1024x1024_20it "k_wpool<false, 5, 2, false, false>" > /dev/null &&
  python3 tools/valu.py "$OUT/pmcv_hetvol" hetvol_k_wpool_1024x1024_20it "k_wpool<false, 5, 3, false, false>" > /dev/null &&
  python3 tools/valu.py "$OUT/pmcv_cloud" cloud_k_wpool_4096x4096_20it "k_wpool<false, 5, 1, false, false>" > /dev/null || exit 1
step c2_bench 200 python3 bench.py --steps 20 --warmup 5
step c1_bench 200 python3 bench.py --scene bucky --steps 20 --warmup 5
step c3_bench 200 python3 bench.py --scene hetvol --steps 20 --warmup 5
step c5_bench 400 python3 bench.py --scene cloud --steps 5 --warmup 1
step c4_bench 400 $B --shard tiles --resolution 2048 2048 --iterations 256 --steps 2 --warmup 1
fi
[ "$PART" = 1 ] && { echo "final profile part 1 done"; exit 0; }
step pmc_a 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/pmc_a" -o run --output-format csv -- $B --serial --steps 3 --warmup 1
step pmc_b 200 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_TA_BUSY --kernel-trace -d "$OUT/pmc_b" -o run --output-format csv -- $B --serial --steps 3 --warmup 1
step pmc_c 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d "$OUT/pmc_c" -o run --output-format csv -- $B --serial --steps 3 --warmup 1
step pmc_d 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_LDS_BANK_CONFLICT --kernel-trace -d "$OUT/pmc_d" -o run --output-format csv -- $B --serial --steps 3 --warmup 1
C5="$B --scene cloud --serial --no-count-words --steps 2 --warmup 1"
step pmc5_a 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/pmc5_a" -o run --output-format csv -- $C5
step pmc5_b 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_TA_BUSY --kernel-trace -d "$OUT/pmc5_b" -o run --output-format csv -- $C5
step pmc5_c 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d "$OUT/pmc5_c" -o run --output-format csv -- $C5
# every kernel id's C2 line (all on the wave pool by default)
for k in streamingSK sortingSK streamingMK naiveSK naiveMK; do
  step k_$k 300 python3 bench.py --kernel $k --steps 20 --warmup 5 --no-shard-emulation --no-cpu-baseline
done
echo "final profile done"
