#!/bin/bash
# Runs GPU steps on the gpurun box, each under its own timeout; stops after a
# timeout / abort / crash (rc >= 124).  Usage: tools/gpu_job.sh step [step...]
#   steps: info smoke pytest bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name (limit ${secs}s): $*"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    info) run info 60 bash -c 'nproc; grep -m1 "model name" /proc/cpuinfo; grep -o -m1 -w fma /proc/cpuinfo; rocm-smi --showproductname 2>/dev/null | head -20; python3 -c "import torch;print(torch.__version__, torch.cuda.device_count())"' ;;
    smoke) run smoke 400 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1100 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    pytestall) run pytest_gpu 1100 python3 -m pytest tests -m gpu -q --timeout 900 -p no:cacheprovider ;;
    bench) run bench 600 python3 bench.py --steps 10 --warmup 2 ;;
    benchd) run benchd 600 python3 bench.py --steps 20 --warmup 5 ;;
    bench_c3) run bench_c3 600 python3 bench.py --steps 10 --warmup 2 --scene hetvol ;;
    bench_c4) run bench_c4 600 python3 bench.py --steps 3 --warmup 1 --shard tiles --resolution 2048 2048 --iterations 256 --no-cpu-baseline ;;
    bench_c5) run bench_c5 600 python3 bench.py --steps 5 --warmup 1 --scene cloud ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmclist) run pmclist 120 rocprofv3 -L ;;
    tune) run tune 600 python3 tools/tune.py ;;
    stamps) run stamps 300 python3 tools/stamps.py ;;
    poolstamps) run poolstamps 300 python3 tools/poolstamps.py ;;
    pmc_sq) run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 1 --variants "regenerationSK:ev=16,chunk=128" ;;
    pmc_a) run pmc_a 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/pmc_a" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    pmc_b) run pmc_b 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_TA_BUSY --kernel-trace -d "$OUT/pmc_b" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    pmc_c) run pmc_c 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d "$OUT/pmc_c" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    pmc_f) run pmc_f 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_f" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    pmc_w) run pmc_w 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_w" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    pmc_d) run pmc_d 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_LDS_BANK_CONFLICT --kernel-trace -d "$OUT/pmc_d" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    pmc_e) run pmc_e 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace -d "$OUT/pmc_e" -o run --output-format csv -- python3 "$ROOT/tools/tune.py" --rounds 2 --variants "regenerationSK:" ;;
    # per-scene profiles: prof:SCENE, pmcf:SCENE (FETCH_SIZE), pmcw:SCENE (WRITE_SIZE)
    prof:*) sc=${step#prof:}; run prof_$sc 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$sc" -o run --output-format csv -- python3 "$ROOT/bench.py" --scene $sc --steps 10 --warmup 2 --no-cpu-baseline --no-shard-emulation ;;
    pmcf:*) sc=${step#pmcf:}; mkdir -p "$OUT/pmcf_$sc"; sha256sum cudavolumerenderer_amd/libcvr.so > "$OUT/pmcf_$sc/libcvr.sha256"; run pmcf_$sc 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_$sc" -o run --output-format csv -- python3 "$ROOT/bench.py" --scene $sc --steps 3 --warmup 1 --no-cpu-baseline --no-shard-emulation ;;
    pmcw:*) sc=${step#pmcw:}; mkdir -p "$OUT/pmcw_$sc"; sha256sum cudavolumerenderer_amd/libcvr.so > "$OUT/pmcw_$sc/libcvr.sha256"; run pmcw_$sc 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_$sc" -o run --output-format csv -- python3 "$ROOT/bench.py" --scene $sc --steps 3 --warmup 1 --no-cpu-baseline --no-shard-emulation ;;
    # synchronous render variants (tools/frame_probe.py): frame:SCENE:v1,v2[:LIB]
    frame:*) IFS=: read -r _ sc vs lib <<< "$step"; tag=default; [ -n "$lib" ] && tag=$(basename $(dirname $lib)); run frame_${sc}_$tag 400 python3 tools/frame_probe.py --scene $sc --variants $vs ${lib:+--lib $lib} ;;
    # experiment builds (build/variants/NAME), one process each, interleaved: abr:SCENE:RES:ROUNDS:v1;v2
    abr:*) IFS=: read -r _ sc res rounds vs <<< "$step"; run abr_${sc}_$res 900 env AB_ARGS="--res $res" bash tools/ab.sh $sc $rounds ${vs//;/ } ;;
    # VALU issue (tools/valu.py): pmcv:SCENE
    pmcv:*) sc=${step#pmcv:}; mkdir -p "$OUT/pmcv_$sc"; sha256sum cudavolumerenderer_amd/libcvr.so > "$OUT/pmcv_$sc/libcvr.sha256"; run pmcv_$sc 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmcv_$sc" -o run --output-format csv -- python3 "$ROOT/bench.py" --scene $sc --steps 3 --warmup 1 --no-cpu-baseline --no-shard-emulation ;;
    # one kernel id's C2 bench line: benchk:KERNEL
    benchk:*) k=${step#benchk:}; run benchk_$k 400 python3 bench.py --kernel $k --steps 10 --warmup 2 --no-cpu-baseline --no-shard-emulation ;;
    # in-process interleaved variants: tunev:SCENE:ROUNDS:variant;variant (e.g. regenerationSK:pair=1)
    tunev:*) IFS=: read -r _ sc rounds vs <<< "$step"; run tunev_$sc 400 python3 tools/tune.py --scene $sc --rounds $rounds --variants ${vs//;/ } ;;
    # selected GPU test files: pytestf:tests/a.py,tests/b.py
    pytestf:*) fs=${step#pytestf:}; run pytestf 900 python3 -u -m pytest ${fs//,/ } -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    # the same at a resolution: tunevr:SCENE:RES:ROUNDS:variant;variant
    tunevr:*) IFS=: read -r _ sc res rounds vs <<< "$step"; run tunevr_${sc}_$res 400 python3 tools/tune.py --scene $sc --res $res --rounds $rounds --variants ${vs//;/ } ;;
    # the driver's default bench line
    benchdef) run benchdef 600 python3 bench.py ;;
    # arbitrary counters on a scene's bench run: pmcx:SCENE:CTR1,CTR2,...
    pmcx:*) IFS=: read -r _ sc ctrs <<< "$step"; d=pmcx_${sc}_${ctrs//,/_}; mkdir -p "$OUT/$d"; sha256sum cudavolumerenderer_amd/libcvr.so > "$OUT/$d/libcvr.sha256"; run $d 300 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace -d "$OUT/$d" -o run --output-format csv -- python3 "$ROOT/bench.py" --scene $sc --steps 3 --warmup 1 --no-cpu-baseline --no-shard-emulation ;;
    # A/B of experiment builds: ab:SCENE:ROUNDS:variant1,variant2,...
    ab:*) IFS=: read -r _ sc rounds vs <<< "$step"; run ab_$sc 400 bash tools/ab.sh $sc $rounds ${vs//,/ } ;;
    *) echo "unknown step $step" ;;
  esac
done
