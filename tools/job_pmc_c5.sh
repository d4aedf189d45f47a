# C5 (sparse cloud, 4096^2, 20 it): the C2 PMC groups on k_wpool<false,4,true,false>
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc5
mkdir -p $OUT
sha256sum cudavolumerenderer_amd/libcvr.so > $OUT/libcvr.sha256
B="python3 bench.py --no-cpu-baseline --scene cloud --serial --steps 2 --warmup 1"
run() { local n=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$n -o run --output-format csv -- $B > $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$n.log; exit 1; }; }
run pmc_a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run pmc_b SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_TA_BUSY
run pmc_c TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
run pmc_d SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_LDS_BANK_CONFLICT
run pmc_f FETCH_SIZE
run pmc_w WRITE_SIZE
python3 tools/pmc_summary.py $OUT/pmc_k_wpool_cloud.json k_wpool $OUT/pmc_a $OUT/pmc_b $OUT/pmc_c $OUT/pmc_d
