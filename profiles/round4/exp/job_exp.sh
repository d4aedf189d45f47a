# Round-4 experiments: C5 LDS brick-word cache (wc64/wc256) and non-temporal cell/albedo loads (nt1/2/3)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/exp
mkdir -p $O
cp cudavolumerenderer_amd/libcvr.so $O/libcvr_default.so
AB_ARGS="--res 4096" bash tools/ab.sh cloud 1 default wc64 wc256 default wc64 wc256 > $O/wcache_ab.log 2>&1; cat $O/wcache_ab.log
bash tools/ab.sh hetvol 2 default nt1 nt2 nt3 default nt1 nt2 nt3 > $O/nt_ab_hetvol.log 2>&1; cat $O/nt_ab_hetvol.log
bash tools/ab.sh manix 2 default nt1 nt3 default nt1 nt3 > $O/nt_ab_manix.log 2>&1; cat $O/nt_ab_manix.log
pmc() {  # variant scene tag counters...
  v=$1; sc=$2; tag=$3; shift 3
  if [ $v = default ]; then cp $O/libcvr_default.so cudavolumerenderer_amd/libcvr.so; else cp build/variants/$v/libcvr.so cudavolumerenderer_amd/libcvr.so; fi
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace -d $O/pmc_${sc}_${v}_$tag -o run --output-format csv -- python3 bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline --no-shard-emulation > $O/pmc_${sc}_${v}_$tag.log 2>&1
  echo "pmc $v $sc $tag done"
}
for v in default nt1 nt3; do pmc $v hetvol w WRITE_SIZE; pmc $v hetvol f FETCH_SIZE; done
for v in default wc64; do
  pmc $v cloud sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS
  pmc $v cloud c TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
  pmc $v cloud f FETCH_SIZE
done
cp $O/libcvr_default.so cudavolumerenderer_amd/libcvr.so
