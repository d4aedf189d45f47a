# Where k_wpool's memory-side writes come from: WRITE_SIZE with and without the framebuffer atomics
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sc in manix hetvol; do
  for L in default nosplat; do
    if [ $L = default ]; then LA=""; else LA="--lib build/variants/$L/libcvr.so"; fi
    timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/wr_${sc}_$L -o run --output-format csv -- python3 tools/tune.py $LA --scene $sc --rounds 2 --variants "regenerationSK:" > gpurun_out/wr_${sc}_$L.log 2>&1
    python3 - <<PY
import csv
v={}
for r in csv.DictReader(open("gpurun_out/wr_${sc}_$L/run_counter_collection.csv")):
    if "k_wpool" in r["Kernel_Name"] and r["Counter_Name"]=="WRITE_SIZE":
        v[r["Dispatch_Id"]]=v.get(r["Dispatch_Id"],0.0)+float(r["Counter_Value"])
x=[v[k] for k in sorted(v,key=int)][1:]
print("$sc $L WRITE_SIZE GB per launch", round(sum(x)/len(x)*1024/1e9,3), len(x))
PY
  done
done
bash tools/job_ab2.sh 4 '"regenerationSK:" "regenerationSK:shard=8"' default major km32 default major km32
