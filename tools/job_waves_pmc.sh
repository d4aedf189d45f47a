# Lane fill vs pool size: VALU instructions and lane cycles at 3 / 4 / 5 waves per SIMD (C2)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/wpmc
mkdir -p $OUT
for w in 5 3 4; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/w$w -o run --output-format csv -- python3 tools/tune.py --rounds 2 --variants "regenerationSK:waves=$w" > $OUT/w$w.log 2>&1 || { echo "w$w failed"; tail -5 $OUT/w$w.log; exit 1; }
  python3 - <<PY
import csv
v={}
for r in csv.DictReader(open("$OUT/w$w/run_counter_collection.csv")):
    if "k_wpool" in r["Kernel_Name"]:
        v.setdefault(r["Counter_Name"],{}); d=v[r["Counter_Name"]]; d[r["Dispatch_Id"]]=d.get(r["Dispatch_Id"],0.0)+float(r["Counter_Value"])
m={k:sum(list(x.values())[1:])/max(1,len(x)-1) for k,x in v.items()}
print("waves $w", "VALU %.3g" % m["SQ_INSTS_VALU"], "lanes %.1f" % (m["SQ_THREAD_CYCLES_VALU"]/m["SQ_INSTS_VALU"]), "wait %.3f" % (m["SQ_WAIT_ANY"]/m["SQ_WAVE_CYCLES"]), "issue %.3f" % (m["SQ_INSTS_VALU"]/1024/(m["GRBM_GUI_ACTIVE"]/8)))
PY
  grep "regen" $OUT/w$w.log | cut -c1-70
done
