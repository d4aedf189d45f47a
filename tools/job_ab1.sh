set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_job.sh pytest
for sc in manix hetvol; do bash tools/ab.sh $sc 3 r3 default r3 default > gpurun_out/ab1_$sc.log 2>&1; cat gpurun_out/ab1_$sc.log; done
bash tools/ab.sh cloud 1 r3 default r3 default > gpurun_out/ab1_cloud.log 2>&1; cat gpurun_out/ab1_cloud.log
