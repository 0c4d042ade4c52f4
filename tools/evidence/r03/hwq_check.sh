set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hwq
for q in 4 8 16; do
  for lag in 5 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --lag $lag >> gpurun_out/hwq/q${q}_lag$lag.json 2>> gpurun_out/hwq/err.log
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --lag $lag >> gpurun_out/hwq/q${q}_lag$lag.json 2>> gpurun_out/hwq/err.log
    echo q $q lag $lag done
  done
done
