set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lag
LCPC_PROF_HOST_ONLY=1 LCPC_PROF_TIMELINE=$PWD/gpurun_out/lag/host_tl.csv timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --prof-timed > gpurun_out/lag/tl.json 2> gpurun_out/lag/tl.err
for lag in 2 3 4 2 3 4; do
  timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --lag $lag >> gpurun_out/lag/lag$lag.json 2>> gpurun_out/lag/lag.err
  echo lag $lag done
done
