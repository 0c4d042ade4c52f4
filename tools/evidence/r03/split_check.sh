set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shard_native.py tests/test_gpu_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/split/pytest.log 2>&1
tail -2 gpurun_out/split/pytest.log
LCPC_PROF_HOST_ONLY=1 LCPC_PROF_TIMELINE=$PWD/gpurun_out/split/host_tl.csv timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --prof-timed > gpurun_out/split/tl.json 2> gpurun_out/split/tl.err
for lag in 3 4 5 3 4 5; do
  timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --lag $lag >> gpurun_out/split/lag$lag.json 2>> gpurun_out/split/lag.err
  echo lag $lag done
done
