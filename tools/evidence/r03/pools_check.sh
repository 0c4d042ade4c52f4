set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pools
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shard_native.py tests/test_gpu_shard.py tests/test_gpu_pos_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pools/pytest.log 2>&1
tail -1 gpurun_out/pools/pytest.log
LCPC_PROF_HOST_ONLY=1 LCPC_PROF_TIMELINE=$PWD/gpurun_out/pools/host_tl.csv timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 --prof-timed > gpurun_out/pools/tl.json 2> gpurun_out/pools/tl.err
for i in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --roofline-steps 1 >> gpurun_out/pools/sh.json 2>> gpurun_out/pools/sh.err
done
echo ok
