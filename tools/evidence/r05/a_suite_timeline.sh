#!/bin/bash
# Round 5, first box: the GPU suite on the stream-ordered pool / one-priority tree, the driver's
# K = 20 line with a per-step timeline, the same line under a rocprofv3 kernel trace (GPU busy
# intervals), and the world-8 mixed-priority (mode 2) pipeline test ONCE (review item 1d).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --timeline $O/timeline_k20.json > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0 --timeline $O/timeline_k20_prof.json > $O/bench_k20_prof.json 2> $O/bench_k20_prof.err || { tail -20 $O/bench_k20_prof.err; exit 1; }
LCPC_PRIORITY_STREAMS=1 LCPC_SHARD_PRIO=2 LCPC_SHARD_PRIO_AB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_shard_native.py -m gpu -x -v --timeout 300 --timeout-method thread -k "world8_rccl_one_gpu and pipeline" > $O/world8_mode2_once.log 2>&1
echo "world8 mode2 rc $?"
tail -3 $O/world8_mode2_once.log
echo done
