#!/bin/bash
# round 4: the pipelined sharded driver with two encode streams (LCPC_SHARD_BULK_STREAMS=2) --
# its pipelined-driver parity tests, then the one-rank K = 20 line against one stream, interleaved
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
LCPC_SHARD_BULK_STREAMS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_native.py -x -q -k "pipeline or many" --timeout 300 --timeout-method thread > $O/pytest_pipeline_bulk2.log 2>&1 && \
for r in a b; do
  for n in 1 2; do
    LCPC_SHARD_BULK_STREAMS=$n timeout -k 10 300 python -u bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $O/sharded_n1_bulk${n}_$r.json 2> $O/sharded_n1_bulk${n}_$r.err || exit 1
  done
done
