#!/bin/bash
# round 4: the self-checking N > 1 lines rehearsed on one GPU (review item 1's "done" criterion):
# the row-sharded cfg3 line with 2, 4 and 8 ranks whose exchanges go through RCCL (per-rank
# NCCL_HOSTID, loopback sockets), and the sharded PoS request with 2 ranks -- plumbing rates, but
# every line carries the oracle parity keys and cpu_baseline
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
export LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1
for n in 2 4 8; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 4 --warmup 1 > $O/sharded_rccl_${n}ranks.json 2> $O/sharded_rccl_${n}ranks.err || exit 1
done
LCPC_BENCH_RCCL_SAME_GPU=0 timeout -k 10 400 python -u bench.py --gpus 2 --code pos --mode sharded --steps 2 --warmup 1 --pos-bytes $((1<<26)) > $O/pos_sharded_2ranks.json 2> $O/pos_sharded_2ranks.err
