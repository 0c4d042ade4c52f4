#!/bin/bash
# Round 5, final tree: the driver's multi-GPU command form (torch.distributed.run, one rank per
# "GPU") rehearsed with 2, 4 and 8 ranks sharing the box's one GPU over RCCL (plumbing and parity,
# not rates), then the encode-only lines with their new steady-state roofline fields.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
port=29511
# the ranks share GPU 0 (LCPC_BENCH_SHARE_GPU), the launcher's group is gloo, and the library's
# exchanges run over RCCL with a distinct host id per rank (LCPC_BENCH_RCCL_SAME_GPU)
export LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1
for n in 2 4 8; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_torchrun_${n}ranks.json 2> $O/bench_torchrun_${n}ranks.err \
    || { tail -30 $O/bench_torchrun_${n}ranks.err; exit 1; }
  port=$((port + 1))
  tail -c 600 $O/bench_torchrun_${n}ranks.json
done
unset LCPC_BENCH_BACKEND LCPC_BENCH_SHARE_GPU LCPC_BENCH_RCCL_SAME_GPU
timeout -k 10 300 python bench.py --code encode --steps 512 --warmup 16 > $O/bench_encode.json 2> $O/bench_encode.err || { tail -20 $O/bench_encode.err; exit 1; }
timeout -k 10 300 python bench.py --code sdig-encode --steps 64 --warmup 8 > $O/bench_sdig_encode.json 2> $O/bench_sdig_encode.err || { tail -20 $O/bench_sdig_encode.err; exit 1; }
echo done
