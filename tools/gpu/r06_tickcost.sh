#!/bin/bash
# per-tick host phases of the weak-scaled sharded line with 2 and 4 ranks sharing the GPU over
# RCCL (the library's real ncclGroup path; loopback sockets, so only the host phases mean anything)
set -o pipefail
O=gpurun_out/${1:-r06r}
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4; do
  LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1 timeout -k 10 400 \
    python bench.py --gpus $n --steps 6 --warmup 2 --log-len 22 --prof-timed --cpu-baseline off --verify-reps 0 > $O/tick_${n}r.json 2> $O/tick_${n}r.err || { tail -30 $O/tick_${n}r.err; exit 1; }
done
echo done
