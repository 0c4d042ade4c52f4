#!/bin/bash
# per-class issue costs of the BLAKE3 leaf kernel's instruction mix (v_xor / v_alignbit / v_add3
# / v_perm / v_bitop3 beside the encode's classes), and the weak-scaled sharded line rehearsed with
# 2 and 4 ranks sharing the one GPU over RCCL (plumbing: loopback sockets, not a rate)
set -o pipefail
O=gpurun_out/${1:-r06f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 ./tools/microbench/issue_cost $O/issue_cost.json > $O/issue_cost.txt 2>&1 || { tail $O/issue_cost.txt; exit 1; }
timeout -k 10 60 ./tools/microbench/b3rot > $O/b3rot.txt 2>&1 || { cat $O/b3rot.txt; exit 1; }
for n in 2 4; do
  LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1 timeout -k 10 300 \
    python bench.py --gpus $n --steps 4 --warmup 2 --log-len 20 > $O/sharded_weak_${n}r.json 2> $O/sharded_weak_${n}r.err || { tail -30 $O/sharded_weak_${n}r.err; exit 1; }
done
echo done
