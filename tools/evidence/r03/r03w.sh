#!/bin/bash
# 8-rank pipelined root mismatch: RCCL vs host-staged collectives vs RCCL with every tick drained
# (checks, not faults: a failing run does not stop the next; a timeout / abort / crash ends it)
export TMPDIR=/tmp
OUT=gpurun_out/r03w; mkdir -p $OUT
T="timeout -k 10 200 python -u tools/rccl_same_gpu.py --world 8 --job many --fid 1 --n 4194304 --polys 9 --lag 0 --timeout 180"
run() {  # name, extra args, env
  for i in 1 2 3 4 5 6; do
    env $3 $T $2 > $OUT/$1_$i.log 2>&1
    rc=$?
    echo "$1 run $i rc=$rc $(grep -o 'bad_root_polys[^]]*]' $OUT/$1_$i.log | sort | uniq -c | tr '\n' ' ')"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo stopping; exit $rc; fi
  done
}
run rccl "" "X=1"
run host "--host" "X=1"
run rccl_sync "" "LCPC_SHARD_SYNC_TICKS=1"
echo ok
