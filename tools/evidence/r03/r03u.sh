#!/bin/bash
# isolate the 8-rank pipelined root mismatch: polynomial count vs schedule lag.  A case that
# fails its checks (rc 1) does not stop the others; a timeout, abort or crash ends the script.
export TMPDIR=/tmp
OUT=gpurun_out/r03u; mkdir -p $OUT
for c in "9 2" "6 0" "9 0" "9 10"; do
  set -- $c
  timeout -k 10 200 python -u tools/rccl_same_gpu.py --world 8 --job many --fid 1 --n 4194304 --polys $1 --lag $2 --timeout 180 > $OUT/p$1_lag$2.log 2>&1
  rc=$?
  echo "polys $1 lag $2 rc=$rc"; grep '^{' $OUT/p$1_lag$2.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping"; exit $rc; fi
done
echo ok
