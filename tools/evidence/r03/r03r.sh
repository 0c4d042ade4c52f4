#!/bin/bash
# the RCCL exchanges with 8 ranks on one GPU (per-rank NCCL_HOSTID): cfg3 (2^24 Ft127, 512 rows:
# 9 leaf chunks over 8 ranks) commit + prove against the single-GPU commitment and the oracle,
# then the pipelined driver over 8 ranks on 2^22 polynomials (256 rows, 5 chunks)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03r; mkdir -p $OUT
timeout -k 10 300 python -u tools/rccl_same_gpu.py --world 8 --job rank --fid 1 --n 16777216 --timeout 280 > $OUT/rccl_8ranks_cfg3.log 2>&1
cat $OUT/rccl_8ranks_cfg3.log
timeout -k 10 300 python -u tools/rccl_same_gpu.py --world 8 --job many --fid 1 --n 4194304 --timeout 280 > $OUT/rccl_8ranks_many.log 2>&1
cat $OUT/rccl_8ranks_many.log
echo ok
