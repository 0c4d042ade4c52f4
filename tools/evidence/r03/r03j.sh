#!/bin/bash
# Brakedown / Ft191 row shards (native shard tests, SDIG, PoS shards), then the RCCL multi-rank
# path with ranks on the one GPU (tools/rccl_same_gpu.py: per-rank NCCL_HOSTID, loopback sockets)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03j}; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_shard_native.py tests/test_gpu_sdig.py tests/test_gpu_pos_shard.py -m "gpu and not slow" -k "not rccl_one_gpu" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_shard.log 2>&1
tail -1 $OUT/pytest_shard.log
$T 150 python tools/rccl_same_gpu.py --world 2 --job rank --case ft127 --timeout 120 > $OUT/rccl_w2_ft127.log 2>&1
cat $OUT/rccl_w2_ft127.log | grep rank
$T 150 python tools/rccl_same_gpu.py --world 2 --job many --case ft127 --timeout 120 > $OUT/rccl_w2_many.log 2>&1
$T 150 python tools/rccl_same_gpu.py --world 2 --job rank --case sdig_ft127 --root 1 --timeout 120 > $OUT/rccl_w2_sdig.log 2>&1
$T 150 python tools/rccl_same_gpu.py --world 4 --job rank --case ft127_ragged --root 3 --timeout 120 > $OUT/rccl_w4_ragged.log 2>&1
echo ok
