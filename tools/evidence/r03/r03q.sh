#!/bin/bash
# leaf merge (single pass <= 16 chunks, 64-thread blocks) + PoS whole-row buffer: parity subset, PoS/cfg3 lines
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03q; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pos.py tests/test_gpu_shard_native.py tests/test_gpu_sdig.py -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
B="python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off"
$T 300 $B --pipeline 1 > $OUT/pos_p1.json 2>> $OUT/b.err
$T 300 $B --pipeline 2 > $OUT/pos_p2.json 2>> $OUT/b.err
$T 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20.json 2>> $OUT/b.err
echo ok
