#!/bin/bash
# Packed-destination transpose (k_transpose_packed) against the 32 x 32 tiles
# (LCPC_TRANSPOSE_TILED=1): the Brakedown transpose's time from rocprofv3 kernel traces of
# bench.py --code sdig, alternating, then the GPU tests that run it (SDIG, full size, commit paths).
# The packed kernel was not kept (within noise of the tiles); LCPC_TRANSPOSE_TILED is no
# longer read, so the script now records how the A/B was made.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-trp}; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -k "sdig or brakedown or fullsize or commit or shard" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
i=0
for tiled in 0 1 0 1; do
  i=$((i+1)); D=$OUT/prof_${i}_tiled$tiled
  LCPC_TRANSPOSE_TILED=$tiled $T 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- \
    python3 bench.py --code sdig --steps 8 --warmup 4 --cpu-baseline off --verify-reps 0 --sharded-n1 0 > $D.json 2> $D.err
  echo "tiled=$tiled"; python3 tools/sdig_levels.py $(find $D -name "*kernel_trace.csv" | head -1) | grep -E "transpose|total"
done
