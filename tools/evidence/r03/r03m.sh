#!/bin/bash
set -e
bash tools/r03_final.sh r03fin
export TMPDIR=/tmp
OUT=gpurun_out/r03pos; mkdir -p $OUT
T="timeout -k 10"
B="python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off"
$T 300 $B --pipeline 1 > $OUT/p1.json 2>> $OUT/b.err
$T 300 $B --pipeline 2 > $OUT/p2.json 2>> $OUT/b.err
$T 300 $B --pipeline 4 --commit-slots 1 > $OUT/p4_cs1.json 2>> $OUT/b.err
$T 300 $B --pipeline 4 --commit-slots 2 > $OUT/p4_cs2.json 2>> $OUT/b.err
$T 300 $B --pipeline 8 --commit-slots 2 > $OUT/p8_cs2.json 2>> $OUT/b.err
$T 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --code pos --steps 8 --warmup 2 --cpu-baseline off --no-prof > $OUT/under_prof.json 2>> $OUT/b.err
echo ok
