#!/bin/bash
# replicas K=20: step timelines and a few admission / worker settings
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03h}; mkdir -p $OUT
T="timeout -k 10"
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0"
for i in 1 2; do $T 200 $B --timeline $OUT/tl_$i.json > $OUT/k20_$i.json 2>> $OUT/b.err; done
for cs in 2 3 6; do $T 200 $B --commit-slots $cs > $OUT/k20_cs$cs.json 2>> $OUT/b.err; done
for w in 12 20; do $T 200 $B --workers $w > $OUT/k20_w$w.json 2>> $OUT/b.err; done
$T 200 $B --steps 256 > $OUT/k256.json 2>> $OUT/b.err
echo ok
