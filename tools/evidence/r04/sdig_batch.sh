#!/bin/bash
# round 4: the Brakedown encode alone (bench.py --code sdig-encode), one / two / four commitments'
# rows per call, at the default 8-tile cap and with 9 tiles per wave (two commitments in one wave)
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
B="python -u bench.py --code sdig-encode --verify-reps 0"
timeout -k 10 200 $B --batch 1 --steps 24 --warmup 4 > $O/b1.json 2> $O/b1.err && \
timeout -k 10 200 $B --batch 2 --steps 12 --warmup 2 --cpu-baseline off > $O/b2.json 2> $O/b2.err && \
LCPC_SDIG_TILES=9 timeout -k 10 200 $B --batch 2 --steps 12 --warmup 2 --cpu-baseline off > $O/b2_t9.json 2> $O/b2_t9.err && \
timeout -k 10 200 $B --batch 4 --steps 6 --warmup 2 --cpu-baseline off > $O/b4.json 2> $O/b4.err && \
LCPC_SDIG_TILES=9 timeout -k 10 200 $B --batch 4 --steps 6 --warmup 2 --cpu-baseline off > $O/b4_t9.json 2> $O/b4_t9.err
