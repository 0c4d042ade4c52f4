#!/bin/bash
# Round 5: runtime allocations (hipMalloc / hipHostMalloc / stream creation) inside the timed
# regions of the cfg4 and cfg5 lines, from the library's host-phase timeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
rm -f $O/ph_sdig.csv $O/ph_pos.csv
LCPC_PROF_TIMELINE=$O/ph_sdig.csv LCPC_PROF_HOST_ONLY=1 timeout -k 10 300 python bench.py --code sdig --steps 20 --warmup 5 --prof-timed --timeline $O/tl_sdig.json --cpu-baseline off --verify-reps 0 > $O/sdig.json 2> $O/sdig.err || { tail -20 $O/sdig.err; exit 1; }
LCPC_PROF_TIMELINE=$O/ph_pos.csv LCPC_PROF_HOST_ONLY=1 timeout -k 10 300 python bench.py --code pos --steps 16 --warmup 4 --prof-timed --cpu-baseline off > $O/pos.json 2> $O/pos.err || { tail -20 $O/pos.err; exit 1; }
echo done
