#!/bin/bash
# A/B of the Brakedown SpMM prefetch depth (LCPC_SDIG_PF=1: one 4-nonzero group in flight while
# one is multiplied; 2: two, three register sets in rotation): per-level times from a rocprofv3
# kernel trace of bench.py --code sdig, and the cfg4 parity tests under the depth-2 kernel.
# The depth-2 kernel was measured slower and removed after this run; LCPC_SDIG_PF is no
# longer read, so the script now records how the A/B was made.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-spmm_pf}; mkdir -p $OUT
T="timeout -k 10"
i=0
for pf in 1 2 1 2; do
  i=$((i+1)); D=$OUT/prof_${i}_pf$pf
  LCPC_SDIG_PF=$pf $T 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- \
    python3 bench.py --code sdig --steps 8 --warmup 4 --cpu-baseline off --verify-reps 0 > $D.json 2> $D.err
  echo "pf=$pf"; python3 tools/sdig_levels.py $(find $D -name "*kernel_trace.csv" | head -1) | grep -E "pre0|post0|total"
done
LCPC_SDIG_PF=2 $T 400 python -u -m pytest tests -m gpu -k "sdig or brakedown or fullsize" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_pf2.log 2>&1
tail -1 $OUT/pytest_pf2.log
