#!/bin/bash
# round 4: effective GPU clock per kernel (GRBM_GUI_ACTIVE cycles / kernel duration) on the cfg5
# request, after the one-pass row kernel and after the four-step pair: is the leaf kernel's
# 0.81 vs 1.02 ms difference a clock (power) effect?
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
for m in 1 0; do
  LCPC_NTT_ROW1=$m timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/clk_m$m -o run --output-format csv -- \
    python3 bench.py --code pos --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 > /dev/null 2> $O/clk_m$m.err || exit 1
done
