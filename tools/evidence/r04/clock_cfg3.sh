#!/bin/bash
# round 4: effective GPU clock per kernel on cfg3 (serial steps, and the pipelined K = 20 region)
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/clk_serial -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 --sharded-n1 0 > /dev/null 2> $O/clk_serial.err && \
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/clk_k20 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --no-prof --verify-reps 0 --sharded-n1 0 > $O/clk_k20.json 2> $O/clk_k20.err
