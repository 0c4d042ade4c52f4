#!/bin/bash
# where the cfg2 encode line (2^20 Ft127, 16 calls in flight) goes: a kernel trace of the line
set -o pipefail
O=gpurun_out/${1:-r06z}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python3 bench.py --code encode --steps 512 --warmup 32 --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
echo done
