#!/bin/bash
# Round 5: where a cfg5 request's 5 ms goes -- a kernel trace of the PoS line (K = 16, 4 in flight)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off > $O/bench_pos.json 2> $O/bench_pos.err || { tail -20 $O/bench_pos.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/pos_kt -o run --output-format csv -- python3 bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off --no-prof > $O/bench_pos_prof.json 2> $O/pos_kt.err || { tail -20 $O/pos_kt.err; exit 1; }
echo done
