#!/bin/bash
# the encode's cycle model after the carry-free mads: its SQ / GRBM counters (tools/pmc_ntt.sh),
# a kernel trace of the cfg3-size encode, and the default K = 256 line (GPU-throughput bound)
set -o pipefail
O=gpurun_out/${1:-r06k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/femul2 > $O/femul2.txt 2>&1 || { cat $O/femul2.txt; exit 1; }
bash tools/pmc_ntt.sh ${1:-r06k}/pmc --code encode --log-len 24 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --code encode --log-len 24 --steps 20 --warmup 5 --cpu-baseline off > $O/trace_bench.json 2> $O/trace_bench.err || { tail $O/trace_bench.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --code encode > $O/bench_encode.json 2> $O/bench_encode.err || { tail -20 $O/bench_encode.err; exit 1; }
echo done
