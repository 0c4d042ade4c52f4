#!/bin/bash
# where the K = 20 line goes after the carry-free mads: the bench timeline under a kernel trace
set -o pipefail
O=gpurun_out/${1:-r06o}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0 --timeline $O/tl.json > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 tools/timeline_k20.py $O/tl.json --trace $(ls $O/trace/*kernel_trace.csv | head -1) --json $O/tl_analysis.json > $O/tl_analysis.txt 2>&1 || { cat $O/tl_analysis.txt; exit 1; }
cat $O/tl_analysis.txt
echo done
