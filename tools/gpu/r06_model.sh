#!/bin/bash
# the encode's cycle model: per-class issue costs (issue_cost v3) and the cfg3 encode's own SQ /
# GRBM counters (tools/pmc_ntt.sh, one rocprofv3 pass per group), plus a kernel trace of it
set -o pipefail
O=gpurun_out/${1:-r06d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 150 ./tools/microbench/issue_cost $O/issue_cost.json > $O/issue_cost.txt 2>&1 || { tail $O/issue_cost.txt; exit 1; }
bash tools/pmc_ntt.sh ${1:-r06d}/pmc --code encode --log-len 24 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --code encode --log-len 24 --steps 20 --warmup 5 --cpu-baseline off > $O/trace_bench.json 2> $O/trace_bench.err || { tail $O/trace_bench.err; exit 1; }
echo done
