#!/bin/bash
# kernel traces of both one-GPU engines at K = 160 (where the sharded driver's 4 % goes)
set -o pipefail
O=gpurun_out/${1:-r06s}
mkdir -p $O
export TMPDIR=/tmp
for m in sharded replicas; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace_$m -o run --output-format csv -- \
    python3 bench.py --mode $m --steps 160 --warmup 10 --cpu-baseline off --verify-reps 0 --sharded-n1 0 > $O/bench_$m.json 2> $O/bench_$m.err || { tail -20 $O/bench_$m.err; exit 1; }
done
echo done
