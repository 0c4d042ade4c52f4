#!/bin/bash
# steady state of both engines on one GPU: K = 160 (the weak-scaled N = 8 line's commitment count)
set -o pipefail
O=gpurun_out/${1:-r06p}
mkdir -p $O
export TMPDIR=/tmp
for m in sharded replicas; do
  timeout -k 10 400 python bench.py --mode $m --steps 160 --warmup 10 --cpu-baseline off --verify-reps 0 --sharded-n1 0 --prof-timed > $O/bench_$m.json 2> $O/bench_$m.err || { tail -20 $O/bench_$m.err; exit 1; }
done
echo done
