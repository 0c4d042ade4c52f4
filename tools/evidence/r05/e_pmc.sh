#!/bin/bash
# Round 5: HBM counters (FETCH_SIZE, WRITE_SIZE; separate passes, serial steps) for every bench
# workload on the final kernels, then the driver's K = 20 line under a kernel trace + stats pass.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
C="--steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 --sharded-n1 0"
for w in "ligero:" "encode:--code encode" "sdig_encode:--code sdig-encode" "sdig:--code sdig" "pos:--code pos"; do
  tag=${w%%:*}; args=${w#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    n=$(echo "$c" | cut -d_ -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc "$c" -d $O/$tag/pmc_$n -o run --output-format csv -- python3 bench.py $args $C > /dev/null 2> $O/${tag}_pmc_$n.err || { echo "pmc $tag $c failed"; tail -20 $O/${tag}_pmc_$n.err; exit 1; }
  done
  echo "pmc $tag ok"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k20_kt -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20_under_prof.json 2> $O/k20_kt.err || { tail -20 $O/k20_kt.err; exit 1; }
echo done
