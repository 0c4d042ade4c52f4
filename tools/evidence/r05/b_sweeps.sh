#!/bin/bash
# Round 5, second box: the cfg2 shape sweep (nttbench 2), the Brakedown encode's per-level HBM
# counters (two PMC passes + a kernel trace of the same sdig-encode command), and the cfg5
# eight-rank RCCL rehearsal on one GPU (plumbing rate; parity against the oracle).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 120 ./tools/microbench/nttbench 2 > $O/nttbench_cfg2.txt 2>&1 || { tail $O/nttbench_cfg2.txt; exit 1; }
cat $O/nttbench_cfg2.txt
A="--code sdig-encode --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof"
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo "$c" | cut -d_ -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 90 rocprofv3 --pmc "$c" -d $O/sdig/pmc_$n -o run --output-format csv -- python3 bench.py $A > /dev/null 2> $O/sdig_pmc_$n.err || { tail -20 $O/sdig_pmc_$n.err; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/sdig/kt -o run --output-format csv -- python3 bench.py $A > /dev/null 2> $O/sdig_kt.err || { tail -20 $O/sdig_kt.err; exit 1; }
LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1 timeout -k 10 500 python bench.py --code pos --mode sharded --gpus 8 --steps 2 --warmup 1 > $O/bench_pos_sharded_8ranks_rccl_one_gpu.json 2> $O/bench_pos8.err || { tail -30 $O/bench_pos8.err; exit 1; }
tail -c 1500 $O/bench_pos_sharded_8ranks_rccl_one_gpu.json
echo done
