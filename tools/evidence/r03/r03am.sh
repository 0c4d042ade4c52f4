#!/bin/bash
# the N > 1 bench paths on the final tree, ranks sharing GPU 0 over RCCL (plumbing, not rates):
# cfg3 sharded at 2 and 4 ranks, the PoS request sharded at 2
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03am; mkdir -p $OUT
export LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1
T="timeout -k 10 400"
$T python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_2.json 2> $OUT/b.err
$T python bench.py --gpus 4 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_4.json 2>> $OUT/b.err
$T python bench.py --gpus 2 --code pos --mode sharded --steps 6 --warmup 2 --cpu-baseline off > $OUT/pos_sharded_2.json 2>> $OUT/b.err
for f in sharded_2 sharded_4 pos_sharded_2; do
  python -c "import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);print('$f', d['n_gpus'], d.get('world_formed'), round(d['value']/1e9,3), round(d['ms_per_step'],2), d['config'].get('parallelism','')[:60], d['config'].get('exchanges','')[:40])"
done
echo ok
