#!/bin/bash
# Round 5: lcpc_sharded_reserve now also pins the proofs' host blocks; the sharded tests, then
# the one-rank sharded K = 20 line three times with its host phases
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_native.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_shard.log 2>&1
rc=$?; tail -3 $O/pytest_shard.log; [ $rc -eq 0 ] || exit $rc
for r in a b c; do
  rm -f $O/phases_$r.csv
  LCPC_PROF_TIMELINE=$O/phases_$r.csv LCPC_PROF_HOST_ONLY=1 timeout -k 10 200 python bench.py --mode sharded --gpus 1 --steps 20 --warmup 5 \
    --prof-timed --cpu-baseline off --verify-reps 0 > $O/sh_$r.json 2> $O/sh_$r.err || { tail -20 $O/sh_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/sh_$r.json').read().strip().splitlines()[-1]);print('$r', round(d['value']/1e9,3), d['ms_per_step'])"
done
for r in a b; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/k20_$r.json 2> $O/k20_$r.err || { tail -20 $O/k20_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/k20_$r.json').read().strip().splitlines()[-1]);print('k20 $r', round(d['value']/1e9,3), 'sharded_n1', round(d['sharded_n1']['value']/1e9,3), d['parity_ok'])"
done
echo done
