#!/bin/bash
# Round 5: one-wave collapse blocks (4.3 KiB LDS, co-resident with four encode blocks per CU)
# against the four-wave default; parity first, then K = 20 alternating, and a timeline of each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
LCPC_COLLAPSE_WAVES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_collapse.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_w1.log 2>&1
rc=$?; tail -3 $O/pytest_w1.log; [ $rc -eq 0 ] || exit $rc
common="--gpus 1 --steps 20 --warmup 5 --cpu-baseline off --sharded-n1 0 --verify-reps 0"
for rep in 1 2 3 4; do
  for w in 4 1; do
    LCPC_COLLAPSE_WAVES=$w timeout -k 10 200 python bench.py $common > $O/k20_w${w}_$rep.json 2> $O/k20_w${w}_$rep.err || { tail -20 $O/k20_w${w}_$rep.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/k20_w${w}_$rep.json').read().strip().splitlines()[-1]);print('waves $w rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],4), d['kernels']['collapse_partial']['avg_ms'])"
  done
done
for w in 4 1; do
  LCPC_COLLAPSE_WAVES=$w timeout -k 10 200 python bench.py $common --timeline $O/tl_w$w.json > $O/k20_w${w}_tl.json 2> $O/k20_w${w}_tl.err || { tail -20 $O/k20_w${w}_tl.err; exit 1; }
done
echo done
