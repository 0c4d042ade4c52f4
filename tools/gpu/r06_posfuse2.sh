#!/bin/bash
# the fused evaluation with fe_dot groups: the fused-request tests, then fused vs separate (64 steps,
# three interleaved rounds) and one request's serial latency each way
set -o pipefail
O=gpurun_out/${1:-r06w}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pos.py -k "fused" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
  for m in fused separate; do
    timeout -k 10 300 python bench.py --code pos --pos-eval $m --steps 64 --warmup 8 --cpu-baseline off > $O/pos_${m}_${rep}.json 2> $O/pos_${m}_${rep}.err || { tail -20 $O/pos_${m}_${rep}.err; exit 1; }
  done
done
for m in fused separate; do
  timeout -k 10 300 python bench.py --code pos --pos-eval $m --steps 16 --warmup 4 --pipeline 1 --cpu-baseline off > $O/pos_${m}_serial.json 2> $O/pos_${m}_serial.err || { tail -20 $O/pos_${m}_serial.err; exit 1; }
done
echo done
