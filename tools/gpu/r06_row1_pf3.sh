#!/bin/bash
# Where the one-pass kernel issues its L2 prefetch: round 3's start (1), round 2's start (2), the
# output phase's start (3); three interleaved rounds, 4 in flight, K = 64, plus a short parity check
set -o pipefail
O=gpurun_out/${1:-r06_row1_pf3}
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for m in 2 3; do
  LCPC_ROW1_PREFETCH=$m $T 300 python -u -m pytest tests/test_gpu_ntt_row1.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$m.log 2>&1 || { tail -30 $O/pytest_$m.log; exit 1; }
done
for rep in 1 2 3; do
  for m in 1 2 3; do
    LCPC_ROW1_PREFETCH=$m $T 300 python bench.py --code pos --steps 64 --warmup 8 --cpu-baseline off > $O/pos_m${m}_$rep.json 2> $O/pos_m${m}_$rep.err || { tail -20 $O/pos_m${m}_$rep.err; exit 1; }
    echo "m=$m rep=$rep done"
  done
done
echo done
