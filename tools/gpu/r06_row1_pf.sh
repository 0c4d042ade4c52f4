#!/bin/bash
# The one-pass PoS row kernel with and without the L2 prefetch of the row 256 ahead
# (LCPC_ROW1_PREFETCH): the row-kernel and PoS GPU suites with it on, then interleaved PoS lines
# (4 in flight, K = 64) and one-at-a-time lines (the kernel's own duration).
set -o pipefail
O=gpurun_out/${1:-r06_row1_pf}
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
LCPC_ROW1_PREFETCH=1 $T 400 python -u -m pytest tests/test_gpu_ntt_row1.py tests/test_gpu_pos.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
  for pf in 0 1; do
    LCPC_ROW1_PREFETCH=$pf $T 300 python bench.py --code pos --steps 64 --warmup 8 --cpu-baseline off > $O/pos_pf${pf}_$rep.json 2> $O/pos_pf${pf}_$rep.err || { tail -20 $O/pos_pf${pf}_$rep.err; exit 1; }
    echo "pf=$pf rep=$rep done"
  done
done
for pf in 0 1; do
  LCPC_ROW1_PREFETCH=$pf $T 300 python bench.py --code pos --steps 16 --warmup 4 --pipeline 1 --cpu-baseline off > $O/pos_pf${pf}_serial.json 2> $O/pos_pf${pf}_serial.err || { tail -20 $O/pos_pf${pf}_serial.err; exit 1; }
done
echo done
