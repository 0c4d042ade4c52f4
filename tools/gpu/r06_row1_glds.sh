#!/bin/bash
# The one-pass row kernel's byte staging by LDS-DMA (LCPC_ROW1_GLDS=1) against loads + ds_write
# (prefetch at round 3 in both): the row-kernel / PoS GPU suites with it, then four interleaved
# pairs of the cfg5 line (4 in flight, K = 64)
set -o pipefail
O=gpurun_out/${1:-r06_row1_glds}
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
LCPC_ROW1_GLDS=1 $T 400 python -u -m pytest tests/test_gpu_ntt_row1.py tests/test_gpu_pos.py tests/test_gpu_fullsize.py tests/test_c_client.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3 4; do
  for g in 1 0; do
    LCPC_ROW1_GLDS=$g $T 300 python bench.py --code pos --steps 64 --warmup 8 --cpu-baseline off > $O/pos_g${g}_$rep.json 2> $O/pos_g${g}_$rep.err || { tail -20 $O/pos_g${g}_$rep.err; exit 1; }
    echo "g=$g rep=$rep done"
  done
done
echo done
