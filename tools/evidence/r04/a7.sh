#!/bin/bash
# round 4: the file image through the four-step pair with the unpack in pass A (LCPC_NTT_ROW1=4)
# against the one-pass row kernel (the default) and the round-3 path, interleaved; then the
# per-kernel effective clocks
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt_row1.py -x -q --timeout 120 --timeout-method thread > $O/pytest_row1.log 2>&1 && \
for r in a b; do
  for m in 4 1 0; do
    LCPC_NTT_ROW1=$m timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_m${m}_$r.json 2> $O/pos_m${m}_$r.err || exit 1
  done
done && \
./tools/evidence/r04/clock_pmc.sh
