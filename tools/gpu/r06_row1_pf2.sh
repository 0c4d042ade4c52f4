#!/bin/bash
# Second round of the prefetch A/B: five interleaved pairs (prefetch first), 4 in flight, K = 64
set -o pipefail
O=gpurun_out/${1:-r06_row1_pf2}
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for rep in 1 2 3 4 5; do
  for pf in 1 0; do
    LCPC_ROW1_PREFETCH=$pf $T 300 python bench.py --code pos --steps 64 --warmup 8 --cpu-baseline off > $O/pos_pf${pf}_$rep.json 2> $O/pos_pf${pf}_$rep.err || { tail -20 $O/pos_pf${pf}_$rep.err; exit 1; }
    echo "pf=$pf rep=$rep done"
  done
done
echo done
