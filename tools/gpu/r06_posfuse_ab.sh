#!/bin/bash
# fused vs separate u^T Enc(M) in the 1 GiB PoS request line, 64 steps, three interleaved rounds
set -o pipefail
O=gpurun_out/${1:-r06v}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for m in fused separate; do
    timeout -k 10 300 python bench.py --code pos --pos-eval $m --steps 64 --warmup 8 --cpu-baseline off > $O/pos_${m}_${rep}.json 2> $O/pos_${m}_${rep}.err || { tail -20 $O/pos_${m}_${rep}.err; exit 1; }
  done
done
echo done
