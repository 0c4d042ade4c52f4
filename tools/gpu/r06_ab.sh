#!/bin/bash
# round 6 A/B: the pageable host-input path (staged through page-locked slots vs the runtime's own
# pageable copy), alternating; and the issue-cost microbench with the select variants.
set -o pipefail
O=gpurun_out/${1:-r06c}
mkdir -p $O
T="timeout -k 10"
$T 120 ./tools/microbench/issue_cost $O/issue_cost.json > $O/issue_cost.txt 2>&1 || { tail $O/issue_cost.txt; exit 1; }
B="python bench.py --steps 20 --warmup 5 --sharded-n1 0 --cpu-baseline off --verify-reps 0"
for rep in 1 2; do
  for mode in staged direct; do
    LCPC_H2D_PAGEABLE=$mode $T 300 $B --input host > $O/host_${mode}_$rep.json 2> $O/host_${mode}_$rep.err || { tail $O/host_${mode}_$rep.err; exit 1; }
    LCPC_H2D_PAGEABLE=$mode $T 300 python bench.py --code pos --steps 8 --warmup 2 --input host --cpu-baseline off > $O/pos_host_${mode}_$rep.json 2> $O/pos_host_${mode}_$rep.err || { tail $O/pos_host_${mode}_$rep.err; exit 1; }
  done
done
echo done
