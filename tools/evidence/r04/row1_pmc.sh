#!/bin/bash
# issue-level PMC counters of the one-pass row kernel (fused file-image commit) and of the
# four-step pair on the same cfg5 request; two K = 20 lines first (run-to-run spread)
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sharded-n1 0 > $O/k20_a.json 2> $O/k20_a.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sharded-n1 0 > $O/k20_b.json 2> $O/k20_b.err && \
LCPC_NTT_ROW1=1 bash tools/pmc_ntt.sh r04h/row1 --code pos > $O/row1.log 2>&1 && \
LCPC_NTT_ROW1=0 bash tools/pmc_ntt.sh r04h/four --code pos --pos-commit elements > $O/four.log 2>&1
