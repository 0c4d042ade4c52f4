#!/bin/bash
# round 4: the persistent, prefetching row kernel (LCPC_NTT_ROW1=2): parity, the cfg5 line in each
# mode, then issue counters of modes 1 and 2; two K = 20 lines for the run-to-run spread
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt_row1.py -x -v --timeout 120 --timeout-method thread > $O/pytest_row1.log 2>&1 && \
LCPC_NTT_ROW1=2 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_row2_bytes.json 2> $O/pos_row2_bytes.err && \
LCPC_NTT_ROW1=1 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_row1_bytes.json 2> $O/pos_row1_bytes.err && \
LCPC_NTT_ROW1=2 timeout -k 10 300 python -u bench.py --code pos --steps 16 --pos-commit elements > $O/pos_row2_elems.json 2> $O/pos_row2_elems.err && \
LCPC_NTT_ROW1=0 timeout -k 10 300 python -u bench.py --code pos --steps 16 --pos-commit elements > $O/pos_fourstep.json 2> $O/pos_fourstep.err && \
LCPC_NTT_ROW1=2 bash tools/pmc_ntt.sh r04i/pmc_row2 --code pos > $O/pmc_row2.log 2>&1 && \
LCPC_NTT_ROW1=1 bash tools/pmc_ntt.sh r04i/pmc_row1 --code pos > $O/pmc_row1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sharded-n1 0 > $O/k20_a.json 2> $O/k20_a.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sharded-n1 0 > $O/k20_b.json 2> $O/k20_b.err && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --field Ft255 --rho 1/4 --sharded-n1 0 > $O/ft255_rho14.json 2> $O/ft255_rho14.err
