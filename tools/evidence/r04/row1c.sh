#!/bin/bash
# round 4: row-kernel modes 1 / 3 against the four-step pair, interleaved, on the cfg5 request
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt_row1.py -x -q --timeout 120 --timeout-method thread > $O/pytest_row1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_default_a.json 2> $O/pos_default_a.err && \
LCPC_NTT_ROW1=0 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_fourstep_a.json 2> $O/pos_fourstep_a.err && \
LCPC_NTT_ROW1=3 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_direct_a.json 2> $O/pos_direct_a.err && \
timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_default_b.json 2> $O/pos_default_b.err && \
LCPC_NTT_ROW1=0 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_fourstep_b.json 2> $O/pos_fourstep_b.err && \
LCPC_NTT_ROW1=3 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_direct_b.json 2> $O/pos_direct_b.err && \
timeout -k 10 300 python -u bench.py --code pos --steps 64 > $O/pos_default_k64.json 2> $O/pos_default_k64.err && \
LCPC_NTT_ROW1=0 timeout -k 10 300 python -u bench.py --code pos --steps 64 > $O/pos_fourstep_k64.json 2> $O/pos_fourstep_k64.err
