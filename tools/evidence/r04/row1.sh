#!/bin/bash
# round 4: the one-pass Ft63 row kernel -- parity first, then the cfg5 line with it and with the
# four-step pair (LCPC_NTT_ROW1=0), then its kernel trace + PMC traffic, then the round's suite
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt_row1.py -x -v --timeout 120 --timeout-method thread > $O/pytest_row1.log 2>&1 && \
LCPC_NTT_ROW1=1 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_row1.json 2> $O/pos_row1.err && \
LCPC_NTT_ROW1=0 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_fourstep.json 2> $O/pos_fourstep.err && \
LCPC_NTT_ROW1=1 bash tools/prof_workload.sh r04g/prof_pos_row1 16 --code pos > $O/prof_pos_row1.log 2>&1 && \
./tools/evidence/r04/suite.sh
