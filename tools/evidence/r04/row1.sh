#!/bin/bash
# round 4: the one-pass Ft63 row kernel and the fused file-image commit -- parity first, then the
# cfg5 line three ways (one-pass + fused unpack; one-pass on packed elements; the four-step pair on
# packed elements = round 3's path), then its kernel trace + PMC traffic, then the round's suite
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt_row1.py -x -v --timeout 120 --timeout-method thread > $O/pytest_row1.log 2>&1 && \
LCPC_NTT_ROW1=1 timeout -k 10 300 python -u bench.py --code pos --steps 16 > $O/pos_row1_bytes.json 2> $O/pos_row1_bytes.err && \
LCPC_NTT_ROW1=1 timeout -k 10 300 python -u bench.py --code pos --steps 16 --pos-commit elements > $O/pos_row1_elems.json 2> $O/pos_row1_elems.err && \
LCPC_NTT_ROW1=0 timeout -k 10 300 python -u bench.py --code pos --steps 16 --pos-commit elements > $O/pos_fourstep.json 2> $O/pos_fourstep.err && \
LCPC_NTT_ROW1=1 bash tools/prof_workload.sh r04g/prof_pos_row1 16 --code pos > $O/prof_pos_row1.log 2>&1 && \
./tools/evidence/r04/suite.sh
