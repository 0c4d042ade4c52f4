#!/bin/bash
# round 4 final tree: the other configurations' lines (bench.py with no flags = cfg3 K = 256,
# cfg2 encode alone, cfg4 commit + open at K = 20 and K = 64)
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err && \
timeout -k 10 300 python -u bench.py --code encode --steps 512 > $O/encode_k512.json 2> $O/encode_k512.err && \
timeout -k 10 400 python -u bench.py --code sdig --steps 20 --warmup 5 > $O/sdig_k20.json 2> $O/sdig_k20.err && \
timeout -k 10 400 python -u bench.py --code sdig --steps 64 --warmup 5 > $O/sdig_k64.json 2> $O/sdig_k64.err
