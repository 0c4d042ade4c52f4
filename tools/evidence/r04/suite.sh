#!/bin/bash
# round 4: the GPU suite in one process (as the driver runs it), then the K = 20 line and the
# like-for-like context lines (rho = 1/4 as the reference's commit_bench, Ft255)
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 60 ./tools/microbench/nttmfma63 $((1<<20)) 8 > $O/nttmfma63.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --rho 1/4 --sharded-n1 0 > $O/bench_rho14.json 2> $O/bench_rho14.err && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --field Ft255 --sharded-n1 0 > $O/bench_ft255.json 2> $O/bench_ft255.err
