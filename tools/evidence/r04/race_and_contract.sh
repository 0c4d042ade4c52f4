#!/bin/bash
# round 4: per-(poly, stage) events -- the re-record microbench, the eight-rank RCCL pipeline test
# at the default priorities and in the mixed-priority A/B mode, the bench contract (N > 1 lines
# self-checking), and the K = 20 line.
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/microbench/prio_wait 200 > $O/prio_wait.txt 2>&1 && \
timeout -k 10 400 $T tests/test_gpu_shard_native.py -k "world8_rccl_one_gpu and pipeline" > $O/world8_default.log 2>&1 && \
LCPC_SHARD_PRIO=2 LCPC_SHARD_PRIO_AB=1 timeout -k 10 400 $T tests/test_gpu_shard_native.py -k "world8_rccl_one_gpu and pipeline" > $O/world8_mode2_a.log 2>&1 && \
LCPC_SHARD_PRIO=2 LCPC_SHARD_PRIO_AB=1 timeout -k 10 400 $T tests/test_gpu_shard_native.py -k "world8_rccl_one_gpu and pipeline" > $O/world8_mode2_b.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_bench_contract.py tests/test_gpu_shard_native.py tests/test_gpu_pos_shard.py -m "gpu and not slow" > $O/contract_shard.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err
