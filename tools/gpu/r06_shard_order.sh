#!/bin/bash
# the prove buffers' comm-stream writers ordered after their takes: the sharded GPU suites
# (one rank, ranks sharing the GPU over gloo and over RCCL, the pipelined driver, PoS requests)
# and the weak-scaled two-rank bench lines
set -o pipefail
O=gpurun_out/${1:-r06m}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_shard_native.py tests/test_gpu_pos_shard.py \
  tests/test_gpu_bench_contract.py tests/test_gpu_transcript_ops.py tests/test_gpu_host_input.py tests/test_gpu_sdig.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo done
