#!/bin/bash
# the 8-rank RCCL tests (pipelined 2^22, cfg3 full size), one GPU
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard_native.py -k "world8" -x -v --timeout 600 --timeout-method thread > $OUT/pytest_world8.log 2>&1
tail -4 $OUT/pytest_world8.log
echo ok
