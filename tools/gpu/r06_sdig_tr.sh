#!/bin/bash
# SDIG encode_rows with the message part written by the input transpose (only the parity part
# transposed back): the SDIG GPU parity tests, then the cfg4 encode line twice
set -o pipefail
O=gpurun_out/${1:-r06h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sdig.py > $O/pytest_sdig.log 2>&1 || { tail -30 $O/pytest_sdig.log; exit 1; }
tail -2 $O/pytest_sdig.log
for i in a b; do
  timeout -k 10 300 python bench.py --code sdig-encode > $O/bench_sdig_encode_$i.json 2> $O/bench_sdig_encode_$i.err || { tail -20 $O/bench_sdig_encode_$i.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --code sdig-encode --cpu-baseline off > $O/bench_trace.json 2> $O/bench_trace.err || { tail -20 $O/bench_trace.err; exit 1; }
echo done
