#!/bin/bash
# Round 5: the GPU suite on the cfg2-shape + split-SpMM tree, then the cfg2 / sdig-encode lines,
# the SDIG level times, and two driver-style K = 20 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --code encode --steps 512 --warmup 16 > $O/bench_encode.json 2> $O/bench_encode.err || { tail -20 $O/bench_encode.err; exit 1; }
timeout -k 10 300 python bench.py --code sdig-encode --steps 64 --warmup 8 > $O/bench_sdig_encode.json 2> $O/bench_sdig_encode.err || { tail -20 $O/bench_sdig_encode.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/sdig_kt -o run --output-format csv -- python3 bench.py --code sdig-encode --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof > /dev/null 2> $O/sdig_kt.err || { tail -20 $O/sdig_kt.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/enc_kt -o run --output-format csv -- python3 bench.py --code encode --steps 8 --warmup 2 --pipeline 1 --cpu-baseline off > /dev/null 2> $O/enc_kt.err || { tail -20 $O/enc_kt.err; exit 1; }
for r in a b; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20_$r.json 2> $O/bench_k20_$r.err || { tail -20 $O/bench_k20_$r.err; exit 1; }
done
echo done
