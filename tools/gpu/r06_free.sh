#!/bin/bash
# carry-free mads in fe_mul_fips: the multiply against CIOS on every field, the encode / commit
# parity suites, the cfg3-size encode alone and the K = 20 line twice
set -o pipefail
O=gpurun_out/${1:-r06j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/femul_free > $O/femul_free.txt 2>&1 || { cat $O/femul_free.txt; exit 1; }
cat $O/femul_free.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py \
  tests/test_gpu_ntt_row1.py tests/test_gpu_sdig.py tests/test_gpu_properties.py tests/test_gpu_transcript_ops.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --code encode --log-len 24 --steps 64 --warmup 8 > $O/bench_encode24.json 2> $O/bench_encode24.err || { tail -20 $O/bench_encode24.err; exit 1; }
for i in a b; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20_$i.json 2> $O/bench_k20_$i.err || { tail -20 $O/bench_k20_$i.err; exit 1; }
done
echo done
