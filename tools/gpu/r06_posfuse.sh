#!/bin/bash
# the PoS request with u^T Enc(M) summed in the leaf pass: the PoS GPU suites, the fused and the
# separate request lines (1 GiB, interleaved), and the bench-contract PoS cases
set -o pipefail
O=gpurun_out/${1:-r06u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pos.py tests/test_gpu_pos_shard.py \
  "tests/test_gpu_bench_contract.py::test_bench_pos_small" tests/test_gpu_fullsize.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for m in fused separate; do
    timeout -k 10 300 python bench.py --code pos --pos-eval $m --cpu-baseline off > $O/pos_${m}_${rep}.json 2> $O/pos_${m}_${rep}.err || { tail -20 $O/pos_${m}_${rep}.err; exit 1; }
  done
done
timeout -k 10 300 python bench.py --code pos > $O/pos_default.json 2> $O/pos_default.err || { tail -20 $O/pos_default.err; exit 1; }
echo done
