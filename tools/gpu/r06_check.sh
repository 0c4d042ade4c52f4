#!/bin/bash
# round 6: the new boundary (caller transcripts), host-resident inputs, the pool-ordering fix,
# smoke, then the default K = 20 line and the host-input lines beside it.
set -o pipefail
O=gpurun_out/${1:-r06b}
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_transcript_ops.py tests/test_gpu_host_input.py tests/test_pool_ordering.py \
  tests/test_gpu_pos_shard.py tests/test_gpu_bench_contract.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
$T 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
$T 400 python bench.py --steps 20 --warmup 5 --input host --sharded-n1 0 --cpu-baseline off --verify-reps 0 > $O/bench_k20_host.json 2> $O/bench_k20_host.err || { tail -20 $O/bench_k20_host.err; exit 1; }
$T 400 python bench.py --steps 20 --warmup 5 --input host-pinned --sharded-n1 0 --cpu-baseline off --verify-reps 0 > $O/bench_k20_hostpinned.json 2> $O/bench_k20_hostpinned.err || { tail -20 $O/bench_k20_hostpinned.err; exit 1; }
$T 400 python bench.py --steps 20 --warmup 5 --transcript caller --sharded-n1 0 --cpu-baseline off --verify-reps 0 > $O/bench_k20_caller_tr.json 2> $O/bench_k20_caller_tr.err || { tail -20 $O/bench_k20_caller_tr.err; exit 1; }
$T 400 python bench.py --code pos --steps 8 --warmup 2 --input host --cpu-baseline off > $O/bench_pos_host.json 2> $O/bench_pos_host.err || { tail -20 $O/bench_pos_host.err; exit 1; }
echo done
