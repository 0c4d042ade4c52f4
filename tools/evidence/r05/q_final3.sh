#!/bin/bash
# Round 5, final tree (third pass: the sharded reserve pins proof blocks): the driver's
# sequence -- GPU suite, smoke, the default bench line and two K = 20 lines -- plus the kernel
# trace of the K = 20 command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -m pytest tests/test_pool_ordering.py -m gpu -q -s --timeout 60 --timeout-method thread > $O/pool_selftest.log 2>&1 || { tail -20 $O/pool_selftest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
for r in a b; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20_$r.json 2> $O/bench_k20_$r.err || { tail -20 $O/bench_k20_$r.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k20_kt -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20_prof.json 2> $O/k20_kt.err || { tail -20 $O/k20_kt.err; exit 1; }
LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --steps 20 --warmup 5 > $O/bench_torchrun_8ranks.json 2> $O/bench_torchrun_8ranks.err \
  || { tail -30 $O/bench_torchrun_8ranks.err; exit 1; }
echo done
