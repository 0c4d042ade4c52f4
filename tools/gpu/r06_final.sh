#!/bin/bash
# driver-style final check: the whole GPU suite in one process, smoke, the default bench line
# (K = 20, W = 5) twice, and a rocprofv3 kernel trace of the same command for profiles/
set -o pipefail
O=gpurun_out/${1:-r06_final}
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 1500 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
$T 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20_a.json 2> $O/bench_k20_a.err || { tail -20 $O/bench_k20_a.err; exit 1; }
$T 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20_b.json 2> $O/bench_k20_b.err || { tail -20 $O/bench_k20_b.err; exit 1; }
$T 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > $O/bench_k20_trace.json 2> $O/bench_k20_trace.err || { tail -20 $O/bench_k20_trace.err; exit 1; }
echo done
