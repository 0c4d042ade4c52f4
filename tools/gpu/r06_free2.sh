#!/bin/bash
# the library rebuilt with the asm carry-free mads: parity suites, the cfg3-size encode alone,
# the encode's SQ / GRBM counters and kernel trace (cycle model), K = 20 twice, K = 256, cfg2
set -o pipefail
O=gpurun_out/${1:-r06l}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py \
  tests/test_gpu_ntt_row1.py tests/test_gpu_sdig.py tests/test_gpu_properties.py tests/test_gpu_transcript_ops.py tests/test_gpu_pos.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --code encode --log-len 24 --steps 64 --warmup 8 > $O/bench_encode24.json 2> $O/bench_encode24.err || { tail -20 $O/bench_encode24.err; exit 1; }
bash tools/pmc_ntt.sh ${1:-r06l}/pmc --code encode --log-len 24 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --code encode --log-len 24 --steps 20 --warmup 5 --cpu-baseline off > $O/trace_bench.json 2> $O/trace_bench.err || { tail $O/trace_bench.err; exit 1; }
for i in a b; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20_$i.json 2> $O/bench_k20_$i.err || { tail -20 $O/bench_k20_$i.err; exit 1; }
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --code encode > $O/bench_encode.json 2> $O/bench_encode.err || { tail -20 $O/bench_encode.err; exit 1; }
timeout -k 10 300 python bench.py --code pos > $O/bench_pos.json 2> $O/bench_pos.err || { tail -20 $O/bench_pos.err; exit 1; }
echo done
