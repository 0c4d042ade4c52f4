set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03a; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
$T 400 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
$T 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
echo ok
