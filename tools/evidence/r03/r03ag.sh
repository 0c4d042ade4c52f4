#!/bin/bash
# default mode 3 (every sharded-driver stream high priority): the 8-rank pipelined test twelve
# times (checks: a failing run does not stop the next; a timeout / abort / crash ends the script),
# then the GPU suite (fast + full-size) and the K = 20 line
export TMPDIR=/tmp
OUT=gpurun_out/r03ag; mkdir -p $OUT
fails=0
for i in $(seq 1 12); do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/w8_$i.log 2>&1
  rc=$?
  if [ $rc -eq 1 ]; then fails=$((fails+1)); fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "run $i rc=$rc stopping"; exit $rc; fi
done
echo "world8 failures: $fails of 12"
set -e
timeout -k 10 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
timeout -k 10 800 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
tail -1 $OUT/pytest_gpu_slow.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20.json 2> $OUT/b.err
python -c "import json;d=json.loads(open('$OUT/k20.json').read().strip().splitlines()[-1]);print('k20', round(d['value']/1e9,3), 'sharded_n1', round(d['sharded_n1']['value']/1e9,3))"
echo ok
