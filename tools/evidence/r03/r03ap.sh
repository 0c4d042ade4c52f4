#!/bin/bash
# grouped leaves for long row-major messages (PoS 74 chunks): parity (leaf chunk counts, PoS,
# commit), then the PoS line with and without (LCPC_LEAF_GROUPS=0), interleaved
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03ap; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pos.py tests/test_gpu_pos_files.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
B="timeout -k 10 300 python bench.py --code pos --pipeline 2 --steps 16 --warmup 4 --cpu-baseline off"
for i in 1 2; do
  $B > $OUT/grp_$i.json 2>> $OUT/b.err
  LCPC_LEAF_GROUPS=0 $B > $OUT/nogrp_$i.json 2>> $OUT/b.err
  for f in grp_$i nogrp_$i; do
    python -c "import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],3), 'leaf', round(k['leaf_chunks']['ms_per_step'],4), round(k.get('leaf_merge',{}).get('ms_per_step',0),4), 'frac', round(d['roofline_leaf']['frac'],3))"
  done
done
echo ok
