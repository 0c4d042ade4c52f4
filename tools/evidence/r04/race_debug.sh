#!/bin/bash
# round 4: the mixed-priority wrong root with LCPC_SHARD_DEBUG=1 (per rank and polynomial: the
# codeword shard and the sent chaining values recomputed, the subtree roots), mode 2.  A test
# failure (rc 1) is a result; any other status ends the script.
O=gpurun_out/r04d3
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_shard_native.py -k pipeline_world8_rccl"
for i in 1 2 3 4 5 6; do
  env LCPC_SHARD_DEBUG=1 LCPC_SHARD_PRIO=2 LCPC_SHARD_PRIO_AB=1 timeout -k 10 240 $T > $O/dbg_$i.log 2>&1
  rc=$?
  echo "dbg_$i rc=$rc" >> $O/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
