#!/bin/bash
# Round 5: the row-sharded engine at one rank (the N > 1 engine's own N = 1 point), K = 20: its
# host phases per tick (LCPC_PROF_TIMELINE, host scopes only) and a kernel trace of the same run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
for r in a b; do
  rm -f $O/phases_$r.csv
  LCPC_PROF_TIMELINE=$O/phases_$r.csv LCPC_PROF_HOST_ONLY=1 timeout -k 10 200 python bench.py --mode sharded --gpus 1 --steps 20 --warmup 5 \
    --prof-timed --cpu-baseline off --verify-reps 0 > $O/sh_$r.json 2> $O/sh_$r.err || { tail -20 $O/sh_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/sh_$r.json').read().strip().splitlines()[-1]);print('$r', round(d['value']/1e9,3), d['ms_per_step'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --mode sharded --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --no-prof > $O/sh_prof.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
echo done
