#!/bin/bash
# Round-1 closing GPU pass: the full gpu suite, the cfg3 bench + rocprof evidence (tools/gpu_check.sh),
# then the cfg5 PoS bench with its rocprof kernel stats.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_check.sh r01f 1024 || exit 1
OUT=gpurun_out/r01f
timeout -k 10 400 python bench.py --code pos --steps 8 --warmup 4 --pipeline 4 > "$OUT/pos.json" 2> "$OUT/pos.err" || { tail -20 "$OUT/pos.err"; exit 1; }
cat "$OUT/pos.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pos" -o run --output-format csv -- \
  python3 bench.py --code pos --steps 8 --warmup 4 --pipeline 4 --cpu-baseline off --verify-reps 0 > "$OUT/pos_under_prof.json" 2> "$OUT/prof_pos.err" || { tail -20 "$OUT/prof_pos.err"; exit 1; }
echo final done
