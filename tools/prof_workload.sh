#!/bin/bash
# One bench workload with its evidence: the bench line, a rocprofv3 kernel-trace + stats run of
# the same command, and the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE; serial steps).
# Usage (repo root, on the box): bash tools/prof_workload.sh <tag> <steps> [bench args...]
set -o pipefail
TAG=${1:-wl}; STEPS=${2:-256}; shift; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps "$STEPS" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps "$STEPS" --cpu-baseline off --verify-reps 0 "$@" > "$OUT/bench_under_prof.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo "$c" | cut -d_ -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 120 rocprofv3 --pmc "$c" -d "$OUT/pmc_$n" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 "$@" > /dev/null 2> "$OUT/pmc_$n.err" \
    || { tail -20 "$OUT/pmc_$n.err"; exit 1; }
done
echo done
