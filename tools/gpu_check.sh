#!/bin/bash
# One GPU-box pass: parity tests, the bench line, the rocprofv3 kernel-trace summary of the same
# bench command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic figure.
# Usage (from the repo root, on the box): bash tools/gpu_check.sh <tag> [steps]
set -o pipefail
TAG=${1:-run}
STEPS=${2:-64}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "[gpu_check] pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "[gpu_check] bench"
timeout -k 10 400 python bench.py --steps "$STEPS" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "[gpu_check] rocprofv3 kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps "$STEPS" --cpu-baseline off --verify-reps 0 > "$OUT/bench_under_prof.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
echo "[gpu_check] rocprofv3 pmc FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 > /dev/null 2> "$OUT/pmc_fetch.err" || { tail -30 "$OUT/pmc_fetch.err"; exit 1; }
echo "[gpu_check] rocprofv3 pmc WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 > /dev/null 2> "$OUT/pmc_write.err" || { tail -30 "$OUT/pmc_write.err"; exit 1; }
find "$OUT" -name "*.csv" | head -20
echo "[gpu_check] done"
