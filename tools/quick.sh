#!/bin/bash
# Quick GPU-box iteration: parity suite + one cfg3 bench line, key numbers printed.
# Usage (repo root, on the box): bash tools/quick.sh <tag> [steps] [extra bench args...]
set -o pipefail
TAG=${1:-quick}; STEPS=${2:-128}; shift; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python bench.py --steps "$STEPS" --cpu-baseline off "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.3f G/s  ms/step %.4f  roofline frac %.4f  valu frac %.3f" % (d["value"] / 1e9, d["ms_per_step"], d["roofline"]["frac"], d.get("roofline_valu", {}).get("frac", 0)))
for k, v in sorted(d.get("kernels", {}).items()):
    print("  %-22s %.4f ms" % (k, v["avg_ms"]))
PY
