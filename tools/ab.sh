#!/bin/bash
# A/B of one environment switch on the same box: bench A (default) and B (with VAR=VALUE), twice each.
# Usage (repo root, on the box): bash tools/ab.sh <tag> <VAR=VALUE> [steps] [extra bench args...]
set -o pipefail
TAG=${1:-ab}; SW=$2; STEPS=${3:-128}; shift; shift; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then E=""; else E="$SW"; fi
    timeout -k 10 300 env $E python bench.py --steps "$STEPS" --cpu-baseline off "$@" > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -20 "$OUT/$v$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));k=d['kernels'];print('$v$i', '%.3f G/s'%(d['value']/1e9), '%.4f ms/step'%d['ms_per_step'], ' '.join('%s=%.4f'%(n,k[n]['avg_ms']) for n in sorted(k) if not n.startswith('host')))"
  done
done
