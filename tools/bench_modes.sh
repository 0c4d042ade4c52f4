#!/bin/bash
# Runs every bench workload once (cfg3 Ligero, cfg4 Brakedown, cfg5 proof-of-storage).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-modes}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py > "$OUT/ligero.json" 2> "$OUT/ligero.err" || { tail -20 "$OUT/ligero.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/ligero.json'));print('ligero',d['value']/1e9,'G/s',d['ms_per_step'],'ms frac',d['roofline']['frac'],'cpu',d['cpu_baseline']['value']/1e6,'M/s parity',d.get('parity_root_vs_oracle'))"
for p in 12 16 24; do
timeout -k 10 300 python bench.py --code sdig --steps 48 --warmup 24 --pipeline $p --cpu-baseline off > "$OUT/sdig_$p.json" 2> "$OUT/sdig_$p.err" || { tail -20 "$OUT/sdig_$p.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/sdig_$p.json'));print('sdig p$p',d['value']/1e9,'G/s',d['ms_per_step'],'ms frac',d['roofline']['frac'])"
done
timeout -k 10 400 python bench.py --code pos --steps 8 --warmup 4 --pipeline 4 > "$OUT/pos.json" 2> "$OUT/pos.err" || { tail -20 "$OUT/pos.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/pos.json'));print('pos',d['value']/1e9,'G/s',d['ms_per_step'],'ms frac',d['roofline']['frac'],'cpu',d['cpu_baseline'])"
