set -o pipefail
for a in "20 10 16" "20 10 4" "50 10 16" "50 10 8" "100 10 16" "100 10 8" "200 20 16"; do
  set -- $a
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --pipeline $3 --cpu-baseline off --verify-reps 0 --no-prof > gpurun_out/sk_$1_$3.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sk_$1_$3.json'));print('K=$1 W=$2 P=$3', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms')"
done
