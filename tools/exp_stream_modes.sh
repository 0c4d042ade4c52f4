set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/exp1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/exp1/pytest.log 2>&1 || { tail -30 gpurun_out/exp1/pytest.log; exit 1; }
tail -2 gpurun_out/exp1/pytest.log
for mode in pool serial; do
 for p in 4 8 12; do
  timeout -k 10 300 python bench.py --steps 48 --warmup 16 --pipeline $p --stream-mode $mode --cpu-baseline off > gpurun_out/exp1/b_${mode}_$p.json 2>gpurun_out/exp1/b_${mode}_$p.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp1/b_${mode}_$p.json'));print('$mode',$p,round(d['value']/1e9,3),'G/s',round(d['ms_per_step'],3),'ms', 'frac',round(d['roofline']['frac'],4))"
 done
done
