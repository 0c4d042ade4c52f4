set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sdigb
timeout -k 10 600 python bench.py --code sdig --steps 32 --warmup 12 > gpurun_out/sdigb/bench.json 2> gpurun_out/sdigb/bench.err || { tail -30 gpurun_out/sdigb/bench.err; exit 1; }
cat gpurun_out/sdigb/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sdigb/prof -o run --output-format csv -- python3 bench.py --code sdig --steps 8 --warmup 4 --cpu-baseline off > /dev/null 2> gpurun_out/sdigb/prof.err || { tail -30 gpurun_out/sdigb/prof.err; exit 1; }
