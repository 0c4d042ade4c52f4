#!/bin/bash
# Issue-level PMC counters of the encode kernels (one counter group per rocprofv3 pass).
# Usage (repo root, on the box): bash tools/pmc_ntt.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-ntt}; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES" \
           "SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 "$@" > /dev/null 2> "$OUT/p$i.err" \
    || { tail -20 "$OUT/p$i.err"; exit 1; }
done
echo done
