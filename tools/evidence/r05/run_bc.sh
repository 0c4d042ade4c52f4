#!/bin/bash
# b (sweeps, PMC, 8-rank cfg5) then c (K = 20 A/B); a heartbeat file shows progress while a
# long step (the 8-rank rehearsal) runs
mkdir -p gpurun_out/r05b
( while true; do date +%s > gpurun_out/r05b/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/evidence/r05/b_sweeps.sh && bash tools/evidence/r05/c_k20_ab.sh
