#!/bin/bash
# round 4: the transcript's Keccak on the box's EPYC under -mtune generic / znver4 / znver5, each
# permutation forced (scalar, avx512), three repetitions
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
for rep in 1 2 3; do
  for t in generic znver4 znver5; do
    for k in scalar avx512; do
      echo "$t $k $(LCPC_KECCAK=$k timeout 60 ./tools/microbench/transcript_bench_$t 2>&1 | tail -1)" >> $O/keccak_tune.txt || exit 1
    done
  done
done
