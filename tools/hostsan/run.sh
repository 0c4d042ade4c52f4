#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer runs of the library's host-only code
# (CPU, this container): the Merlin/STROBE transcript (both Keccak implementations; the batched
# record absorb against one append_message per record, at every block offset) and the
# Brakedown matgen (CSR invariants for SdigCode 1..6).  GPU sanitizers are not available.
set -e
cd "$(dirname "$0")/../../lcpc_proof_of_storage_amd/csrc"
OUT=${TMPDIR:-/tmp}/lcpc_hostsan; mkdir -p "$OUT"
SAN="-O1 -g -std=c++20 -march=x86-64-v3 -fsanitize=address,undefined -fno-omit-frame-pointer -I."
g++ $SAN ../../tools/hostsan/transcript_san.cpp transcript.cpp -o "$OUT/transcript_san"
g++ $SAN -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include ../../tools/hostsan/matgen_san.cpp sdig_host.cpp transcript.cpp \
  -o "$OUT/matgen_san" -lpthread
export ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=halt_on_error=1
LCPC_KECCAK=scalar "$OUT/transcript_san"
LCPC_KECCAK=avx512 "$OUT/transcript_san"
"$OUT/matgen_san" | tail -1
