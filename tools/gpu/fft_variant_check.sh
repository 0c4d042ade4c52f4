#!/bin/bash
# The FFT-convention switches (include/lcpc_fft_convention.h) flipped in BOTH the product and the
# oracle: the product built with omega^-1 and natural-order output
#   make -C lcpc_proof_of_storage_amd OUT=build_natural LIB=build_natural/liblcpc_mi.so \
#        EXTRA_FLAGS="-DLCPC_FFT_OUTPUT_BITREV=0 -DLCPC_FFT_OMEGA_INVERSE=1"
# and the oracle variant of tests/test_fft_convention.py (oracle/build/omega_inv_natural), then the
# GPU parity tests that touch the encode, the commitment, prove / verify and ifft_oi run against
# each other.  (test_golden is left out: the committed fixtures are the default convention's.)
set -o pipefail
O=gpurun_out/${1:-r06_fft_variant}
mkdir -p $O
export LCPC_MI_LIB=$PWD/lcpc_proof_of_storage_amd/build_natural/liblcpc_mi.so
export LCPC_ORACLE_LIB=$PWD/oracle/build/omega_inv_natural/liblcpc_oracle.so
test -f $LCPC_MI_LIB && test -f $LCPC_ORACLE_LIB || { echo "variant builds missing"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pos.py tests/test_gpu_ntt_row1.py tests/test_gpu_host_input.py \
  -k "not golden" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
