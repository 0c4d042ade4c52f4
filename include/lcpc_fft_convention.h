/*
 * lcpc_fft_convention.h -- the two choices of fffft's fft_io that can change output bits, as
 * compile-time switches shared by the product's NTT plans (lcpc_proof_of_storage_amd/csrc/ntt.hip)
 * and the test oracle (oracle/of_ntt.c).
 *
 * LigeroEncodingRho::encode is fffft's FieldFFT::fft_io_pc (lcpc-ligero-pc/src/lib.rs:162-164),
 * precomputed by precomp_fft(n_cols) (:138-148).  fffft is a path dependency absent from the
 * reference tree (Cargo.toml:17; the 2021 logs name fffft v0.4.0), so its convention is restated,
 * not read.  The reference's own tests pin only relations that hold under every choice below
 * (lcpc-2d/src/tests.rs:193-234: ifft_oi inverts the encode and encoded rows are Reed-Solomon
 * evaluations), so VALUE parity with the Rust crates is unpinned at exactly these two bits.
 * tools/rust_golden/ prints the values that decide them on a machine with a Rust toolchain;
 * flip a switch here, rebuild (make -C lcpc_proof_of_storage_amd; make -C oracle) and
 * regenerate tests/golden/golden.json if they disagree.
 *
 * LCPC_FFT_OMEGA_INVERSE
 *   0 (restated default): omega = ROOT_OF_UNITY^(2^(S - k)), k = log2(n_cols);
 *   1: omega^-1 instead (ifft_oi then uses omega).
 * LCPC_FFT_OUTPUT_BITREV
 *   1 (restated default): decimation in frequency, natural-order input, bit-reversed output:
 *      out[bitrev_k(j)] = sum_i in[i] omega^(i j)   (ifft_oi: bit-reversed in, natural out);
 *   0: natural-order output, out[j] = sum_i in[i] omega^(i j) (ifft_oi: natural in).
 */
#ifndef LCPC_FFT_CONVENTION_H
#define LCPC_FFT_CONVENTION_H

#ifndef LCPC_FFT_OMEGA_INVERSE
#define LCPC_FFT_OMEGA_INVERSE 0
#endif
#ifndef LCPC_FFT_OUTPUT_BITREV
#define LCPC_FFT_OUTPUT_BITREV 1
#endif

#endif /* LCPC_FFT_CONVENTION_H */
