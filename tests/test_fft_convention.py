"""The fffft convention switches (include/lcpc_fft_convention.h), CPU only.

fffft (a path dependency absent from the reference tree, Cargo.toml:17) decides two things the
reference's tests never pin: the root (omega or omega^-1) and the output order of fft_io
(bit-reversed or natural).  Both are compile-time switches shared by the product's NTT plans and
the oracle.  Here the oracle is rebuilt with each non-default setting and shown to (1) compute
exactly the DFT that setting names (against the independent big-integer restatement in pyref.py),
(2) still satisfy the reference's invariants (ifft_oi inverts fft_io; verify accepts; the
evaluation is p(x)), and (3) change the committed fixtures -- so a Rust run that disagrees with
tests/golden/golden.json on the root names which switch to flip (tools/rust_golden/).
"""
import json
import os

import numpy as np
import pytest

import pyref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))

VARIANTS = {  # name: (compiler flags, omega_inverse, bit-reversed output)
    "omega_inv": ("-DLCPC_FFT_OMEGA_INVERSE=1", True, True),
    "natural_out": ("-DLCPC_FFT_OUTPUT_BITREV=0", False, False),
    "omega_inv_natural": ("-DLCPC_FFT_OMEGA_INVERSE=1 -DLCPC_FFT_OUTPUT_BITREV=0", True, False),
}


@pytest.fixture(scope="module")
def variant_libs(oracle):
    return {k: oracle.build_variant(k, flags) for k, (flags, _, _) in VARIANTS.items()}


def _canon(oracle, fid, a):
    return [int(v) for v in oracle.from_mont(fid, a)]


@pytest.mark.parametrize("name", list(VARIANTS) + ["default"])
@pytest.mark.parametrize("fid", [0, 1, 4])
def test_variant_is_the_dft_it_names(oracle, variant_libs, name, fid):
    omega_inv, bitrev = (False, True) if name == "default" else VARIANTS[name][1:]
    f = pyref.Field(fid)
    n, nl = 64, oracle.limbs(fid)
    x = oracle.ChaCha(seed_u64=5 + fid).field_random(fid, n)
    want = pyref.fft_io_naive(f, _canon(oracle, fid, x), omega_inverse=omega_inv, bitrev_out=bitrev)
    path = oracle.LIB_PATH if name == "default" else variant_libs[name]
    with oracle.use_lib(path):
        y = oracle.fft_io(fid, x)
        assert _canon(oracle, fid, y) == want
        back = oracle.ifft_oi(fid, y)
    assert np.array_equal(back.reshape(-1, nl), x.reshape(-1, nl))  # ifft_oi inverts fft_io


@pytest.mark.parametrize("name", list(VARIANTS))
def test_flipping_a_switch_changes_the_fixtures(oracle, variant_libs, name):
    """the Ft63 2^14 fixture under another convention: a different codeword, tree and column choice
    (the transcript absorbs the root), the same evaluation p(x) (it does not depend on the code)"""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import gen_golden
    g = GOLDEN["ft63_2_14"]
    with oracle.use_lib(variant_libs[name]):
        v = gen_golden.ligero_case(0, 14)  # (asserts that the variant's verify accepts its proof)
    assert v["dims"] == g["dims"]
    for k in ("root", "comm_sha256", "hashes_sha256"):
        assert v[k] != g[k], k
    assert v["eval"] == g["eval"] and v["p_eval_sha256"] == g["p_eval_sha256"]
    # and the default build reproduces the committed fixture
    d = gen_golden.ligero_case(0, 14)
    assert d["root"] == g["root"] and d["comm_sha256"] == g["comm_sha256"]


def test_product_and_oracle_share_the_switches():
    """one header, included by the product's NTT plans and by the oracle (no second copy)"""
    root = os.path.dirname(HERE)
    hdr = "lcpc_fft_convention.h"
    assert os.path.exists(os.path.join(root, "include", hdr))
    for rel in ("lcpc_proof_of_storage_amd/csrc/kernels.hpp", "oracle/of_ntt.c"):
        assert hdr in open(os.path.join(root, rel)).read(), rel
    for rel in ("lcpc_proof_of_storage_amd/csrc/ntt.hip", "oracle/of_ntt.c"):
        txt = open(os.path.join(root, rel)).read()
        assert "LCPC_FFT_OMEGA_INVERSE" in txt and "LCPC_FFT_OUTPUT_BITREV" in txt, rel
