"""GPU parity of the one-pass Ft63 row encode (csrc/ntt_row1.hpp) at the proof-of-storage
default dims (2^15-point rows, rate 1/2: 16384 coefficients -> 32768), against the oracle's
fft_io and commit (lcpc-ligero-pc/src/lib.rs:162-164, lcpc-2d/src/lib.rs:651-700), and against
the four-step pair (lcpc_encoding_set_row_kernel selects the kernel per encoding)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

AUTO, FOURSTEP, ONEPASS = 0, 1, 2
NP, NC = 16384, 32768


def rand_elems(oracle, n, seed):
    return oracle.ChaCha(seed_u64=seed).field_random(0, n)


def test_row1_encode_rows_match_fffft(gpu, oracle):
    """batched rows (Montgomery output, no coefficient copy) against fft_io row by row, through
    the one-pass kernel and the four-step pair"""
    enc = gpu.RsEncoding.new(0, NP, NC, 4, 1).set_row_kernel(ONEPASS)
    rows = np.zeros((5, NC), np.uint64)
    rows[:, :NP] = rand_elems(oracle, 5 * NP, 61).reshape(5, NP)
    got = enc.encode_rows(rows.copy()).reshape(5, NC)
    for r in range(5):
        assert np.array_equal(got[r], oracle.fft_io(0, rows[r])), r
    got4 = enc.set_row_kernel(FOURSTEP).encode_rows(rows.copy()).reshape(5, NC)
    assert np.array_equal(got, got4)


@pytest.mark.parametrize("pattern", ["max", "alternating", "one", "impulse_last"])
def test_row1_extreme_values(gpu, oracle, pattern):
    """p - 1 everywhere, alternating 0 / p - 1, a single 1 and a single p - 1 at the last valid
    coefficient: the [0, 2p) butterflies at their carry / borrow boundaries"""
    pm1 = oracle.modulus(0) - 1
    row = np.zeros(NC, np.uint64)
    if pattern == "max":
        row[:NP] = pm1
    elif pattern == "alternating":
        row[1:NP:2] = pm1
    elif pattern == "one":
        row[0] = 1
    else:
        row[NP - 1] = pm1
    want = oracle.fft_io(0, row)
    for kernel in (ONEPASS, FOURSTEP):
        enc = gpu.RsEncoding.new(0, NP, NC, 4, 1).set_row_kernel(kernel)
        got = row.copy()
        enc.encode(got)
        assert np.array_equal(got, want), kernel


@pytest.mark.parametrize("length", [37 * NP, 37 * NP + 5, 3 * NP - 1, 1000, 300 * NP])
def test_row1_commit_device_matches_oracle(gpu, oracle, hipmem, length):
    """the commit path (canonical output + the commitment's coefficient copy), full and ragged
    last rows, against the oracle's coefficient matrix, codeword, hashes and root"""
    coeffs = rand_elems(oracle, length, 17)
    g_enc = gpu.RsEncoding.new(0, NP, NC, 16, 2).set_row_kernel(ONEPASS)
    o_enc = oracle.Encoding.ligero(0, NP, NC, 16, 2)
    d = hipmem.to_device(coeffs)
    try:
        g = gpu.LcCommit.commit_device(d, length, g_enc)
        o = oracle.Commit(o_enc, coeffs)
        assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
        assert np.array_equal(g.comm.reshape(-1), o.comm)
        assert g.hashes == o.hashes
        assert g.get_root() == o.root()
        g4 = gpu.LcCommit.commit_device(d, length, g_enc.set_row_kernel(FOURSTEP))
        assert g4.get_root() == g.get_root()
        del g, g4
    finally:
        hipmem.free(d)


@pytest.mark.parametrize("kernel", [AUTO, FOURSTEP], ids=["auto_onepass", "fourstep_packed"])
@pytest.mark.parametrize("dims,n_bytes", [
    ((NP, NC), 7 * NP * 5),            # whole rows, one-pass fused unpack
    ((NP, NC), 7 * NP * 300 + 11),     # more rows than CUs (persistent workgroups loop), a ragged last row
    ((NP, NC), 7 * NP * 5 + 1001),     # a partial last row, a partial last element
    ((NP, NC), 13),                    # two elements, one row
    ((100, 256), 7 * 100 * 3 + 5),     # other dims: packed first
])
def test_pos_commit_bytes_device(gpu, oracle, hipmem, kernel, dims, n_bytes):
    """lcpc_pos_commit_bytes_device == DataField::from_byte_vec + LcCommit::commit (the oracle's
    pos_bytes_to_field + Commit), and == the two-call device path; AUTO = the one-pass kernel with
    the fused unpack at the PoS dims, FOURSTEP = k_pack7 + the four-step pair"""
    np_, nc = dims
    data = np.random.default_rng(n_bytes).integers(0, 256, n_bytes, dtype=np.uint8)
    data[-1] = 0xff
    el = oracle.pos_bytes_to_field(data.tobytes())
    g_enc = gpu.RsEncoding.new(0, np_, nc, 16, 2).set_row_kernel(kernel)
    o_enc = oracle.Encoding.ligero(0, np_, nc, 16, 2)
    d = hipmem.to_device(np.concatenate([data, np.zeros((-n_bytes) % 8, np.uint8)]).view(np.uint64))
    de = hipmem.to_device(el)
    try:
        g = gpu.LcCommit.commit_pos_bytes_device(d, n_bytes, g_enc)
        o = oracle.Commit(o_enc, el)
        assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
        assert np.array_equal(g.comm.reshape(-1), o.comm)
        assert g.get_root() == o.root()
        assert gpu.LcCommit.commit_device(de, el.size, g_enc.set_row_kernel(AUTO)).get_root() == g.get_root()
        del g
    finally:
        hipmem.free(d)
        hipmem.free(de)


def test_pos_commit_bytes_device_rejects(gpu, hipmem):
    d = hipmem.to_device(np.zeros(16, np.uint64))
    try:
        enc127 = gpu.RsEncoding.new(1, 64, 128, 4, 1)
        with pytest.raises(Exception):
            gpu.LcCommit.commit_pos_bytes_device(d, 64, enc127)       # not WriteableFt63
        enc = gpu.RsEncoding.new(0, 64, 128, 4, 1)
        with pytest.raises(Exception):
            gpu.LcCommit.commit_pos_bytes_device(d + 1, 64, enc)      # misaligned
        with pytest.raises(Exception):
            gpu.LcCommit.commit_pos_bytes_device(d, 0, enc)           # empty
    finally:
        hipmem.free(d)


def test_pos_commit_bytes_device_sdig(gpu, oracle, hipmem):
    """a Brakedown (SDIG) WriteableFt63 encoding takes the packed path: the same commitment as
    packing first and committing the elements"""
    n_bytes = 7 * 3000 + 3
    data = np.random.default_rng(7).integers(0, 256, n_bytes, dtype=np.uint8)
    el = oracle.pos_bytes_to_field(data.tobytes())
    enc = gpu.SdigEncoding.new(0, el.size, 0)
    d = hipmem.to_device(np.concatenate([data, np.zeros((-n_bytes) % 8, np.uint8)]).view(np.uint64))
    de = hipmem.to_device(el)
    try:
        g = gpu.LcCommit.commit_pos_bytes_device(d, n_bytes, enc)
        assert gpu.LcCommit.commit_device(de, el.size, enc).get_root() == g.get_root()
        assert g.get_root() == gpu.LcCommit.commit(el, enc).get_root()
    finally:
        hipmem.free(d)
        hipmem.free(de)


def test_row1_runtime_modes_agree(gpu, oracle):
    """the file-image kernel's runtime knobs (ntt_row1.hpp row1_prefetch / row1_glds, read once
    per process, so one child process per setting): every prefetch placement, with and without
    the LDS-DMA staging, gives the default's commitment -- whole rows, a ragged last row that the
    prefetch of row + 256 reaches, a partial last element, a one-row file -- and the default's
    root is the oracle's"""
    import json
    import os
    import subprocess
    import sys
    sizes = [7 * NP * 5 + 1001, 7 * NP * 300 + 11, 7 * NP * 600, 13]
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_row1_modes_child.py")
    results = {}
    for pf, glds in [(None, None), ("0", None), ("2", None), ("3", None), ("1", "0"), ("0", "0")]:
        env = {k: v for k, v in os.environ.items() if k not in ("LCPC_ROW1_PREFETCH", "LCPC_ROW1_GLDS")}
        if pf is not None:
            env["LCPC_ROW1_PREFETCH"] = pf
        if glds is not None:
            env["LCPC_ROW1_GLDS"] = glds
        r = subprocess.run([sys.executable, child, *map(str, sizes)], env=env, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, (pf, glds, r.stderr[-2000:])
        results[(pf, glds)] = json.loads(r.stdout.strip().splitlines()[-1])
    default = results[(None, None)]
    for key, got in results.items():
        assert got == default, key
    n_bytes = sizes[0]
    data = np.random.default_rng(n_bytes).integers(0, 256, n_bytes, dtype=np.uint8)
    data[-1] = 0xff
    o = oracle.Commit(oracle.Encoding.ligero(0, NP, NC, 16, 2), oracle.pos_bytes_to_field(data.tobytes()))
    assert default[str(n_bytes)][0] == o.root().hex()
