"""CPU: the C-ABI boundary (include/lcpc_mi.h) without a GPU.

* liblcpc_mi.so loads, exports every function the header declares, and the Python binding
  (_native.SIGNATURES) covers exactly that set;
* the library carries gfx950 device code;
* the host-only entry points (dims, soundness counts, Field::random, the Merlin transcript)
  agree with the oracle;
* with no HIP device every compute entry point fails loudly (DeviceError) -- there is no
  CPU fallback in the product;
* the product package never imports the oracle.
"""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "lcpc_proof_of_storage_amd")


@pytest.fixture(scope="module")
def native():
    from lcpc_proof_of_storage_amd import _native as N
    if not os.path.exists(N.LIB_PATH):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)
    N.load()
    return N


@pytest.fixture(scope="module")
def api(native):
    from lcpc_proof_of_storage_amd import lcpc2d
    return lcpc2d


def test_header_symbols_exported_and_bound(native):
    import ctypes as C
    declared = native.header_symbols()
    assert len(declared) >= 60
    raw = C.CDLL(native.LIB_PATH)
    missing = [s for s in declared if not hasattr(raw, s)]
    assert not missing, missing
    assert sorted(native.SIGNATURES) == declared


def test_abi_version_matches_header(native):
    text = open(native.HEADER_PATH).read()
    want = int(re.search(r"#define LCPC_ABI_VERSION (\d+)", text).group(1))
    assert native.load().lcpc_abi_version() == want


def test_library_carries_gfx950_code(native):
    blob = open(native.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_header_is_plain_c():
    """No torch / C++ types in the boundary: it must compile as C99."""
    src = "#include \"lcpc_mi.h\"\nint main(void){return lcpc_abi_version();}\n"
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", "-",
                        "-I", os.path.join(ROOT, "include")], input=src.encode(), capture_output=True)
    assert r.returncode == 0, r.stderr.decode()


def test_product_never_imports_oracle():
    for dirpath, _, files in os.walk(PKG):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".hpp", ".h")) or fn == "Makefile":
                text = open(os.path.join(dirpath, fn), errors="replace").read()
                assert "oracle" not in text.lower(), fn


@pytest.mark.parametrize("fid", [0, 1, 2, 3, 4])
def test_field_params(api, oracle, fid):
    assert api.limbs(fid) == oracle.limbs(fid)
    assert api.num_bits(fid) == oracle.lib().of_field_num_bits(fid)


@pytest.mark.parametrize("fid", [0, 1, 2, 3, 4])
def test_field_random_matches_oracle(api, oracle, fid):
    for seed in [0, 7, 0x1CDC2024]:
        got = api.field_random(fid, 257, seed).reshape(-1)
        want = oracle.random_coeffs(fid, 257, seed)
        assert np.array_equal(got, want)


def test_dims_and_counts_match_oracle(api, oracle):
    L = oracle.lib()
    rng = np.random.default_rng(3)
    for fid in [0, 1, 3]:
        for rho in [(1, 2), (1, 4), (3, 4)]:
            for _ in range(40):
                n = int(rng.integers(1, 1 << 26))
                assert api.LigeroEncoding.get_dims_for(fid, n, rho) == oracle.ligero_dims(fid, n, rho)
    for rho in [(1, 2), (1, 4), (3, 4), (1, 8)]:
        assert api.LigeroEncoding.n_col_opens(rho) == L.of_ligero_n_col_opens(*rho)
    for n_cols in [4, 1024, 65536, 363568, 1 << 22]:
        for flog2 in [62, 126, 190, 254, 252]:
            assert api.n_degree_tests(128, n_cols, flog2) == L.of_n_degree_tests(128, n_cols, flog2)
    for v in [1, 2, 3, 1000, 1 << 20, (1 << 20) + 1]:
        assert api.log2(v) == L.of_log2(v)


def test_sdig_parameters_match_oracle(api, oracle):
    """SdigEncodingS::_n_col_opens and new()'s n_per_row choice (lcpc-brakedown-pc/src/lib.rs:
    57-110) are host-only."""
    L = oracle.lib()
    for code in range(1, 7):
        assert api.SdigEncoding.n_col_opens(code) == L.of_sdig_n_col_opens(code)
        for fid in [0, 1, 2, 3, 4]:
            for n in [100, 5000, 1 << 16, 1 << 20, (1 << 24) + 17, 1 << 26]:
                assert api.SdigEncoding.n_per_row_for(fid, n, code) == L.of_sdig_new_np(fid, code, n)


def test_pos_host_functions_match_oracle(native, oracle):
    """get_aspect_ratio_default_from_field_len and get_column_indicies_from_random_seed are
    host-only (networking/server.rs:1139-1170, client.rs:443-456)."""
    from lcpc_proof_of_storage_amd import pos
    for n in [1, 2, 5, 86, 1000, 4097, (1 << 30) // 8, 153391690, 10**9]:
        assert pos.get_aspect_ratio_default_from_field_len(n) == oracle.pos_default_dims(n)
    for seed, amount, mx in [(1337, 256, 32768), (1, 4, 10), (9, 10, 5), (3, 0, 7)]:
        assert pos.get_column_indicies_from_random_seed(seed, amount, mx) == \
            oracle.pos_column_indices(seed, amount, mx)


def test_transcript_matches_oracle(api, oracle):
    """Merlin framing through both STROBE paths (records inside / across the 166-byte rate)."""
    rng = np.random.default_rng(4)
    a, b = api.Transcript(b"test transcript"), oracle.Transcript(b"test transcript")
    for i in range(200):
        n = int(rng.choice([0, 1, 8, 16, 32, 100, 150, 166, 167, 400]))
        msg = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        lab = [b"$l//PR", b"polycommit", b"x" * int(rng.integers(1, 40))][i % 3]
        a.append_message(lab, msg)
        b.append_message(lab, msg)
        if i % 17 == 0:
            k = int(rng.choice([1, 32, 64, 200]))
            assert a.challenge_bytes(b"$l//DT", k) == b.challenge_bytes(b"$l//DT", k)
    c = a.clone()
    want = b.challenge_bytes(b"$l//CO", 32)
    assert c.challenge_bytes(b"$l//CO", 32) == want == a.challenge_bytes(b"$l//CO", 32)
    assert a.challenge_bytes(b"end", 48) == b.challenge_bytes(b"end", 48)


@pytest.mark.parametrize("label,msg_len", [(b"$l//PR", 16), (b"$l//PE", 8), (b"$l//PR", 32), (b"lbl", 5),
                                           (b"x" * 40, 64), (b"", 1), (b"$l//PR", 0)])
def test_transcript_append_messages_matches_oracle(api, oracle, label, msg_len):
    """The block-buffered record path (one record after another at every offset of the 166-byte
    rate, records split across it) against the oracle's message-by-message absorption."""
    rng = np.random.default_rng(msg_len + len(label))
    for pre in (0, 1, 7, 100, 131, 165):
        a, b = api.Transcript(b"test transcript"), oracle.Transcript(b"test transcript")
        head = rng.integers(0, 256, pre, dtype=np.uint8).tobytes()
        a.append_message(b"pre", head)
        b.append_message(b"pre", head)
        n = 300
        msgs = rng.integers(0, 256, n * msg_len, dtype=np.uint8).tobytes()
        if msg_len:
            a.append_messages(label, msgs, msg_len)
        else:
            for _ in range(n):
                a.append_message(label, b"")
        for i in range(n):
            b.append_message(label, msgs[i * msg_len:(i + 1) * msg_len])
        a.append_message(b"post", head[:3])
        b.append_message(b"post", head[:3])
        assert a.challenge_bytes(b"$l//CO", 40) == b.challenge_bytes(b"$l//CO", 40)


def test_compute_fails_loudly_without_device(api):
    if api.device_count() > 0:
        pytest.skip("a HIP device is visible; the GPU tests cover this path")
    calls = [
        lambda: api.LigeroEncoding.new(1, 1 << 12),
        lambda: api.merkle_tree(bytes(32 * 4)),
        lambda: api.collapse_columns(1, np.zeros(16, np.uint64), np.zeros(2, np.uint64), 2, 4),
        lambda: api.hash_columns(1, np.zeros(16, np.uint64), 2, 4),
    ]
    for fn in calls:
        with pytest.raises(api.DeviceError):
            fn()
