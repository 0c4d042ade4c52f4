"""CPU: pin the oracle against known-answer tests and an independent Python restatement.

The reference (Rust) cannot be built or imported here: no cargo/rustc,
fffft / ff-derive-num path dependencies absent, blake3 / merlin / rand_chacha crates not
vendored.  The oracle's third-party pieces are therefore pinned by published vectors
(BLAKE3 official test_vectors.json, RFC 7539 / rand_chacha ChaCha20 values, SHA3 through
hashlib for Keccak-f[1600]) and by a second, independent restatement in tests/pyref.py.
"""
import hashlib

import numpy as np
import pytest

import pyref

# BLAKE3 official test vectors: input = bytes(i % 251), 32-byte hash (test_vectors.json)
BLAKE3_VECTORS = {
    0: "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    1: "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213",
    1023: "10108970eeda3eb932baac1428c7a2163b0e924c9a9e25b35bba72b28f70bd11",
    1024: "42214739f095a406f3fc83deb889744ac00df831c10daa55189b5d121c855af7",
    1025: "d00278ae47eb27b34faecf67b4fe263f82d5412916c1ffd97c8cb7fb814b8444",
    2048: "e776b6028c7cd22a4d0ba182a8bf62205d2ef576467e838ed6f2529b85fba24a",
    2049: "5f4d72f40d7a5f82b15ca2b2e44b1de3c2ef86c426c95c1af0b6879522563030",
    3072: "b98cb0ff3623be03326b373de6b9095218513e64f1ee2edd2525c7ad1e5cffd2",
    3073: "7124b49501012f81cc7f11ca069ec9226cecb8a2c850cfe644e327d22d3e1cd3",
    4096: "015094013f57a5277b59d8475c0501042c0b642e531b0a1c8f58d2163229e969",
    4097: "9b4052b38f1c5fc8b1f9ff7ac7b27cd242487b3d890d15c96a1c25b8aa0fb995",
    5120: "9cadc15fed8b5d854562b26a9536d9707cadeda9b143978f319ab34230535833",
    8192: "aae792484c8efe4f19e2ca7d371d8c467ffb10748d8a5a1ae579948f718a2a63",
    8193: "bab6c09cb8ce8cf459261398d2e7aef35700bf488116ceb94a36d0f5f1b7bc3b",
    16384: "f875d6646de28985646f34ee13be9a576fd515f76b5b0a26bb324735041ddde4",
    31744: "62b6960e1a44bcc1eb1a611a8d6235b6b4b78f32e7abc4fb4c6cdcce94895c47",
    102400: "bc3e3d41a1146b069abffad3c0d44860cf664390afce4d9661f7902e7943e085",
}


def test_blake3_official_vectors(oracle):
    pattern = bytes(i % 251 for i in range(102400))
    for n, want in BLAKE3_VECTORS.items():
        assert oracle.blake3(pattern[:n]).hex() == want, n
    assert oracle.blake3(b"abc").hex() == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"


def test_blake3_python_restatement(oracle):
    pattern = bytes(i % 251 for i in range(9000))
    for n in [0, 1, 63, 64, 65, 1023, 1024, 1025, 2080, 3072, 8224]:  # 8224 = 512-row Ft127 leaf
        assert pyref.blake3(pattern[:n]) == oracle.blake3(pattern[:n]), n


def test_keccak_via_sha3(oracle):
    data = bytes(range(256)) * 3
    for n in [0, 1, 135, 136, 137, 271, 272, 700]:
        assert oracle.sha3_256(data[:n]) == hashlib.sha3_256(data[:n]).digest(), n


def test_chacha20_true_values(oracle):
    # rand_chacha test_chacha_true_values_a == RFC 7539 A.1 test vectors #1/#2 (zero key/nonce)
    r = oracle.ChaCha(bytes(32))
    block0 = [r.next_u32() for _ in range(16)]
    block1 = [r.next_u32() for _ in range(16)]
    assert block0 == [0xade0b876, 0x903df1a0, 0xe56a5d40, 0x28bd8653, 0xb819d2bd, 0x1aed8da0, 0xccef36a8,
                      0xc70d778b, 0x7c5941da, 0x8d485751, 0x3fe02477, 0x374ad8b8, 0xf4b8436a, 0x1ca11815,
                      0x69b687c3, 0x8665eeb2]
    assert block1 == [0xbee7079f, 0x7a385155, 0x7c97ba98, 0x0d082d73, 0xa0290fcb, 0x6965e348, 0x3e53c612,
                      0xed7aee32, 0x7621b729, 0x434ee69c, 0xb03371d5, 0xd539d874, 0x281fed31, 0x45fb0a51,
                      0x1f0ae1ac, 0x6f4d794b]


def test_chacha_u64_and_fill_are_keystream_views(oracle):
    a, b, c = oracle.ChaCha(bytes(range(32))), oracle.ChaCha(bytes(range(32))), oracle.ChaCha(bytes(range(32)))
    u32 = [a.next_u32() for _ in range(200)]
    u64 = [b.next_u64() for _ in range(100)]
    assert u64 == [u32[2 * i] | (u32[2 * i + 1] << 32) for i in range(100)]
    fb = c.fill_bytes(800)
    assert fb == b"".join(x.to_bytes(4, "little") for x in u32)


def test_uniform_power_of_two_is_top_bits(oracle):
    a, b = oracle.ChaCha(bytes(32)), oracle.ChaCha(bytes(32))
    for _ in range(100):
        assert a.uniform(0, 65536) == b.next_u64() >> 48


def test_uniform_rejection_zone(oracle):
    # rand 0.8 UniformInt<usize>: widening multiply, reject lo > zone
    a, b = oracle.ChaCha(bytes([7] * 32)), oracle.ChaCha(bytes([7] * 32))
    n = 363568  # a Brakedown codeword length (not a power of two)
    zone = (2**64 - 1) - ((2**64 - n) % n)
    for _ in range(200):
        got = a.uniform(0, n)
        while True:
            v = b.next_u64()
            m = v * n
            if m & (2**64 - 1) <= zone:
                assert got == m >> 64
                break


@pytest.mark.parametrize("fid", [0, 1, 2, 3, 4])
def test_field_constants_and_arith(oracle, fid):
    f = pyref.Field(fid)
    assert oracle.modulus(fid) == f.p
    assert oracle.lib().of_field_s(fid) == f.S
    assert oracle.lib().of_field_num_bits(fid) == f.p.bit_length()
    r = np.zeros(f.nl, np.uint64)
    oracle.lib().of_field_root_of_unity(fid, oracle.p64(r))
    assert oracle.from_mont(fid, r)[0] == f.root
    rng = np.random.default_rng(fid)
    vals = [int(rng.integers(0, 2**62)) * int(rng.integers(1, 2**62)) % f.p for _ in range(50)] + [0, 1, f.p - 1]
    m = oracle.to_mont(fid, vals)
    assert oracle.ints_from_limbs(m, f.nl) == [f.to_mont(v) for v in vals]
    assert oracle.from_mont(fid, m) == vals
    prod = oracle.mul(fid, m, m.copy())
    assert oracle.from_mont(fid, prod) == [v * v % f.p for v in vals]


def test_survey_root_values(oracle):
    # SURVEY.md §8(a-1/a-2) derived values for Ft127
    assert pyref.Field(1).root == 0x3280b719bea9b43abb9ee4e683614688
    w = np.zeros(2, np.uint64)
    oracle.lib().of_ntt_omega(1, 16, oracle.p64(w))
    assert oracle.from_mont(1, w)[0] == 0x3d1dafd4d962d8c57070ba75e1ebdda9
    oracle.lib().of_ntt_omega(1, 12, oracle.p64(w))
    assert oracle.from_mont(1, w)[0] == 0x5f368ee4e3516fa8ecb8d895fdf8060


@pytest.mark.parametrize("fid", [0, 1, 3, 4])
@pytest.mark.parametrize("log_n", [0, 1, 2, 3, 5, 7])
def test_fft_io_matches_naive_dft(oracle, fid, log_n):
    f = pyref.Field(fid)
    n = 1 << log_n
    rng = np.random.default_rng(100 * fid + log_n)
    xs = [int(rng.integers(0, 2**62)) * int(rng.integers(1, 2**62)) % f.p for _ in range(n)]
    got = oracle.from_mont(fid, oracle.fft_io(fid, oracle.to_mont(fid, xs)))
    assert got == pyref.fft_io_naive(f, xs)
    back = oracle.from_mont(fid, oracle.ifft_oi(fid, oracle.to_mont(fid, got)))
    assert back == xs


def test_fft_errors(oracle):
    with pytest.raises(ValueError):
        oracle.fft_io(1, np.zeros(2 * 6, np.uint64))  # not a power of two


def test_field_random_semantics(oracle):
    """ff_derive random(): limbs straight from next_u64, top masked, reject >= p, no conversion."""
    for fid in [0, 1, 3]:
        f = pyref.Field(fid)
        r1, r2 = oracle.ChaCha(bytes([3] * 32)), oracle.ChaCha(bytes([3] * 32))
        got = oracle.ints_from_limbs(r1.field_random(fid, 64), f.nl)
        shave = 64 * f.nl - f.p.bit_length()
        want = []
        while len(want) < 64:
            limbs = [r2.next_u64() for _ in range(f.nl)]
            limbs[-1] &= (2**64 - 1) >> shave
            v = sum(l << (64 * i) for i, l in enumerate(limbs))
            if v < f.p:
                want.append(v)
        assert got == want
