"""Independent pure-Python restatement (big integers) of the field / NTT / BLAKE3 pieces,
used only by tests to cross-check the C oracle on small inputs.  TEST INFRASTRUCTURE ONLY.

Written separately from oracle/*.c so an implementation slip in one is caught by the other:
  field: ff_derive PrimeField semantics (lcpc-test-fields/src/lib.rs:13-70)
  ntt:   fffft fft_io contract, computed as a naive DFT + bit reversal (O(n^2))
  blake3: the BLAKE3 spec (chunk chaining, left-balanced tree)
"""
from __future__ import annotations

FIELD_DECL = {  # fid: (modulus, generator, u64 limbs, big-endian repr)
    0: (5102708120182849537, 10, 1, False),
    1: (146823888364060453008360742206866194433, 3, 2, False),
    2: (1697146272512170708389931801544665676545308500647389167617, 5, 3, False),
    3: (46242760681095663677370860714659204618859642560429202607213929836750194081793, 5, 4, False),
    4: (14474011154664524421669271390699307717822958659997404088829842556525106692097, 3, 4, True),
}


class Field:
    def __init__(self, fid: int):
        self.p, self.g, self.nl, self.be = FIELD_DECL[fid]
        self.R = 1 << (64 * self.nl)
        t, s = self.p - 1, 0
        while t % 2 == 0:
            t //= 2
            s += 1
        self.S = s
        self.root = pow(self.g, t, self.p)  # ROOT_OF_UNITY (canonical)

    def to_mont(self, x: int) -> int:
        return x * self.R % self.p

    def from_mont(self, x: int) -> int:
        return x * pow(self.R, -1, self.p) % self.p

    def omega(self, log_n: int) -> int:
        return pow(self.root, 1 << (self.S - log_n), self.p)

    def repr_bytes(self, canonical: int) -> bytes:
        b = canonical.to_bytes(8 * self.nl, "little")
        return b[::-1] if self.be else b


def bitrev(x: int, bits: int) -> int:
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def fft_io_naive(f: Field, xs, omega_inverse: bool = False, bitrev_out: bool = True):
    """out[bitrev(j)] = sum_i x_i w^(ij) on canonical values (the two switches of
    include/lcpc_fft_convention.h: w^-1 instead of w; natural instead of bit-reversed output)."""
    n = len(xs)
    lg = n.bit_length() - 1
    w = f.omega(lg)
    if omega_inverse:
        w = pow(w, -1, f.p)
    out = [0] * n
    for j in range(n):
        wj = pow(w, j, f.p)
        acc, pw = 0, 1
        for x in xs:
            acc = (acc + x * pw) % f.p
            pw = pw * wj % f.p
        out[bitrev(j, lg) if bitrev_out else j] = acc
    return out


# ---------------------------------------------------------------- BLAKE3 (spec)
IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
M32 = 0xFFFFFFFF


def _g(s, a, b, c, d, x, y):
    s[a] = (s[a] + s[b] + x) & M32
    s[d] = ((s[d] ^ s[a]) >> 16 | (s[d] ^ s[a]) << 16) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 12 | (s[b] ^ s[c]) << 20) & M32
    s[a] = (s[a] + s[b] + y) & M32
    s[d] = ((s[d] ^ s[a]) >> 8 | (s[d] ^ s[a]) << 24) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 7 | (s[b] ^ s[c]) << 25) & M32


def compress(cv, block: bytes, counter: int, blen: int, flags: int):
    m = [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]
    s = list(cv) + IV[:4] + [counter & M32, counter >> 32, blen, flags]
    for r in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1]); _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5]); _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9]); _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13]); _g(s, 3, 4, 9, 14, m[14], m[15])
        m = [m[PERM[i]] for i in range(16)]
    return [s[i] ^ s[i + 8] for i in range(8)]


def _chunk_cv(data: bytes, counter: int, root: bool):
    cv = list(IV)
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)] or [b""]
    for i, blk in enumerate(blocks):
        flags = (1 if i == 0 else 0) | (2 | (8 if root else 0) if i == len(blocks) - 1 else 0)
        cv = compress(cv, blk.ljust(64, b"\0"), counter, len(blk), flags)
    return cv


def blake3(data: bytes) -> bytes:
    chunks = [data[i:i + 1024] for i in range(0, len(data), 1024)] or [b""]
    if len(chunks) == 1:
        cv = _chunk_cv(chunks[0], 0, True)
    else:
        stack = []
        for i, ch in enumerate(chunks[:-1]):  # BLAKE3 reference: merge by trailing zeros
            cv = _chunk_cv(ch, i, False)
            total = i + 1
            while total & 1 == 0:
                left = stack.pop()
                cv = compress(IV, b"".join(x.to_bytes(4, "little") for x in left + cv), 0, 64, 4)
                total >>= 1
            stack.append(cv)
        cv = _chunk_cv(chunks[-1], len(chunks) - 1, False)
        while stack:
            left = stack.pop()
            root = not stack
            cv = compress(IV, b"".join(x.to_bytes(4, "little") for x in left + cv), 0, 64, 4 | (8 if root else 0))
    return b"".join(x.to_bytes(4, "little") for x in cv)
