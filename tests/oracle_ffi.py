"""ctypes binding of the TEST ORACLE (oracle/build/liblcpc_oracle.so).

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The oracle is the CPU restatement of the reference path (see
oracle/oracle.h); it is the checker, never the thing measured as the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# LCPC_ORACLE_LIB: an oracle variant (build_variant below) for a whole test run
LIB_PATH = os.environ.get("LCPC_ORACLE_LIB") or os.path.join(ORACLE_DIR, "build", "liblcpc_oracle.so")

FIELDS = {"Ft63": 0, "Ft127": 1, "Ft191": 2, "Ft255": 3, "Ft253_192": 4}
LABEL = {"DT": b"$l//DT", "PR": b"$l//PR", "PE": b"$l//PE", "CO": b"$l//CO"}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _setup(_lib)
    return _lib


def build_variant(name: str, flags: str) -> str:
    """an oracle built with other compile-time switches (e.g. the FFT conventions of
    include/lcpc_fft_convention.h) into oracle/build/<name>/; returns the library path"""
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "variant", f"VARIANT={name}", f"VARIANT_FLAGS={flags}"],
                   check=True)
    return os.path.join(ORACLE_DIR, "build", name, "liblcpc_oracle.so")


class use_lib:
    """with use_lib(path): every wrapper in this module calls that oracle build instead"""

    def __init__(self, path: str):
        self.path = path

    def __enter__(self):
        global _lib
        self.prev = lib()
        v = C.CDLL(self.path)
        _setup(v)
        _lib = v
        return v

    def __exit__(self, *exc):
        global _lib
        _lib = self.prev
        return False


u64p = C.POINTER(C.c_uint64)
u8p = C.POINTER(C.c_uint8)
szp = C.POINTER(C.c_size_t)


class OfCommit(C.Structure):
    _fields_ = [("fid", C.c_int), ("nl", C.c_int), ("n_rows", C.c_size_t), ("n_cols", C.c_size_t),
                ("n_per_row", C.c_size_t), ("n_hashes", C.c_size_t), ("comm", u64p),
                ("coeffs", u64p), ("hashes", u8p)]


class OfProof(C.Structure):
    _fields_ = [("fid", C.c_int), ("nl", C.c_int), ("n_cols", C.c_size_t), ("n_per_row", C.c_size_t),
                ("n_rows", C.c_size_t), ("n_degree_tests", C.c_size_t), ("n_col_opens", C.c_size_t),
                ("path_len", C.c_size_t), ("p_eval", u64p), ("p_random", u64p), ("cols", u64p),
                ("paths", u8p), ("col_idx", u64p)]


class OfEnc(C.Structure):
    _fields_ = [("fid", C.c_int), ("kind", C.c_int), ("n_per_row", C.c_size_t), ("n_cols", C.c_size_t),
                ("n_col_opens", C.c_size_t), ("n_degree_tests", C.c_size_t), ("bd", C.c_void_p)]


def _setup(L):
    sig = {
        "of_field_limbs": (C.c_int, [C.c_int]),
        "of_field_num_bits": (C.c_int, [C.c_int]),
        "of_field_s": (C.c_int, [C.c_int]),
        "of_field_modulus": (None, [C.c_int, u64p]),
        "of_field_root_of_unity": (None, [C.c_int, u64p]),
        "of_from_canonical": (None, [C.c_int, u64p, u64p, C.c_size_t]),
        "of_to_canonical": (None, [C.c_int, u64p, u64p, C.c_size_t]),
        "of_add": (None, [C.c_int, u64p, u64p, u64p, C.c_size_t]),
        "of_sub": (None, [C.c_int, u64p, u64p, u64p, C.c_size_t]),
        "of_mul": (None, [C.c_int, u64p, u64p, u64p, C.c_size_t]),
        "of_to_repr": (None, [C.c_int, u64p, u8p, C.c_size_t]),
        "of_fft_io": (C.c_int, [C.c_int, u64p, C.c_size_t]),
        "of_ifft_oi": (C.c_int, [C.c_int, u64p, C.c_size_t]),
        "of_ntt_omega": (None, [C.c_int, C.c_int, u64p]),
        "of_blake3": (None, [u8p, C.c_size_t, u8p]),
        "of_sha3_256": (None, [u8p, C.c_size_t, u8p]),
        "of_transcript_new": (C.c_void_p, [u8p, C.c_size_t]),
        "of_transcript_clone": (C.c_void_p, [C.c_void_p]),
        "of_transcript_free": (None, [C.c_void_p]),
        "of_transcript_append_message": (None, [C.c_void_p, u8p, C.c_size_t, u8p, C.c_size_t]),
        "of_transcript_challenge_bytes": (None, [C.c_void_p, u8p, C.c_size_t, u8p, C.c_size_t]),
        "of_chacha_from_seed": (C.c_void_p, [u8p, C.c_int]),
        "of_chacha_seed_from_u64": (C.c_void_p, [C.c_uint64, C.c_int]),
        "of_chacha_free": (None, [C.c_void_p]),
        "of_chacha_next_u32": (C.c_uint32, [C.c_void_p]),
        "of_chacha_next_u64": (C.c_uint64, [C.c_void_p]),
        "of_chacha_fill_bytes": (None, [C.c_void_p, u8p, C.c_size_t]),
        "of_chacha_set_stream": (None, [C.c_void_p, C.c_uint64]),
        "of_uniform_usize": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_uint64]),
        "of_gen_range_u32": (C.c_uint32, [C.c_void_p, C.c_uint32, C.c_uint32]),
        "of_field_random": (None, [C.c_int, C.c_void_p, u64p, C.c_size_t]),
        "of_log2": (C.c_size_t, [C.c_size_t]),
        "of_n_degree_tests": (C.c_size_t, [C.c_size_t, C.c_size_t, C.c_size_t]),
        "of_ligero_n_col_opens": (C.c_size_t, [C.c_size_t, C.c_size_t]),
        "of_ligero_get_dims": (C.c_int, [C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, szp, szp, szp]),
        "of_enc_ligero": (C.POINTER(OfEnc), [C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]),
        "of_enc_sdig": (C.POINTER(OfEnc), [C.c_int, C.c_size_t, C.c_size_t, C.c_uint64, C.c_int,
                                           C.c_size_t, C.c_size_t]),
        "of_enc_free": (None, [C.POINTER(OfEnc)]),
        "of_enc_encode": (C.c_int, [C.POINTER(OfEnc), u64p]),
        "of_enc_encode_rows": (C.c_int, [C.POINTER(OfEnc), u64p, C.c_size_t, C.c_size_t, u64p]),
        "of_set_threads": (None, [C.c_int]),
        "of_commit_new": (C.POINTER(OfCommit), [C.POINTER(OfEnc), u64p, C.c_size_t]),
        "of_commit_free": (None, [C.POINTER(OfCommit)]),
        "of_prove": (C.POINTER(OfProof), [C.POINTER(OfCommit), C.POINTER(OfEnc), u64p, C.c_void_p,
                                         C.POINTER(C.c_int)]),
        "of_proof_alloc": (C.POINTER(OfProof), [C.c_int, C.c_size_t, C.c_size_t, C.c_size_t,
                                               C.c_size_t, C.c_size_t, C.c_size_t]),
        "of_proof_free": (None, [C.POINTER(OfProof)]),
        "of_verify": (C.c_int, [u8p, u64p, C.c_size_t, u64p, C.c_size_t, C.POINTER(OfProof),
                                C.POINTER(OfEnc), C.c_void_p, u64p]),
        "of_collapse_columns": (None, [C.c_int, u64p, u64p, u64p, C.c_size_t, C.c_size_t]),
        "of_hash_columns": (None, [C.c_int, u64p, C.c_size_t, C.c_size_t, u8p]),
        "of_merkle_tree": (None, [u8p, C.c_size_t, u8p]),
        "of_open_column": (C.c_int, [C.POINTER(OfCommit), C.c_size_t, u64p, u8p]),
        "of_verify_column_path": (C.c_int, [C.c_int, u64p, C.c_size_t, u8p, C.c_size_t, C.c_size_t, u8p]),
        "of_verify_column_value": (C.c_int, [C.c_int, u64p, u64p, C.c_size_t, u64p]),
        "of_blake3_chunk_cv": (None, [u8p, C.c_size_t, C.c_uint64, C.c_int, u8p]),
        "of_blake3_merge_cvs": (None, [u8p, C.c_size_t, u8p]),
        "of_pos_bytes_to_field": (C.c_size_t, [u8p, C.c_size_t, u64p]),
        "of_pos_field_to_bytes": (None, [u64p, C.c_size_t, u8p, C.c_size_t]),
        "of_pos_default_dims": (None, [C.c_size_t, szp, szp, szp]),
        "of_pos_column_indices": (C.c_size_t, [C.c_uint64, C.c_size_t, C.c_size_t, u64p]),
        "of_pos_side_vectors": (None, [C.c_int, u64p, C.c_size_t, C.c_size_t, u64p, u64p]),
        "of_sdig_n_col_opens": (C.c_size_t, [C.c_int]),
        "of_sdig_new_np": (C.c_size_t, [C.c_int, C.c_int, C.c_size_t]),
        "of_sdig_levels": (C.c_int, [C.POINTER(OfEnc)]),
        "of_sdig_matrix": (C.c_size_t, [C.POINTER(OfEnc), C.c_int, C.c_int, szp, szp, szp, szp, u64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


# ---------------------------------------------------------------- helpers
def p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u64p)


def p8(a):
    if isinstance(a, (bytes, bytearray)):
        buf = (C.c_uint8 * len(a)).from_buffer_copy(bytes(a))
        return C.cast(buf, u8p), buf
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u8p), a


def limbs(fid: int) -> int:
    return lib().of_field_limbs(fid)


def modulus(fid: int) -> int:
    nl = limbs(fid)
    out = np.zeros(nl, np.uint64)
    lib().of_field_modulus(fid, p64(out))
    return ints_from_limbs(out, nl)[0]


def ints_from_limbs(a: np.ndarray, nl: int):
    a = a.reshape(-1, nl)
    return [sum(int(a[i, k]) << (64 * k) for k in range(nl)) for i in range(a.shape[0])]


def limbs_from_ints(vals, nl: int) -> np.ndarray:
    out = np.zeros((len(vals), nl), np.uint64)
    for i, v in enumerate(vals):
        for k in range(nl):
            out[i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    return out.reshape(-1)


def to_mont(fid: int, vals) -> np.ndarray:
    nl = limbs(fid)
    can = limbs_from_ints(vals, nl)
    out = np.zeros_like(can)
    lib().of_from_canonical(fid, p64(can), p64(out), len(vals))
    return out


def from_mont(fid: int, a: np.ndarray):
    nl = limbs(fid)
    a = np.ascontiguousarray(a, dtype=np.uint64)
    out = np.zeros_like(a)
    lib().of_to_canonical(fid, p64(a), p64(out), a.size // nl)
    return ints_from_limbs(out, nl)


def blake3(data: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    ptr, keep = p8(data if len(data) else b"\x00")
    lib().of_blake3(ptr, len(data), out.ctypes.data_as(u8p))
    return out.tobytes()


def sha3_256(data: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    ptr, keep = p8(data if len(data) else b"\x00")
    lib().of_sha3_256(ptr, len(data), out.ctypes.data_as(u8p))
    return out.tobytes()


class Transcript:
    """Merlin transcript (oracle restatement)."""

    def __init__(self, label: bytes = None, _h=None):
        if _h is not None:
            self.h = _h
        else:
            ptr, keep = p8(label)
            self.h = lib().of_transcript_new(ptr, len(label))

    def clone(self):
        return Transcript(_h=lib().of_transcript_clone(self.h))

    def append_message(self, label: bytes, msg: bytes):
        lp, k1 = p8(label)
        mp, k2 = p8(msg if len(msg) else b"\x00")
        lib().of_transcript_append_message(self.h, lp, len(label), mp, len(msg))

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        lp, k1 = p8(label)
        out = np.zeros(max(n, 1), np.uint8)
        lib().of_transcript_challenge_bytes(self.h, lp, len(label), out.ctypes.data_as(u8p), n)
        return out[:n].tobytes()

    def __del__(self):
        try:
            lib().of_transcript_free(self.h)
        except Exception:
            pass


class ChaCha:
    def __init__(self, seed: bytes = None, rounds: int = 20, seed_u64: int = None):
        if seed_u64 is not None:
            self.h = lib().of_chacha_seed_from_u64(seed_u64, rounds)
        else:
            ptr, keep = p8(seed)
            self.h = lib().of_chacha_from_seed(ptr, rounds)

    def next_u32(self):
        return lib().of_chacha_next_u32(self.h)

    def next_u64(self):
        return lib().of_chacha_next_u64(self.h)

    def fill_bytes(self, n):
        out = np.zeros(n, np.uint8)
        lib().of_chacha_fill_bytes(self.h, out.ctypes.data_as(u8p), n)
        return out.tobytes()

    def set_stream(self, s):
        lib().of_chacha_set_stream(self.h, s)

    def uniform(self, low, high):
        return lib().of_uniform_usize(self.h, low, high)

    def gen_range_u32(self, low, high):
        return lib().of_gen_range_u32(self.h, low, high)

    def field_random(self, fid, n):
        out = np.zeros(n * limbs(fid), np.uint64)
        lib().of_field_random(fid, self.h, p64(out), n)
        return out

    def __del__(self):
        try:
            lib().of_chacha_free(self.h)
        except Exception:
            pass


def random_coeffs(fid: int, n: int, seed_u64: int = 0x1CDC2024) -> np.ndarray:
    """F::random draws from ChaCha20Rng::seed_from_u64(seed) (SURVEY §8d synthetic inputs)."""
    return ChaCha(seed_u64=seed_u64).field_random(fid, n)


def fft_io(fid: int, data: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(data.copy(), dtype=np.uint64)
    rc = lib().of_fft_io(fid, p64(a), a.size // limbs(fid))
    if rc:
        raise ValueError(f"FFTError {rc}")
    return a


def ifft_oi(fid: int, data: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(data.copy(), dtype=np.uint64)
    rc = lib().of_ifft_oi(fid, p64(a), a.size // limbs(fid))
    if rc:
        raise ValueError(f"FFTError {rc}")
    return a


def ligero_dims(fid: int, length: int, rho=(1, 2)):
    nr, np_, nc = C.c_size_t(), C.c_size_t(), C.c_size_t()
    ok = lib().of_ligero_get_dims(fid, rho[0], rho[1], length, C.byref(nr), C.byref(np_), C.byref(nc))
    if not ok:
        return None
    return nr.value, np_.value, nc.value


class Encoding:
    def __init__(self, ptr):
        self.ptr = ptr
        e = ptr.contents
        self.fid, self.n_per_row, self.n_cols = e.fid, e.n_per_row, e.n_cols
        self.n_col_opens, self.n_degree_tests = e.n_col_opens, e.n_degree_tests

    @classmethod
    def ligero(cls, fid, n_per_row, n_cols, n_col_opens=None, n_degree_tests=None, rho=(1, 2)):
        L = lib()
        if n_col_opens is None:
            n_col_opens = L.of_ligero_n_col_opens(*rho)
        if n_degree_tests is None:
            n_degree_tests = L.of_n_degree_tests(128, n_cols, L.of_field_num_bits(fid) - 1)
        return cls(L.of_enc_ligero(fid, n_per_row, n_cols, n_col_opens, n_degree_tests))

    @classmethod
    def ligero_new(cls, fid, length, rho=(1, 2)):
        nr, np_, nc = ligero_dims(fid, length, rho)
        return cls.ligero(fid, np_, nc, rho=rho)

    @classmethod
    def sdig(cls, fid, n_per_row, seed, code_id=3, n_cols=0):
        p = lib().of_enc_sdig(fid, n_per_row, n_cols, seed, code_id, 0, 0)
        if not p:
            raise ValueError("sdig dims")
        return cls(p)

    def encode(self, row: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(row.copy(), dtype=np.uint64)
        assert a.size == self.n_cols * limbs(self.fid)
        rc = lib().of_enc_encode(self.ptr, p64(a))
        if rc:
            raise ValueError(f"encode error {rc}")
        return a

    def encode_rows(self, src: np.ndarray, n_rows: int, out: np.ndarray = None) -> np.ndarray:
        """every row's n_per_row leading coefficients (rows n_per_row apart in src) encoded, rows in
        parallel on of_set_threads threads; out: [n_rows][n_cols] limbs"""
        nl = limbs(self.fid)
        s = np.ascontiguousarray(src, dtype=np.uint64).reshape(-1)
        assert s.size >= n_rows * self.n_per_row * nl
        if out is None:
            out = np.empty(n_rows * self.n_cols * nl, np.uint64)
        rc = lib().of_enc_encode_rows(self.ptr, p64(s), self.n_per_row, n_rows, p64(out))
        if rc:
            raise ValueError(f"encode error {rc}")
        return out

    def __del__(self):
        try:
            lib().of_enc_free(self.ptr)
        except Exception:
            pass


class Commit:
    def __init__(self, enc: Encoding, coeffs: np.ndarray):
        coeffs = np.ascontiguousarray(coeffs, dtype=np.uint64)
        nl = limbs(enc.fid)
        self.ptr = lib().of_commit_new(enc.ptr, p64(coeffs), coeffs.size // nl)
        if not self.ptr:
            raise ValueError("commit: bad dimensions")
        c = self.ptr.contents
        self.fid, self.nl = c.fid, c.nl
        self.n_rows, self.n_cols, self.n_per_row, self.n_hashes = c.n_rows, c.n_cols, c.n_per_row, c.n_hashes

    @property
    def comm(self):
        c = self.ptr.contents
        return np.ctypeslib.as_array(c.comm, (self.n_rows * self.n_cols * self.nl,)).copy()

    @property
    def coeffs(self):
        c = self.ptr.contents
        return np.ctypeslib.as_array(c.coeffs, (self.n_rows * self.n_per_row * self.nl,)).copy()

    @property
    def hashes(self):
        c = self.ptr.contents
        return bytes(np.ctypeslib.as_array(c.hashes, (self.n_hashes * 32,)))

    def root(self) -> bytes:
        return self.hashes[-32:]

    def prove(self, enc: Encoding, outer: np.ndarray, tr: Transcript):
        err = C.c_int(0)
        outer = np.ascontiguousarray(outer, dtype=np.uint64)
        p = lib().of_prove(self.ptr, enc.ptr, p64(outer), tr.h, C.byref(err))
        if not p:
            raise ValueError(f"ProverError {err.value}")
        return Proof(p)

    def __del__(self):
        try:
            lib().of_commit_free(self.ptr)
        except Exception:
            pass


class Proof:
    def __init__(self, ptr):
        self.ptr = ptr
        p = ptr.contents
        self.fid, self.nl = p.fid, p.nl
        self.n_cols, self.n_per_row, self.n_rows = p.n_cols, p.n_per_row, p.n_rows
        self.n_degree_tests, self.n_col_opens, self.path_len = p.n_degree_tests, p.n_col_opens, p.path_len

    def _arr(self, name, n, dt=np.uint64):
        return np.ctypeslib.as_array(getattr(self.ptr.contents, name), (max(n, 1),))[:n]

    @property
    def p_eval(self):
        return self._arr("p_eval", self.n_per_row * self.nl)

    @property
    def p_random(self):
        return self._arr("p_random", self.n_degree_tests * self.n_per_row * self.nl)

    @property
    def cols(self):
        return self._arr("cols", self.n_col_opens * self.n_rows * self.nl)

    @property
    def paths(self):
        return self._arr("paths", self.n_col_opens * self.path_len * 32)

    @property
    def col_idx(self):
        return self._arr("col_idx", self.n_col_opens)

    @classmethod
    def from_parts(cls, fid, n_cols, n_per_row, n_rows, p_eval, p_random, cols, paths, ndt, nco, path_len):
        p = lib().of_proof_alloc(fid, n_cols, n_per_row, n_rows, ndt, nco, path_len)
        pr = cls(p)
        pr._arr("p_eval", len(p_eval))[:] = p_eval
        pr._arr("p_random", len(p_random))[:] = p_random
        pr._arr("cols", len(cols))[:] = cols
        pr._arr("paths", len(paths))[:] = paths
        return pr

    def verify(self, root: bytes, outer, inner, enc: Encoding, tr: Transcript):
        outer = np.ascontiguousarray(outer, dtype=np.uint64)
        inner = np.ascontiguousarray(inner, dtype=np.uint64)
        rp, keep = p8(root)
        out = np.zeros(self.nl, np.uint64)
        rc = lib().of_verify(rp, p64(outer), outer.size // self.nl, p64(inner), inner.size // self.nl,
                             self.ptr, enc.ptr, tr.h, p64(out))
        return rc, out

    def __del__(self):
        try:
            lib().of_proof_free(self.ptr)
        except Exception:
            pass


def powers(fid: int, x: np.ndarray, n: int) -> np.ndarray:
    """[1, x, x^2, ...] (n terms), Montgomery form."""
    nl = limbs(fid)
    out = np.zeros(n * nl, np.uint64)
    cur = to_mont(fid, [1])
    for i in range(n):
        out[i * nl:(i + 1) * nl] = cur
        nxt = np.zeros(nl, np.uint64)
        lib().of_mul(fid, p64(cur), p64(np.ascontiguousarray(x)), p64(nxt), 1)
        cur = nxt
    return out


def mul(fid, a, b):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros_like(a)
    lib().of_mul(fid, p64(a), p64(b), p64(out), a.size // limbs(fid))
    return out


def eval_tensors(fid: int, x: np.ndarray, n_per_row: int, n_rows: int):
    """inner = [1, x, ..., x^(n_per_row-1)], outer = [1, xr, xr^2, ...] with xr = x^n_per_row
    (lcpc-ligero-pc/src/tests.rs:234-242)."""
    nl = limbs(fid)
    inner = powers(fid, x, n_per_row)
    xr = mul(fid, x, inner[(n_per_row - 1) * nl:])
    outer = powers(fid, xr, n_rows)
    return inner, outer


def standard_transcript(n_col_opens: int, root: bytes) -> Transcript:
    """Transcript prefix of lcpc-ligero-pc/src/tests.rs:245-247."""
    tr = Transcript(b"test transcript")
    tr.append_message(b"polycommit", root)
    tr.append_message(b"ncols", int(n_col_opens).to_bytes(8, "big"))
    return tr


# ---------------------------------------------------------------- proof-of-storage producers
def pos_bytes_to_field(data: bytes) -> np.ndarray:
    n = (len(data) + 6) // 7
    out = np.zeros(max(n, 1), np.uint64)
    ptr, keep = p8(data if data else b"\x00")
    lib().of_pos_bytes_to_field(ptr, len(data), p64(out))
    return out[:n]


def pos_field_to_bytes(elems: np.ndarray, expected_len: int) -> bytes:
    a = np.ascontiguousarray(elems, dtype=np.uint64).reshape(-1)
    out = np.zeros(max(expected_len, 1), np.uint8)
    lib().of_pos_field_to_bytes(p64(a) if a.size else None, a.size, out.ctypes.data_as(u8p), expected_len)
    return out[:expected_len].tobytes()


def pos_default_dims(field_len: int):
    a, b, c = C.c_size_t(), C.c_size_t(), C.c_size_t()
    lib().of_pos_default_dims(field_len, C.byref(a), C.byref(b), C.byref(c))
    return a.value, b.value, c.value


def pos_column_indices(seed: int, amount: int, max_index: int):
    out = np.zeros(max(amount, 1), np.uint64)
    n = lib().of_pos_column_indices(seed, amount, max_index, p64(out))
    return [int(v) for v in out[:n]]


def pos_side_vectors(fid: int, x: np.ndarray, n_rows: int, n_cols: int):
    nl = limbs(fid)
    left = np.zeros(max(n_rows, 1) * nl, np.uint64)
    right = np.zeros(max(n_cols, 1) * nl, np.uint64)
    lib().of_pos_side_vectors(fid, p64(np.ascontiguousarray(x, dtype=np.uint64)), n_rows, n_cols,
                              p64(left), p64(right))
    return left[:n_rows * nl], right[:n_cols * nl]


def collapse(fid: int, m: np.ndarray, tensor: np.ndarray, n_rows: int, width: int) -> np.ndarray:
    out = np.zeros(width * limbs(fid), np.uint64)
    lib().of_collapse_columns(fid, p64(np.ascontiguousarray(m, dtype=np.uint64)),
                              p64(np.ascontiguousarray(tensor, dtype=np.uint64)), p64(out), n_rows, width)
    return out


def hash_columns(fid: int, m: np.ndarray, n_rows: int, n_cols: int) -> bytes:
    out = np.zeros(32 * n_cols, np.uint8)
    lib().of_hash_columns(fid, p64(np.ascontiguousarray(m, dtype=np.uint64)), n_rows, n_cols,
                          out.ctypes.data_as(u8p))
    return out.tobytes()


# ---------------------------------------------------------------- proof-of-storage encoded files
def pos_encode_file(data: bytes, pre: int, enc: int, row_capacity: int = None):
    """EncodedFileWriter::convert_unencoded_file restated (encoded_file_writer.rs:134-231,
    264-389; column_digest_accumulator.rs:62-118; merkle_tree.rs:14-27): the data's 7-byte
    elements in rows of `pre` (the last row partial), each zero padded to `enc` and Ligero
    encoded (fft_io); the file is column-major with `row_capacity` (default 2 * rows) canonical
    8-byte LE elements per column; leaves = BLAKE3(32 zero bytes || column repr); the tree is
    leaves || parents.  Returns (porenc bytes, tree bytes, rows, capacity)."""
    elems = pos_bytes_to_field(data)
    rows = -(-len(elems) // pre)
    cap = 2 * rows if row_capacity is None else row_capacity
    coder = Encoding.ligero(0, pre, enc, 1, 1)
    comm = np.zeros((rows, enc), np.uint64)
    for r in range(rows):
        row = np.zeros(enc, np.uint64)
        part = elems[r * pre:(r + 1) * pre]
        row[:len(part)] = part
        comm[r] = coder.encode(row)
    canon = np.zeros(rows * enc, np.uint64)
    if rows:
        lib().of_to_canonical(0, p64(np.ascontiguousarray(comm.reshape(-1))), p64(canon), rows * enc)
    img = np.zeros((enc, cap), "<u8")
    img[:, :rows] = canon.reshape(rows, enc).T
    leaves = np.frombuffer(hash_columns(0, comm.reshape(-1) if rows else np.zeros(1, np.uint64), rows, enc),
                           np.uint8).copy()
    parents = np.zeros(32 * (enc - 1), np.uint8)
    lib().of_merkle_tree(leaves.ctypes.data_as(u8p), enc, parents.ctypes.data_as(u8p))
    return img.tobytes(), leaves.tobytes() + parents.tobytes(), rows, cap


def pos_decode_rows(img: bytes, pre: int, enc: int, cap: int, rows: int) -> bytes:
    """EncodedFileReader::decode_to_target_file restated (encoded_file_reader.rs:59-91,
    lcpc_online.rs:568-574): each row gathered from the columns, ifft_oi, first `pre`
    coefficients, 7 data bytes each."""
    a = np.frombuffer(img, "<u8").reshape(enc, cap)
    out = []
    for r in range(rows):
        mont = to_mont(0, [int(v) for v in a[:, r]])
        coeffs = ifft_oi(0, mont)
        out.append(pos_field_to_bytes(coeffs[:pre], 7 * pre))
    return b"".join(out)


def verify_path(leaf: bytes, col: int, path: bytes, root: bytes) -> bool:
    """lcpc-2d verify_column_path's climb (lib.rs:985-1012) from a leaf digest."""
    h = leaf
    for i in range(0, len(path), 32):
        sib = path[i:i + 32]
        h = blake3(h + sib) if col % 2 == 0 else blake3(sib + h)
        col >>= 1
    return h == root
