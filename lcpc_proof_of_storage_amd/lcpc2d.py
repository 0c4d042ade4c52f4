"""Python mirror of the reference's lcpc-2d / lcpc-ligero-pc API over liblcpc_mi.so.

Reference interface (TrevorGKann/lcpc_proof_of_storage):
  LcEncoding trait              lcpc-2d/src/lib.rs:75-105
  LigeroEncodingRho             lcpc-ligero-pc/src/lib.rs:32-186 (LigeroEncoding = rho 1/2)
  LcCommit::{commit, prove, get_root, get_n_rows, get_n_cols, get_n_per_row}   :285-327
  LcEvalProof::{verify, get_n_cols, get_n_per_row}                             :531-557
  LcColumn {col, path}                                                         :424-433
  ProverError / VerifierError                                                  :113-167
  free functions open_column, merkle_tree, verify_column_path/value,
  collapse_columns, n_degree_tests, log2                                       :642-1154

Field elements are numpy uint64 arrays of shape (n, limbs) in ff_derive's Montgomery form
(bit-identical to the reference's ``struct FtX([u64; N])``).  All compute runs on the GPU
through the C ABI; nothing here does field arithmetic.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass, field as dc_field
from typing import List, Optional

import numpy as np

from . import _native as N

FT63, FT127, FT191, FT255, FT253_192 = 0, 1, 2, 3, 4
FIELD_NAMES = {FT63: "Ft63", FT127: "Ft127", FT191: "Ft191", FT255: "Ft255", FT253_192: "Ft253_192"}

# status codes (include/lcpc_mi.h)
PROVER = {1: "TooBig", 2: "Encode", 3: "Commit", 4: "ColumnNumber", 5: "OuterTensor"}
TRANSCRIPT_CALLBACK = 35  # LCPC_ERR_TRANSCRIPT: a CallerTranscript callback failed
VERIFIER = {10: "NumColOpens", 11: "ColumnPath", 12: "ColumnEval", 13: "ColumnDegree", 14: "OuterTensor",
            15: "InnerTensor", 16: "EncodingDims", 17: "Encode"}
FFT = {20: "NotPowerOfTwo", 21: "TooBig", 22: "WrongSizePrecomp"}


class LcpcError(Exception):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{self.kind} ({code}): {msg}")

    @property
    def kind(self) -> str:
        return {**PROVER, **VERIFIER, **FFT}.get(self.code, "Error")


class ProverError(LcpcError):
    pass


class VerifierError(LcpcError):
    pass


class FFTError(LcpcError):
    pass


class DeviceError(LcpcError):
    pass


def _raise(code: int, cls=None):
    if code == 0:
        return
    msg = N.last_error()
    if cls is None:
        if code in PROVER:
            cls = ProverError
        elif code in VERIFIER:
            cls = VerifierError
        elif code in FFT:
            cls = FFTError
        else:
            cls = DeviceError
    raise cls(code, msg)


def _p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(N.u64p)


def _bytes_ptr(b: bytes):
    buf = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(bytes(b) if len(b) else b"\0")
    return C.cast(buf, N.u8p), buf


def limbs(field: int) -> int:
    return N.load().lcpc_field_limbs(field)


def num_bits(field: int) -> int:
    return N.load().lcpc_field_num_bits(field)


def _elems(a, field: int) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return a.reshape(-1, limbs(field))


def field_random(field: int, n: int, seed: int) -> np.ndarray:
    """n draws of F::random(ChaCha20Rng::seed_from_u64(seed)), shape (n, limbs)."""
    out = np.zeros((n, limbs(field)), np.uint64)
    _raise(N.load().lcpc_field_random(field, seed, _p64(out), n))
    return out


def prof_enable(on: bool = True):
    N.load().lcpc_prof_enable(1 if on else 0)


def prof_reset():
    N.load().lcpc_prof_reset()


def prof_stats() -> dict:
    """{kernel name: (total ms, launches)} recorded with HIP events since the last reset."""
    L = N.load()
    n = L.lcpc_prof_names(None, 0)
    buf = C.create_string_buffer(n + 1)
    L.lcpc_prof_names(buf, n + 1)
    out = {}
    for name in buf.value.decode().split("\n"):
        if not name:
            continue
        ms, cnt = C.c_double(), C.c_uint64()
        L.lcpc_prof_get(name.encode(), C.byref(ms), C.byref(cnt))
        out[name] = (ms.value, cnt.value)
    return out


def selftest_pool_ordering(rounds: int = 8, spin_us: int = 300) -> dict:
    """On-device check of the stream-ordered buffer pool (lcpc_selftest_pool_ordering):
    {"violations": words clobbered across a fence (must be 0), "control_violations": the same
    without the fence, "reused": takes that returned the released block}."""
    v, cv, r = C.c_uint64(), C.c_uint64(), C.c_uint64()
    _raise(N.load().lcpc_selftest_pool_ordering(rounds, spin_us, C.byref(v), C.byref(cv), C.byref(r)))
    return {"violations": v.value, "control_violations": cv.value, "reused": r.value}


def set_device(device: int):
    _raise(N.load().lcpc_set_device(device), DeviceError)


def device_count() -> int:
    return N.load().lcpc_device_count()


# ---------------------------------------------------------------- parameters
def n_degree_tests(lam: int, length: int, flog2: int) -> int:
    """lcpc-2d/src/lib.rs:642-645"""
    return N.load().lcpc_n_degree_tests(lam, length, flog2)


def log2(v: int) -> int:
    """lcpc-2d/src/lib.rs:857-859"""
    return N.load().lcpc_log2(v)


# ---------------------------------------------------------------- transcript
class Transcript:
    """merlin::Transcript (merlin 2.0)."""

    def __init__(self, label: bytes = b"", _h=None):
        L = N.load()
        if _h is None:
            p, keep = _bytes_ptr(label)
            _h = L.lcpc_transcript_new(p, len(label))
        self._h = _h

    def clone(self) -> "Transcript":
        return Transcript(_h=N.load().lcpc_transcript_clone(self._h))

    def append_message(self, label: bytes, message: bytes):
        lp, k1 = _bytes_ptr(label)
        mp, k2 = _bytes_ptr(message)
        N.load().lcpc_transcript_append_message(self._h, lp, len(label), mp, len(message))

    def append_messages(self, label: bytes, messages: bytes, msg_len: int):
        """append_message(label, m) for each msg_len-byte m of `messages` (one call)."""
        if msg_len <= 0 or len(messages) % msg_len:
            raise ValueError("messages must be whole msg_len-byte records")
        lp, k1 = _bytes_ptr(label)
        mp, k2 = _bytes_ptr(messages)
        N.load().lcpc_transcript_append_messages(self._h, lp, len(label), mp, msg_len, len(messages) // msg_len)

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        lp, k1 = _bytes_ptr(label)
        out = (C.c_uint8 * max(n, 1))()
        N.load().lcpc_transcript_challenge_bytes(self._h, lp, len(label), C.cast(out, N.u8p), n)
        return bytes(out)[:n]

    def __del__(self):
        try:
            N.load().lcpc_transcript_free(self._h)
        except Exception:
            pass


class CallerTranscript:
    """A transcript the CALLER owns, driven by prove / verify through lcpc_transcript_ops.

    The reference's prove / verify mutate the caller's ``&mut merlin::Transcript``
    (lcpc-2d/src/lib.rs:319-326, 547-556) and the caller goes on using it.  ``obj`` is any object
    with ``append_message(label, msg)`` and ``challenge_bytes(label, n) -> bytes`` (merlin's
    methods), optionally ``append_messages(label, msgs, msg_len)`` for the prover's batched
    per-coefficient absorption; every absorb and squeeze of the call goes to it, in the
    reference's order.  An exception raised inside a callback fails the call (LCPC_ERR_TRANSCRIPT)
    and is re-raised from prove / verify."""

    def __init__(self, obj):
        self.obj = obj
        self.error: Optional[BaseException] = None

        def guard(fn):
            def cb(*a):
                if self.error is not None:
                    return 1
                try:
                    fn(*a)
                    return 0
                except BaseException as e:  # noqa: BLE001 -- handed back to the caller after the C call
                    self.error = e
                    return 1
            return cb

        def am(ctx, lp, ln, mp, mn):
            obj.append_message(C.string_at(lp, ln), C.string_at(mp, mn))

        def ams(ctx, lp, ln, mp, ml, n):
            label, data = C.string_at(lp, ln), C.string_at(mp, ml * n)
            obj.append_messages(label, data, ml)

        def ch(ctx, lp, ln, dp, n):
            out = bytes(obj.challenge_bytes(C.string_at(lp, ln), n))
            if len(out) != n:
                raise ValueError(f"challenge_bytes returned {len(out)} bytes, {n} asked")
            C.memmove(dp, out, n)

        many = N.TR_APPEND_MANY_FN(guard(ams)) if hasattr(obj, "append_messages") else N.TR_APPEND_MANY_FN()
        self._cbs = (N.TR_APPEND_FN(guard(am)), many, N.TR_CHALLENGE_FN(guard(ch)))
        self._ops = N.TranscriptOps(None, *self._cbs)
        self._h = N.load().lcpc_transcript_from_ops(C.byref(self._ops))
        if not self._h:
            raise LcpcError(30, N.last_error())

    def reraise(self, code: int):
        """after a failed call: the callback's own exception if it caused the failure"""
        if code == 35 and self.error is not None:
            err, self.error = self.error, None
            raise err

    def __del__(self):
        try:
            N.load().lcpc_transcript_free(self._h)
        except Exception:
            pass


def _transcript(tr):
    """the library's Transcript as is; any other transcript object behind CallerTranscript"""
    if isinstance(tr, (Transcript, CallerTranscript)):
        return tr
    return CallerTranscript(tr)


def _call_with_transcript(tr, fn):
    rc = fn(tr._h)
    if isinstance(tr, CallerTranscript):
        tr.reraise(rc)
    _raise(rc)


# ---------------------------------------------------------------- encodings
class LcEncoding:
    """Handle to a GPU-resident encoding (LcEncoding trait, lcpc-2d/src/lib.rs:75-105)."""

    LABEL_DT = b"$l//DT"  # def_labels! (lcpc-2d/src/macros.rs:29-36) never substitutes $l
    LABEL_PR = b"$l//PR"
    LABEL_PE = b"$l//PE"
    LABEL_CO = b"$l//CO"

    def __init__(self, handle):
        self._h = handle
        L = N.load()
        self.field = L.lcpc_encoding_field(handle)

    def __del__(self):
        try:
            N.load().lcpc_encoding_free(self._h)
        except Exception:
            pass

    @property
    def n_per_row(self) -> int:
        return N.load().lcpc_encoding_n_per_row(self._h)

    @property
    def n_cols(self) -> int:
        return N.load().lcpc_encoding_n_cols(self._h)

    def get_dims(self, length: int):
        a, b, c = C.c_size_t(), C.c_size_t(), C.c_size_t()
        N.load().lcpc_encoding_get_dims(self._h, length, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def dims_ok(self, n_per_row: int, n_cols: int) -> bool:
        return bool(N.load().lcpc_encoding_dims_ok(self._h, n_per_row, n_cols))

    def get_n_col_opens(self) -> int:
        return N.load().lcpc_encoding_n_col_opens(self._h)

    def get_n_degree_tests(self) -> int:
        return N.load().lcpc_encoding_n_degree_tests(self._h)

    ROW_KERNEL_AUTO, ROW_KERNEL_FOURSTEP, ROW_KERNEL_ONEPASS = 0, 1, 2

    def set_row_kernel(self, kernel: int):
        """lcpc_encoding_set_row_kernel: the kernel for 2^15-point Ft63 rate-1/2 rows (AUTO: one-pass
        for file images, four-step for element rows; results identical)."""
        _raise(N.load().lcpc_encoding_set_row_kernel(self._h, kernel))
        return self

    def prepare_thread(self, n_rows: int):
        """Pre-allocate the calling thread's pinned staging for prove (lcpc_prepare_thread)."""
        _raise(N.load().lcpc_prepare_thread(self._h, n_rows))

    def reserve(self, length: int, count: int):
        """Pre-allocate device buffers and streams for `count` concurrent commit + prove calls."""
        _raise(N.load().lcpc_reserve(self._h, length, count))

    @property
    def kind(self) -> str:
        return ["rs", "sdig"][N.load().lcpc_encoding_kind(self._h)]

    @property
    def matrix_nnz(self) -> int:
        """Nonzeros of the SDIG code matrices (0 for R-S)."""
        return N.load().lcpc_encoding_matrix_nnz(self._h)

    def encode(self, inp: np.ndarray) -> np.ndarray:
        """LcEncoding::encode: in place on one row of n_cols elements (uint64, C-contiguous)."""
        a = np.asarray(inp)
        if a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
            raise TypeError("encode needs a C-contiguous uint64 array (modified in place)")
        _raise(N.load().lcpc_encode(self._h, _p64(a.reshape(-1)), a.size // limbs(self.field)))
        return a

    def encode_rows(self, rows: np.ndarray) -> np.ndarray:
        """Batched in-place encode of a (n_rows, n_cols, limbs) array."""
        a = np.ascontiguousarray(rows, dtype=np.uint64)
        nl = limbs(self.field)
        a = a.reshape(-1, self.n_cols * nl)
        _raise(N.load().lcpc_encode_rows(self._h, _p64(a), a.shape[0], self.n_cols))
        return a.reshape(-1, self.n_cols, nl)

    def encode_rows_device(self, src_ptr: int, src_stride: int, n_valid: int, dst_ptr: int,
                           dst_stride: int, n_rows: int, stream: int = 0):
        _raise(N.load().lcpc_encode_rows_device(self._h, src_ptr, src_stride, n_valid, dst_ptr,
                                                 dst_stride, n_rows, stream or None))


class LigeroEncoding(LcEncoding):
    """LigeroEncodingRho<F, Rn, Rd> (lcpc-ligero-pc/src/lib.rs:32-186); default rate 1/2."""

    LAMBDA = 128

    @staticmethod
    def _new(fn, *args) -> "LigeroEncoding":
        h = C.c_void_p()
        _raise(fn(*args, C.byref(h)))
        return LigeroEncoding(h.value)

    @classmethod
    def new(cls, field: int, length: int, rho=(1, 2)) -> "LigeroEncoding":
        return cls._new(N.load().lcpc_ligero_new, field, rho[0], rho[1], length)

    @classmethod
    def new_ml(cls, field: int, n_vars: int, rho=(1, 2)) -> "LigeroEncoding":
        return cls._new(N.load().lcpc_ligero_new_ml, field, rho[0], rho[1], n_vars)

    @classmethod
    def new_from_dims(cls, field: int, n_per_row: int, n_cols: int, rho=(1, 2)) -> "LigeroEncoding":
        return cls._new(N.load().lcpc_ligero_new_from_dims, field, rho[0], rho[1], n_per_row, n_cols)

    @staticmethod
    def n_col_opens(rho=(1, 2)) -> int:
        return N.load().lcpc_ligero_n_col_opens(*rho)

    @staticmethod
    def get_dims_for(field: int, length: int, rho=(1, 2)):
        """LigeroEncodingRho::_get_dims (lib.rs:70-112)."""
        a, b, c = C.c_size_t(), C.c_size_t(), C.c_size_t()
        _raise(N.load().lcpc_ligero_get_dims(field, rho[0], rho[1], length, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value


class RsEncoding(LcEncoding):
    """fft_io encoding with explicit soundness counts (lcpc-2d/src/tests.rs:23-121)."""

    @classmethod
    def new(cls, field: int, n_per_row: int, n_cols: int, n_col_opens: int, n_degree_tests: int):
        h = C.c_void_p()
        _raise(N.load().lcpc_rs_encoding_new(field, n_per_row, n_cols, n_col_opens, n_degree_tests, C.byref(h)))
        return cls(h.value)


class SdigEncoding(LcEncoding):
    """SdigEncodingS<F, SdigCodeK> (lcpc-brakedown-pc/src/lib.rs:40-176): Brakedown's expander
    code; `code` K in 1..6 (codespec.rs:169-232), default 3 as the crate's SdigEncoding."""

    @staticmethod
    def _new(fn, *args) -> "SdigEncoding":
        h = C.c_void_p()
        _raise(fn(*args, C.byref(h)))
        return SdigEncoding(h.value)

    @classmethod
    def new(cls, field: int, length: int, seed: int, code: int = 3) -> "SdigEncoding":
        return cls._new(N.load().lcpc_sdig_new, field, code, length, seed)

    @classmethod
    def new_ml(cls, field: int, n_vars: int, seed: int, code: int = 3) -> "SdigEncoding":
        return cls._new(N.load().lcpc_sdig_new_ml, field, code, n_vars, seed)

    @classmethod
    def new_from_dims(cls, field: int, n_per_row: int, n_cols: int, seed: int,
                      code: int = 3) -> "SdigEncoding":
        return cls._new(N.load().lcpc_sdig_new_from_dims, field, code, n_per_row, n_cols, seed)

    @staticmethod
    def n_col_opens(code: int = 3) -> int:
        return N.load().lcpc_sdig_n_col_opens(code)

    @staticmethod
    def n_per_row_for(field: int, length: int, code: int = 3) -> int:
        out = C.c_size_t()
        _raise(N.load().lcpc_sdig_get_n_per_row(field, code, length, C.byref(out)))
        return out.value


# ---------------------------------------------------------------- commitment / proof
# serde + bincode 1.3 encodings of the reference's wrapped types (fixed-width little-endian
# integers, u64 lengths; an element is ff_derive's [u64; N] newtype, i.e. its Montgomery limbs;
# a digest is WrappedOutput { bytes: serde_bytes }, lib.rs:376-381)
_q = struct.Struct("<Q").pack


def _ser_vec_f(a, nl: int) -> bytes:
    a = np.ascontiguousarray(a, dtype="<u8").reshape(-1, nl)
    return _q(a.shape[0]) + a.tobytes()


def _ser_digest(d: bytes) -> bytes:
    return _q(len(d)) + bytes(d)


class _Reader:
    def __init__(self, data: bytes):
        self.data, self.off = data, 0

    def u64(self) -> int:
        if self.off + 8 > len(self.data):
            raise LcpcError(30, "truncated bincode input")
        v = struct.unpack_from("<Q", self.data, self.off)[0]
        self.off += 8
        return v

    def vec_f(self, nl: int) -> np.ndarray:
        n = self.u64()
        if self.off + 8 * n * nl > len(self.data):
            raise LcpcError(30, "truncated bincode input")
        a = np.frombuffer(self.data, dtype="<u8", count=n * nl, offset=self.off).astype(np.uint64).reshape(n, nl)
        self.off += 8 * n * nl
        return a

    def digest(self) -> bytes:
        n = self.u64()
        # Output<Blake3> is a 32-byte GenericArray: collecting another length panics (lib.rs:388-389)
        if n != 32 or self.off + n > len(self.data):
            raise LcpcError(30, "a serialized digest is not 32 bytes")
        d = bytes(self.data[self.off:self.off + n])
        self.off += n
        return d

    def end(self):
        if self.off != len(self.data):
            raise LcpcError(30, "trailing bytes after a serialized value")


class LcRoot:
    """LcRoot<Blake3, E> (lcpc-2d/src/lib.rs:331-422): a commitment root digest, with its serde
    form (WrappedOutput: 8-byte length 32, then the bytes)."""

    def __init__(self, root: bytes):
        if len(root) != 32:
            raise LcpcError(30, "a root is 32 bytes")
        self.root = bytes(root)

    @classmethod
    def new_from_root_digest(cls, root: bytes) -> "LcRoot":
        return cls(root)

    def into_raw(self) -> bytes:
        return self.root

    def as_ref(self) -> bytes:
        return self.root

    def __eq__(self, other) -> bool:
        return isinstance(other, LcRoot) and self.root == other.root

    def to_bincode(self) -> bytes:
        return _ser_digest(self.root)

    @classmethod
    def from_bincode(cls, data: bytes) -> "LcRoot":
        r = _Reader(data)
        root = r.digest()
        r.end()
        return cls(root)


@dataclass
class LcColumn:
    col: np.ndarray          # (n_rows, limbs)
    path: List[bytes]        # log2(n_cols) digests

    def to_bincode(self, field: int) -> bytes:
        """WrappedLcColumn (lib.rs:457-463): col as Vec<F>, path as Vec<WrappedOutput>."""
        return (_ser_vec_f(self.col, limbs(field)) + _q(len(self.path))
                + b"".join(_ser_digest(d) for d in self.path))

    @classmethod
    def from_bincode(cls, field: int, data: bytes) -> "LcColumn":
        r = _Reader(data)
        col = r.vec_f(limbs(field))
        path = [r.digest() for _ in range(r.u64())]
        r.end()
        return cls(col, path)


class LcCommit:
    """LcCommit<Blake3, E> resident in HBM (lcpc-2d/src/lib.rs:174-191, 285-327)."""

    def __init__(self, handle, field: int):
        self._h = handle
        self.field = field

    def __del__(self):
        try:
            N.load().lcpc_commit_free(self._h)
        except Exception:
            pass

    @classmethod
    def commit(cls, coeffs: np.ndarray, enc: LcEncoding) -> "LcCommit":
        a = _elems(coeffs, enc.field)
        h = C.c_void_p()
        _raise(N.load().lcpc_commit_new(enc._h, _p64(a), a.shape[0], C.byref(h)))
        return cls(h.value, enc.field)

    @classmethod
    def commit_device(cls, d_coeffs: int, length: int, enc: LcEncoding) -> "LcCommit":
        h = C.c_void_p()
        _raise(N.load().lcpc_commit_new_device(enc._h, d_coeffs, length, C.byref(h)))
        return cls(h.value, enc.field)

    @classmethod
    def commit_pos_bytes_device(cls, d_bytes: int, n_bytes: int, enc: LcEncoding) -> "LcCommit":
        """the proof-of-storage server's commitment to a file image in device memory:
        DataField::from_byte_vec + LcCommit::commit (lcpc_online.rs:80-239), one call
        (lcpc_pos_commit_bytes_device; WriteableFt63 encodings only)"""
        h = C.c_void_p()
        _raise(N.load().lcpc_pos_commit_bytes_device(enc._h, d_bytes, n_bytes, C.byref(h)))
        return cls(h.value, enc.field)

    @classmethod
    def commit_pos_bytes_device_eval(cls, d_bytes: int, n_bytes: int, enc: LcEncoding, left):
        """one proof-of-storage request's commitment and u^T Enc(M) in one call
        (lcpc_pos_commit_eval_bytes_device; networking/server.rs:670-730): the commitment of
        commit_pos_bytes_device and the n_cols values of pos.verifiable_polynomial_evaluation
        with `left` (n_rows elements), the evaluation summed during the leaf hashing's pass"""
        nl = limbs(enc.field)
        u = np.ascontiguousarray(left, dtype=np.uint64).reshape(-1, nl)
        out = np.zeros((enc.n_cols, nl), np.uint64)
        h = C.c_void_p()
        _raise(N.load().lcpc_pos_commit_eval_bytes_device(enc._h, d_bytes, n_bytes, _p64(u), u.shape[0], _p64(out),
                                                          C.byref(h)))
        return cls(h.value, enc.field), out

    @classmethod
    def commit_pos_bytes(cls, data, enc: LcEncoding) -> "LcCommit":
        """the same commitment from a file image in host memory (lcpc_pos_commit_bytes: the
        server's per-request commit of the file it just read, networking/server.rs:670-679);
        data: bytes or a uint8 array"""
        a = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, np.uint8)
        h = C.c_void_p()
        _raise(N.load().lcpc_pos_commit_bytes(enc._h, a.ctypes.data_as(N.u8p), a.size, C.byref(h)))
        return cls(h.value, enc.field)

    def get_root(self) -> bytes:
        out = (C.c_uint8 * 32)()
        _raise(N.load().lcpc_commit_get_root(self._h, C.cast(out, N.u8p)))
        return bytes(out)

    def to_bincode(self) -> bytes:
        """serde Serialize via WrappedLcCommit (lib.rs:193-283): comm, coeffs (Vec<F>), n_rows,
        n_cols, n_per_row (u64), hashes (Vec<WrappedOutput>)."""
        nl = limbs(self.field)
        h = self.hashes
        return b"".join([_ser_vec_f(self.comm, nl), _ser_vec_f(self.coeffs, nl), _q(self.get_n_rows()),
                         _q(self.get_n_cols()), _q(self.get_n_per_row()), _q(len(h) // 32)]
                        + [_ser_digest(h[i:i + 32]) for i in range(0, len(h), 32)])

    @classmethod
    def from_bincode(cls, field: int, data: bytes) -> "LcCommit":
        """serde Deserialize (WrappedLcCommit::unwrap): the fields loaded into HBM
        (lcpc_commit_from_parts), so prove / open_column work on the result."""
        nl = limbs(field)
        r = _Reader(data)
        comm, coeffs = r.vec_f(nl), r.vec_f(nl)
        n_rows, n_cols, n_per_row = r.u64(), r.u64(), r.u64()
        hashes = b"".join(r.digest() for _ in range(r.u64()))
        r.end()
        if comm.shape[0] != n_rows * n_cols or coeffs.shape[0] != n_rows * n_per_row:
            raise LcpcError(30, "serialized commitment: vector lengths disagree with its dims")
        hp, keep = _bytes_ptr(hashes)
        h = C.c_void_p()
        _raise(N.load().lcpc_commit_from_parts(field, n_rows, n_cols, n_per_row,
                                               _p64(np.ascontiguousarray(comm)), _p64(np.ascontiguousarray(coeffs)),
                                               hp, len(hashes) // 32, C.byref(h)))
        return cls(h.value, field)

    def get_n_rows(self) -> int:
        return N.load().lcpc_commit_n_rows(self._h)

    def get_n_cols(self) -> int:
        return N.load().lcpc_commit_n_cols(self._h)

    def get_n_per_row(self) -> int:
        return N.load().lcpc_commit_n_per_row(self._h)

    @property
    def comm(self) -> np.ndarray:
        out = np.zeros((self.get_n_rows() * self.get_n_cols(), limbs(self.field)), np.uint64)
        _raise(N.load().lcpc_commit_copy_comm(self._h, _p64(out)))
        return out

    @property
    def coeffs(self) -> np.ndarray:
        out = np.zeros((self.get_n_rows() * self.get_n_per_row(), limbs(self.field)), np.uint64)
        _raise(N.load().lcpc_commit_copy_coeffs(self._h, _p64(out)))
        return out

    @property
    def hashes(self) -> bytes:
        n = N.load().lcpc_commit_n_hashes(self._h)
        out = (C.c_uint8 * (32 * n))()
        _raise(N.load().lcpc_commit_copy_hashes(self._h, C.cast(out, N.u8p)))
        return bytes(out)

    def device_comm_ptr(self) -> int:
        return N.load().lcpc_commit_device_comm(self._h)

    def check(self, enc: LcEncoding):
        _raise(N.load().lcpc_check_comm(self._h, enc._h))

    def open_column(self, column: int) -> LcColumn:
        nr, nl = self.get_n_rows(), limbs(self.field)
        pl = log2(self.get_n_cols())
        col = np.zeros((nr, nl), np.uint64)
        path = (C.c_uint8 * max(32 * pl, 1))()
        _raise(N.load().lcpc_open_column(self._h, column, _p64(col), C.cast(path, N.u8p)))
        pb = bytes(path)
        return LcColumn(col, [pb[32 * i:32 * i + 32] for i in range(pl)])

    def open_columns(self, columns) -> List[LcColumn]:
        """open_column for many columns in one device pass."""
        idx = np.ascontiguousarray(list(columns), dtype=np.uint64)
        n = len(idx)
        nr, nl = self.get_n_rows(), limbs(self.field)
        pl = log2(self.get_n_cols())
        cols = np.zeros((max(n, 1), nr, nl), np.uint64)
        paths = (C.c_uint8 * max(32 * pl * n, 1))()
        _raise(N.load().lcpc_open_columns(self._h, _p64(idx) if n else None, n, _p64(cols),
                                          C.cast(paths, N.u8p)))
        pb = bytes(paths)
        return [LcColumn(cols[k].copy(), [pb[32 * (k * pl + i):32 * (k * pl + i + 1)] for i in range(pl)])
                for k in range(n)]

    def prove(self, outer_tensor: np.ndarray, enc: LcEncoding, tr) -> "LcEvalProof":
        """LcCommit::prove (lib.rs:319-326).  tr: the library's Transcript, or the caller's own
        transcript object (CallerTranscript: every absorb / squeeze goes to it)."""
        o = _elems(outer_tensor, self.field)
        h = C.c_void_p()
        tr = _transcript(tr)
        _call_with_transcript(tr, lambda th: N.load().lcpc_prove(self._h, _p64(o), o.shape[0], enc._h, th,
                                                                 C.byref(h)))
        return LcEvalProof(h.value)


class LcEvalProof:
    """LcEvalProof<Blake3, E> (lcpc-2d/src/lib.rs:516-557)."""

    def __init__(self, handle):
        self._h = handle
        L = N.load()
        self.field = L.lcpc_proof_field(handle)
        self.n_cols = L.lcpc_proof_n_cols(handle)
        self.n_per_row = L.lcpc_proof_n_per_row(handle)
        self.n_rows = L.lcpc_proof_n_rows(handle)
        self.n_degree_tests = L.lcpc_proof_n_degree_tests(handle)
        self.n_col_opens = L.lcpc_proof_n_col_opens(handle)
        self.path_len = L.lcpc_proof_path_len(handle)

    def __del__(self):
        try:
            N.load().lcpc_proof_free(self._h)
        except Exception:
            pass

    def get_n_cols(self) -> int:
        return self.n_cols

    def get_n_per_row(self) -> int:
        return self.n_per_row

    @property
    def p_eval(self) -> np.ndarray:
        out = np.zeros((self.n_per_row, limbs(self.field)), np.uint64)
        _raise(N.load().lcpc_proof_copy_p_eval(self._h, _p64(out)))
        return out

    @property
    def p_random_vec(self) -> List[np.ndarray]:
        res = []
        for i in range(self.n_degree_tests):
            out = np.zeros((self.n_per_row, limbs(self.field)), np.uint64)
            _raise(N.load().lcpc_proof_copy_p_random(self._h, i, _p64(out)))
            res.append(out)
        return res

    @property
    def columns(self) -> List[LcColumn]:
        res = []
        nl = limbs(self.field)
        for k in range(self.n_col_opens):
            col = np.zeros((self.n_rows, nl), np.uint64)
            path = (C.c_uint8 * max(32 * self.path_len, 1))()
            _raise(N.load().lcpc_proof_copy_column(self._h, k, _p64(col), C.cast(path, N.u8p)))
            pb = bytes(path)
            res.append(LcColumn(col, [pb[32 * i:32 * i + 32] for i in range(self.path_len)]))
        return res

    @staticmethod
    def _check_shapes(field: int, p_eval, p_random_vec, col_lens, path_lens, digest_lens):
        """A proof from untrusted bytes must be rectangular before its flat buffers reach
        lcpc_proof_from_parts (which copies n_col_opens x n_rows elements, etc.).  The reference
        cannot even represent a digest that is not 32 bytes (Output<Blake3> is a fixed array:
        bincode rejects it); a ragged proof it does represent fails verify (lib.rs:862-982) --
        a short column changes the tensor dot product (ColumnDegree), a long column or a wrong
        path length changes the recomputed root (ColumnPath), a p_random of another length
        changes the absorbed transcript (ColumnDegree).  (A wrong NUMBER of p_random vectors,
        which panics at lib.rs:914 when too few, is rejected by lcpc_verify as EncodingDims.)"""
        n_per_row = _elems(p_eval, field).shape[0]
        if any(int(d) != 32 for d in digest_lens):
            raise LcpcError(30, "malformed proof: a Merkle digest is not 32 bytes")
        if any(_elems(x, field).shape[0] != n_per_row for x in p_random_vec):
            raise VerifierError(13, "malformed proof: p_random length differs from p_eval")
        if col_lens:
            n_rows = col_lens[0]
            if any(n < n_rows for n in col_lens):
                raise VerifierError(13, "malformed proof: ragged columns")
            if any(n > n_rows for n in col_lens):
                raise VerifierError(11, "malformed proof: ragged columns")
            if any(pl != path_lens[0] for pl in path_lens):
                raise VerifierError(11, "malformed proof: Merkle paths of different lengths")

    @classmethod
    def from_parts(cls, field: int, n_cols: int, p_eval, p_random_vec, columns: List[LcColumn]):
        nl = limbs(field)
        cls._check_shapes(field, p_eval, p_random_vec, [_elems(c.col, field).shape[0] for c in columns],
                          [len(c.path) for c in columns], [len(d) for c in columns for d in c.path])
        pe = _elems(p_eval, field)
        pr = np.ascontiguousarray(np.concatenate([_elems(x, field) for x in p_random_vec]) if p_random_vec
                                  else np.zeros((1, nl), np.uint64))
        n_rows = _elems(columns[0].col, field).shape[0] if columns else 0
        path_len = len(columns[0].path) if columns else 0
        cols = np.ascontiguousarray(np.concatenate([_elems(c.col, field) for c in columns]) if columns
                                    else np.zeros((1, nl), np.uint64))
        paths = b"".join(b"".join(c.path) for c in columns)
        pp, keep = _bytes_ptr(paths)
        h = C.c_void_p()
        _raise(N.load().lcpc_proof_from_parts(field, n_cols, pe.shape[0], n_rows, len(p_random_vec), len(columns),
                                              path_len, _p64(pe), _p64(pr), _p64(cols), pp, C.byref(h)))
        return cls(h.value)

    # ---- serialization: bincode 1.3 (fixed-width little-endian integers, u64 lengths) of the
    # reference's WrappedLcEvalProof (lcpc-2d/src/lib.rs:576-590, 457-463, 377-381), the bytes
    # `bincode::serialize(&pf)` produces (lcpc-ligero-pc/src/tests.rs:137): n_cols as u64;
    # p_eval and each p_random as Vec<F>, an element being the serde newtype of ff_derive's
    # [u64; N] (its Montgomery limbs); each column as Vec<F> plus a Vec of serde_bytes digests.
    @staticmethod
    def serialized_size_for(field: int, n_rows: int, n_per_row: int, n_cols: int, n_col_opens: int,
                            n_degree_tests: int) -> int:
        fb = 8 * limbs(field)
        path_len = log2(n_cols)
        return (8 + (8 + n_per_row * fb) + 8 + n_degree_tests * (8 + n_per_row * fb) + 8
                + n_col_opens * ((8 + n_rows * fb) + 8 + path_len * (8 + 32)))

    def to_bincode(self) -> bytes:
        nl = limbs(self.field)
        q = struct.Struct("<Q").pack

        def vec_f(a):
            a = np.ascontiguousarray(a, dtype="<u8").reshape(-1, nl)
            return q(a.shape[0]) + a.tobytes()

        parts = [q(self.n_cols), vec_f(self.p_eval), q(self.n_degree_tests)]
        parts += [vec_f(x) for x in self.p_random_vec]
        cols = self.columns
        parts.append(q(len(cols)))
        for c in cols:
            parts.append(vec_f(c.col))
            parts.append(q(len(c.path)))
            parts += [q(len(d)) + bytes(d) for d in c.path]
        return b"".join(parts)

    @classmethod
    def from_bincode(cls, field: int, data: bytes) -> "LcEvalProof":
        """Inverse of to_bincode (the reference's bincode::deserialize of a proof)."""
        nl = limbs(field)
        off = 0

        def u64():
            nonlocal off
            v = struct.unpack_from("<Q", data, off)[0]
            off += 8
            return v

        def vec_f():
            nonlocal off
            n = u64()
            a = np.frombuffer(data, dtype="<u8", count=n * nl, offset=off).astype(np.uint64).reshape(n, nl)
            off += 8 * n * nl
            return a

        n_cols = u64()
        p_eval = vec_f()
        p_random = [vec_f() for _ in range(u64())]
        columns = []
        for _ in range(u64()):
            col = vec_f()
            path = []
            for _ in range(u64()):
                ln = u64()
                path.append(bytes(data[off:off + ln]))
                off += ln
            columns.append(LcColumn(col, path))
        if off != len(data):
            raise LcpcError(30, "trailing bytes after a serialized proof")  # LCPC_ERR_INVALID_ARG
        return cls.from_parts(field, n_cols, p_eval, p_random, columns)

    @classmethod
    def from_arrays(cls, field: int, n_cols: int, p_eval, p_random_vec, cols, paths):
        """from_parts with the columns as one (n_col_opens, n_rows, limbs) array and the paths
        as one (n_col_opens, path_len, 32) byte array."""
        nl = limbs(field)
        cls._check_shapes(field, p_eval, p_random_vec, [], [], [])
        pe = _elems(p_eval, field)
        pr = np.ascontiguousarray(np.concatenate([_elems(x, field) for x in p_random_vec]) if p_random_vec
                                  else np.zeros((1, nl), np.uint64))
        cols = np.ascontiguousarray(cols, dtype=np.uint64)
        paths = np.ascontiguousarray(paths, dtype=np.uint8)
        nco, n_rows = cols.shape[0], (cols.shape[1] if cols.ndim > 1 else 0)
        path_len = paths.shape[1] if paths.ndim > 1 else 0
        if nco and (cols.ndim != 3 or cols.shape[2] != nl):
            raise LcpcError(30, f"columns must be (n_col_opens, n_rows, {nl}) limbs")
        if nco and (paths.shape[0] != nco or (path_len and (paths.ndim != 3 or paths.shape[2] != 32))):
            raise LcpcError(30, "paths must be (n_col_opens, path_len, 32) bytes")
        if nco == 0:
            cols = np.zeros((1, nl), np.uint64)
            paths = np.zeros(1, np.uint8)
        h = C.c_void_p()
        _raise(N.load().lcpc_proof_from_parts(field, n_cols, pe.shape[0], n_rows, len(p_random_vec), nco, path_len,
                                              _p64(pe), _p64(pr), _p64(cols), paths.ctypes.data_as(N.u8p),
                                              C.byref(h)))
        return cls(h.value)

    def verify(self, root: bytes, outer_tensor, inner_tensor, enc: LcEncoding, tr) -> np.ndarray:
        """LcEvalProof::verify (lib.rs:547-556); tr as for LcCommit.prove."""
        o = _elems(outer_tensor, self.field)
        i = _elems(inner_tensor, self.field)
        rp, keep = _bytes_ptr(root)
        out = np.zeros(limbs(self.field), np.uint64)
        tr = _transcript(tr)
        _call_with_transcript(tr, lambda th: N.load().lcpc_verify(rp, _p64(o), o.shape[0], _p64(i), i.shape[0],
                                                                  self._h, enc._h, th, _p64(out)))
        return out


# ---------------------------------------------------------------- free functions
def collapse_columns(field: int, coeffs, tensor, n_rows: int, n_per_row: int) -> np.ndarray:
    c = _elems(coeffs, field)
    t = _elems(tensor, field)
    out = np.zeros((n_per_row, limbs(field)), np.uint64)
    _raise(N.load().lcpc_collapse_columns(field, _p64(c), _p64(t), _p64(out), n_rows, n_per_row))
    return out


def merkle_tree(ins: bytes) -> bytes:
    n = len(ins) // 32
    ip, keep = _bytes_ptr(ins)
    out = (C.c_uint8 * max(32 * (n - 1), 1))()
    _raise(N.load().lcpc_merkle_tree(ip, n, C.cast(out, N.u8p)))
    return bytes(out)[:32 * (n - 1)]


def hash_columns(field: int, comm, n_rows: int, n_cols: int) -> bytes:
    c = _elems(comm, field)
    out = (C.c_uint8 * (32 * n_cols))()
    _raise(N.load().lcpc_hash_columns(field, _p64(c), n_rows, n_cols, C.cast(out, N.u8p)))
    return bytes(out)


def verify_column_path(field: int, column: LcColumn, col_num: int, root: bytes) -> bool:
    c = _elems(column.col, field)
    pb = b"".join(column.path)
    pp, k1 = _bytes_ptr(pb)
    rp, k2 = _bytes_ptr(root)
    return bool(N.load().lcpc_verify_column_path(field, _p64(c), c.shape[0], pp, len(column.path), col_num, rp))


def verify_column_value(field: int, column: LcColumn, tensor, poly_eval) -> bool:
    c = _elems(column.col, field)
    t = _elems(tensor, field)
    e = _elems(poly_eval, field)
    return bool(N.load().lcpc_verify_column_value(field, _p64(c), _p64(t), c.shape[0], _p64(e)))
