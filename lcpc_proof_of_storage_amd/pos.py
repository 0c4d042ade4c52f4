"""proof-of-storage producers of the commitment path, restated over liblcpc_mi.so.

Mirrors the functions of the reference's proof-of-storage crate that feed / consume the lcpc-2d
commitment (names kept):
  fields::convert_byte_vec_to_field_elements_vec        fields.rs:109-112, data_field.rs:38-46
  fields::convert_field_elements_vec_to_byte_vec        fields.rs:114-121
  fields::field_generator_iter::FieldGeneratorIter      fields/field_generator_iter.rs:5-55
  fields::{read_file_to_field_elements_vec, stream_file_to_field_elements_vec_sync,
           read_file_path_to_field_elements_vec, field_elements_vec_to_file,
           random_writeable_field_vec, evaluate_field_polynomial_at_point[_with_elevated_degree],
           vector_multiply, is_power_of_two}          fields.rs:25-194
  lcpc_online::dims_ok                                   lcpc_online.rs:71-76
  networking::server::get_aspect_ratio_default_from_field_len / _from_file_len
                                                         networking/server.rs:1139-1182
  networking::client::get_column_indicies_from_random_seed   networking/client.rs:443-456
  lcpc_online::{convert_file_data_to_commit, verifiable_polynomial_evaluation, decode_row,
                form_side_vectors_for_polynomial_evaluation_from_point,
                server_retreive_columns, hash_column_to_digest,
                client_online_verify_column_paths[_without_full_columns],
                client_online_verify_column_leaves, client_verify_commitment[_without_full_columns],
                hash_column_to_digest, hash_field_vec_to_digest, _get_POS_soundness_n_cols,
                verify_proper_partial_polynomial_evaluation, verifiable_full_polynomial_evaluation,
                verify_full_polynomial_evaluation_wrapper_with_single_eval_point}
                                                         lcpc_online.rs:80-627
  lcpc_online::file_handler::left_multiply_unencoded_matrix_by_vector   file_handler.rs:614-638
The field is WriteableFt63: the modulus, arithmetic and repr of FT63.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N
from .lcpc2d import (FT63, VERIFIER, LcColumn, LcCommit, LigeroEncoding, ProverError, VerifierError,
                     _p64, _raise, collapse_columns, limbs, verify_column_path)

WRITTEN_BYTES_WIDTH = 8   # size_of::<WriteableFt63>() (data_field.rs:24)
DATA_BYTE_CAPACITY = 7    # CAPACITY / 8 (data_field.rs:22)


def _u8p(b: bytes):
    buf = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0")
    return C.cast(buf, N.u8p), buf


def convert_byte_vec_to_field_elements_vec(data: bytes) -> np.ndarray:
    """7 LE bytes per element, raw limb (WriteableFt63::from_data_bytes); shape (n, 1)."""
    n = (len(data) + 6) // 7
    out = np.zeros((n, 1), np.uint64)
    p, keep = _u8p(data)
    got = C.c_size_t()
    _raise(N.load().lcpc_pos_bytes_to_field(p, len(data), _p64(out), C.byref(got)))
    return out


def convert_field_elements_vec_to_byte_vec(elems: np.ndarray, expected_length: int) -> bytes:
    a = np.ascontiguousarray(elems, dtype=np.uint64).reshape(-1)
    out = (C.c_uint8 * max(expected_length, 1))()
    _raise(N.load().lcpc_pos_field_to_bytes(_p64(a), a.size, C.cast(out, N.u8p), expected_length))
    return bytes(out)[:expected_length]


class FieldGeneratorIter:
    """FieldGeneratorIter<I, WriteableFt63> (fields/field_generator_iter.rs:5-55): an iterator of
    bytes (ints 0..255, or bytes-like blocks) to field elements, DATA_BYTE_CAPACITY = 7 bytes each,
    the last one zero padded -- the elements convert_byte_vec_to_field_elements_vec gives for the
    same bytes.  Bytes are packed a block at a time by the library (lcpc_pos_bytes_to_field);
    elements come out as uint64 raw limbs.  `byte_blocks()` hands a consumer the remaining bytes
    themselves in blocks of whole elements (RowGeneratorIter's digest path)."""

    BLOCK = DATA_BYTE_CAPACITY * 65536

    def __init__(self, inner):
        if isinstance(inner, (bytes, bytearray, memoryview)):
            mv = memoryview(inner).cast("B")
            inner = (bytes(mv[i:i + self.BLOCK]) for i in range(0, len(mv), self.BLOCK))
        self._inner = iter(inner)
        self._carry = b""          # bytes read but not yet packed (fewer than a whole block)
        self._elems = np.zeros(0, np.uint64)
        self._pos = 0
        self._done = False

    def _read(self, want: int) -> bytes:
        """Up to `want` bytes (fewer only at the end of the input)."""
        parts, have = [self._carry], len(self._carry)
        while have < want and not self._done:
            try:
                x = next(self._inner)
            except StopIteration:
                self._done = True
                break
            b = bytes(x) if isinstance(x, (bytes, bytearray, memoryview)) else bytes((x,))
            parts.append(b)
            have += len(b)
        buf = b"".join(parts)
        self._carry = buf[want:]
        return buf[:want]

    def __iter__(self):
        return self

    def __next__(self) -> np.uint64:
        if self._pos == self._elems.size:
            block = self._read(self.BLOCK)
            if not block:
                raise StopIteration
            self._elems = convert_byte_vec_to_field_elements_vec(block).reshape(-1)
            self._pos = 0
        v = self._elems[self._pos]
        self._pos += 1
        return v

    def byte_blocks(self):
        """The rest of the input as bytes: first the elements already packed but not yet taken
        (7 little-endian bytes each), then the unread bytes in blocks."""
        if self._pos < self._elems.size:
            rest = self._elems[self._pos:]
            self._pos = self._elems.size
            yield rest.astype("<u8").view(np.uint8).reshape(-1, 8)[:, :DATA_BYTE_CAPACITY].tobytes()
        while True:
            block = self._read(self.BLOCK)
            if not block:
                return
            yield block


def read_file_to_field_elements_vec(file) -> tuple:
    """fields.rs:25-35: (bytes read, elements) of a whole binary file object."""
    data = file.read()
    return len(data), convert_byte_vec_to_field_elements_vec(data)


def stream_file_to_field_elements_vec_sync(file) -> tuple:
    """fields.rs:72-106: the same elements, read in buffers of 1000 whole elements (7000 bytes,
    the reference's BufReader size), each buffer packed by the library.  (file size, elements)."""
    buf = 1000 * DATA_BYTE_CAPACITY
    parts, total = [], 0
    while True:
        b = file.read(buf)
        if not b:
            break
        total += len(b)
        parts.append(convert_byte_vec_to_field_elements_vec(b))
    return total, (np.concatenate(parts) if parts else np.zeros((0, 1), np.uint64))


def read_file_path_to_field_elements_vec(path: str) -> np.ndarray:
    """fields.rs:122-127."""
    with open(path, "rb") as f:
        return read_file_to_field_elements_vec(f)[1]


def field_elements_vec_to_file(path: str, field_elements) -> None:
    """fields.rs:129-146: each element's 7 data bytes in turn; the last element's trailing zero
    bytes are dropped (an empty vector gives an empty file)."""
    a = np.ascontiguousarray(field_elements, dtype=np.uint64).reshape(-1)
    data = convert_field_elements_vec_to_byte_vec(a, a.size * DATA_BYTE_CAPACITY) if a.size else b""
    if a.size:
        head, last = data[:-DATA_BYTE_CAPACITY], data[-DATA_BYTE_CAPACITY:].rstrip(b"\0")
        data = head + last
    with open(path, "wb") as f:
        f.write(data)


def random_writeable_field_vec(log_len: int, seed: int = 0) -> np.ndarray:
    """fields.rs:148-158: 7 * 2^log_len random bytes packed to 2^log_len elements (the
    reference draws them from a thread RNG; here a seeded one)."""
    data = np.random.default_rng(seed).integers(0, 256, DATA_BYTE_CAPACITY << log_len, dtype=np.uint8).tobytes()
    return convert_byte_vec_to_field_elements_vec(data)


def is_power_of_two(x: int) -> bool:
    """fields.rs:192-194 (true for 0, as x & (x - 1) is)."""
    return x & (x - 1) == 0 if x else True


def dims_ok(num_pre_encoded_columns: int, num_encoded_columns: int) -> bool:
    """lcpc_online.rs:71-76: a power-of-two width >= 2, >= 1 column, rate at most 1/2."""
    return (num_encoded_columns > 0 and num_encoded_columns & (num_encoded_columns - 1) == 0
            and num_pre_encoded_columns >= 1 and num_encoded_columns >= 2
            and num_encoded_columns >= 2 * num_pre_encoded_columns)


def get_aspect_ratio_default_from_field_len(field_len: int):
    """(num_pre_encoded_columns, num_encoded_matrix_columns, soundness)."""
    a, b, c = C.c_size_t(), C.c_size_t(), C.c_size_t()
    N.load().lcpc_pos_default_dims(field_len, C.byref(a), C.byref(b), C.byref(c))
    return a.value, b.value, c.value


def get_aspect_ratio_default_from_file_len(file_len: int):
    return get_aspect_ratio_default_from_field_len(-(-file_len // WRITTEN_BYTES_WIDTH))


def get_column_indicies_from_random_seed(random_seed: int, number_of_columns_to_extract: int,
                                         max_column_index: int) -> List[int]:
    out = np.zeros(max(number_of_columns_to_extract, 1), np.uint64)
    n = C.c_size_t()
    _raise(N.load().lcpc_pos_column_indices(random_seed, number_of_columns_to_extract, max_column_index,
                                            _p64(out), C.byref(n)))
    return [int(v) for v in out[:n.value]]


def form_side_vectors_for_polynomial_evaluation_from_point(evaluation_point: np.ndarray, n_rows: int,
                                                           n_cols: int, field: int = FT63):
    """(left, right): left = [1, x^n_cols, ...] (n_rows), right = [1, x, ...] (n_cols)."""
    nl = limbs(field)
    x = np.ascontiguousarray(evaluation_point, dtype=np.uint64).reshape(-1)[:nl].copy()
    left = np.zeros((max(n_rows, 1), nl), np.uint64)
    right = np.zeros((max(n_cols, 1), nl), np.uint64)
    _raise(N.load().lcpc_pos_side_vectors(field, _p64(x), n_rows, n_cols, _p64(left), _p64(right)))
    return left[:n_rows], right[:n_cols]


def verifiable_polynomial_evaluation(commitment: LcCommit, left_evaluation_column) -> np.ndarray:
    """u^T Enc(M): n_cols results over the encoded matrix (lcpc_online.rs:454-484)."""
    u = np.ascontiguousarray(left_evaluation_column, dtype=np.uint64).reshape(-1, limbs(commitment.field))
    out = np.zeros((commitment.get_n_cols(), limbs(commitment.field)), np.uint64)
    _raise(N.load().lcpc_pos_eval_encoded(commitment._h, _p64(u), u.shape[0], _p64(out)))
    return out


def ifft_oi_rows(rows: np.ndarray, field: int = FT63) -> np.ndarray:
    """fffft::ifft_oi on every row of a (n_rows, len, limbs) or (len, limbs) array."""
    nl = limbs(field)
    a = np.ascontiguousarray(rows, dtype=np.uint64).copy()
    shape = a.shape
    a2 = a.reshape(-1, (a.size // nl) if a.ndim <= 2 else shape[-2] * nl)
    length = a2.shape[1] // nl
    _raise(N.load().lcpc_ifft_oi_rows(field, _p64(a2), a2.shape[0], length))
    return a2.reshape(shape)


def decode_row(row: np.ndarray, field: int = FT63) -> np.ndarray:
    """lcpc_online::decode_row = ifft_oi (lcpc_online.rs:568-574)."""
    return ifft_oi_rows(row, field)


# ---------------------------------------------------------------- convert_file_data_to_commit
@dataclass
class Commit:
    pass


@dataclass
class Leaves:
    columns: Sequence[int]


@dataclass
class ColumnsWithPath:
    columns: Sequence[int]


@dataclass
class ColumnsWithoutPath:
    columns: Sequence[int]


@dataclass
class Specified:
    num_pre_encoded_columns: int
    num_encoded_columns: int


class Square:
    pass


def commit_dimensions(data_len: int, dims) -> tuple:
    """The (num_pre_encoded_columns, num_encoded_columns) of convert_file_data_to_commit
    (lcpc_online.rs:91-132), with its `ensure!` checks as ProverError(Commit)."""
    if data_len <= 0:
        raise ValueError("Cannot convert empty file to commit")
    if isinstance(dims, Specified):
        np_, nc = dims.num_pre_encoded_columns, dims.num_encoded_columns
        if np_ < 1 or nc < 2 or nc & (nc - 1) or not nc > np_:
            raise ValueError(f"bad commit dimensions {np_}/{nc}")
        return np_, nc
    w = math.ceil(float(np.sqrt(np.float32(data_len))))  # (data_len as f32).sqrt().ceil()
    np_ = w if (w & (w - 1)) == 0 else 1 << (w - 1).bit_length()
    nc = 1 << np_.bit_length()  # (np + 1).next_power_of_two()
    return np_, nc


def convert_file_data_to_commit(field_data: np.ndarray, what_to_extract, dimensions):
    """Commit -> LcCommit; Leaves -> list of 32-byte digests; ColumnsWithPath -> [LcColumn];
    ColumnsWithoutPath -> (n, n_rows, limbs) array."""
    data = np.ascontiguousarray(field_data, dtype=np.uint64).reshape(-1, limbs(FT63))
    np_, nc = commit_dimensions(data.shape[0], dimensions)
    enc = LigeroEncoding.new_from_dims(FT63, np_, nc)
    if isinstance(what_to_extract, Commit):
        return LcCommit.commit(data, enc)
    if isinstance(what_to_extract, ColumnsWithPath):
        comm = LcCommit.commit(data, enc)
        return comm.open_columns(list(what_to_extract.columns))
    idx = np.ascontiguousarray(list(what_to_extract.columns), dtype=np.uint64)
    n_rows = -(-data.shape[0] // np_)
    nl = limbs(FT63)
    cols = np.zeros((max(len(idx), 1), n_rows, nl), np.uint64)
    leaves = (C.c_uint8 * max(32 * len(idx), 1))()
    want_leaves = isinstance(what_to_extract, Leaves)
    _raise(N.load().lcpc_pos_columns(enc._h, _p64(data), data.shape[0], _p64(idx) if len(idx) else None,
                                     len(idx), _p64(cols),
                                     C.cast(leaves, N.u8p) if want_leaves else None))
    if want_leaves:
        b = bytes(leaves)
        return [b[32 * i:32 * i + 32] for i in range(len(idx))]
    return cols[:len(idx)]


def vector_multiply(a, b, field: int = FT63) -> np.ndarray:
    """fields.rs:188-190 = field_dot."""
    return field_dot(a, b, field)


def evaluate_field_polynomial_at_point_with_elevated_degree(field_elements, point, degree_offset: int,
                                                            field: int = FT63) -> np.ndarray:
    """fields.rs:172-186: sum_i c_i x^(i + degree_offset), on the GPU (the powers from
    lcpc_pos_side_vectors, the sum a one-column collapse)."""
    nl = limbs(field)
    c = np.ascontiguousarray(field_elements, dtype=np.uint64).reshape(-1, nl)
    n = c.shape[0]
    if n == 0:
        return np.zeros((1, nl), np.uint64)
    # left = [1, x^d] (n_rows 2, n_cols d) gives x^d; right = [1, x, ..., x^(n-1)]
    _, right = form_side_vectors_for_polynomial_evaluation_from_point(point, 1, n, field)
    v = field_dot(c, right, field)
    if degree_offset:
        left, _ = form_side_vectors_for_polynomial_evaluation_from_point(point, 2, degree_offset, field)
        v = field_dot(v, left[1], field)
    return v


def evaluate_field_polynomial_at_point(field_elements, point, field: int = FT63) -> np.ndarray:
    """fields.rs:160-170: sum_i c_i x^i (coefficients little-endian: c_0 first)."""
    return evaluate_field_polynomial_at_point_with_elevated_degree(field_elements, point, 0, field)


def server_retreive_columns(comm: LcCommit, requested_columns: Sequence[int]) -> List[LcColumn]:
    return comm.open_columns(list(requested_columns))


def field_dot(a, b, field: int = FT63) -> np.ndarray:
    """fields::vector_multiply (fields.rs): sum_i a[i] b[i], on the GPU (a one-column collapse)."""
    nl = limbs(field)
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1))
    b = np.ascontiguousarray(np.asarray(b, dtype=np.uint64).reshape(-1))
    n = min(a.size, b.size) // nl
    if n == 0:
        return np.zeros((1, nl), np.uint64)
    return collapse_columns(field, a[:n * nl], b[:n * nl], n, 1)


def _verifier_error(kind: str, msg: str) -> VerifierError:
    code = {v: k for k, v in VERIFIER.items()}[kind]
    return VerifierError(code, msg)


def client_online_verify_column_paths(root: bytes, requested_columns: Sequence[int],
                                      received_columns: Sequence[LcColumn], field: int = FT63) -> None:
    """lcpc_online.rs:251-277: every received column's Merkle path leads to root.
    Raises VerifierError(ColumnEval) otherwise, as the reference's Err."""
    if len(requested_columns) != len(received_columns):
        raise _verifier_error("ColumnEval", "column count")
    if not received_columns:
        return
    leaves = hash_columns_to_digests(received_columns, field)
    client_online_verify_column_paths_without_full_columns(
        root, requested_columns, leaves, [c.path for c in received_columns])


def client_online_verify_column_paths_without_full_columns(
        root: bytes, requested_columns: Sequence[int], received_columns_digests: Sequence[bytes],
        received_column_paths: Sequence[Sequence[bytes]]) -> None:
    """lcpc_online.rs:280-318 (the paths checked on the GPU in one launch)."""
    n = len(requested_columns)
    if len(received_column_paths) != n or len(received_columns_digests) < n:
        raise _verifier_error("ColumnEval", "column count")
    if n == 0:
        return
    plen = len(received_column_paths[0])
    if any(len(p) != plen for p in received_column_paths):
        raise _verifier_error("ColumnEval", "path lengths differ")
    # untrusted server data: every digest is exactly one BLAKE3 output (the reference's
    # Output<Blake3> is a fixed 32-byte array, so anything else never deserializes)
    if any(len(d) != 32 for d in received_columns_digests[:n]) or \
            any(len(d) != 32 for p in received_column_paths for d in p):
        raise _verifier_error("ColumnEval", "digest is not 32 bytes")
    leaves = np.frombuffer(b"".join(received_columns_digests[:n]), np.uint8).copy()
    paths = np.frombuffer(b"".join(b"".join(p) for p in received_column_paths) or b"\0", np.uint8).copy()
    idx = np.ascontiguousarray(np.array(requested_columns, dtype=np.uint64))
    ok = np.zeros(n, np.uint8)
    rp, keep = _u8p(root)
    _raise(N.load().lcpc_verify_leaf_paths(leaves.ctypes.data_as(N.u8p), paths.ctypes.data_as(N.u8p), n, plen,
                                           _p64(idx), rp, ok.ctypes.data_as(N.u8p)))
    if not ok.all():
        raise _verifier_error("ColumnEval", "Merkle path mismatch")


def hash_field_vec_to_digest(column, field: int = FT63) -> bytes:
    """lcpc_online.rs:439-452: BLAKE3(32 zero bytes || repr of every element)."""
    return hash_columns_to_digests([column], field)[0]


def hash_column_to_digest(column: LcColumn, field: int = FT63) -> bytes:
    """lcpc_online.rs:431-437."""
    return hash_field_vec_to_digest(column.col, field)


def hash_columns_to_digests(columns, field: int = FT63) -> List[bytes]:
    """hash_column_to_digest over many columns in one GPU launch."""
    cols = [np.ascontiguousarray(getattr(c, "col", c), dtype=np.uint64).reshape(-1) for c in columns]
    if not cols:
        return []
    n_rows = cols[0].size // limbs(field)
    if any(c.size != cols[0].size for c in cols):
        raise ValueError("columns of different lengths")
    m = np.ascontiguousarray(np.concatenate(cols)) if n_rows else np.zeros(1, np.uint64)
    out = np.zeros(32 * len(cols), np.uint8)
    _raise(N.load().lcpc_hash_field_columns(field, _p64(m), n_rows, len(cols), out.ctypes.data_as(N.u8p)))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(len(cols))]


def client_online_verify_column_leaves(locally_derived_column_leaves: Sequence[bytes],
                                       requested_columns: Sequence[int],
                                       received_column_leaves: Sequence[bytes]) -> None:
    """lcpc_online.rs:321-356 (errors are NumColOpens there, kept)."""
    if (len(locally_derived_column_leaves) != len(requested_columns)
            or len(received_column_leaves) != len(requested_columns)):
        raise _verifier_error("NumColOpens", "leaf count")
    if any(bytes(a) != bytes(b) for a, b in zip(locally_derived_column_leaves, received_column_leaves)):
        raise _verifier_error("NumColOpens", "leaf mismatch")


def _get_POS_soundness_n_cols(pre_encoded_columns: int, encoded_columns: int) -> int:  # noqa: N802
    """lcpc_online.rs:363-368 (f64 arithmetic as in Rust)."""
    den = math.log2((1.0 + pre_encoded_columns / encoded_columns) / 2.0)
    return min(math.ceil(-128.0 / den), encoded_columns)


def get_PoS_soudness_n_cols(num_columns: int, num_encoded_columns: int) -> int:  # noqa: N802
    """lcpc_online.rs:359-361 (FileMetadata's two widths passed directly)."""
    return _get_POS_soundness_n_cols(num_columns, num_encoded_columns)


def client_verify_commitment(root: bytes, locally_derived_column_leaves: Sequence[bytes],
                             requested_columns: Sequence[int], received_columns: Sequence[LcColumn],
                             required_columns_for_soundness: int, field: int = FT63) -> None:
    """lcpc_online.rs:370-398: the received columns hash to the locally derived leaves and their
    paths lead to root."""
    if (required_columns_for_soundness < len(locally_derived_column_leaves)
            or required_columns_for_soundness < len(requested_columns)
            or required_columns_for_soundness < len(received_columns)):
        raise _verifier_error("NumColOpens", "more columns than the soundness count")
    received_leaves = hash_columns_to_digests(received_columns, field)
    client_online_verify_column_leaves(locally_derived_column_leaves, requested_columns, received_leaves)
    client_online_verify_column_paths(root, requested_columns, received_columns, field)


def client_verify_commitment_without_full_columns(root: bytes, locally_derived_column_leaves: Sequence[bytes],
                                                  requested_columns: Sequence[int],
                                                  received_column_digests: Sequence[bytes],
                                                  received_column_paths: Sequence[Sequence[bytes]],
                                                  required_columns_for_soundness: int) -> None:
    """lcpc_online.rs:400-429."""
    if (required_columns_for_soundness < len(locally_derived_column_leaves)
            or required_columns_for_soundness < len(requested_columns)
            or required_columns_for_soundness < len(received_column_digests)):
        raise _verifier_error("NumColOpens", "more columns than the soundness count")
    client_online_verify_column_leaves(locally_derived_column_leaves, requested_columns, received_column_digests)
    client_online_verify_column_paths_without_full_columns(root, requested_columns, received_column_digests,
                                                           received_column_paths)


def verify_proper_partial_polynomial_evaluation(left_evaluation_column, evaluation_result_vector,
                                                requested_columns_indices: Sequence[int],
                                                received_columns: Sequence[LcColumn],
                                                field: int = FT63) -> None:
    """lcpc_online.rs:487-516: vector_multiply(left, column) == the result entry of that column.
    As in the reference, the result entries are taken in increasing column index (the filter
    over the result vector) and zipped with the columns in the order received."""
    nl = limbs(field)
    res = np.ascontiguousarray(np.asarray(evaluation_result_vector, dtype=np.uint64).reshape(-1))
    n_res = res.size // nl
    wanted = set(int(i) for i in requested_columns_indices)
    picked = [i for i in range(n_res) if i in wanted]
    k = min(len(received_columns), len(picked))
    if k == 0:
        return
    cols = np.ascontiguousarray(np.concatenate(
        [np.asarray(getattr(c, "col", c), dtype=np.uint64).reshape(-1) for c in received_columns[:k]]))
    n_rows = cols.size // nl // k
    left = np.ascontiguousarray(np.asarray(left_evaluation_column, dtype=np.uint64).reshape(-1))
    if left.size // nl < n_rows:
        raise _verifier_error("ColumnEval", "left vector shorter than the columns")
    idx = np.array(picked[:k], dtype=np.uint64)
    ok = np.zeros(k, np.uint8)
    _raise(N.load().lcpc_verify_column_values(field, _p64(cols), k, n_rows, _p64(left), _p64(res), n_res,
                                              _p64(idx), ok.ctypes.data_as(N.u8p)))
    if not ok.all():
        raise _verifier_error("ColumnEval", "column value mismatch")


def verifiable_full_polynomial_evaluation(left_evaluation_column, right_evaluation_column,
                                          received_decoded_result_vector, requested_column_indices,
                                          received_columns, pre_encoded_len: int, encoded_len: int,
                                          field: int = FT63):
    """lcpc_online.rs:519-543.  The reference body does not compile as written (it passes an
    undefined `received_result_vector`); this restates its evident intent: the result is
    <decoded u^T M, right>, and the decoded vector re-encoded (Enc(u^T M) = u^T Enc(M)) must
    agree with u^T col at every opened column.  Parity unpinned (no reference output exists)."""
    nl = limbs(field)
    dec = np.ascontiguousarray(np.asarray(received_decoded_result_vector, dtype=np.uint64).reshape(-1, nl))
    right = np.ascontiguousarray(np.asarray(right_evaluation_column, dtype=np.uint64).reshape(-1, nl))
    result = field_dot(dec[:pre_encoded_len], right[:pre_encoded_len], field)
    enc = LigeroEncoding.new_from_dims(field, pre_encoded_len, encoded_len)
    row = np.zeros((encoded_len, nl), np.uint64)
    row[:min(pre_encoded_len, dec.shape[0])] = dec[:pre_encoded_len]
    encoded = enc.encode(row)
    verify_proper_partial_polynomial_evaluation(left_evaluation_column, encoded, requested_column_indices,
                                                received_columns, field)
    return result


def verify_full_polynomial_evaluation_wrapper_with_single_eval_point(
        evaluation_point, received_result_vector, n_rows: int, n_cols: int, requested_column_indices,
        received_columns, pre_encoded_len: int, field: int = FT63):
    """lcpc_online.rs:545-566 (side vectors from the point, then the check above)."""
    left, right = form_side_vectors_for_polynomial_evaluation_from_point(evaluation_point, n_rows, n_cols, field)
    return verifiable_full_polynomial_evaluation(left, right, received_result_vector, requested_column_indices,
                                                 received_columns, pre_encoded_len, n_cols, field)


def left_multiply_unencoded_matrix_by_vector(data: bytes, pre_encoded_size: int, left_vector) -> np.ndarray:
    """file_handler.rs:614-638: u^T M over the file's unencoded rows (7 bytes per element, rows of
    pre_encoded_size).  The reference returns an empty vector (its result is `with_capacity`
    and never resized); this returns the sum it is written to accumulate."""
    el = convert_byte_vec_to_field_elements_vec(data).reshape(-1)
    n_rows = -(-el.size // pre_encoded_size)
    left = np.ascontiguousarray(np.asarray(left_vector, dtype=np.uint64).reshape(-1))
    if left.size != n_rows:
        raise ValueError(f"left_vector incorrect size, expected {n_rows} and received {left.size}")
    m = np.zeros(n_rows * pre_encoded_size, np.uint64)
    m[:el.size] = el
    return collapse_columns(FT63, m, left, n_rows, pre_encoded_size)
