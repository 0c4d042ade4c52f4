"""proof-of-storage producers of the commitment path, restated over liblcpc_mi.so.

Mirrors the functions of the reference's proof-of-storage crate that feed / consume the lcpc-2d
commitment (names kept):
  fields::convert_byte_vec_to_field_elements_vec        fields.rs:109-112, data_field.rs:38-46
  fields::convert_field_elements_vec_to_byte_vec        fields.rs:114-121
  networking::server::get_aspect_ratio_default_from_field_len / _from_file_len
                                                         networking/server.rs:1139-1182
  networking::client::get_column_indicies_from_random_seed   networking/client.rs:443-456
  lcpc_online::{convert_file_data_to_commit, verifiable_polynomial_evaluation, decode_row,
                form_side_vectors_for_polynomial_evaluation_from_point,
                server_retreive_columns, hash_column_to_digest,
                client_online_verify_column_paths}       lcpc_online.rs:80-627
The field is WriteableFt63: the modulus, arithmetic and repr of FT63.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N
from .lcpc2d import (FT63, LcColumn, LcCommit, LigeroEncoding, ProverError, _p64, _raise,
                     limbs, verify_column_path)

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


def server_retreive_columns(comm: LcCommit, requested_columns: Sequence[int]) -> List[LcColumn]:
    return comm.open_columns(list(requested_columns))


def client_online_verify_column_paths(root: bytes, requested_columns: Sequence[int],
                                      received_columns: Sequence[LcColumn], field: int = FT63) -> bool:
    if len(requested_columns) != len(received_columns):
        return False
    return all(verify_column_path(field, c, i, root) for i, c in zip(requested_columns, received_columns))
