"""ctypes binding of liblcpc_mi.so (include/lcpc_mi.h).

The shared library is built in-tree (``make -C lcpc_proof_of_storage_amd``) and loaded from
this package directory.  There is no fallback: if the library or a HIP device is missing,
every compute call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
# LCPC_MI_LIB: another in-tree build of the same sources (e.g. an FFT-convention variant,
# tools/gpu/fft_variant_check.sh); the default is the shipped library
LIB_PATH = os.environ.get("LCPC_MI_LIB") or os.path.join(PKG_DIR, "liblcpc_mi.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "lcpc_mi.h")

_lib = None

u64p = C.POINTER(C.c_uint64)
u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
szp = C.POINTER(C.c_size_t)
vp = C.c_void_p
sz = C.c_size_t
i32 = C.c_int

# caller-supplied collectives of lcpc_comm_from_ops and the transcript factory of
# lcpc_sharded_commit_prove_many (include/lcpc_mi.h)
ALL_GATHER_FN = C.CFUNCTYPE(C.c_int, vp, vp, vp, sz)
ALL_TO_ALL_V_FN = C.CFUNCTYPE(C.c_int, vp, vp, szp, vp, szp)
BROADCAST_FN = C.CFUNCTYPE(C.c_int, vp, vp, sz, C.c_int)
MAKE_TRANSCRIPT_FN = C.CFUNCTYPE(vp, vp, sz, u8p)
# lcpc_transcript_ops: a caller-owned transcript's absorb / squeeze callbacks
TR_APPEND_FN = C.CFUNCTYPE(C.c_int, vp, u8p, sz, u8p, sz)
TR_APPEND_MANY_FN = C.CFUNCTYPE(C.c_int, vp, u8p, sz, u8p, sz, sz)
TR_CHALLENGE_FN = C.CFUNCTYPE(C.c_int, vp, u8p, sz, u8p, sz)


class P2pRecord(C.Structure):
    """lcpc_p2p_record (include/lcpc_mi.h)"""
    _fields_ = [("tick", C.c_uint32), ("pos", C.c_uint32), ("poly", C.c_uint32), ("stage", C.c_uint32),
                ("is_send", C.c_int32), ("peer", C.c_int32), ("bytes", C.c_uint64)]


class TranscriptOps(C.Structure):
    """lcpc_transcript_ops (include/lcpc_mi.h)"""
    _fields_ = [("ctx", vp), ("append_message", TR_APPEND_FN), ("append_messages", TR_APPEND_MANY_FN),
                ("challenge_bytes", TR_CHALLENGE_FN)]


class CommOps(C.Structure):
    _fields_ = [("user", vp), ("all_gather", ALL_GATHER_FN), ("all_to_all_v", ALL_TO_ALL_V_FN),
                ("broadcast", BROADCAST_FN)]


# name: (restype, argtypes)
SIGNATURES = {
    "lcpc_abi_version": (i32, []),
    "lcpc_last_error": (C.c_char_p, []),
    "lcpc_set_device": (i32, [i32]),
    "lcpc_device_count": (i32, []),
    "lcpc_field_limbs": (i32, [i32]),
    "lcpc_field_num_bits": (i32, [i32]),
    "lcpc_field_random": (i32, [i32, C.c_uint64, u64p, sz]),
    "lcpc_n_degree_tests": (sz, [sz, sz, sz]),
    "lcpc_log2": (sz, [sz]),
    "lcpc_ligero_n_col_opens": (sz, [sz, sz]),
    "lcpc_ligero_get_dims": (i32, [i32, sz, sz, sz, szp, szp, szp]),
    "lcpc_ligero_new": (i32, [i32, sz, sz, sz, C.POINTER(vp)]),
    "lcpc_ligero_new_ml": (i32, [i32, sz, sz, sz, C.POINTER(vp)]),
    "lcpc_ligero_new_from_dims": (i32, [i32, sz, sz, sz, sz, C.POINTER(vp)]),
    "lcpc_rs_encoding_new": (i32, [i32, sz, sz, sz, sz, C.POINTER(vp)]),
    "lcpc_sdig_n_col_opens": (sz, [i32]),
    "lcpc_sdig_get_n_per_row": (i32, [i32, i32, sz, szp]),
    "lcpc_sdig_new": (i32, [i32, i32, sz, C.c_uint64, C.POINTER(vp)]),
    "lcpc_sdig_new_ml": (i32, [i32, i32, sz, C.c_uint64, C.POINTER(vp)]),
    "lcpc_sdig_new_from_dims": (i32, [i32, i32, sz, sz, C.c_uint64, C.POINTER(vp)]),
    "lcpc_encoding_kind": (i32, [vp]),
    "lcpc_encoding_matrix_nnz": (sz, [vp]),
    "lcpc_encoding_free": (None, [vp]),
    "lcpc_encoding_field": (i32, [vp]),
    "lcpc_encoding_get_dims": (None, [vp, sz, szp, szp, szp]),
    "lcpc_encoding_dims_ok": (i32, [vp, sz, sz]),
    "lcpc_encoding_n_col_opens": (sz, [vp]),
    "lcpc_encoding_n_degree_tests": (sz, [vp]),
    "lcpc_prepare_thread": (i32, [vp, sz]),
    "lcpc_reserve": (i32, [vp, sz, sz]),
    "lcpc_encoding_n_per_row": (sz, [vp]),
    "lcpc_encoding_n_cols": (sz, [vp]),
    "lcpc_encoding_set_row_kernel": (i32, [vp, i32]),
    "lcpc_encode": (i32, [vp, u64p, sz]),
    "lcpc_encode_rows": (i32, [vp, u64p, sz, sz]),
    "lcpc_encode_rows_device": (i32, [vp, vp, sz, sz, vp, sz, sz, vp]),
    "lcpc_commit_new": (i32, [vp, u64p, sz, C.POINTER(vp)]),
    "lcpc_commit_new_device": (i32, [vp, vp, sz, C.POINTER(vp)]),
    "lcpc_commit_free": (None, [vp]),
    "lcpc_commit_get_root": (i32, [vp, u8p]),
    "lcpc_commit_n_rows": (sz, [vp]),
    "lcpc_commit_n_cols": (sz, [vp]),
    "lcpc_commit_n_per_row": (sz, [vp]),
    "lcpc_commit_n_hashes": (sz, [vp]),
    "lcpc_commit_from_parts": (i32, [i32, sz, sz, sz, u64p, u64p, u8p, sz, C.POINTER(vp)]),
    "lcpc_commit_copy_comm": (i32, [vp, u64p]),
    "lcpc_commit_copy_coeffs": (i32, [vp, u64p]),
    "lcpc_commit_copy_hashes": (i32, [vp, u8p]),
    "lcpc_commit_col_major": (i32, [vp]),
    "lcpc_commit_device_comm": (vp, [vp]),
    "lcpc_commit_comm_canonical": (i32, [vp]),
    "lcpc_commit_device_coeffs": (vp, [vp]),
    "lcpc_check_comm": (i32, [vp, vp]),
    "lcpc_open_column": (i32, [vp, sz, u64p, u8p]),
    "lcpc_transcript_new": (vp, [u8p, sz]),
    "lcpc_transcript_clone": (vp, [vp]),
    "lcpc_transcript_free": (None, [vp]),
    "lcpc_transcript_append_message": (None, [vp, u8p, sz, u8p, sz]),
    "lcpc_transcript_append_messages": (None, [vp, u8p, sz, u8p, sz, sz]),
    "lcpc_transcript_challenge_bytes": (None, [vp, u8p, sz, u8p, sz]),
    "lcpc_transcript_from_ops": (vp, [C.POINTER(TranscriptOps)]),
    "lcpc_transcript_status": (i32, [vp]),
    "lcpc_prove": (i32, [vp, u64p, sz, vp, vp, C.POINTER(vp)]),
    "lcpc_prove_ops": (i32, [vp, u64p, sz, vp, C.POINTER(TranscriptOps), C.POINTER(vp)]),
    "lcpc_verify_ops": (i32, [u8p, u64p, sz, u64p, sz, vp, vp, C.POINTER(TranscriptOps), u64p]),
    "lcpc_proof_free": (None, [vp]),
    "lcpc_proof_n_cols": (sz, [vp]),
    "lcpc_proof_n_per_row": (sz, [vp]),
    "lcpc_proof_n_rows": (sz, [vp]),
    "lcpc_proof_n_degree_tests": (sz, [vp]),
    "lcpc_proof_n_col_opens": (sz, [vp]),
    "lcpc_proof_path_len": (sz, [vp]),
    "lcpc_proof_field": (i32, [vp]),
    "lcpc_proof_copy_p_eval": (i32, [vp, u64p]),
    "lcpc_proof_copy_p_random": (i32, [vp, sz, u64p]),
    "lcpc_proof_copy_column": (i32, [vp, sz, u64p, u8p]),
    "lcpc_proof_from_parts": (i32, [i32, sz, sz, sz, sz, sz, sz, u64p, u64p, u64p, u8p, C.POINTER(vp)]),
    "lcpc_verify": (i32, [u8p, u64p, sz, u64p, sz, vp, vp, vp, u64p]),
    "lcpc_collapse_columns": (i32, [i32, u64p, u64p, u64p, sz, sz]),
    "lcpc_merkle_tree": (i32, [u8p, sz, u8p]),
    "lcpc_verify_column_path": (i32, [i32, u64p, sz, u8p, sz, sz, u8p]),
    "lcpc_verify_column_value": (i32, [i32, u64p, u64p, sz, u64p]),
    "lcpc_hash_columns": (i32, [i32, u64p, sz, sz, u8p]),
    "lcpc_pos_bytes_to_field": (i32, [u8p, sz, u64p, szp]),
    "lcpc_pos_bytes_to_field_device": (i32, [vp, sz, vp, vp]),
    "lcpc_pos_commit_bytes_device": (i32, [vp, vp, sz, C.POINTER(vp)]),
    "lcpc_pos_commit_eval_bytes_device": (i32, [vp, vp, sz, u64p, sz, u64p, C.POINTER(vp)]),
    "lcpc_pos_commit_bytes": (i32, [vp, u8p, sz, C.POINTER(vp)]),
    "lcpc_last_upload_pinned": (i32, []),
    "lcpc_pos_field_to_bytes": (i32, [u64p, sz, u8p, sz]),
    "lcpc_pos_default_dims": (None, [sz, szp, szp, szp]),
    "lcpc_pos_column_indices": (i32, [C.c_uint64, sz, sz, u64p, szp]),
    "lcpc_pos_side_vectors": (i32, [i32, u64p, sz, sz, u64p, u64p]),
    "lcpc_pos_eval_encoded": (i32, [vp, u64p, sz, u64p]),
    "lcpc_ifft_oi_rows": (i32, [i32, u64p, sz, sz]),
    "lcpc_open_columns": (i32, [vp, u64p, sz, u64p, u8p]),
    "lcpc_pos_columns": (i32, [vp, u64p, sz, u64p, sz, u64p, u8p]),
    "lcpc_hash_field_columns": (i32, [i32, u64p, sz, sz, u8p]),
    "lcpc_verify_leaf_paths": (i32, [u8p, u8p, sz, sz, u64p, u8p, u8p]),
    "lcpc_verify_column_values": (i32, [i32, u64p, sz, sz, u64p, u64p, sz, u64p, u8p]),
    "lcpc_pos_encode_file": (i32, [u8p, sz, sz, sz, sz, u8p, u8p, szp]),
    "lcpc_pos_encode_file_batched": (i32, [u8p, sz, sz, sz, sz, u8p, u8p, szp, sz]),
    "lcpc_pos_writer_new": (i32, [sz, sz, u8p, sz, sz, C.POINTER(vp)]),
    "lcpc_pos_writer_free": (None, [vp]),
    "lcpc_column_digests_new": (i32, [i32, sz, sz, C.POINTER(vp)]),
    "lcpc_column_digests_free": (None, [vp]),
    "lcpc_column_digests_width": (sz, [vp]),
    "lcpc_column_digests_update": (i32, [vp, u64p, sz]),
    "lcpc_column_digests_finalize": (i32, [vp, u8p, u8p]),
    "lcpc_pos_writer_set_target": (i32, [vp, u8p, sz]),
    "lcpc_pos_writer_rows_written": (sz, [vp]),
    "lcpc_pos_writer_push_bytes": (i32, [vp, u8p, sz]),
    "lcpc_pos_writer_finalize": (i32, [vp, u8p, u8p, szp, szp]),
    "lcpc_pos_porenc_tree": (i32, [u8p, sz, sz, sz, u8p]),
    "lcpc_pos_decode_porenc": (i32, [u8p, sz, sz, sz, sz, sz, u8p]),
    "lcpc_leaf_n_chunks": (sz, [i32, sz]),
    "lcpc_leaf_chunk_first_row": (sz, [i32, sz]),
    "lcpc_shard_new": (i32, [vp, u64p, sz, sz, sz, C.POINTER(vp)]),
    "lcpc_shard_new_device": (i32, [vp, vp, sz, sz, sz, C.POINTER(vp)]),
    "lcpc_shard_free": (None, [vp]),
    "lcpc_shard_chunk_cvs": (i32, [vp, sz, sz, u8p]),
    "lcpc_leaves_from_cvs": (i32, [u8p, sz, sz, u8p]),
    "lcpc_shard_collapse": (i32, [vp, u64p, sz, u64p]),
    "lcpc_shard_gather_columns": (i32, [vp, u64p, sz, u64p]),
    "lcpc_field_sum": (i32, [i32, u64p, sz, sz, u64p]),
    "lcpc_shard_chunk_cvs_device": (i32, [vp, sz, sz, vp]),
    "lcpc_leaves_tree_device": (i32, [vp, sz, sz, vp]),
    "lcpc_shard_collapse_device": (i32, [vp, vp, sz, vp]),
    "lcpc_shard_gather_columns_device": (i32, [vp, u64p, sz, vp]),
    "lcpc_field_sum_device": (i32, [i32, vp, sz, sz, u64p]),
    "lcpc_pos_reencode_rows": (i32, [u8p, sz, sz, sz, sz, u8p, sz]),
    "lcpc_challenge_tensor": (i32, [vp, i32, sz, u64p]),
    "lcpc_transcript_append_field_elems": (i32, [vp, u8p, sz, i32, u64p, sz]),
    "lcpc_challenge_columns": (i32, [vp, sz, sz, u64p]),
    "lcpc_comm_rccl_unique_id": (i32, [u8p]),
    "lcpc_comm_rccl_new": (i32, [u8p, i32, i32, C.POINTER(vp)]),
    "lcpc_comm_from_ops": (i32, [C.POINTER(CommOps), i32, i32, C.POINTER(vp)]),
    "lcpc_comm_nranks": (i32, [vp]),
    "lcpc_comm_rank": (i32, [vp]),
    "lcpc_comm_is_rccl": (i32, [vp]),
    "lcpc_comm_free": (None, [vp]),
    "lcpc_sharded_rows": (i32, [i32, sz, i32, i32, szp, szp]),
    "lcpc_sharded_commit_new_device": (i32, [vp, vp, sz, vp, C.POINTER(vp)]),
    "lcpc_sharded_commit_free": (None, [vp]),
    "lcpc_sharded_commit_get_root": (i32, [vp, u8p]),
    "lcpc_sharded_commit_n_hashes": (sz, [vp]),
    "lcpc_sharded_commit_copy_hashes": (i32, [vp, u8p]),
    "lcpc_sharded_prove": (i32, [vp, u64p, sz, vp, vp, i32, C.POINTER(vp)]),
    "lcpc_sharded_commit_prove_many": (i32, [vp, C.POINTER(vp), sz, sz, u64p, vp, MAKE_TRANSCRIPT_FN, vp, sz,
                                             C.POINTER(vp), u8p]),
    "lcpc_sharded_reserve": (i32, [vp, sz, vp, sz, sz]),
    "lcpc_sharded_pos_request": (i32, [vp, u64p, sz, u64p, sz, i32, u64p, u64p, u8p]),
    "lcpc_sharded_p2p_schedule": (i32, [i32, sz, sz, sz, sz, sz, i32, i32, sz, sz, C.POINTER(P2pRecord), sz,
                                        szp]),
    "lcpc_prof_enable": (None, [i32]),
    "lcpc_prof_reset": (None, []),
    "lcpc_prof_get": (i32, [C.c_char_p, C.POINTER(C.c_double), u64p]),
    "lcpc_prof_names": (sz, [C.c_char_p, sz]),
    "lcpc_selftest_pool_ordering": (i32, [i32, C.c_uint32, u64p, u64p, u64p]),
}


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/lcpc_mi.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lcpc_[a-z0-9_]+)\s*\(", text)))


def load(path: str = LIB_PATH):
    """Load liblcpc_mi.so; raises OSError if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise OSError(f"{path} not built: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
        # torch-ROCm bundles its own libamdhip64.so (soname libamdhip64.so.7, as ours).  Loaded
        # first, it satisfies this library's dependency, so torch tensors and RCCL (shard.py)
        # share one HIP runtime with the kernels here; loaded after us, torch would bring a
        # second runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def last_error() -> str:
    msg = load().lcpc_last_error()
    return msg.decode() if msg else ""
