"""lcpc_proof_of_storage_amd -- MI355X-native lcpc-2d commit/prove/verify row-encoding path.

Drop-in for the reference's LcEncoding / LcCommit / LcEvalProof path
(TrevorGKann/lcpc_proof_of_storage, lcpc-2d + lcpc-ligero-pc) behind the C ABI in
include/lcpc_mi.h, implemented by liblcpc_mi.so (gfx950 HIP kernels + C++ host).
"""
from .lcpc2d import (  # noqa: F401
    FT63, FT127, FT191, FT255, FT253_192, FIELD_NAMES,
    LcpcError, ProverError, VerifierError, FFTError, DeviceError,
    Transcript, CallerTranscript, LcEncoding, LigeroEncoding, RsEncoding, SdigEncoding, LcCommit, LcEvalProof, LcColumn,
    collapse_columns, merkle_tree, hash_columns, verify_column_path, verify_column_value,
    n_degree_tests, log2, limbs, num_bits, set_device, device_count, field_random,
    prof_enable, prof_reset, prof_stats, selftest_pool_ordering,
)
