"""GPU: the row combinations (collapse_columns, lcpc-2d/src/lib.rs:1126-1154) for 1 to 4
tensors at once, through a row shard holding every row (lcpc_shard_collapse and its
device-resident form), against the oracle tensor by tensor.  For Ft127 with up to 3 tensors
this is the int8 matrix-core kernel (collapse_mfma.hpp); 4 tensors and the other fields take
the VALU kernel.  Shapes cover ragged rows and columns (not multiples of the 4-row MFMA step or
the 64-column wave tile), one row, and more rows than one 512-row split."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = [(37, 100), (1, 64), (4, 1000), (600, 70), (512, 4096)]


@pytest.mark.parametrize("fid", [1, 0, 2, 3])
@pytest.mark.parametrize("n_rows,n_per_row", SHAPES)
@pytest.mark.parametrize("n_t", [1, 2, 3, 4])
def test_collapse_tensors_match_oracle(gpu, oracle, fid, n_rows, n_per_row, n_t):
    from lcpc_proof_of_storage_amd.shard import GpuBackend
    if fid in (2, 3) and n_rows * n_per_row > 100000:
        pytest.skip("Ft191 / Ft255: the small shapes suffice")
    nl = oracle.limbs(fid)
    n_cols = 1 << (n_per_row.bit_length())
    enc = gpu.LigeroEncoding.new_from_dims(fid, n_per_row, n_cols)
    be = GpuBackend(enc)
    rng = oracle.ChaCha(seed_u64=n_rows * 1000 + n_per_row + n_t)
    coeffs = rng.field_random(fid, n_rows * n_per_row).reshape(n_rows, n_per_row * nl)
    tens = rng.field_random(fid, n_t * n_rows).reshape(n_t, n_rows, nl)
    sh = be.shard_new(coeffs, 0, n_rows)
    try:
        got = be.collapse(sh, tens)
        for t in range(n_t):
            want = oracle.collapse(fid, coeffs, tens[t], n_rows, n_per_row)
            assert np.array_equal(got[t].reshape(-1), want), f"tensor {t}"
    finally:
        be.shard_free(sh)


@pytest.mark.parametrize("n_t", [1, 2, 3])
def test_collapse_device_form_matches_host_form(gpu, oracle, n_t):
    import torch
    from lcpc_proof_of_storage_amd.shard import GpuBackend
    fid, n_rows, n_per_row = 1, 300, 2048
    nl = oracle.limbs(fid)
    enc = gpu.LigeroEncoding.new_from_dims(fid, n_per_row, 4096)
    be = GpuBackend(enc)
    rng = oracle.ChaCha(seed_u64=77 + n_t)
    coeffs = rng.field_random(fid, n_rows * n_per_row).reshape(n_rows, n_per_row * nl)
    tens = rng.field_random(fid, n_t * n_rows).reshape(n_t, n_rows, nl)
    sh = be.shard_new(coeffs, 0, n_rows)
    try:
        host = be.collapse(sh, tens)
        dt = torch.from_numpy(np.ascontiguousarray(tens).view(np.int64)).to("cuda:0")
        dev = be.collapse_dev(sh, dt).cpu().numpy().view(np.uint64)
        assert np.array_equal(dev, host)
    finally:
        be.shard_free(sh)
