"""GPU parity of the proof-of-storage field helpers in pos.py (fields.rs:25-194,
lcpc_online.rs:71-76), with ports of the reference's own fields.rs tests:
  test_polynomial_eval                        fields.rs:201-229
  test_polynomial_eval_with_elevated_degree   :231-287
  bytes_into_then_out_of_field_elements       :289-301
plus file reads at ragged sizes and evaluations at random points against a big-int Horner."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FT63 = 0


@pytest.fixture(scope="module")
def pos(gpu):
    from lcpc_proof_of_storage_amd import pos
    return pos


def _ev(pos, oracle, coeffs, x, offset=None):
    c = oracle.to_mont(FT63, coeffs)
    p = oracle.to_mont(FT63, [x])
    if offset is None:
        v = pos.evaluate_field_polynomial_at_point(c, p)
    else:
        v = pos.evaluate_field_polynomial_at_point_with_elevated_degree(c, p, offset)
    return oracle.from_mont(FT63, v)[0]


def test_polynomial_eval(pos, oracle):
    assert _ev(pos, oracle, [0, 0, 0], 1) == 0
    assert _ev(pos, oracle, [1, 1, 1], 1) == 3
    assert _ev(pos, oracle, [0, 1, 2], 2) == 2 * 2 ** 2 + 2 + 0


def test_polynomial_eval_with_elevated_degree(pos, oracle):
    assert _ev(pos, oracle, [0, 0, 0], 1, 1) == 0
    assert _ev(pos, oracle, [1, 1, 1], 1, 1) == 3
    assert _ev(pos, oracle, [0, 0, 2], 2) == _ev(pos, oracle, [2], 2, 2)
    assert _ev(pos, oracle, [0, 0, 2, 2], 2) == _ev(pos, oracle, [2, 2], 2, 2)


@pytest.mark.parametrize("n,offset", [(1, 0), (17, 3), (1000, 0), (4096, 12345)])
def test_polynomial_eval_random(pos, oracle, n, offset):
    p = oracle.modulus(FT63)
    rng = np.random.default_rng(n)
    coeffs = [int(v) % p for v in rng.integers(0, 1 << 62, n)]
    x = int(rng.integers(0, 1 << 62)) % p
    want = 0
    for c in reversed(coeffs):
        want = (want * x + c) % p
    want = want * pow(x, offset, p) % p
    assert _ev(pos, oracle, coeffs, x, offset) == want
    a = oracle.to_mont(FT63, coeffs)
    b = oracle.to_mont(FT63, [int(v) % p for v in rng.integers(0, 1 << 62, n)])
    dot = sum(u * v for u, v in zip(oracle.from_mont(FT63, a), oracle.from_mont(FT63, b))) % p
    assert oracle.from_mont(FT63, pos.vector_multiply(a, b))[0] == dot


def test_bytes_into_then_out_of_field_elements(pos):
    data = np.random.default_rng(1).integers(0, 256, 999, dtype=np.uint8).tobytes()
    field = pos.convert_byte_vec_to_field_elements_vec(data)
    assert pos.convert_field_elements_vec_to_byte_vec(field, 999) == data


@pytest.mark.parametrize("n", [0, 1, 6999, 7000, 7001, 100003])
def test_file_reads(pos, tmp_path, n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    path = tmp_path / "f.bin"
    path.write_bytes(data)
    want = pos.convert_byte_vec_to_field_elements_vec(data) if n else np.zeros((0, 1), np.uint64)
    with open(path, "rb") as f:
        size, el = pos.read_file_to_field_elements_vec(f)
    assert size == n and np.array_equal(el, want)
    with open(path, "rb") as f:
        size, el = pos.stream_file_to_field_elements_vec_sync(f)
    assert size == n and np.array_equal(el, want)
    assert np.array_equal(pos.read_file_path_to_field_elements_vec(str(path)), want)


@pytest.mark.parametrize("tail", [b"", b"\x05", b"\x05\x00\x00", b"\x00" * 7, b"\x01\x00\x00\x00\x00\x00\x02"])
def test_field_elements_vec_to_file(pos, tmp_path, tail):
    """Each element's 7 data bytes; only the last element's trailing zeros are dropped."""
    head = np.random.default_rng(2).integers(1, 256, 70, dtype=np.uint8).tobytes()
    data = head + tail
    el = pos.convert_byte_vec_to_field_elements_vec(data)
    path = tmp_path / "out.bin"
    pos.field_elements_vec_to_file(str(path), el)
    full = pos.convert_field_elements_vec_to_byte_vec(el, el.size * 7)
    assert path.read_bytes() == full[:-7] + full[-7:].rstrip(b"\0")
    pos.field_elements_vec_to_file(str(path), np.zeros((0, 1), np.uint64))
    assert path.read_bytes() == b""


def test_random_writeable_field_vec_and_dims(pos):
    v = pos.random_writeable_field_vec(4, seed=3)
    assert v.shape == (16, 1) and int(v.max()) < 1 << 56
    assert pos.dims_ok(4, 8) and pos.dims_ok(1, 2) and not pos.dims_ok(5, 8) and not pos.dims_ok(4, 12)
    assert not pos.dims_ok(0, 8) and not pos.dims_ok(1, 1)
    assert pos.is_power_of_two(0) and pos.is_power_of_two(64) and not pos.is_power_of_two(96)
