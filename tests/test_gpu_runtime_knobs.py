"""GPU: the library's runtime knobs change how the work is scheduled or which kernel variant runs,
never the result.  Each knob is read once per process, so each setting gets its own child process
(tests/_runtime_knobs_child.py: Ligero commit / prove / verify over all five fields, Brakedown over
Ft63 and Ft127, a proof-of-storage file-image commit, the sharded driver at one rank); every setting must return what the default
returns, and the default's roots are the oracle's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KNOBS = ("LCPC_NO_MFMA", "LCPC_STREAM_MODE", "LCPC_PRIORITY_STREAMS", "LCPC_HOST_WAIT", "LCPC_KECCAK",
         "LCPC_ROW1_PREFETCH", "LCPC_ROW1_GLDS", "LCPC_SHARD_BULK_STREAMS")
SETTINGS = [
    {"LCPC_NO_MFMA": "1"},              # VALU row combinations and SDIG levels instead of the int8 MFMA ones
    {"LCPC_STREAM_MODE": "serial"},     # every call on one stream
    {"LCPC_PRIORITY_STREAMS": "1"},     # the prover's streams above the bulk ones
    {"LCPC_HOST_WAIT": "blocking"},     # host threads sleep on the GPU instead of the runtime's default
    {"LCPC_KECCAK": "scalar"},          # the transcript's scalar permutation
    {"LCPC_KECCAK": "avx512"},          # the vector one where the host has AVX-512
    {"LCPC_SHARD_BULK_STREAMS": "1"},   # the sharded driver's bulk streams: one ...
    {"LCPC_SHARD_BULK_STREAMS": "4"},   # ... or the most it takes
]


def _run(env_extra):
    env = {k: v for k, v in os.environ.items() if k not in KNOBS}
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "_runtime_knobs_child.py")], env=env,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, (env_extra, r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_results(gpu):
    return _run({})


def test_default_roots_are_the_oracles(default_results, gpu, oracle):
    """the child's default Ligero roots against the oracle's commit of the same coefficients"""
    for field in range(5):
        coeffs = gpu.field_random(field, (1 << 14) + 77, 11 + field)
        g_enc = gpu.LigeroEncoding.new(field, coeffs.shape[0])
        o_enc = oracle.Encoding.ligero(field, g_enc.n_per_row, g_enc.n_cols, g_enc.get_n_col_opens(),
                                       g_enc.get_n_degree_tests())
        assert default_results[f"ligero_f{field}"][0] == oracle.Commit(o_enc, coeffs.reshape(-1)).root().hex(), field


@pytest.mark.parametrize("setting", SETTINGS, ids=lambda s: ",".join(f"{k}={v}" for k, v in s.items()))
def test_knob_gives_the_default_results(default_results, setting):
    assert _run(setting) == default_results
