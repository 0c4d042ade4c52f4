"""The C-ABI boundary from plain C: tests/c/drop_in_client.c is compiled with gcc -std=c99 against
include/lcpc_mi.h and linked to the in-tree liblcpc_mi.so -- the binding a Rust FFI crate makes --
and drives commit / prove / verify through the caller-owned-transcript ops table.

CPU: it compiles warning-free, links, and fails loudly without a HIP device (no CPU fallback).
GPU: it runs to "drop-in client ok" (prove through ops == prove with the library's transcript,
the caller's transcript ends in the same state, verify accepts, a wrong root is rejected).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "lcpc_proof_of_storage_amd")


def _build(tmp_path):
    exe = str(tmp_path / "drop_in_client")
    r = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror",
                        os.path.join(ROOT, "tests", "c", "drop_in_client.c"), "-I", os.path.join(ROOT, "include"),
                        "-L", LIBDIR, "-llcpc_mi", f"-Wl,-rpath,{LIBDIR}", "-o", exe],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_client_builds_and_fails_loudly_without_gpu(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "liblcpc_mi.so")):
        pytest.skip("liblcpc_mi.so not built")
    exe = _build(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([exe, "12"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 1 and "no HIP device" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("log_len", [12, 16, 20])
def test_c_client_runs_on_gpu(gpu, tmp_path, log_len):
    exe = _build(tmp_path)
    r = subprocess.run([exe, str(log_len)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "drop-in client ok" in r.stdout
