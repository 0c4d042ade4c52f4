"""The C-ABI boundary from plain C: the clients under tests/c/ are compiled with gcc -std=c99
against include/lcpc_mi.h and linked to the in-tree liblcpc_mi.so -- the binding a Rust FFI crate
makes.  drop_in_client.c drives lcpc-2d commit / prove / verify through the caller-owned-transcript
ops table; pos_audit_client.c runs one proof-of-storage audit round (upload to .porenc/.portree,
commit, column challenge, evaluation, client checks, decode, a one-row edit).

CPU: both compile warning-free, link, and fail loudly without a HIP device (no CPU fallback).
GPU: drop_in_client runs to "drop-in client ok" (prove through ops == prove with the library's
transcript, the caller's transcript ends in the same state, verify accepts, a wrong root is
rejected); pos_audit_client runs to "pos audit ok" (the .portree root is the commitment root,
paths and column values verify, tampering is caught, the image decodes, the edit re-roots).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "lcpc_proof_of_storage_amd")


def _build(tmp_path, name="drop_in_client"):
    exe = str(tmp_path / name)
    r = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror",
                        os.path.join(ROOT, "tests", "c", name + ".c"), "-I", os.path.join(ROOT, "include"),
                        "-L", LIBDIR, "-llcpc_mi", f"-Wl,-rpath,{LIBDIR}", "-o", exe],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.parametrize("name,arg", [("drop_in_client", "12"), ("pos_audit_client", "100000")])
def test_c_client_builds_and_fails_loudly_without_gpu(tmp_path, name, arg):
    if not os.path.exists(os.path.join(LIBDIR, "liblcpc_mi.so")):
        pytest.skip("liblcpc_mi.so not built")
    exe = _build(tmp_path, name)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([exe, arg], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 1 and "no HIP device" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("log_len", [12, 16, 20])
def test_c_client_runs_on_gpu(gpu, tmp_path, log_len):
    exe = _build(tmp_path)
    r = subprocess.run([exe, str(log_len)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "drop-in client ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("n_bytes", [1000, (1 << 20) + 3, 16 << 20, 64 << 20])
def test_pos_audit_client_runs_on_gpu(gpu, tmp_path, n_bytes):
    exe = _build(tmp_path, "pos_audit_client")
    r = subprocess.run([exe, str(n_bytes)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "pos audit ok" in r.stdout
