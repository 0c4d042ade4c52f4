"""Host-only code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU): the transcript's
batched record absorb (both Keccak implementations, against one append_message per record at
every block offset) and the Brakedown matgen's CSR invariants.  tools/hostsan/run.sh."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                    reason="needs g++ and the ROCm headers")
def test_host_code_under_asan_ubsan(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "hostsan", "run.sh")], capture_output=True,
                       text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "impl scalar mismatches 0" in r.stdout
    assert "bad 0" in r.stdout
