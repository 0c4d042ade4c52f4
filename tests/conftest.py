import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
# the sharded calls' watchdog is off in the library by default; the tests (and the processes they
# spawn, which inherit the environment) turn it on so a stuck exchange ends with a message
os.environ.setdefault("LCPC_SHARD_WATCHDOG_S", "120")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    oracle_ffi.lib()
    return oracle_ffi


@pytest.fixture(scope="session")
def gpu():
    """The product package with a live device; fails loudly (no fallback) if absent."""
    import lcpc_proof_of_storage_amd as L
    n = L.device_count()
    assert n > 0, "no HIP device visible: the -m gpu tests need an MI355X"
    L.set_device(0)
    return L


class _HipMem:
    """Raw device buffers through the HIP runtime liblcpc_mi.so itself links (tests only).

    torch wheels bundle a second HIP runtime; initialising it after ours can fail, so the GPU
    tests do not use torch for device memory."""

    H2D, D2H = 1, 2

    def __init__(self):
        import ctypes as C
        self.C = C
        self.L = C.CDLL("libamdhip64.so.7")
        self.L.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.L.hipFree.argtypes = [C.c_void_p]

    def to_device(self, a):
        p = self.C.c_void_p()
        assert self.L.hipMalloc(self.C.byref(p), max(a.nbytes, 16)) == 0
        assert self.L.hipMemcpy(p, a.ctypes.data, a.nbytes, self.H2D) == 0
        return p.value

    def to_host(self, ptr, out):
        assert self.L.hipMemcpy(out.ctypes.data, ptr, out.nbytes, self.D2H) == 0
        return out

    def free(self, ptr):
        self.L.hipFree(ptr)


@pytest.fixture(scope="session")
def hipmem(gpu):
    return _HipMem()


def collect_ranks(procs, q, world, timeout=280, label="ranks"):
    """The reports of `world` spawned ranks from queue q, as {rank: report}.  A rank that exits
    without reporting (a crash, or the sharded watchdog's status 75) fails the caller within
    seconds, with the exit codes, instead of leaving it waiting out the timeout; ranks still alive
    at the end are killed."""
    import queue
    import time
    res, deadline = {}, time.monotonic() + timeout
    try:
        while len(res) < world:
            try:
                r, v = q.get(timeout=5)
                res[r] = v
                continue
            except queue.Empty:
                pass
            silent = [(i, p.exitcode) for i, p in enumerate(procs) if i not in res and p.exitcode is not None]
            if silent:
                raise AssertionError(f"{label}: rank(s) exited without reporting (rank, exit code): {silent}")
            if time.monotonic() > deadline:
                raise AssertionError(f"{label}: no report from ranks {sorted(set(range(world)) - set(res))} "
                                     f"within {timeout} s")
    finally:
        for p in procs:
            p.join(timeout=60 if len(res) == world else 5)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return res


# rendezvous bound for spawned gloo groups: a rank that cannot form the group reports instead of
# waiting forever
RENDEZVOUS_TIMEOUT_S = 60
