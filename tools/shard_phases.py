"""Per-phase host timing of one rank's row-sharded commit + prove (bench.py --shard rows, N = 1):
wraps every GpuBackend / Comm method with a wall-clock timer.  Usage: python tools/shard_phases.py"""
import collections
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import lcpc_proof_of_storage_amd as L  # noqa: E402
from lcpc_proof_of_storage_amd import shard as S  # noqa: E402

acc = collections.defaultdict(float)


def wrap(cls, name):
    f = getattr(cls, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[f"{cls.__name__}.{name}"] += time.perf_counter() - t
    setattr(cls, name, g)


for n in [m for m in dir(S.GpuBackend) if not m.startswith("_")]:
    if callable(getattr(S.GpuBackend, n)):
        wrap(S.GpuBackend, n)
for n in ["bcast", "all_gather", "t_all_to_all", "t_all_gather"]:
    wrap(S.Comm, n)
for n in ["commit", "prove"]:
    wrap(S.RowShardedCommit, n)

L.set_device(0)
fid, n = L.FT127, 1 << 24
enc = L.LigeroEncoding.new(fid, n)
n_rows, n_per_row, n_cols = enc.get_dims(n)
coeffs = L.field_random(fid, n, 0x1CDC2024).reshape(n_rows, -1)
outer = L.field_random(fid, n_rows, 7)
be = S.GpuBackend(enc)
comm = S.Comm(None, "cuda:0")
d = torch.from_numpy(np.ascontiguousarray(coeffs).view(np.int64)).to("cuda:0")
steps = 8
for i in range(steps + 2):
    if i == 2:
        acc.clear()
        t0 = time.perf_counter()
    sc = S.RowShardedCommit(be, comm, n_rows, 16)
    root = sc.commit((d.data_ptr(), n_rows))
    tr = L.Transcript(b"test transcript")
    tr.append_message(b"polycommit", root)
    tr.append_message(b"ncols", enc.get_n_col_opens().to_bytes(8, "big"))
    sc.prove(outer, tr)
    sc.close()
tot = time.perf_counter() - t0
print(f"total {1e3 * tot / steps:.3f} ms/step")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:40s} {1e3 * v / steps:8.3f} ms")
