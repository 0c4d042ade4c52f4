"""Child process of test_gpu_ntt_row1.py::test_row1_runtime_modes_agree: the file-image commits of
a few sizes under whatever LCPC_ROW1_PREFETCH / LCPC_ROW1_GLDS this process was started with (the
library reads them once), printed as one JSON line of {n_bytes: [root, sha256(comm), sha256(coeffs)]}."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lcpc_proof_of_storage_amd as L  # noqa: E402

NP, NC = 16384, 32768


def main():
    assert L.device_count() > 0, "no HIP device"
    L.set_device(0)
    enc = L.RsEncoding.new(0, NP, NC, 16, 2)
    out = {}
    for n_bytes in map(int, sys.argv[1:]):
        data = np.random.default_rng(n_bytes).integers(0, 256, n_bytes, dtype=np.uint8)
        data[-1] = 0xff
        c = L.LcCommit.commit_pos_bytes(data, enc)
        out[n_bytes] = [c.get_root().hex(), hashlib.sha256(c.comm.tobytes()).hexdigest(),
                        hashlib.sha256(c.coeffs.tobytes()).hexdigest()]
        del c
    print(json.dumps(out))


if __name__ == "__main__":
    main()
