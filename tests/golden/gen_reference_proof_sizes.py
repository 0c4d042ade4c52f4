#!/usr/bin/env python3
"""Extract the proof sizes the reference itself recorded into reference_proof_sizes.json.

The reference's `prove_verify_size_bench` tests (lcpc-ligero-pc/src/tests.rs:102-170,
lcpc-brakedown-pc/src/tests.rs:98-166) print, per log2 length lgl in 13, 15, ..., 29,
"lgl: prove_ns verify_ns proof_bytes xor_byte", where proof_bytes =
bincode::serialize(&LcEvalProof).len() of a real Ft255 proof.  The 2021-08-07 logs under
doc/benchmark-results/ are from the current serialization (the earlier ones carry an older
path encoding); their Ligero runs are the rates the `hlf` (1/2), default (1/4) and `isz`
(38/39) features select, and the sdig run is SdigCode3 with seed 0.  Only the numbers are kept
(data, not source).  Run here, where /root/reference exists:
    python tests/golden/gen_reference_proof_sizes.py
"""
import json
import os
import re

SRC = "/root/reference/doc/benchmark-results"
FILES = {
    "ligero_rho_1_2": ("20210807_1c_255bit_ligero_hlf_pvs.txt", [1, 2]),
    "ligero_rho_1_4": ("20210807_1c_255bit_ligero_dfl_pvs.txt", [1, 4]),
    "ligero_rho_38_39": ("20210807_1c_255bit_ligero_isz_pvs.txt", [38, 39]),
    "sdig_code3_seed0": ("20210807_1c_255bit_sdig_pvs.txt", None),
}


def main():
    out = {"field": "Ft255", "source": "doc/benchmark-results/*_pvs.txt (reference run, 2021-08-07)",
           "runs": {}}
    for key, (fname, rho) in FILES.items():
        sizes = {}
        for line in open(os.path.join(SRC, fname)):
            m = re.match(r"^(\d+): \d+ \d+ (\d+) \d+\s*$", line)
            if m:
                sizes[m.group(1)] = int(m.group(2))
        out["runs"][key] = {"file": fname, "rho": rho, "proof_bytes_by_log_len": sizes}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_proof_sizes.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
