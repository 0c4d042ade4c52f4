#!/usr/bin/env python3
"""The proof-of-storage one-pass row encode (ntt_row1.hpp k_row_ntt15<Ft63, CANON, COPY, BYTES>)
against the VALU issue floor of its own instruction stream -- the round-6 cycle model of
tools/encode_cycle_model.py applied to the cfg5 kernel.

Compiles csrc/ntt_ft63.hip for gfx950 to assembly (no GPU needed), counts the kernel's static
instructions by class (tools/isa_count.py), prices each VALU class with the measured per-class
issue cost at 4 waves/SIMD (profiles/r06_issue_cost.json; the kernel's occupancy: 1024-thread
workgroups, 123 VGPRs, 132 KiB of LDS, one workgroup per CU), and scales to the 1 GiB request
(9363 rows, one 16-wave workgroup each, 1024 SIMDs).  The kernel is fully unrolled apart from the
byte staging, so the static count stands in for the dynamic one.

    python tools/row1_cycle_model.py MEASURED_MS [OUT.txt]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lcpc_proof_of_storage_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import encode_cycle_model as M  # noqa: E402
import isa_count as IC  # noqa: E402

ROWS = 9363                      # 1 GiB file at the default dims (16384 -> 32768 Ft63 per row)
WAVES_PER_ROW = 16
# CANON, COPY (the commit's coeffs), BYTES, PF = 1 (the L2 prefetch at round 3), GLDS (LDS-DMA
# staging): the file-image kernel's defaults since round 6
KERNEL = "k_row_ntt15<lcpc::Ft63, true, true, true, 1, true>"


def main():
    measured = float(sys.argv[1])
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "ntt63.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-Wno-unused-function", "-I" + CSRC, "-o", s, os.path.join(CSRC, "ntt_ft63.hip")],
                       check=True, capture_output=True)
        ks = IC.kernels(s)
        dem = dict(zip(ks, IC.demangle(list(ks))))
        name = next(k for k in ks if KERNEL in dem[k])
        text = open(s).read()
        vgpr = re.search(re.escape(name) + r":.*?\.amdhsa_next_free_vgpr (\d+)", text, re.S)
        lds = re.search(re.escape(name) + r":.*?\.amdhsa_group_segment_fixed_size (\d+)", text, re.S)
        counts = IC.classify(ks[name])
    cost = M.issue_costs(os.path.join(ROOT, "profiles", "r06_issue_cost.json"))
    full = cost["v_add_u32 (reference: full-rate)"]
    per_wave = 0.0
    print(f"# {dem[name]}", file=out)
    print(f"# {vgpr.group(1) if vgpr else '?'} VGPRs, {lds.group(1) if lds else '?'} B of LDS per 1024-thread "
          f"workgroup: one workgroup (4 waves/SIMD) per CU", file=out)
    print(f"# static instructions per thread by class (priced at 4 waves/SIMD, ns per wave-instruction per SIMD)",
          file=out)
    for c, n in sorted(counts.items(), key=lambda kv: -kv[1]):
        price = cost[M.PRICE[c]] if c in M.PRICE else (full if c == "other valu" else None)
        if price is not None:
            per_wave += n * price
        print(f"   {c:26s} {n:6d}" + (f"   x {price:.3f} ns" if price is not None else "   (not VALU)"), file=out)
    model = ROWS * WAVES_PER_ROW / 1024 * per_wave * 1e-6
    print(f"VALU issue time per wave {per_wave / 1e3:.1f} us; x {ROWS * WAVES_PER_ROW / 1024:.1f} waves per SIMD "
          f"-> model {model:.3f} ms per 1 GiB request; measured {measured:.3f} ms -> the kernel runs at "
          f"{model / measured:.0%} of its VALU issue floor", file=out)
    print("The rest is the phases a 1024-thread workgroup spends off the VALU with no other workgroup on its CU to "
          "fill them: the row's 112 KiB byte load, the three LDS exchanges (ds_read / ds_write counts above) and the "
          "barriers between them (DESIGN.md §4, the one-pass kernel).", file=out)


if __name__ == "__main__":
    main()
