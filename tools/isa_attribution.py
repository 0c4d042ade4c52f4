#!/usr/bin/env python3
"""Instruction attribution of the Ligero encode (review item: the ~41 non-multiply VALU
instructions per butterfly).  Compiles, for gfx950 and to assembly only (no GPU needed):
  * tools/microbench/isa_prims.hip -- fe_mul_lazy, fe_add_2p, fe_sub_2p and one whole DIF
    butterfly (add_2p + sub_2p + mul_lazy) as stand-alone kernels;
  * csrc/ntt_ft127.hip -- the cfg3 passes k_pass_a<Ft127, 8, 3, 8, HALFZ, CANON> and
    k_pass_b<Ft127, 8, 3, 8>;
and prints per-primitive VALU counts by class and each pass's counts per thread, per twiddle
product and per butterfly.

    python tools/isa_attribution.py [OUT.txt]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lcpc_proof_of_storage_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++20", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-Wno-unused-function",
         "-I" + CSRC]
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_count as IC  # noqa: E402

# butterflies per thread of the cfg3 shapes (ntt_v2.hpp; R = 3, 256 threads, 8 elements per
# round): pass B <8,3,8> rounds of 3, 3, 2 stages -> 12 + 12 + 8; pass A <8,3,8,HALFZ> the same
# minus stage 0's 4, which are (a, a w) with no add / sub.  Twiddle products per thread are
# counted from the code itself: 28 v_mad_u64_u32 per Montgomery product (16 a_i b_j + 12 m_i p_j)
SHAPES = {"k_pass_b": {"butterflies": 32}, "k_pass_a": {"butterflies": 28}}


def compile_s(src, out):
    subprocess.run([HIPCC] + FLAGS + ["-o", out, src], check=True, capture_output=True)


def valu_classes(ops):
    c = IC.classify(ops)
    return {k: v for k, v in c.items() if not k.startswith(("ds_", "global", "s_", "salu"))}


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
    with tempfile.TemporaryDirectory() as d:
        ps, ns = os.path.join(d, "prims.s"), os.path.join(d, "ntt.s")
        compile_s(os.path.join(ROOT, "tools", "microbench", "isa_prims.hip"), ps)
        compile_s(os.path.join(CSRC, "ntt_ft127.hip"), ns)
        prims = {}
        cur = None
        for line in open(ps):
            m = re.match(r"^(k_\w+):", line)
            if m:
                cur = m.group(1)
                prims[cur] = []
                continue
            if cur is None:
                continue
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            t = line.strip()
            if t and not t.startswith((";", ".")) and not t.endswith(":"):
                prims[cur].append(t.split()[0])
        print("# Ft127 field primitives, gfx950 VALU instructions (stand-alone kernels; the load /", file=out)
        print("# store address setup, 1 instruction, is included)", file=out)
        for k in ("k_mul_lazy", "k_add2p", "k_sub2p", "k_bfly"):
            c = valu_classes(prims[k])
            print(f"{k:12s} VALU {sum(c.values()):4d}  " + ", ".join(f"{n} {v}" for n, v in
                                                                      sorted(c.items(), key=lambda kv: -kv[1])),
                  file=out)
        ks = IC.kernels(ns)
        dem = dict(zip(ks, IC.demangle(list(ks))))
        print("\n# cfg3 passes, static VALU instructions per thread (one tile item per thread)", file=out)
        for want, key in (("k_pass_a<lcpc::Ft127, 8, 3, 8, true, true>", "k_pass_a"),
                          ("k_pass_b<lcpc::Ft127, 8, 3, 8>", "k_pass_b")):
            mk = next(k for k in ks if want in dem[k])
            c = valu_classes(ks[mk])
            tot = sum(c.values())
            sh = dict(SHAPES[key])
            mads = c.get("mad_u64_u32", 0)
            sh["products"] = mads // 28
            print(f"{want}: VALU {tot}, s_nop {IC.classify(ks[mk]).get('s_nop', 0)}", file=out)
            print(f"   {sh['products']} twiddle products, {sh['butterflies']} butterflies per thread: "
                  f"{tot / sh['products']:.1f} VALU per product, {tot / sh['butterflies']:.1f} per butterfly, "
                  f"{mads / sh['products']:.1f} mads per product", file=out)
            for n, v in sorted(c.items(), key=lambda kv: -kv[1]):
                print(f"   {n:28s} {v:6d}  ({100.0 * v / tot:4.1f} %)", file=out)


if __name__ == "__main__":
    main()
