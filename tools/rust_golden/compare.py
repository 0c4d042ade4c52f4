"""Compare rust_golden's output (the Rust reference's values) with tests/golden/golden.json (the
oracle's), and for a differing Ligero root name the FFT convention that reproduces it.

    python tools/rust_golden/compare.py rust_golden.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

VARIANTS = {"omega_inv": "-DLCPC_FFT_OMEGA_INVERSE=1", "natural_out": "-DLCPC_FFT_OUTPUT_BITREV=0",
            "omega_inv_natural": "-DLCPC_FFT_OMEGA_INVERSE=1 -DLCPC_FFT_OUTPUT_BITREV=0"}
LIGERO_ARGS = {"cfg1_ft127_2_16": (1, 16), "ft63_2_14": (0, 14), "ft255_2_12": (3, 12), "ft253_192_2_12": (4, 12)}


def diff(a, b, path=""):
    out = []
    if isinstance(a, dict) and isinstance(b, dict):
        for k in sorted(set(a) | set(b)):
            if k not in a or k not in b:
                out.append(f"{path}/{k}: only in {'rust' if k in a else 'golden'}")
            else:
                out += diff(a[k], b[k], f"{path}/{k}")
    elif a != b:
        out.append(f"{path}: rust {str(a)[:80]} != golden {str(b)[:80]}")
    return out


def main(path):
    rust = json.load(open(path))
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    bad = 0
    for case in sorted(gold):
        if rust.get(case) is None:
            print(f"{case}: not produced by rust_golden (not covered)")
            continue
        d = diff(rust[case], gold[case], case)
        bad += bool(d)
        print(f"{case}: {'MATCH' if not d else 'DIFFERS'}")
        for line in d[:12]:
            print("   ", line)
        if d and case in LIGERO_ARGS and rust[case].get("root") != gold[case].get("root"):
            import gen_golden
            import oracle_ffi as O
            fid, lg = LIGERO_ARGS[case]
            for name, flags in VARIANTS.items():
                with O.use_lib(O.build_variant(name, flags)):
                    if gen_golden.ligero_case(fid, lg)["root"] == rust[case]["root"]:
                        print(f"    -> the Rust root is the oracle's under {flags}: set it in "
                              f"include/lcpc_fft_convention.h")
    print("all covered cases match" if not bad else f"{bad} case(s) differ")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
