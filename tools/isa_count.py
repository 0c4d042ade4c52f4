#!/usr/bin/env python3
"""Per-kernel instruction-class counts of a gfx950 assembly file (hipcc --cuda-device-only -S).

Static counts over each kernel's text, by class: the 64-bit mads, the carry folds, the modular
add/sub chains, selects, moves, LDS / global memory, address arithmetic and scalar work.  Used to
attribute the Ligero encode's VALU instructions per butterfly.

    python tools/isa_count.py FILE.s [kernel-substring ...]
"""
import collections
import re
import subprocess
import sys

CLASSES = [
    ("mad_u64_u32", re.compile(r"^v_mad_u64_u32")),
    ("addc/subb (carry)", re.compile(r"^v_(addc|subb|subbrev)_co_u32")),
    ("add/sub_co (carry out)", re.compile(r"^v_(add|sub|subrev)_co_u32")),
    ("cndmask (select)", re.compile(r"^v_cndmask")),
    ("cmp", re.compile(r"^v_cmp")),
    ("mov", re.compile(r"^v_(mov|accvgpr)")),
    ("add/sub u32 (no carry)", re.compile(r"^v_(add|sub|subrev)_u32")),
    ("lshl_add_u64 / 64-bit", re.compile(r"^v_(lshl_add_u64|add_u64|lshlrev_b64|lshrrev_b64)")),
    ("shift/logic/bfe", re.compile(r"^v_(lshl|lshr|ashr|and|or|xor|bfe|bfi|perm|alignbit|alignbyte|not|bitrev|mad_u32_u24|mul_lo|mul_hi|lshl_or|and_or|or3|xad|add3|lshl_add)")),
    ("mul/mad other", re.compile(r"^v_(mad|mul)")),
    ("ds_read", re.compile(r"^ds_read")),
    ("ds_write", re.compile(r"^ds_write")),
    ("global/buffer load", re.compile(r"^(global|buffer|flat)_load")),
    ("global/buffer store", re.compile(r"^(global|buffer|flat)_store")),
    ("s_nop", re.compile(r"^s_nop")),
    ("s_waitcnt/barrier", re.compile(r"^s_(waitcnt|barrier)")),
    ("salu", re.compile(r"^s_")),
    ("other valu", re.compile(r"^v_")),
]


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return out.splitlines()


def kernels(path):
    """{mangled: [instruction mnemonics]} for every kernel body in the file."""
    ks, cur = {}, None
    for line in open(path):
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            ks[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith("\t.section") or line.startswith(".Lfunc_end"):
            cur = None
            continue
        t = line.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        ks[cur].append(t.split()[0])
    return ks


def classify(ops):
    c = collections.Counter()
    for op in ops:
        for name, rx in CLASSES:
            if rx.match(op):
                c[name] += 1
                break
        else:
            c["?" + op] += 1
    return c


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    ks = kernels(path)
    names = list(ks)
    dem = dict(zip(names, demangle(names)))
    for k in names:
        d = dem[k]
        if subs and not all(s in d for s in subs):
            continue
        c = classify(ks[k])
        valu = sum(v for n, v in c.items() if not n.startswith(("ds_", "global", "s_", "salu")))
        print(f"== {d}\n   total {len(ks[k])}, VALU {valu}")
        for name, _ in CLASSES:
            if c.get(name):
                print(f"   {name:28s} {c[name]:6d}")
        for n, v in sorted(c.items()):
            if n.startswith("?"):
                print(f"   {n:28s} {v:6d}")


if __name__ == "__main__":
    main()
