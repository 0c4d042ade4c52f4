"""tools/rust_golden (the Rust program that prints golden.json's keys from the reference crates;
not compiled here) promises exactly golden.json's layout: its KEYS table, case by case."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rust_keys():
    src = open(os.path.join(ROOT, "tools", "rust_golden", "src", "main.rs")).read()
    lists = {m.group(1): re.findall(r'"([^"]+)"', m.group(2))
             for m in re.finditer(r"const (\w+_KEYS): &\[&str\] = &\[(.*?)\];", src, re.S)}
    table = re.search(r"const KEYS: &\[\(&str, &\[&str\]\)\] = &\[(.*?)\];", src, re.S).group(1)
    return {case: lists[name] for case, name in re.findall(r'\("([^"]+)",\s*(\w+_KEYS)\)', table)}, src


def test_rust_golden_layout_matches_fixtures():
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    keys, src = _rust_keys()
    assert set(keys) == set(gold)
    for case, ks in keys.items():
        assert sorted(ks) == sorted(gold[case]), case
    # every case is produced by main() (inserted under its own name)
    for case in keys:
        assert f'out.insert("{case}"' in src, case


def test_rust_golden_pins_the_reference_versions():
    toml = open(os.path.join(ROOT, "tools", "rust_golden", "Cargo.toml")).read()
    for dep in ("lcpc-2d", "lcpc-ligero-pc", "lcpc-brakedown-pc", "lcpc-test-fields", "fffft"):
        assert re.search(rf"^{dep} = \{{ path = ", toml, re.M), dep
    for dep, ver in (("ff", "0.13"), ("merlin", "2.0"), ("rand_chacha", "0.3"), ("blake3", "1.5")):
        assert re.search(rf'^{dep} = (\{{ version = )?"{re.escape(ver)}"', toml, re.M), dep
