"""GPU: bench.py's output contract on small shapes, one child process per workload.

The driver parses one JSON line per run; these runs check its keys (metric, value, unit,
roofline with bound / achieved / peak / unit / frac / traffic, cpu_baseline with value / unit /
cores / kind / sample) and the parity flags the bench computes against the oracle.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=100):
    env = dict(os.environ)
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_common(d, steps):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["value"] > 0 and d["higher_is_better"] is True
    assert d["scaling"] in ("weak", "strong") and "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] in ("GB/s", "TFLOP/s")
    assert rf["achieved"] > 0 and rf["peak"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert "traffic" in rf


def _check_cpu(d):
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["sample"]
    assert cb["unit"] == d["unit"]


def test_bench_ligero_sharded_small(gpu):
    d = _bench("--mode", "sharded", "--steps", "4", "--warmup", "2", "--log-len", "16", "--verify-reps", "1")
    _check_common(d, 4)
    _check_cpu(d)
    assert d["parity_root_vs_oracle"] is True
    assert d["verify"]["parity_vs_oracle"] is True and d["verify"]["ms"] > 0
    assert d["config"]["n_rows"] * d["config"]["n_per_row"] == 1 << 16
    # the sharded driver line: the kept proof equals the oracle's, one commitment's latency
    assert d["scaling"] == "weak" and d["commitments_per_step"] == 1 and d["parity_proof_vs_oracle"] is True
    assert d["latency"]["commit_ms"] > 0 and d["latency"]["prove_ms"] > 0
    assert "traffic_source" in d["roofline"] and d["world_formed"] == 1
    assert d["parity_ok"] is True and d["steps_agree"] is True


def test_bench_ligero_default_small(gpu):
    """the default engine at --gpus 1 is independent commitments in flight (replicas)"""
    d = _bench("--steps", "4", "--warmup", "2", "--log-len", "16", "--verify-reps", "1")
    _check_common(d, 4)
    _check_cpu(d)
    assert d["scaling"] == "weak" and d["parity_root_vs_oracle"] is True and d["pipeline"] == 4
    assert d["verify"]["parity_vs_oracle"] is True
    assert d["latency"]["commit_ms"] > 0 and d["world_formed"] == 1
    assert d["parity_ok"] is True and d["sharded_n1"]["root_equals_replicas"] is True


@pytest.mark.parametrize("source", ["host", "host-pinned"])
def test_bench_ligero_host_input_small(gpu, source):
    """--input host / host-pinned: every timed step commits from host memory (lcpc_commit_new,
    the reference's commit(&[F])); the line carries the PCIe figures and stays right"""
    d = _bench("--steps", "4", "--warmup", "2", "--log-len", "16", "--verify-reps", "1", "--sharded-n1", "0",
               "--input", source)
    _check_common(d, 4)
    assert d["parity_ok"] is True and d["steps_agree"] is True
    pc = d["pcie"]
    assert pc["input"] == source and pc["bytes_per_step"] == (1 << 16) * 16
    assert pc["achieved_gbs"] > 0 and pc["pinned_copy_peak_gbs"] > 0 and pc["pageable_copy_gbs"] > 0
    assert pc["library_read_pinned_source"] is (source == "host-pinned")
    assert "host" in d["data"] and "host-resident" in d["config"]["workload"]


def test_bench_ligero_caller_transcript_small(gpu):
    """--transcript caller: prove drives a caller-owned transcript through lcpc_transcript_ops;
    same roots, the oracle's proof and verifier value"""
    d = _bench("--steps", "4", "--warmup", "2", "--log-len", "16", "--verify-reps", "1", "--sharded-n1", "0",
               "--transcript", "caller")
    _check_common(d, 4)
    assert d["parity_ok"] is True and d["verify"]["parity_vs_oracle"] is True


def test_bench_pos_host_input_small(gpu):
    d = _bench("--code", "pos", "--steps", "2", "--warmup", "2", "--pos-bytes", str(1 << 20), "--input", "host")
    _check_common(d, 2)
    assert d["parity_ok"] is True and d["pcie"]["bytes_per_step"] == 1 << 20
    assert "lcpc_pos_commit_bytes" in d["config"]["commit_call"]


def _bench_ranks(world, extra_env, *args, timeout=280):
    env = dict(os.environ, LCPC_BENCH_BACKEND="gloo", LCPC_BENCH_SHARE_GPU="1", **extra_env)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), *args], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_self_checking(d, world):
    """an N > 1 line carries its own evidence of a right answer: the oracle's root against every
    warm-up and timed step, the kept proof and the verifier's value (the timed cpu_baseline is the
    N = 1 line's: at N > 1 the oracle runs once, as the checker)"""
    # one GPU box: the ranks share GPU 0 (the rehearsal), and the line says so rank by rank
    assert d["devices"] == [0] * world and d["rehearsal"] is True and len(d["ranks"]) == world
    assert d["n_gpus"] == world and d["world_formed"] == world
    # weak (the default): N row-sharded commitments per step; strong: one
    pps = world if d["scaling"] == "weak" else 1
    assert d["scaling"] in ("weak", "strong") and d["commitments_per_step"] == pps
    assert d["commitments_timed"] == d["steps"] * pps
    assert d["parity_root_vs_oracle"] is True and d["parity_proof_vs_oracle"] is True
    ps = d["parity_steps_vs_oracle"]
    assert ps["steps"] == (d["steps"] + d["warmup"]) * pps and ps["equal"] == ps["steps"]
    assert d["steps_agree"] is True and d["parity_ok"] is True
    assert d["verify"]["parity_vs_oracle"] is True
    assert "cpu_baseline" not in d


@pytest.mark.timeout(300)
def test_bench_sharded_two_ranks_one_gpu(gpu):
    """`bench.py --gpus 2` spawns two ranks; on a one-GPU box they share the GPU and exchange over
    host-staged gloo collectives (RCCL refuses two ranks on one device)."""
    d = _bench_ranks(2, {}, "--steps", "4", "--warmup", "2", "--log-len", "16", "--verify-reps", "1")
    _check_self_checking(d, 2)
    assert "gloo" in d["config"]["exchanges"] and d["scaling"] == "weak"


@pytest.mark.timeout(300)
def test_bench_sharded_two_ranks_one_gpu_strong(gpu):
    """--sharded-scaling strong: one commitment per step at every N (the round-5 line)"""
    d = _bench_ranks(2, {}, "--steps", "4", "--warmup", "2", "--log-len", "16", "--verify-reps", "1",
                     "--sharded-scaling", "strong")
    _check_self_checking(d, 2)
    assert d["scaling"] == "strong"


@pytest.mark.timeout(300)
def test_bench_sharded_two_ranks_rccl_one_gpu(gpu):
    """the same line through the library's RCCL communicator (per-rank NCCL_HOSTID: RCCL's socket
    transport over loopback), with the default cpu_baseline setting: every N > 1 line self-checks against the oracle"""
    d = _bench_ranks(2, {"LCPC_BENCH_RCCL_SAME_GPU": "1"}, "--steps", "4", "--warmup", "2", "--log-len", "16",
                     "--verify-reps", "1")
    _check_self_checking(d, 2)
    assert "RCCL" in d["config"]["exchanges"]


def test_bench_encode_small(gpu):
    d = _bench("--code", "encode", "--steps", "4", "--warmup", "2", "--log-len", "14")
    _check_common(d, 4)
    _check_cpu(d)
    assert d["parity_vs_oracle"] is True


def test_bench_sdig_small(gpu):
    d = _bench("--code", "sdig", "--steps", "2", "--warmup", "2", "--log-len", "14", "--cpu-baseline", "off",
               "--verify-reps", "1")
    _check_common(d, 2)
    assert "cpu_baseline" not in d


@pytest.mark.parametrize("pos_eval", ["fused", "separate"])
def test_bench_pos_small(gpu, pos_eval):
    d = _bench("--code", "pos", "--steps", "2", "--warmup", "2", "--pos-bytes", str(1 << 20), "--pos-eval", pos_eval)
    assert ("lcpc_pos_commit_eval_bytes_device" in d["config"]["commit_call"]) == (pos_eval == "fused")
    _check_common(d, 2)
    _check_cpu(d)
    assert d["parity_root_vs_oracle"] and d["parity_eval_vs_oracle"] and d["parity_cols_vs_oracle"]
    assert d["parity_ok"] is True
