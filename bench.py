#!/usr/bin/env python3
"""bench.py -- committed field-elements/s (commit + open) of a 2^24-coefficient Ligero
commitment over Ft127 on MI355X (BASELINE.json metric; config 3).

One step = LcCommit::commit of 2^24 Ft127 coefficients already resident in HBM (encode every
row with the R-S NTT, hash every column with BLAKE3, build the Merkle tree) followed by
LcCommit::prove (2 degree tests + evaluation row combination, Merlin transcript over every
row-combination coefficient, 309 column openings with Merkle paths): lcpc-2d/src/lib.rs:651-700
and :1034-1123, dims 512 x 32768 -> 65536 (rho = 1/2, lcpc-ligero-pc/src/lib.rs:70-112).

Engines (--mode; the default, auto, is sharded for --gpus > 1 and replicas on one GPU):
  sharded (cfg3): every commitment's rows are split over the N ranks (one process per GPU,
    RCCL over xGMI through liblcpc_mi's own communicator), run by the library's pipelined driver
    lcpc_sharded_commit_prove_many (csrc/shard_native.cpp): the exchanges of the commitments in
    flight go out in one fixed order per tick, the transcript of commitment i runs on rank i % N.
    At N = 1 the same driver runs with no exchanges.  --sharded-scaling weak (default): a step is
    N commitments (one commitment's work per GPU per step, "scaling": "weak"); strong: a step is
    one commitment whatever N ("scaling": "strong", the round-5 line).
  replicas: every rank commits and opens its own polynomial (independent objects), host
    threads keep --pipeline commitments in flight; "scaling": "weak".

Launch: `python bench.py --gpus N` spawns N ranks under torch.distributed.run itself (before any
torch / HIP import); under torch.distributed.run (WORLD_SIZE set) --gpus must equal the world
size.  The barrier and the max-over-ranks reduction of the timed region use torch.distributed.

Printed JSON line: the metric, a "roofline" object for the dominant kernel (the encode; HIP
events on the launching stream, on serial launches after the timed region) and a
"cpu_baseline" object (the C restatement under oracle/, run on the host cores of rank 0 at
N = 1: warm-up + median of 5, which doubles as the bit-exactness check of the root).
"""
import argparse
import glob
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
LEAF_PEAK_GCPS = 54.2    # BLAKE3 compressions/s with no loads (tools/microbench/leafbench.hip, MI355X)
SEED = 0x1CDC2024       # coefficients = F::random(ChaCha20Rng::seed_from_u64(SEED))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--mode", choices=["auto", "sharded", "replicas"], default="auto",
                    help="sharded: every commitment's rows split over the ranks, N commitments per step by "
                         "default (--sharded-scaling; the library's "
                         "pipelined driver; the BASELINE cfg3 configuration); replicas: independent "
                         "commitments per rank on host threads; auto (default): sharded for --gpus > 1, "
                         "replicas on one GPU, where there is nothing to split and independent "
                         "commitments in flight are the faster single-GPU engine")
    ap.add_argument("--sharded-n1", type=int, default=1,
                    help="N = 1 replicas lines (ligero): also time the row-sharded engine on the one GPU "
                         "(the N = 1 base of the sharded N > 1 lines) and report it as \"sharded_n1\": "
                         "1 in a fresh child process (as an N > 1 rank starts), 2 in this process after "
                         "the replicas run, 0 off")
    ap.add_argument("--sharded-scaling", choices=["weak", "strong"], default="weak",
                    help="sharded engine: weak (default) = N row-sharded commitments per step, so each GPU "
                         "does one commitment's work per step at every N; strong = one commitment per step "
                         "(K = 20 then holds 20 commitments at every N, and the last one's serial "
                         "transcript dominates an N = 8 run: DESIGN §6)")
    ap.add_argument("--lag", type=int, default=0,
                    help="sharded driver: ticks between a row-combination gather and the next challenge "
                         "broadcast (0: the library's choice)")
    ap.add_argument("--plumbing-only", action="store_true",
                    help="multi-process plumbing check without a GPU (spawn, world size, barrier, "
                         "max-over-ranks over gloo); prints the JSON line with value null")
    ap.add_argument("--log-len", type=int, default=None, help="log2 coefficients (24; 20 for --code encode)")
    ap.add_argument("--field", default="Ft127")
    ap.add_argument("--rho", default="1/2",
                    help="Ligero code rate (LigeroEncodingRho<F, U1, U2>, lcpc-ligero-pc/src/lib.rs:32-37): 1/2 "
                         "is LigeroEncoding (the BASELINE metric, :189); 1/4 is the reference's commit_bench "
                         "(lcpc-ligero-pc/src/bench.rs:43, the 2021 published commit timings)")
    ap.add_argument("--code", choices=["ligero", "sdig", "pos", "encode", "sdig-encode"], default="ligero",
                    help="ligero: R-S / NTT rows (the BASELINE metric, cfg3); sdig: Brakedown "
                         "SdigCode3 expander code, seed 0 (cfg4); pos: proof-of-storage request "
                         "on a resident file (cfg5); encode: the Ligero R-S encode alone (cfg2); "
                         "sdig-encode: the Brakedown encode alone (cfg4's rows, LcEncoding::encode)")
    ap.add_argument("--batch", type=int, default=1,
                    help="sdig-encode: commitments' rows per encode call (72 rows each at 2^24): the "
                         "expander levels gather batch x 72-row runs per nonzero")
    ap.add_argument("--pos-bytes", type=int, default=1 << 30, help="file size for --code pos")
    ap.add_argument("--pos-commit", choices=["bytes", "elements"], default="bytes",
                    help="--code pos: commit the file image in one call (lcpc_pos_commit_bytes_device) or pack "
                         "it to elements first (lcpc_pos_bytes_to_field_device + lcpc_commit_new_device)")
    ap.add_argument("--cpu-baseline", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every core this process may use (affinity and cgroup quota)")
    ap.add_argument("--cpu-reps", type=int, default=5, help="cpu_baseline: timed runs after one warm-up (median)")
    ap.add_argument("--cpu-baseline-1core", choices=["auto", "on", "off"], default="auto",
                    help="also time the oracle on one thread (auto: the ligero workload)")
    ap.add_argument("--no-prof", action="store_true", help="disable HIP-event kernel timing")
    ap.add_argument("--prof-timed", action="store_true",
                    help="also time every kernel inside the timed region with HIP events (their "
                         "recording costs ~10%% of the throughput; off by default, the roofline "
                         "launches after the timed region are always timed unless --no-prof)")
    ap.add_argument("--stream-mode", choices=["pool", "serial"], default="pool",
                    help="pool: each call leases its own HIP stream (kernels of different "
                         "commitments overlap); serial: one in-order stream per GPU")
    ap.add_argument("--verify-reps", type=int, default=8,
                    help="verifies of one proof timed after the timed region (ligero/sdig; 0: skip)")
    ap.add_argument("--roofline-steps", type=int, default=3,
                    help="serial steps after the timed region whose encode launches give the roofline")
    ap.add_argument("--commit-slots", type=int, default=-1,
                    help="replicas (ligero / sdig / pos): commits admitted to the GPU at once, first come first "
                         "served (0: no limit; default 4, 2 for --code sdig, none for pos, from sweeps on the box).  "
                         "Commits then finish in order and each proof's serial host "
                         "transcript starts while later commits run, instead of every commit of a wave "
                         "finishing together at its end")
    ap.add_argument("--pos-eval", choices=("fused", "separate"), default="separate",
                    help="--code pos with a device file image (--pos-commit bytes): separate (default) = "
                         "lcpc_pos_commit_bytes_device, then lcpc_pos_eval_encoded's own HBM-bound pass, which "
                         "overlaps the other requests' VALU-bound kernels; fused = both in one call "
                         "(lcpc_pos_commit_eval_bytes_device: the evaluation summed in the leaf hashing's pass), "
                         "4 %% faster for one request alone, not faster with 4 in flight (DESIGN §5a)")
    ap.add_argument("--input", choices=("device", "host", "host-pinned"), default="device",
                    help="replicas (ligero / sdig / pos): where each step's input is when it starts.  device "
                         "(default, the headline): resident in HBM.  host: pageable host memory, the caller's "
                         "&[F] of LcCommit::commit (lcpc-2d/src/lib.rs:651) or the file image a PoS server read "
                         "from disk (networking/server.rs:670-679) -- lcpc_commit_new / lcpc_pos_commit_bytes "
                         "move it across PCIe inside the timed step.  host-pinned: the same from page-locked "
                         "memory (the DMA engine reads it directly)")
    ap.add_argument("--transcript", choices=("library", "caller"), default="library",
                    help="ligero / sdig replicas: prove with the library's own Merlin transcript, or with a "
                         "caller-owned one driven through lcpc_transcript_ops (CallerTranscript over a "
                         "library transcript: every absorb / squeeze crosses the callback boundary)")
    ap.add_argument("--timeline", default=None,
                    help="replicas (ligero / sdig): write every timed step's gate / commit / prove "
                         "times (s, from the start of the timed region) to this JSON file")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="independent commitments in flight per GPU (host threads); the serial "
                         "Merlin transcript of one overlaps the kernels of the others.  0: 16, 20 for "
                         "--code sdig, or 4 for --code pos (a 1 GiB request's 2.3 GiB codeword per slot: deeper "
                         "pipelines only contend for HBM)")
    args = ap.parse_args()
    if args.code in ("sdig", "encode", "sdig-encode"):
        args.mode = "replicas"  # cfg2 / cfg4 run as independent steps per rank
    if args.mode == "auto":
        args.mode = "sharded" if args.gpus > 1 else "replicas"
    if args.log_len is None:
        args.log_len = 20 if args.code == "encode" else 24
    if args.code == "sdig-encode" and args.pipeline <= 0:
        args.pipeline = 4
    num, den = (int(x) for x in args.rho.split("/"))
    args.rho_t = (num, den)
    if args.commit_slots < 0:
        args.commit_slots = {"sdig": 2, "pos": 0}.get(args.code, 4)
    if args.pipeline <= 0:
        # sdig: 20, its proofs being 26 ms of host transcript each (K = 20: 5.6-6.05 against
        # 5.1-5.3 G/s at 16, 4.5-4.9 at 24; tools/evidence/r03/workers_sweep.sh)
        args.pipeline = {"pos": 4, "sdig": 20}.get(args.code, 16)
    return args


# ---------------------------------------------------------------- multi-process plumbing
def dist_env():
    """(rank, local_rank, world) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_dist(world, local_rank, backend="nccl"):
    """One process per GPU; returns torch.distributed or None at N = 1 (RCCL is "nccl")."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend=backend)
    return dist


def sync_barrier(dist, device_sync=None):
    """barrier over ranks, then drain this rank's device (both sides of the timed region)."""
    if dist is not None:
        dist.barrier()
    if device_sync is not None:
        device_sync()


def max_over_ranks(dist, x, device="cpu"):
    """The job's wall time is its slowest rank's."""
    if dist is None:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replica_seed(rank):
    """Each replica commits its own polynomial (independent objects, no data-path collective)."""
    return SEED + rank


# the variables of the one-GPU rehearsals of N ranks (LCPC_BENCH_SHARE_GPU: every rank on GPU 0;
# LCPC_BENCH_BACKEND=gloo: host-staged exchanges; LCPC_BENCH_RCCL_SAME_GPU / NCCL_HOSTID: RCCL over
# loopback sockets).  A plain `--gpus N` run sets none of them.
REHEARSAL_VARS = ("LCPC_BENCH_BACKEND", "LCPC_BENCH_SHARE_GPU", "LCPC_BENCH_RCCL_SAME_GPU", "NCCL_HOSTID")
COMM_INFO = {}  # the library communicator of this rank's sharded run (nranks, is_rccl), when one exists


def device_binding(local_rank):
    """(the HIP device this rank binds, the rehearsal variables set): one GPU per rank, device =
    LOCAL_RANK, unless the one-GPU rehearsal puts every rank on GPU 0"""
    share = os.environ.get("LCPC_BENCH_SHARE_GPU") == "1"
    return (0 if share else local_rank), {k: os.environ[k] for k in REHEARSAL_VARS if k in os.environ}


def rank_identity(rank, local_rank, device_idx, torch=None):
    """what this rank ran on: its device index and, with a GPU, the device's UUID and PCI bus
    (distinct per physical GPU), the rehearsal variables, and the library communicator"""
    ident = {"rank": rank, "local_rank": local_rank, "device": device_idx,
             "rehearsal_env": device_binding(local_rank)[1],
             "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")}
    if torch is not None:
        props = torch.cuda.get_device_properties(device_idx)
        ident["device_uuid"] = str(getattr(props, "uuid", "") or "")
        ident["pci_bus_id"] = getattr(props, "pci_bus_id", None)
    if COMM_INFO:
        ident["comm_nranks"] = COMM_INFO.get("nranks")
        ident["comm_is_rccl"] = COMM_INFO.get("is_rccl")
    return ident


def fold_identities(dist, ident):
    """every rank's identity on every rank (a collective), and the summary rank 0 prints: the
    devices the ranks bound, how many distinct GPUs those are, the communicator's rank count when
    the exchanges ran over RCCL, and whether any rank ran a one-GPU rehearsal"""
    ids = [ident]
    if dist is not None:
        ids = [None] * dist.get_world_size()
        dist.all_gather_object(ids, ident)
    uu = [i.get("device_uuid") or f"index:{i['device']}" for i in ids]
    rccl = [i.get("comm_nranks") for i in ids if i.get("comm_is_rccl")]
    return {"devices": [i["device"] for i in ids], "distinct_gpus": len(set(uu)),
            "rccl_nranks": rccl[0] if rccl and len(rccl) == len(ids) else None,
            "rehearsal": any(i["rehearsal_env"] for i in ids), "ranks": ids}


def cgroup_throttle():
    """cgroup v2 cpu.stat throttling counters (nr_throttled, throttled_usec), or None."""
    try:
        kv = dict(line.split() for line in open("/sys/fs/cgroup/cpu.stat"))
        return {k: int(kv[k]) for k in ("nr_periods", "nr_throttled", "throttled_usec") if k in kv}
    except (OSError, ValueError):
        return None


def host_cpu_use(c0, c1, elapsed):
    """Host CPU time this process spent in the timed region, in cores (user + system)."""
    quota = None
    try:  # cgroup v2 CPU quota, "max 100000" when unlimited
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    return {"cores_busy": ((c1.user - c0.user) + (c1.system - c0.system)) / max(elapsed, 1e-9),
            "user_s": c1.user - c0.user, "system_s": c1.system - c0.system,
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": quota,
            "host_wait": os.environ.get("LCPC_HOST_WAIT", "default")}


def job_throughput(n_per_step, steps, world, elapsed):
    """Whole-job rate: the units all ranks processed / the max-over-ranks time."""
    return n_per_step * steps * world / elapsed


def ntt_muls(n):
    """Montgomery products of one length-n four-step fft_io (the last stage of each pass is
    multiplication-free): (n/2)(log2 n - 2) butterflies + n inter-pass twiddles."""
    lg = n.bit_length() - 1
    return (n // 2) * max(lg - 2, 0) + n


def row1_active(n, file_image=False):
    """whether the one-pass Ft63 row kernel (csrc/ntt_row1.hpp) encodes these rate-1/2 2^n-point
    rows: the library's AUTO row kernel takes it for the file-image commit
    (lcpc_pos_commit_bytes_device) and the four-step pair for element rows"""
    return n == 1 << 15 and file_image


def pos_ntt_muls(n, file_image=False):
    """(products per row, model) of the Ft63 encode at the PoS dims: the one-pass kernel does
    stage 0 (16384, the sum branch's R^-1 scaling by a reduction counted as half a product),
    stages 1-9 (16384 each) and round 3's 49 nontrivial products per thread; the four-step pair
    ntt_muls(n)"""
    if row1_active(n, file_image):
        return (n // 2) * 10 + 1024 * 49 + n // 4, ("one-pass 2^15 DIF (ntt_row1): stages 0-9 all products, "
                                                    "stages 10-14 the 49 nontrivial per thread, + n/2 half-cost "
                                                    "R^-1 reductions")
    return ntt_muls(n), "four-step fft_io: (n/2)(log2 n - 2) general-twiddle butterflies + n inter-pass twiddles per row"


def leaf_compressions(n_rows, n_cols, elem_bytes):
    """BLAKE3 compressions of the column leaves (lcpc-2d/src/lib.rs:736-775): each leaf message
    is 32 zero bytes + n_rows elements, one compression per 64-byte block (the last one of a
    chunk included), plus the chunk-merge parents (chunks - 1 per column)."""
    msg = 32 + n_rows * elem_bytes
    blocks = -(-msg // 64)
    chunks = -(-msg // 1024)
    return n_cols * (blocks + chunks - 1)


class Workload:
    """One bench configuration: `step(slot)` runs one pass of the hot path on resident inputs."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


INPUT_NOTE = {"device": "resident in HBM",
              "host": "in pageable host memory (numpy; crossed to HBM inside every timed step)",
              "host-pinned": "in page-locked host memory (torch pin_memory; crossed to HBM inside every timed step)"}
INPUT_WORKLOAD = {"device": "", "host": ", host-resident input (pageable)",
                  "host-pinned": ", host-resident input (page-locked)"}


def rho_note(args):
    """the metric name of a non-default rate (the BASELINE metric is rho = 1/2)"""
    return "" if args.rho == "1/2" else f", rho={args.rho}"


def ligero_or_sdig(args, L, torch, rank, local_rank):
    """cfg3 (Ligero, the BASELINE metric) and cfg4 (Brakedown SdigCode3, seed 0): commit + open
    of one polynomial (lcpc-2d/src/lib.rs:651-700, 1034-1123)."""
    fid = {"Ft63": L.FT63, "Ft127": L.FT127, "Ft255": L.FT255}[args.field]
    nl = L.limbs(fid)
    n = 1 << args.log_len
    sdig = args.code == "sdig"
    enc = L.SdigEncoding.new(fid, n, 0) if sdig else L.LigeroEncoding.new(fid, n, args.rho_t)
    n_rows, n_per_row, n_cols = enc.get_dims(n)
    nco, ndt = enc.get_n_col_opens(), enc.get_n_degree_tests()
    # synthetic inputs (host RNG of the product library), then resident in HBM
    coeffs = L.field_random(fid, n, replica_seed(rank))
    outer = L.field_random(fid, n_rows, 7)  # prove accepts any outer tensor of n_rows elements
    host_src = None
    if args.input == "device":
        d_coeffs = torch.from_numpy(coeffs.view(np.int64)).to(f"cuda:{local_rank}")

        def commit():
            return L.LcCommit.commit_device(d_coeffs.data_ptr(), n, enc)
    else:
        # the caller's coefficients in host memory: LcCommit::commit(&[F]) (lib.rs:651-682)
        host_src = (torch.from_numpy(coeffs.view(np.int64)).pin_memory().numpy().view(np.uint64)
                    if args.input == "host-pinned" else coeffs)

        def commit():
            return L.LcCommit.commit(host_src, enc)

    gate = threading.Semaphore(args.commit_slots) if args.commit_slots > 0 else None

    timeline = []  # (slot, t_gate, t_commit_start, t_commit_end, t_prove_end) with --timeline

    def transcript(root):
        tr = L.Transcript(b"test transcript")
        tr.append_message(b"polycommit", root)
        tr.append_message(b"ncols", nco.to_bytes(8, "big"))
        # --transcript caller: the caller owns the transcript and prove drives it through
        # lcpc_transcript_ops (here a library transcript behind Python callbacks)
        return L.CallerTranscript(tr) if args.transcript == "caller" else tr

    def step(slot):
        t_a = time.perf_counter()
        if gate is not None:
            with gate:
                t_b = time.perf_counter()
                c = commit()
        else:
            t_b = t_a
            c = commit()
        t_c = time.perf_counter()
        root = c.get_root()
        c.prove(outer, enc, transcript(root))
        if args.timeline:
            timeline.append((slot, t_a, t_b, t_c, time.perf_counter()))
        return root

    inner = L.field_random(fid, n_per_row, 8)  # verify returns sum_c inner[c] p_eval[c]
    cpu_verify = []  # (ms, accepted, evaluation) per cpu_baseline call

    def latency(reps):
        """one commitment, serial: commit and prove wall clock (median of reps)"""
        cs, ps = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            c = commit()
            root = c.get_root()
            t2 = time.perf_counter()
            c.prove(outer, enc, transcript(root))
            cs.append(1e3 * (t2 - t1))
            ps.append(1e3 * (time.perf_counter() - t2))
        cs.sort()
        ps.sort()
        return {"commit_ms": cs[len(cs) // 2], "prove_ms": ps[len(ps) // 2],
                "what": f"one commitment, serial: LcCommit::{'commit_device' if args.input == 'device' else 'commit'} "
                        f"and LcCommit::prove (median of {reps})"}

    def cpu_baseline(O):
        o_enc = (O.Encoding.sdig(fid, n_per_row, seed=0, code_id=3) if sdig
                 else O.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt, rho=args.rho_t))
        t1 = time.perf_counter()
        oc = O.Commit(o_enc, coeffs.reshape(-1))
        op = oc.prove(o_enc, outer.reshape(-1), O.standard_transcript(nco, oc.root()))
        dt = time.perf_counter() - t1
        # the oracle's verify of its own proof (outside the commit+open figure)
        t2 = time.perf_counter()
        rc, ev = op.verify(oc.root(), outer.reshape(-1), inner.reshape(-1), o_enc,
                           O.standard_transcript(nco, oc.root()))
        cpu_verify.append((1e3 * (time.perf_counter() - t2), rc == 0, ev))
        return dt, oc.root(), f"one full commit+open of the same 2^{args.log_len} {args.field} workload"

    def verify_bench(reps):
        """LcEvalProof::verify (lcpc-2d/src/lib.rs:862-982) of one proof of this workload: the
        verifier's encodes of p_random / p_eval and the column checks, timed over `reps` calls."""
        c = commit()
        root = c.get_root()

        def tr():
            t = L.Transcript(b"test transcript")
            t.append_message(b"polycommit", root)
            t.append_message(b"ncols", nco.to_bytes(8, "big"))
            return t

        pf = c.prove(outer, enc, tr())
        ev = pf.verify(root, outer, inner, enc, tr())
        t1 = time.perf_counter()
        for _ in range(reps):
            pf.verify(root, outer, inner, enc, tr())
        return 1e3 * (time.perf_counter() - t1) / reps, ev

    B = 8 * nl
    name = (f"Brakedown (SdigCode3, seed 0) commit+open, {args.field}, 2^{args.log_len} coeffs, " if sdig
            else f"Ligero commit+open, {args.field}, 2^{args.log_len} coeffs, rho={args.rho}, ")
    return Workload(
        units=n, unit="field-elements/s", bytes_per_unit=B,
        metric=("committed field-elements/s (commit+open), 2^24-coeff Brakedown (cfg4)" if sdig else
                "committed field-elements/s (commit+open), 2^24-coeff Ligero, 1/2/4/8 GPU" + rho_note(args)),
        dtype=f"u64x{nl} ({args.field} Montgomery limbs)",
        data=f"synthetic: F::random(ChaCha20Rng::seed_from_u64({SEED:#x} + rank)), " + INPUT_NOTE[args.input],
        config={"workload": name + f"{n_rows}x{n_per_row}->{n_cols}, {nco} column opens, {ndt} degree tests, "
                                   f"BLAKE3 Merkle" + INPUT_WORKLOAD[args.input],
                "field": args.field, "len": n, "n_rows": n_rows, "n_per_row": n_per_row, "n_cols": n_cols,
                "n_col_opens": nco, "n_degree_tests": ndt},
        step=step, cpu_baseline=cpu_baseline, input_bytes=n * B, verify_bench=verify_bench, cpu_verify=cpu_verify,
        latency=latency,
        prepare=lambda: enc.prepare_thread(n_rows), reserve=lambda count: enc.reserve(n, count),
        timeline=timeline,
        enc_kernels=("transpose", "sdig_encode") if sdig else ("ntt_pass_a", "ntt_pass_b", "ntt_small"),
        enc_kernel_desc=("sdig_encode = transpose + 13 SpMM / Reed-Solomon levels (per commit, all rows)" if sdig
                         else f"ntt_encode = ntt_pass_a + ntt_pass_b (one launch each per commit, all {n_rows} rows)"),
        # encode bytes per commit (read the coefficients, write the codeword; SDIG
        # also streams its code matrices once: 16-B values + 4-B indices)
        algo_bytes=n_rows * n_per_row * B + n_rows * n_cols * B + (enc.matrix_nnz * (B + 4) if sdig else 0),
        leaf_compressions=leaf_compressions(n_rows, n_cols, B),
        gather_bytes=(n_rows * enc.matrix_nnz * B + n_rows * (n_cols - n_per_row) * B + enc.matrix_nnz * 20
                      + 3 * n_rows * n_per_row * B) if sdig else 0,
        traffic_key=(n, args.field, args.code),
        mul_count=(n_rows * enc.matrix_nnz if sdig else n_rows * ntt_muls(n_cols)),
        mul_model=("one product per nonzero per row" if sdig else
                   "four-step fft_io: (n/2)(log2 n - 2) general-twiddle butterflies + n inter-pass twiddles per row"))


def encode_workload(args, L, torch, rank, local_rank):
    """cfg2: the Ligero R-S encode alone (LcEncoding::encode on every row of a 2^20-coefficient
    commitment, lcpc-ligero-pc/src/lib.rs:162-164 -> fft_io), device rows in, device rows out."""
    fid = {"Ft63": L.FT63, "Ft127": L.FT127, "Ft255": L.FT255}[args.field]
    nl = L.limbs(fid)
    n = 1 << args.log_len
    enc = L.LigeroEncoding.new(fid, n, args.rho_t)
    n_rows, n_per_row, n_cols = enc.get_dims(n)
    coeffs = L.field_random(fid, n_rows * n_per_row, replica_seed(rank))
    dev = f"cuda:{local_rank}"
    d_src = torch.from_numpy(coeffs.view(np.int64)).to(dev)
    dst = [torch.empty(n_rows * n_cols * nl, dtype=torch.int64, device=dev) for _ in range(max(1, args.pipeline))]
    torch.cuda.synchronize()

    def step(slot):
        enc.encode_rows_device(d_src.data_ptr(), n_per_row, n_per_row, dst[slot].data_ptr(), n_cols, n_rows)
        return None

    ocache = {}

    def cpu_baseline(O):
        # the oracle's fft_io on every row of the same workload, rows in parallel on the threads
        # of_set_threads gives it (the reference encodes a commitment's rows in parallel,
        # lcpc-2d/src/lib.rs:677-682), output buffer allocated once; whole passes until about 5 s,
        # rate per pass; then every GPU row against the oracle's
        if not ocache:
            ocache["enc"] = O.Encoding.ligero(fid, n_per_row, n_cols, rho=args.rho_t)
            ocache["out"] = np.empty(n_rows * n_cols * nl, np.uint64)
        o_enc, out = ocache["enc"], ocache["out"]
        passes, t1 = 0, time.perf_counter()
        while True:
            o_enc.encode_rows(coeffs, n_rows, out)
            passes += 1
            if time.perf_counter() - t1 >= 5.0 or passes >= 256:
                break
        dt = (time.perf_counter() - t1) / passes
        step(0)
        torch.cuda.synchronize()
        got = dst[0].cpu().numpy().view(np.uint64).reshape(-1)
        ok = bool(np.array_equal(got, out))
        return dt, ok, (f"fft_io of all {n_rows} rows of the same 2^{args.log_len} {args.field} workload "
                        f"(oracle of_enc_encode_rows), {passes} passes, time per pass")

    B = 8 * nl
    return Workload(
        units=n_rows * n_per_row, unit="field-elements/s", bytes_per_unit=B,
        metric=f"encoded field-elements/s (Ligero R-S encode), 2^{args.log_len}-coeff {args.field} (cfg2)",
        dtype=f"u64x{nl} ({args.field} Montgomery limbs)",
        data=f"synthetic: F::random(ChaCha20Rng::seed_from_u64({SEED:#x} + rank)), resident in HBM",
        config={"workload": f"Ligero R-S encode, {args.field}, 2^{args.log_len} coeffs, "
                            f"{n_rows}x{n_per_row}->{n_cols}",
                "field": args.field, "len": n, "n_rows": n_rows, "n_per_row": n_per_row, "n_cols": n_cols},
        step=step, cpu_baseline=cpu_baseline, root_is_parity=True, cpu_reps_ok=False,
        enc_kernels=("ntt_pass_a", "ntt_pass_b", "ntt_small"),
        enc_kernel_desc=f"ntt_encode = ntt_pass_a + ntt_pass_b (one launch each per step, all {n_rows} rows)",
        algo_bytes=n_rows * n_per_row * B + n_rows * n_cols * B,
        traffic_key=(n, args.field, "encode"),
        mul_count=n_rows * ntt_muls(n_cols),
        mul_model="four-step fft_io: (n/2)(log2 n - 2) general-twiddle butterflies + n inter-pass twiddles per row")


def sdig_encode_workload(args, L, torch, rank, local_rank):
    """cfg4's encode alone: LcEncoding::encode of SdigEncodingS (lcpc-brakedown-pc/src/lib.rs:150-153
    -> encode.rs:36-94) on every row of `batch` 2^24-coefficient commitments in one call (row-major
    device rows in and out; the library runs the expander levels on the element-major transpose)."""
    fid = {"Ft63": L.FT63, "Ft127": L.FT127, "Ft255": L.FT255}[args.field]
    nl = L.limbs(fid)
    n = 1 << args.log_len
    enc = L.SdigEncoding.new(fid, n, 0)
    n_rows1, n_per_row, n_cols = enc.get_dims(n)
    k = max(1, args.batch)
    n_rows = n_rows1 * k
    coeffs = L.field_random(fid, n_rows * n_per_row, replica_seed(rank))
    dev = f"cuda:{local_rank}"
    d_src = torch.from_numpy(coeffs.view(np.int64)).to(dev)
    dst = [torch.empty(n_rows * n_cols * nl, dtype=torch.int64, device=dev) for _ in range(max(1, args.pipeline))]
    torch.cuda.synchronize()

    def step(slot):
        enc.encode_rows_device(d_src.data_ptr(), n_per_row, n_per_row, dst[slot].data_ptr(), n_cols, n_rows)
        return None

    ocache = {}

    def cpu_baseline(O):
        # the oracle's encode (encode.rs:36-94) on every row of this workload, rows in parallel on
        # the threads of_set_threads gives it (lcpc-2d/src/lib.rs:677-682), output allocated once;
        # whole passes until about 5 s (at least one); then every GPU row against the oracle's
        if not ocache:
            ocache["enc"] = O.Encoding.sdig(fid, n_per_row, seed=0, code_id=3)
            ocache["out"] = np.empty(n_rows * n_cols * nl, np.uint64)
        o_enc, out = ocache["enc"], ocache["out"]
        passes, t1 = 0, time.perf_counter()
        while True:
            o_enc.encode_rows(coeffs, n_rows, out)
            passes += 1
            if time.perf_counter() - t1 >= 5.0:
                break
        dt = (time.perf_counter() - t1) / passes
        step(0)
        torch.cuda.synchronize()
        got = dst[0].cpu().numpy().view(np.uint64).reshape(-1)
        ok = bool(np.array_equal(got, out))
        return dt, ok, (f"the oracle's encode of all {n_rows} rows (of_enc_encode_rows), {passes} passes, time per "
                        f"pass; every row compared")

    B = 8 * nl
    nnz = enc.matrix_nnz
    return Workload(
        units=n_rows * n_per_row, unit="field-elements/s", bytes_per_unit=B,
        metric=f"encoded field-elements/s (Brakedown SdigCode3 encode), 2^{args.log_len}-coeff {args.field} (cfg4)",
        dtype=f"u64x{nl} ({args.field} Montgomery limbs)",
        data=f"synthetic: F::random(ChaCha20Rng::seed_from_u64({SEED:#x} + rank)), resident in HBM",
        config={"workload": f"Brakedown SdigCode3 (seed 0) encode, {args.field}, {k} x 2^{args.log_len} coeffs per "
                            f"call, {n_rows}x{n_per_row}->{n_cols}",
                "field": args.field, "len": n, "batch": k, "n_rows": n_rows, "n_per_row": n_per_row,
                "n_cols": n_cols, "matrix_nnz": nnz},
        step=step, cpu_baseline=cpu_baseline, root_is_parity=True, cpu_reps_ok=False,
        enc_kernels=("transpose", "sdig_encode"),
        enc_kernel_desc=(f"sdig_encode = transpose to element-major + 13 SpMM / Reed-Solomon levels + transpose "
                         f"back (one call, all {n_rows} rows)"),
        # read the coefficients, write the codeword, stream the code matrices once
        algo_bytes=n_rows * n_per_row * B + n_rows * n_cols * B + nnz * (B + 4),
        gather_bytes=(n_rows * nnz * B + n_rows * (n_cols - n_per_row) * B + nnz * 20
                      + 3 * n_rows * n_per_row * B + 2 * n_rows * n_cols * B),
        traffic_key=(n, args.field, f"sdig-encode-b{k}"),
        mul_count=n_rows * nnz, mul_model="one product per nonzero per row")


def pos_workload(args, L, torch, rank, local_rank):
    """cfg5: one proof-of-storage server request on a resident file (networking/server.rs:670-730):
    pack the bytes into WriteableFt63 elements, commit with the default dims, evaluate u^T Enc(M)
    at a point, and open the client's 256 columns with Merkle paths (client.rs:443-456)."""
    from lcpc_proof_of_storage_amd import pos as P
    n_bytes = args.pos_bytes
    n_el = -(-n_bytes // 7)
    np_, nc, snd = P.get_aspect_ratio_default_from_file_len(n_bytes)
    enc = L.LigeroEncoding.new_from_dims(L.FT63, np_, nc)
    n_rows = -(-n_el // np_)
    rng = np.random.default_rng(1 + rank)
    host = rng.integers(0, 256, n_bytes, dtype=np.uint8)
    dev = f"cuda:{local_rank}"
    if args.input == "device":
        d_bytes = torch.from_numpy(host).to(dev)
    elif args.input == "host-pinned":
        host_img = torch.from_numpy(host).pin_memory().numpy()
    else:
        host_img = host
    # element buffers of whole-row capacity whose tail past n_el stays zero: commit pads the last
    # row with zeros (lcpc-2d/src/lib.rs:665-674), so committing the n_rows x n_per_row buffer is
    # the same commitment, and the ragged row needs no separate one-row encode
    slots = ([torch.zeros(n_rows * np_, dtype=torch.int64, device=dev) for _ in range(max(1, args.pipeline))]
             if args.pos_commit == "elements" else [])
    x = L.field_random(L.FT63, 1, 1337)
    left, _ = P.form_side_vectors_for_polynomial_evaluation_from_point(x, n_rows, nc)
    cols = P.get_column_indicies_from_random_seed(1337, 256, nc)
    from lcpc_proof_of_storage_amd import _native
    lib = _native.load()

    gate = threading.Semaphore(args.commit_slots) if args.commit_slots > 0 else None

    def commit(slot):
        if args.input != "device":  # the file the server just read: lcpc_pos_commit_bytes from host memory
            return L.LcCommit.commit_pos_bytes(host_img, enc)
        if args.pos_commit == "bytes":  # lcpc_pos_commit_bytes_device: the file image in one call
            return L.LcCommit.commit_pos_bytes_device(d_bytes.data_ptr(), n_bytes, enc)
        d_el = slots[slot]
        rc = lib.lcpc_pos_bytes_to_field_device(d_bytes.data_ptr(), n_bytes, d_el.data_ptr(), None)
        if rc:
            raise RuntimeError(f"pack failed {rc}: {_native.last_error()}")
        return L.LcCommit.commit_device(d_el.data_ptr(), n_rows * np_, enc)

    fused = args.input == "device" and args.pos_commit == "bytes" and args.pos_eval == "fused"

    def commit_eval(slot):
        if fused:  # one call: the commitment and u^T Enc(M) (the evaluation rides on the leaf pass)
            return L.LcCommit.commit_pos_bytes_device_eval(d_bytes.data_ptr(), n_bytes, enc, left)
        c = commit(slot)
        return c, P.verifiable_polynomial_evaluation(c, left)

    def step(slot):
        if gate is not None:
            gate.acquire()
        try:
            if fused:
                c, _ = commit_eval(slot)
            else:
                c = commit(slot)
        finally:
            if gate is not None:
                gate.release()
        if not fused:
            P.verifiable_polynomial_evaluation(c, left)
        c.open_columns(cols)
        return c.get_root()

    def cpu_baseline(O):
        # bounded sample: the first 1/16 of the file (rows are independent; same dims)
        sample = host[: n_bytes // 16]
        el = O.pos_bytes_to_field(sample.tobytes())
        o_enc = O.Encoding.ligero(0, np_, nc)
        t1 = time.perf_counter()
        oc = O.Commit(o_enc, el)
        O.collapse(0, oc.comm, O.pos_side_vectors(0, x.reshape(-1), oc.n_rows, nc)[0], oc.n_rows, nc)
        dt = time.perf_counter() - t1
        return dt * n_bytes / len(sample), None, (f"commit + u^T Enc(M) of the first 1/16 of the file "
                                                  f"({len(sample)} B, {dt:.2f} s), scaled to the whole file")

    def parity(O):
        """one request of this workload (untimed) against the oracle's answer on the whole file"""
        c, ev = commit_eval(0)
        opened = c.open_columns(cols)
        return pos_oracle_parity(O, host, np_, nc, n_rows, left, cols, c.get_root(), ev, opened)

    fi = args.pos_commit == "bytes" or args.input != "device"  # the file-image commit (its own row-kernel default)
    return Workload(
        units=n_el, unit="field-elements/s", bytes_per_unit=8,
        metric="proof-of-storage server request: committed field-elements/s (pack+commit+eval+256-col open), "
               f"{n_bytes / 2**30:g} GiB file",
        dtype="u64 (WriteableFt63 Montgomery limbs)",
        data=f"synthetic: {n_bytes} random bytes (numpy default_rng(1 + rank)), " + INPUT_NOTE[args.input],
        config={"workload": f"PoS request on a {n_bytes}-byte file: {n_el} WriteableFt63 elements, default "
                            f"dims {n_rows}x{np_}->{nc}, u^T Enc(M) at a point, 256 opened columns"
                            + INPUT_WORKLOAD[args.input],
                "file_bytes": n_bytes, "n_rows": n_rows, "n_per_row": np_, "n_cols": nc, "soundness": snd,
                "commit_call": ("lcpc_pos_commit_bytes (host file image, pipelined upload)" if args.input != "device"
                                else "lcpc_pos_commit_eval_bytes_device (file image and u^T Enc(M) in one call)"
                                if fused
                                else "lcpc_pos_commit_bytes_device (file image in one call)" if args.pos_commit == "bytes"
                                else "lcpc_pos_bytes_to_field_device + lcpc_commit_new_device"),
                "row_kernel": (("one-pass (ntt_row1), L2 prefetch of the row 256 ahead: "
                                + {"0": "off", "2": "at round 2", "3": "at the output phase"}.get(
                                    os.environ.get("LCPC_ROW1_PREFETCH", "1"), "at round 3"))
                               if row1_active(nc, fi) else "four-step (ntt_pass_a + ntt_pass_b)")},
        step=step, cpu_baseline=cpu_baseline, parity=parity, input_bytes=n_bytes,
        enc_kernels=("ntt_pass_a", "ntt_pass_b", "ntt_small", "ntt_row1"),
        enc_kernel_desc=(f"ntt_encode = ntt_row1 (one launch per commit, all {n_rows} rows)" if row1_active(nc, fi) else
                         f"ntt_encode = ntt_pass_a + ntt_pass_b (one launch each per commit, all {n_rows} rows)"),
        algo_bytes=n_rows * np_ * 8 + n_rows * nc * 8,
        leaf_compressions=leaf_compressions(n_rows, nc, 8),
        traffic_key=(n_el, "Ft63", "pos-row1" if row1_active(nc, fi) else "pos"),
        mul_count=n_rows * pos_ntt_muls(nc, fi)[0], mul_model=pos_ntt_muls(nc, fi)[1])


# ---------------------------------------------------------------- launch, cores, shared output
def spawn_ranks(args):
    """`bench.py --gpus N` outside torch.distributed.run: start N ranks ourselves (no torch or HIP
    has been imported in this process) and exit with their status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def available_cores():
    """(cores, basis): the CPUs this process may run on -- its affinity, capped by a cgroup CPU
    quota when one is set (the GPU box grants each job a share of a large host)."""
    n = len(os.sched_getaffinity(0))
    basis = f"sched_getaffinity = {n}"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            c = max(1, int(int(q) / int(per)))
            if c < n:
                n, basis = c, basis + f", cgroup cpu.max quota = {c}"
    except (OSError, ValueError):
        pass
    return n, basis


def plumbing_check(args, rank, world):
    """--plumbing-only: the multi-process contract without a GPU (CPU tests): gloo group, world
    size check, barrier, max-over-ranks, rank-0 JSON line."""
    dist = init_dist(world, 0, backend="gloo")
    formed = dist.get_world_size() if dist else 1
    sync_barrier(dist)
    t0 = time.perf_counter()
    time.sleep(0.01 * (1 + rank))
    sync_barrier(dist)
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    _, local_rank, _ = dist_env()
    ids = fold_identities(dist, rank_identity(rank, local_rank, device_binding(local_rank)[0]))
    if rank == 0:
        print(json.dumps({"metric": "plumbing check", "value": None, "unit": None, "n_gpus": formed,
                          "world_formed": formed, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1e3 * elapsed / max(args.steps, 1), "plumbing_only": True, **ids}))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if formed == args.gpus else 3


def roofline_objects(wl, iso, stats, args, traffic_rows_frac=1.0):
    """roofline (HBM) + roofline_valu of the encode, roofline_leaf of the column hashing."""
    out = {}
    if not iso or not wl.algo_bytes:
        return out
    # iso holds (total ms, launches) over args.roofline_steps serial steps.  The roofline time is
    # the encode's kernel time PER STEP: a step may launch a kernel more than once (the PoS file's
    # ragged last row is its own one-row NTT), so a per-launch average would mix a one-row launch
    # with the full-size one
    nst = max(args.roofline_steps, 1)
    ki = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1], "ms_per_step": v[0] / nst} for k, v in iso.items()}
    out["kernels"] = ki
    enc_ms = sum(ki[k]["ms_per_step"] for k in wl.enc_kernels if k in ki)
    traffic, tsrc = None, None
    for tpath in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json"))):
        try:
            tj = json.load(open(tpath))
        except (OSError, ValueError):
            continue
        if (tj.get("config_len"), tj.get("field"), tj.get("code", "ligero")) == wl.traffic_key:
            traffic = tj.get("ntt_encode_bytes_per_launch")
            if traffic is not None:
                traffic *= traffic_rows_frac
            tsrc = (f"{os.path.relpath(tpath, ROOT)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this "
                    f"workload's encode (a separate profiling run, not this process)")
            break
    achieved = wl.algo_bytes / (enc_ms * 1e-3) / 1e9 if enc_ms else None
    tr_ms = None
    if stats:
        tr_ms = sum(stats[k][0] / max(stats[k][1], 1) for k in wl.enc_kernels if k in stats)
    out["roofline"] = {
        "kernel": wl.enc_kernel_desc, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic, "traffic_source": tsrc,
        "algorithmic_bytes": wl.algo_bytes, "avg_ms": enc_ms,
        "launches": min((ki[k]["launches"] for k in wl.enc_kernels if k in ki), default=0),
        "launches_per_step": {k: ki[k]["launches"] / nst for k in wl.enc_kernels if k in ki},
        "measured": f"HIP events on the launching stream, {args.roofline_steps} serial steps after the timed "
                    f"region (same process, inputs and kernels); avg_ms = the encode kernels' time per step",
        "timed_region_avg_ms": tr_ms,
    }
    if wl.mul_count:
        # the encode is bound by the 32-bit multiply-add pipe, not HBM: its VALU roofline is the
        # Montgomery-multiply rate of the field measured in isolation (tools/microbench/femul2.hip
        # on MI355X, the library's product with its carry-free mads: Ft63 1909, Ft127 579, Ft255
        # 154 G/s; profiles/r06_femul2.txt -- 1701 / 503 / 137 before, r01_femul2.txt); the hardware
        # v_mad_u64_u32 issue ceiling (20.6 T lane-ops/s, profiles/r01_mulbench.txt) over the 28
        # mads of an Ft127 product is the second peak
        field = args.field if args.code != "pos" else "Ft63"
        peak = {"Ft63": 1909.0, "Ft127": 579.0, "Ft255": 154.0}.get(field)
        ach = wl.mul_count / (enc_ms * 1e-3) / 1e9 if enc_ms else None
        out["roofline_valu"] = {
            "kernel": wl.enc_kernel_desc, "bound": "valu (v_mad_u64_u32 Montgomery products)",
            "achieved": ach, "peak": peak, "unit": "G field-mul/s",
            "frac": ach / peak if ach and peak else None, "muls_per_launch": wl.mul_count, "model": wl.mul_model,
        }
        if field == "Ft127" and ach:
            out["roofline_valu"]["mad_issue_peak"] = 20600.0 / 28
            out["roofline_valu"]["frac_of_mad_issue_peak"] = ach / (20600.0 / 28)
        # the passes against the issue floor of their own instruction stream (round 6 model:
        # per-class issue costs x instruction counts, tools/encode_cycle_model.py)
        fpath = os.path.join(ROOT, "profiles", "issue_floor_encode.json")
        try:
            fl = json.load(open(fpath))
            if (fl.get("config_len"), fl.get("field"), fl.get("code")) == wl.traffic_key and traffic_rows_frac == 1.0:
                out["roofline_valu"]["issue_floor"] = {
                    "frac": fl["frac_of_issue_floor"], "model_ms": fl["model_ms"], "measured_ms": fl["measured_ms"],
                    "source": os.path.relpath(fpath, ROOT)}
        except (OSError, ValueError, KeyError):
            pass
    gb = getattr(wl, "gather_bytes", 0)
    if gb and enc_ms:
        # Brakedown: the levels gather every nonzero's input run (R rows) from HBM -- an expander
        # has no locality for the caches to exploit -- so the traffic the encode cannot avoid is
        # the gathers plus the transpose and the outputs, not one read of the input
        ach = gb / (enc_ms * 1e-3) / 1e9
        out["roofline_gather"] = {
            "kernel": wl.enc_kernel_desc, "bound": "hbm (gathers)", "achieved": ach, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "gather_model_bytes": gb, "avg_ms": enc_ms,
            "model": "nnz x R x B input gathers + R x (n_cols - n_per_row) x B outputs + nnz x 20 B matrix "
                     "+ the transpose (R x n_per_row x B read, element-major and row-major copies written)"}
    lc = getattr(wl, "leaf_compressions", 0)
    if lc and "leaf_chunks" in iso:
        leaf_ms = sum(iso[k][0] / nst for k in ("leaf_chunks", "leaf_merge") if k in iso)
        ach = lc / (leaf_ms * 1e-3) / 1e9
        out["roofline_leaf"] = {
            "kernel": "leaf_chunks + leaf_merge (BLAKE3 column leaves)", "bound": "valu (BLAKE3 compressions)",
            "achieved": ach, "peak": LEAF_PEAK_GCPS, "unit": "G compressions/s", "frac": ach / LEAF_PEAK_GCPS,
            "compressions_per_launch": lc, "avg_ms": leaf_ms,
            "peak_source": "tools/microbench/leafbench.hip compress-only twin of the leaf kernel, MI355X"}
    return out


def h2d_copy_rates(torch, nbytes, device, reps=5):
    """GB/s of one host -> HBM copy of nbytes from page-locked and from pageable memory (torch
    copy_ on the current stream, HIP events; best of reps): the PCIe ceilings a host-input line is
    held against"""
    dst = torch.empty(nbytes, dtype=torch.uint8, device=device)
    out = {}
    for kind in ("pinned", "pageable"):
        src = torch.empty(nbytes, dtype=torch.uint8)
        if kind == "pinned":
            src = src.pin_memory()
        src.fill_(1)
        best = None
        for _ in range(reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dst.copy_(src, non_blocking=(kind == "pinned"))
            b.record()
            b.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        out[kind] = nbytes / (best * 1e-3) / 1e9
        del src
    del dst
    return out


def time_cpu_baseline(wl, O, cores, reps):
    """one warm-up, then the median of `reps` timed runs on `cores` threads"""
    O.lib().of_set_threads(cores)
    wl.cpu_baseline(O)  # warm-up (page faults, thread start)
    runs = []
    oroot = sample = None
    for _ in range(max(1, reps)):
        dt, oroot, sample = wl.cpu_baseline(O)
        runs.append(dt)
    runs.sort()
    return runs[len(runs) // 2], runs, oroot, sample


# ---------------------------------------------------------------- the sharded engine (cfg3)
def ligero_sharded(args, L, torch, dist, rank, world, device, backend, share):
    """cfg3 at any N: steps are single 2^24 commitments, rows split over the ranks, driven by
    lcpc_sharded_commit_prove_many (one RCCL group per pipeline tick)."""
    from lcpc_proof_of_storage_amd import shard
    fid = {"Ft63": L.FT63, "Ft127": L.FT127, "Ft255": L.FT255}[args.field]
    nl = L.limbs(fid)
    n = 1 << args.log_len
    enc = L.LigeroEncoding.new(fid, n, args.rho_t)
    n_rows, n_per_row, n_cols = enc.get_dims(n)
    nco, ndt = enc.get_n_col_opens(), enc.get_n_degree_tests()
    coeffs = L.field_random(fid, n, SEED)                    # one polynomial; rank g keeps its rows
    outer = L.field_random(fid, n_rows, 7)
    inner = L.field_random(fid, n_per_row, 8)
    rows = np.zeros((n_rows * n_per_row, nl), np.uint64)
    rows[:n] = coeffs
    rows = rows.reshape(n_rows, n_per_row * nl)
    r0, nr = shard.sharded_rows(fid, n_rows, world, rank)
    d_mine = torch.from_numpy(np.ascontiguousarray(rows[r0:r0 + nr]).view(np.int64)).to(device)
    d_out = torch.empty(max(nr, 1) * n_cols * nl, dtype=torch.int64, device=device)  # roofline encode target
    torch.cuda.synchronize()
    if world == 1:
        comm, comm_kind = shard.NativeComm.single(), "none (one rank)"
    elif backend == "nccl" and not share:
        comm, comm_kind = shard.NativeComm.rccl(dist), "RCCL (liblcpc_mi lcpc_comm_rccl_new, device send/recv)"
    elif os.environ.get("LCPC_BENCH_RCCL_SAME_GPU") == "1":
        comm, comm_kind = (shard.NativeComm.rccl(dist),
                           "RCCL with the ranks sharing one GPU (per-rank NCCL_HOSTID: socket transport over loopback)")
    else:
        comm, comm_kind = shard.NativeComm.host(dist), "host-staged gloo collectives (ranks share one GPU)"
    assert comm.world == world and comm.rank == rank, (comm.world, comm.rank)
    COMM_INFO.update(nranks=comm.world, is_rccl=comm.is_rccl)

    def make_tr(i, root):
        tr = L.Transcript(b"test transcript")
        tr.append_message(b"polycommit", root)
        tr.append_message(b"ncols", nco.to_bytes(8, "big"))
        return tr

    def run(k, keep=False):
        return shard.sharded_commit_prove_many(enc, comm, [d_mine.data_ptr()] * k, n_rows, outer, make_tr,
                                               lag=args.lag, keep_proofs=keep)

    def serial_commit():
        return shard.ShardedCommit(enc, comm, d_mine.data_ptr(), n_rows)

    def reserve(k):
        shard.sharded_reserve(enc, comm, n_rows, k, args.lag)

    def serial_prove(sc):
        root = sc.get_root()
        return sc.prove(outer, make_tr(0, root) if rank == 0 else None, root=0)

    B = 8 * nl
    return dict(
        fid=fid, enc=enc, n=n, n_rows=n_rows, n_per_row=n_per_row, n_cols=n_cols, nco=nco, ndt=ndt, nr=nr,
        coeffs=coeffs, outer=outer, inner=inner, run=run, serial_commit=serial_commit, reserve=reserve,
        serial_prove=serial_prove, make_tr=make_tr,
        comm_kind=comm_kind, d_mine=d_mine, d_out=d_out, B=B)


def main():
    args = parse()
    rank, local_rank, world = dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher formed WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.plumbing_only:
        sys.exit(plumbing_check(args, rank, world))
    os.environ["LCPC_STREAM_MODE"] = args.stream_mode  # read when the library creates streams
    # the sharded calls' watchdog (off in the library by default): a rank whose exchanges stop for
    # two minutes reports the tick and its peers and exits, instead of holding the run until the
    # driver's own limit
    os.environ.setdefault("LCPC_SHARD_WATCHDOG_S", "120")
    import torch

    # LCPC_BENCH_BACKEND=gloo with LCPC_BENCH_SHARE_GPU=1 rehearses N ranks on one GPU (a
    # one-GPU box; the exchanges then go over host-staged gloo collectives); the default is one
    # rank per GPU over RCCL
    backend = os.environ.get("LCPC_BENCH_BACKEND", "nccl")
    device_idx, _ = device_binding(local_rank)
    share = os.environ.get("LCPC_BENCH_SHARE_GPU") == "1"
    # LCPC_BENCH_RCCL_SAME_GPU=1 (with the two above): the ranks share GPU 0 but the library's
    # exchanges still go through RCCL -- a distinct NCCL_HOSTID per rank makes RCCL treat them as
    # separate nodes (loopback sockets), so its multi-rank send / receive groups run on one GPU
    if os.environ.get("LCPC_BENCH_RCCL_SAME_GPU") == "1" and share:
        os.environ.update(NCCL_HOSTID=f"lcpc-bench-rank-{rank}", NCCL_IB_DISABLE="1", NCCL_SOCKET_IFNAME="lo")
    dist = init_dist(world, device_idx, backend=backend)
    formed = dist.get_world_size() if dist is not None else 1
    if formed != args.gpus:
        print(f"bench.py: formed a world of {formed} ranks, --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(device_idx)
    device = f"cuda:{device_idx}"

    import lcpc_proof_of_storage_amd as L

    L.set_device(device_idx)
    sharded_n1 = None
    if args.mode == "sharded" and args.code == "pos":
        out = run_pos_sharded(args, L, torch, dist, rank, world, device, backend, share)
    elif args.mode == "sharded":
        out = run_sharded(args, L, torch, dist, rank, world, device, backend, share)
    else:
        out = run_replicas(args, L, torch, dist, rank, world, device_idx, backend)
        if world == 1 and args.code == "ligero" and args.sharded_n1 == 2:
            # the row-sharded engine on this one GPU, like for like with the N > 1 lines
            # (--mode auto runs it there): same steps and warm-up, after the replicas' figures
            sharded_n1 = sharded_n1_figure(args, L, torch, device)
        elif world == 1 and args.code == "ligero" and args.sharded_n1 == 1:
            sharded_n1 = sharded_n1_child(args)
    if sharded_n1 is not None:
        # the sharded engine commits the same polynomial (seed SEED) as replica 0: its root must
        # be the replicas' and the oracle's
        sharded_n1["root_equals_replicas"] = sharded_n1.get("root") == out.get("root")
        out["sharded_n1"] = sharded_n1
        if "parity_ok" in out and sharded_n1.get("root") is not None:
            out["parity_ok"] = bool(out["parity_ok"] and sharded_n1["root_equals_replicas"])
        if sharded_n1.get("value"):
            # the N = 1 point of the N > 1 lines' own engine: N > 1 runs the row-sharded driver, so a
            # 1 -> N curve is N's value / this one (the replicas value above is the one-GPU headline)
            out["scale_base"] = {"value": sharded_n1["value"], "unit": out.get("unit"), "engine": "sharded",
                                 "what": "the row-sharded engine (--mode sharded, the N > 1 default) at N = 1, same "
                                         "workload, steps and warm-up: divide an N > 1 line's value by this for its "
                                         "speed-up on one engine"}
    # every rank's device and communicator, folded into the line (a collective: all ranks)
    ids = fold_identities(dist, rank_identity(rank, local_rank, device_idx, torch))
    if rank == 0:
        out["world_formed"] = formed
        out.update(ids)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and out.get("parity_ok") is False:
        print("bench.py: the run's answers differ from the oracle's (see the parity_* keys)", file=sys.stderr)
        sys.exit(4)


def sharded_n1_child(args):
    """The sharded engine's one-GPU figure from a fresh child process running this script with
    --mode sharded (same workload, steps and warm-up): the engine's streams and pools start as an
    N > 1 rank's do, not after this process's replicas run left its stream pools in use (the
    in-process figure, --sharded-n1 2, measured 9.1-9.4 against 10.1-10.4 G/s on one box)."""
    import subprocess
    drop = {"--mode": 1, "--sharded-n1": 1, "--cpu-baseline": 1, "--verify-reps": 1, "--timeline": 1}
    argv, i = [], 0
    src = sys.argv[1:]
    while i < len(src):
        a = src[i]
        key = a.split("=", 1)[0]
        if key in drop:
            i += 1 if "=" in a else 1 + drop[key]
            continue
        argv.append(a)
        i += 1
    cmd = [sys.executable, os.path.abspath(__file__)] + argv + ["--mode", "sharded", "--sharded-n1", "0",
                                                                 "--cpu-baseline", "off", "--verify-reps", "0"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    except subprocess.TimeoutExpired:
        return {"error": "the child process timed out"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode or not lines:
        return {"error": f"child exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
    d = json.loads(lines[-1])
    return {"value": d["value"], "unit": d["unit"], "steps": d["steps"], "warmup": d["warmup"],
            "ms_per_step": d["ms_per_step"], "scaling": "strong",
            "engine": "lcpc_sharded_commit_prove_many, one rank (no exchanges): the N = 1 point of the "
                      "--mode sharded (--gpus N > 1) curve, timed in a fresh child process",
            "lag": args.lag or None, "root": d.get("root"), "steps_agree": d.get("steps_agree")}


def sharded_n1_figure(args, L, torch, device):
    """The sharded engine's one-GPU throughput on the same workload (lcpc_sharded_commit_prove_many
    with a one-rank comm: the N = 1 base of the N > 1 sharded lines): pools reserved, exactly
    --warmup untimed steps, then --steps timed, device-synchronised on both sides."""
    S = ligero_sharded(args, L, torch, None, 0, 1, device, "nccl", False)
    S["reserve"](max(args.steps, args.warmup))
    roots, _ = S["run"](max(1, args.warmup))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    troots, _ = S["run"](args.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    assert all(r == roots[0] for r in troots), "sharded engine: roots differ across steps"
    return {"value": S["n"] * args.steps / elapsed, "unit": "field-elements/s", "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "scaling": "strong",
            "engine": "lcpc_sharded_commit_prove_many, one rank (no exchanges): the N = 1 point of the "
                      "--mode sharded (--gpus N > 1) curve",
            "lag": args.lag or None, "root": roots[0].hex()}


def run_sharded(args, L, torch, dist, rank, world, device, backend, share):
    S = ligero_sharded(args, L, torch, dist, rank, world, device, backend, share)
    n, B, nr = S["n"], S["B"], S["nr"]
    fid, enc = S["fid"], S["enc"]
    n_rows, n_per_row, n_cols, nco, ndt = S["n_rows"], S["n_per_row"], S["n_cols"], S["nco"], S["ndt"]

    def barrier():
        sync_barrier(dist, torch.cuda.synchronize)

    # commitments per step: N (weak scaling: one commitment's work per GPU per step) or 1 (strong)
    pps = world if args.sharded_scaling == "weak" else 1
    n_timed = args.steps * pps
    # the pools the timed run's pipeline depth needs (buffers, page-locked staging, streams: not
    # steps), then the warm-up (RCCL connections); polynomial 0's proof is kept on rank 0
    S["reserve"](max(args.steps, args.warmup) * pps)
    roots, proofs = S["run"](max(1, args.warmup) * pps, keep=True)
    warm_proof = proofs[0]
    assert all(r == roots[0] for r in roots), "nondeterministic root across steps"
    prof_timed = args.prof_timed and not args.no_prof
    L.prof_enable(prof_timed)
    L.prof_reset()
    barrier()
    t0 = time.perf_counter()
    c0, th0 = os.times(), cgroup_throttle()
    troots, _ = S["run"](n_timed)
    barrier()
    elapsed = time.perf_counter() - t0
    c1, th1 = os.times(), cgroup_throttle()
    L.prof_enable(False)
    stats = L.prof_stats() if prof_timed else {}
    # recorded, not asserted: the line still prints, and main() exits non-zero on a mismatch
    steps_agree = len(troots) == n_timed and all(r == roots[0] for r in list(troots) + list(roots))
    elapsed = max_over_ranks(dist, elapsed, "cpu" if backend == "gloo" else device)

    # one commitment's latency (serial, median of 3) and the roofline launches (HIP events on the
    # launching streams, every kernel of those serial steps)
    lat_c, lat_p, iso = [], [], {}
    sc = pf = None
    for rep in range(1 + args.roofline_steps):
        if rep == 1 and not args.no_prof:
            L.prof_reset()
            L.prof_enable(True)
        barrier()
        t1 = time.perf_counter()
        sc = S["serial_commit"]()
        t2 = time.perf_counter()
        pf = S["serial_prove"](sc)
        t3 = time.perf_counter()
        if rep >= 1:
            lat_c.append(1e3 * (t2 - t1))
            lat_p.append(1e3 * (t3 - t2))
    if not args.no_prof:
        L.prof_enable(False)
        iso = L.prof_stats()
    lat_c.sort()
    lat_p.sort()
    value = job_throughput(n, args.steps, pps, elapsed)
    out = {
        "metric": "committed field-elements/s (commit+open), 2^24-coeff Ligero, 1/2/4/8 GPU" + rho_note(args),
        "value": value, "unit": "field-elements/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": args.sharded_scaling,
        "commitments_per_step": pps, "commitments_timed": n_timed,
        "vs_baseline": None, "dtype": f"u64x{B // 8} ({args.field} Montgomery limbs)",
        "data": f"synthetic: F::random(ChaCha20Rng::seed_from_u64({SEED:#x})), one polynomial, each rank's rows "
                f"resident in its HBM",
        "config": {"workload": f"Ligero commit+open, {args.field}, 2^{args.log_len} coeffs, rho={args.rho}, {n_rows}x"
                               f"{n_per_row}->{n_cols}, {nco} column opens, {ndt} degree tests, BLAKE3 Merkle",
                   "field": args.field, "len": n, "n_rows": n_rows, "n_per_row": n_per_row, "n_cols": n_cols,
                   "n_col_opens": nco, "n_degree_tests": ndt,
                   "parallelism": (f"rows sharded x{world} ({pps} commitment{'s' if pps > 1 else ''} per step, each "
                                   f"row-sharded over all {world} ranks; lcpc_sharded_commit_prove_many, "
                                   f"transcript of commitment i on rank i % {world})" if world > 1 else
                                   "one GPU (lcpc_sharded_commit_prove_many with one rank: pipelined steps)"),
                   "exchanges": S["comm_kind"], "lag": args.lag or None, "rows_on_rank0": nr},
        "mb_per_s": value * B / 1e6,
        "latency": {"commit_ms": lat_c[len(lat_c) // 2] if lat_c else None,
                    "prove_ms": lat_p[len(lat_p) // 2] if lat_p else None,
                    "what": "one commitment, serial: lcpc_sharded_commit_new_device and lcpc_sharded_prove "
                            "(host wall clock, median of the roofline steps)"},
    }
    out["host_cpu"] = host_cpu_use(c0, c1, elapsed)
    if th0 and th1:
        out["host_cpu"]["cgroup_throttled"] = {k: th1[k] - th0[k] for k in th0 if k in th1}
    if stats:
        out["kernels_timed_region"] = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1], "total_ms": v[0]}
                                       for k, v in stats.items()}
    # the dominant kernel, the encode, over THIS rank's rows
    wl = Workload(
        algo_bytes=nr * n_per_row * B + nr * n_cols * B, enc_kernels=("ntt_pass_a", "ntt_pass_b", "ntt_small"),
        enc_kernel_desc=f"ntt_encode = ntt_pass_a + ntt_pass_b (one launch each per commit, this rank's {nr} rows)",
        traffic_key=(n, args.field, "ligero"), mul_count=nr * ntt_muls(n_cols),
        mul_model="four-step fft_io: (n/2)(log2 n - 2) general-twiddle butterflies + n inter-pass twiddles per row",
        leaf_compressions=leaf_compressions(n_rows, n_cols, B) if world == 1 else 0)
    out.update(roofline_objects(wl, iso, stats, args, traffic_rows_frac=nr / n_rows))
    out["root"] = roots[0].hex()  # (every step commits the same polynomial)
    out["steps_agree"] = steps_agree

    # the verifier (outside the timed region): the serial step's proof, verified again
    if rank == 0 and args.verify_reps > 0 and pf is not None:
        root = sc.get_root()
        ev = pf.verify(root, S["outer"], S["inner"], enc, S["make_tr"](0, root))
        t1 = time.perf_counter()
        for _ in range(args.verify_reps):
            pf.verify(root, S["outer"], S["inner"], enc, S["make_tr"](0, root))
        out["verify"] = {"ms": 1e3 * (time.perf_counter() - t1) / args.verify_reps, "reps": args.verify_reps,
                         "what": "LcEvalProof::verify of one proof of this workload (host + GPU, serial)"}
    else:
        ev = None

    # Parity: the oracle (C restatement) on the same workload, on rank 0 at EVERY N (after the timed
    # region), so that an N > 1 line carries its own proof of a right answer: every timed step's
    # root, the kept warm-up proof and the verifier's value against the oracle's.  The timed CPU
    # baseline is the N = 1 line's (--cpu-baseline on forces it at every N)
    want_cpu = args.cpu_baseline in ("on", "auto")
    if rank == 0 and want_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O  # checker / CPU baseline only
        o_enc = O.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt, rho=args.rho_t)
        keep = {}

        def cpu_once(O_):
            t1 = time.perf_counter()
            oc = O_.Commit(o_enc, S["coeffs"].reshape(-1))
            op = oc.prove(o_enc, S["outer"].reshape(-1), O_.standard_transcript(nco, oc.root()))
            dt = time.perf_counter() - t1
            keep["oc"], keep["op"] = oc, op
            return dt, oc.root(), f"one full commit+open of the same 2^{args.log_len} {args.field} workload"

        cores, basis = available_cores()
        if args.cpu_threads:
            cores, basis = args.cpu_threads, "--cpu-threads"
        if world == 1 or args.cpu_baseline == "on":
            med, runs, oroot, sample = time_cpu_baseline(Workload(cpu_baseline=cpu_once), O, cores, args.cpu_reps)
            out["cpu_baseline"] = {"value": n / med, "unit": "field-elements/s", "cores": cores, "kind": "port",
                                   "sample": f"{sample}: median of {len(runs)} runs after a warm-up on {cores} "
                                             f"threads ({', '.join(f'{r:.3f}' for r in runs)} s)",
                                   "cores_basis": basis}
        else:  # N > 1: the oracle runs once, as the checker only (the CPU baseline is the N = 1 line's)
            O.lib().of_set_threads(cores)
            _, oroot, _ = cpu_once(O)
        out["parity_root_vs_oracle"] = oroot == roots[0]
        out["parity_steps_vs_oracle"] = {"steps": len(troots) + len(roots),
                                         "equal": sum(r == oroot for r in list(troots) + list(roots)),
                                         "what": "every warm-up and timed step's root against the oracle's"}
        op = keep["op"]
        out["parity_proof_vs_oracle"] = False
        if warm_proof is not None:
            out["parity_proof_vs_oracle"] = bool(
                np.array_equal(warm_proof.p_eval.reshape(-1), op.p_eval)
                and np.array_equal(np.concatenate(warm_proof.p_random_vec).reshape(-1), op.p_random)
                and np.array_equal(np.stack([c.col for c in warm_proof.columns]).reshape(-1), op.cols)
                and b"".join(b"".join(c.path) for c in warm_proof.columns) == op.paths.tobytes())
        if ev is not None:
            t2 = time.perf_counter()
            rc, oev = op.verify(keep["oc"].root(), S["outer"].reshape(-1), S["inner"].reshape(-1), o_enc,
                                O.standard_transcript(nco, keep["oc"].root()))
            out["verify"]["cpu_ms"] = 1e3 * (time.perf_counter() - t2)
            out["verify"]["parity_vs_oracle"] = bool(rc == 0 and np.array_equal(np.asarray(ev).reshape(-1), oev))
        if args.cpu_baseline_1core == "on" or (args.cpu_baseline_1core == "auto" and world == 1):
            O.lib().of_set_threads(1)
            dt1, oroot1, sample1 = cpu_once(O)
            out["cpu_baseline_1core"] = {"value": n / dt1, "unit": "field-elements/s", "cores": 1, "kind": "port",
                                         "sample": f"{sample1}: one run on 1 thread ({dt1:.2f} s)"}
            out["parity_root_vs_oracle"] = out["parity_root_vs_oracle"] and oroot1 == roots[0]
        ps = out["parity_steps_vs_oracle"]
        out["parity_ok"] = bool(steps_agree and out["parity_root_vs_oracle"] and ps["equal"] == ps["steps"]
                                and out["parity_proof_vs_oracle"]
                                and out.get("verify", {}).get("parity_vs_oracle", True))
    return out


# ---------------------------------------------------------------- cfg5 over several GPUs
def run_pos_sharded(args, L, torch, dist, rank, world, device, backend, share):
    """cfg5 with ONE file's rows sharded over the ranks: every step is one proof-of-storage
    request (networking/server.rs:652-737) on the whole file -- each rank packs its rows' bytes
    (data_field.rs:38-46), the rows are committed together (lcpc_sharded_commit_new_device), and
    u^T Enc(M) plus the client's 256 columns with paths come back on rank 0
    (lcpc_sharded_pos_request).  Steps are serial (each is two collectives)."""
    from lcpc_proof_of_storage_amd import pos as P
    from lcpc_proof_of_storage_amd import shard
    n_bytes = args.pos_bytes
    n_el = -(-n_bytes // 7)
    np_, nc, snd = P.get_aspect_ratio_default_from_file_len(n_bytes)
    n_rows = -(-n_el // np_)
    enc = L.LigeroEncoding.new_from_dims(L.FT63, np_, nc)
    r0, nr = shard.sharded_rows(L.FT63, n_rows, world, rank)
    host = np.random.default_rng(1).integers(0, 256, n_bytes, dtype=np.uint8)  # the same file on every rank
    lo, hi = min(n_bytes, 7 * np_ * r0), min(n_bytes, 7 * np_ * (r0 + nr))
    mine = np.zeros(-(-(hi - lo) // 8) * 8 + 8, np.uint8)
    mine[:hi - lo] = host[lo:hi]
    d_bytes = torch.from_numpy(mine).to(device)
    d_rows = torch.zeros(max(nr * np_, 1), dtype=torch.int64, device=device)
    x = L.field_random(L.FT63, 1, 1337)
    left, _ = P.form_side_vectors_for_polynomial_evaluation_from_point(x, n_rows, nc)
    cols = P.get_column_indicies_from_random_seed(1337, 256, nc)
    torch.cuda.synchronize()
    if world == 1:
        comm, comm_kind = shard.NativeComm.single(), "none (one rank)"
    elif backend == "nccl" and not share:
        comm, comm_kind = shard.NativeComm.rccl(dist), "RCCL (liblcpc_mi lcpc_comm_rccl_new, device send/recv)"
    elif os.environ.get("LCPC_BENCH_RCCL_SAME_GPU") == "1":
        comm, comm_kind = (shard.NativeComm.rccl(dist),
                           "RCCL with the ranks sharing one GPU (per-rank NCCL_HOSTID: socket transport over loopback)")
    else:
        comm, comm_kind = shard.NativeComm.host(dist), "host-staged gloo collectives (ranks share one GPU)"
    COMM_INFO.update(nranks=comm.world, is_rccl=comm.is_rccl)

    def step():
        if hi > lo:
            shard.pos_pack_shard(d_bytes.data_ptr() - lo, n_bytes, np_, r0, nr, d_rows.data_ptr())
        sc = shard.ShardedCommit(enc, comm, d_rows.data_ptr() if nr else 0, n_rows)
        res = sc.pos_request(left, cols, root=0)
        return sc.get_root(), res

    def barrier():
        sync_barrier(dist, torch.cuda.synchronize)

    for _ in range(max(1, args.warmup)):
        root, res0 = step()
    L.prof_enable(False)
    barrier()
    t0 = time.perf_counter()
    troots = []
    for _ in range(args.steps):
        r_, _ = step()
        troots.append(r_)
    barrier()
    elapsed = max_over_ranks(dist, time.perf_counter() - t0, "cpu" if backend == "gloo" else device)
    iso = {}
    if not args.no_prof:
        L.prof_reset()
        L.prof_enable(True)
        for _ in range(args.roofline_steps):
            step()
        L.prof_enable(False)
        iso = L.prof_stats()
    value = n_el * args.steps / elapsed
    out = {
        "metric": "proof-of-storage server request: committed field-elements/s (pack+commit+eval+256-col open), "
                  f"{n_bytes / 2**30:g} GiB file, rows sharded over the GPUs",
        "value": value, "unit": "field-elements/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u64 (WriteableFt63 Montgomery limbs)",
        "data": f"synthetic: {n_bytes} random bytes (numpy default_rng(1)), each rank's rows resident in its HBM",
        "config": {"workload": f"PoS request on one {n_bytes}-byte file: {n_el} WriteableFt63 elements, default "
                               f"dims {n_rows}x{np_}->{nc}, u^T Enc(M) at a point, 256 opened columns",
                   "file_bytes": n_bytes, "n_rows": n_rows, "n_per_row": np_, "n_cols": nc, "soundness": snd,
                   "parallelism": f"rows sharded x{world} (lcpc_sharded_commit_new_device + lcpc_sharded_pos_request)",
                   "exchanges": comm_kind, "rows_on_rank0": nr},
        "mb_per_s": n_bytes * args.steps / elapsed / 1e6,
    }
    wl = Workload(algo_bytes=nr * np_ * 8 + nr * nc * 8,
                  enc_kernels=("ntt_pass_a", "ntt_pass_b", "ntt_small", "ntt_row1"),
                  enc_kernel_desc=(f"ntt_encode = ntt_row1 (one launch per commit, this rank's {nr} rows)"
                                   if row1_active(nc) else
                                   f"ntt_encode = ntt_pass_a + ntt_pass_b (one launch each per commit, this rank's "
                                   f"{nr} rows)"),
                  traffic_key=(n_el, "Ft63", "pos-row1" if row1_active(nc) else "pos"),
                  mul_count=nr * pos_ntt_muls(nc)[0], mul_model=pos_ntt_muls(nc)[1], leaf_compressions=0)
    out.update(roofline_objects(wl, iso, {}, args, traffic_rows_frac=nr / n_rows))
    out["steps_agree"] = all(r == root for r in troots)
    want_cpu = args.cpu_baseline in ("on", "auto")
    if rank == 0:
        import hashlib
        ev, opened = res0
        out["answer_digests"] = {"root": root.hex(), "eval_sha256": hashlib.sha256(ev.tobytes()).hexdigest(),
                                 "cols_sha256": hashlib.sha256(b"".join(o.col.tobytes() for o in opened)).hexdigest()}
    if rank == 0 and want_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O  # CPU baseline and parity only
        o_enc = O.Encoding.ligero(0, np_, nc)
        cores, basis = available_cores()
        O.lib().of_set_threads(cores)
        if world == 1 or args.cpu_baseline == "on":  # (N > 1: the N = 1 line's baseline)
            # timed sample: the first 1/16 of the file, scaled to the whole
            sample = host[: n_bytes // 16]
            el = O.pos_bytes_to_field(sample.tobytes())
            t1 = time.perf_counter()
            oc = O.Commit(o_enc, el)
            O.collapse(0, oc.comm, O.pos_side_vectors(0, x.reshape(-1), oc.n_rows, nc)[0], oc.n_rows, nc)
            dt = (time.perf_counter() - t1) * 16
            del oc
            out["cpu_baseline"] = {"value": n_el / dt, "unit": "field-elements/s", "cores": cores, "kind": "port",
                                   "sample": f"commit + u^T Enc(M) of the first 1/16 of the file, scaled to the "
                                             f"whole file ({dt / 16:.2f} s)", "cores_basis": basis}
        out.update(pos_oracle_parity(O, host, np_, nc, n_rows, left, cols, root, ev, opened))
        out["parity_ok"] = bool(out["steps_agree"] and out["parity_root_vs_oracle"]
                                and out["parity_eval_vs_oracle"] and out["parity_cols_vs_oracle"])
    return out


def pos_oracle_parity(O, host, np_, nc, n_rows, left, cols, root, ev, opened):
    """The oracle's answer to the same proof-of-storage request on the WHOLE file (untimed): the
    root, u^T Enc(M) and the opened columns with their Merkle paths (lcpc_online.rs:80-239,
    454-484), against this run's answer."""
    oc = O.Commit(O.Encoding.ligero(0, np_, nc), O.pos_bytes_to_field(host.tobytes()))
    m = oc.comm.reshape(n_rows, nc)
    ohash = bytes(oc.hashes)
    return {
        "parity_root_vs_oracle": root == oc.root(),
        "parity_eval_vs_oracle": bool(np.array_equal(np.asarray(ev).reshape(-1),
                                                     O.collapse(0, oc.comm, left.reshape(-1), n_rows, nc))),
        "parity_cols_vs_oracle": bool(
            all(np.array_equal(o.col.reshape(-1), m[:, c]) for c, o in zip(cols, opened))
            and all(O.verify_path(ohash[32 * c:32 * c + 32], c, b"".join(o.path), oc.root())
                    for c, o in zip(cols, opened))),
        "parity_what": "the oracle's commit + u^T Enc(M) + columns and paths of the whole file, untimed"}


# ---------------------------------------------------------------- the replica engine
def run_replicas(args, L, torch, dist, rank, world, device_idx, backend):
    """Independent commitments per rank (cfg3 replicas, cfg4 Brakedown, cfg5 PoS, cfg2 encode),
    kept in flight on host threads over the library's pooled streams."""
    wl = {"pos": pos_workload, "encode": encode_workload, "sdig-encode": sdig_encode_workload}.get(
        args.code, ligero_or_sdig)(
        args, L, torch, rank, device_idx)
    torch.cuda.synchronize()
    prof = not args.no_prof
    # in-flight depth: --pipeline workers pull steps from one counter; with the commit gate there
    # are no waves to align (a K = 20 sweep on the box: 16 workers 11.7-11.8 G/s, 20 workers
    # 10.5-11.2, 10 workers 10.6-11.8, gpurun_out/r02v)
    P = max(1, min(args.pipeline, args.steps))
    n_workers = P
    warm_left = [max(0, args.warmup)]  # exactly --warmup untimed steps, over whichever workers
    warmup_done = warm_left[0]

    def barrier():
        sync_barrier(dist, torch.cuda.synchronize)

    lock = threading.Lock()
    todo = [args.steps]
    roots, errors = [], []
    ready = threading.Barrier(n_workers + 1)
    start = threading.Event()
    def worker(slot):
        try:
            if getattr(wl, "prepare", None):
                wl.prepare()  # this thread's pinned staging (the library's per-thread slots)
            while True:
                with lock:
                    if warm_left[0] <= 0:
                        break
                    warm_left[0] -= 1
                wl.step(slot)
        except Exception as e:  # surface after the join
            errors.append(e)
        ready.wait()
        start.wait()
        while not errors:
            with lock:
                if todo[0] <= 0:
                    return
                todo[0] -= 1
            try:
                roots.append(wl.step(slot))
            except Exception as e:
                errors.append(e)
                return

    if getattr(wl, "reserve", None):
        wl.reserve(n_workers + 1)  # device pool blocks and streams of every concurrent step (not steps)
    workers = [threading.Thread(target=worker, args=(i,)) for i in range(n_workers)]
    for w in workers:
        w.start()
    ready.wait()
    if errors:
        raise errors[0]
    L.prof_enable(prof and args.prof_timed)
    L.prof_reset()
    barrier()
    t0 = time.perf_counter()
    t0_mono_ns = time.clock_gettime_ns(time.CLOCK_MONOTONIC)  # (--timeline: aligns with a rocprofv3 trace)
    c0, th0 = os.times(), cgroup_throttle()
    start.set()
    for w in workers:
        w.join()
    if errors:
        raise errors[0]
    root = roots[-1] if roots else None
    steps_agree = len(roots) == args.steps and all(r == root for r in roots)
    barrier()
    elapsed = time.perf_counter() - t0
    c1, th1 = os.times(), cgroup_throttle()
    if args.timeline and getattr(wl, "timeline", None) is not None:
        tl = [(s_, a - t0, b - t0, c - t0, d - t0) for s_, a, b, c, d in wl.timeline if a >= t0]
        json.dump({"elapsed": elapsed, "t0_monotonic_ns": t0_mono_ns,
                   "columns": ["slot", "t_gate", "t_commit_start", "t_commit_end", "t_prove_end"],
                   "steps": sorted(tl, key=lambda r: r[2])}, open(args.timeline, "w"))
    L.prof_enable(False)
    stats = L.prof_stats() if (prof and args.prof_timed) else {}
    iso = {}
    if prof:
        # The roofline launches: the same step run serially after the timed region, so each
        # encode launch has the GPU to itself.  One untimed step first: this (main) thread's
        # pinned staging is allocated on first use.
        wl.step(0)
        L.prof_reset()
        L.prof_enable(True)
        for _ in range(args.roofline_steps):
            wl.step(0)
        L.prof_enable(False)
        iso = L.prof_stats()
    lat = wl.latency(3) if getattr(wl, "latency", None) else None
    elapsed = max_over_ranks(dist, elapsed, "cpu" if backend == "gloo" else f"cuda:{device_idx}")
    scaling = getattr(wl, "scaling", "weak")
    value = job_throughput(wl.units, args.steps, world if scaling == "weak" else 1, elapsed)
    out = {
        "metric": wl.metric, "value": value, "unit": wl.unit, "n_gpus": world, "steps": args.steps,
        "warmup": warmup_done, "ms_per_step": 1e3 * elapsed / args.steps, "pipeline": P,
        "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": wl.dtype, "data": wl.data,
        "config": dict(wl.config, parallelism=f"replicas x{world} (independent commitments per GPU, {P} in flight, "
                                              f"{args.stream_mode} streams)"),
        "mb_per_s": value * wl.bytes_per_unit / 1e6,
    }
    if lat:
        out["latency"] = lat
    if args.input != "device":
        from lcpc_proof_of_storage_amd import _native
        ib = wl.input_bytes
        rates = h2d_copy_rates(torch, ib, f"cuda:{device_idx}")
        ach = ib * args.steps * (world if scaling == "weak" else 1) / elapsed / 1e9
        out["pcie"] = {
            "input": args.input, "bytes_per_step": ib, "achieved_gbs": ach,
            "pinned_copy_peak_gbs": rates["pinned"], "pageable_copy_gbs": rates["pageable"],
            "frac_of_pinned_peak": ach / rates["pinned"] if rates["pinned"] else None,
            "library_read_pinned_source": bool(_native.load().lcpc_last_upload_pinned()),
            "what": "input bytes of the timed steps / the timed region, against one whole-buffer torch copy_ of "
                    "the same size to HBM from page-locked and from pageable memory (HIP events, best of 5)"}
    out["host_cpu"] = host_cpu_use(c0, c1, elapsed)
    if th0 and th1:
        out["host_cpu"]["cgroup_throttled"] = {k: th1[k] - th0[k] for k in th0 if k in th1}
    if stats:
        out["kernels_timed_region"] = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1], "total_ms": v[0]}
                                       for k, v in stats.items()}
    out.update(roofline_objects(wl, iso, stats, args))
    if args.code in ("encode", "sdig-encode") and out.get("roofline"):
        # each timed step of these lines is exactly one encode call (inputs resident, no other
        # kernels): the rate over the timed region, with P calls in flight, is the steady state
        # the serial launches above cannot reach when one call holds less than a wave of tiles
        st_ms = 1e3 * elapsed / args.steps
        for key, num in (("roofline", wl.algo_bytes / 1e9), ("roofline_valu", (wl.mul_count or 0) / 1e9),
                         ("roofline_gather", getattr(wl, "gather_bytes", 0) / 1e9)):
            o = out.get(key)
            if o and num and o.get("peak"):
                ach = num / (st_ms * 1e-3)
                o["steady_state"] = {"achieved": ach, "frac": ach / o["peak"], "ms_per_step": st_ms,
                                     "what": f"per-step work / the timed region's ms_per_step ({P} calls in flight)"}

    gev = None
    if getattr(wl, "verify_bench", None) and args.verify_reps > 0:
        vms, gev = wl.verify_bench(args.verify_reps)
        out["verify"] = {"ms": vms, "reps": args.verify_reps,
                         "what": "LcEvalProof::verify of one proof of this workload (host + GPU, serial)"}
    if root is not None:
        out["root"] = root.hex()
    out["steps_agree"] = steps_agree
    want_cpu = args.cpu_baseline in ("on", "auto")  # rank 0's polynomial checked at every N
    if rank == 0 and want_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O  # checker / CPU baseline only
        cores, basis = available_cores()
        if getattr(wl, "cpu_cores", None):
            cores, basis = wl.cpu_cores, "this workload runs the oracle single-threaded"
        elif args.cpu_threads:
            cores, basis = args.cpu_threads, "--cpu-threads"
        reps = args.cpu_reps if getattr(wl, "cpu_reps_ok", True) else 1
        if world == 1 or args.cpu_baseline == "on":
            med, runs, oroot, sample = time_cpu_baseline(wl, O, cores, reps)
            out["cpu_baseline"] = {"value": wl.units / med, "unit": wl.unit, "cores": cores, "kind": "port",
                                   "sample": f"{sample}: median of {len(runs)} runs after a warm-up on {cores} "
                                             f"threads ({', '.join(f'{r:.3f}' for r in runs)} s)",
                                   "cores_basis": basis}
        else:  # N > 1: the oracle runs once, as the checker only (the CPU baseline is the N = 1 line's)
            O.lib().of_set_threads(cores)
            _, oroot, _ = wl.cpu_baseline(O)
        if getattr(wl, "root_is_parity", False):
            out["parity_vs_oracle"] = bool(oroot)
        elif oroot is not None:
            out["parity_root_vs_oracle"] = oroot == root if root is not None else None
        if args.cpu_baseline_1core == "on" or (args.cpu_baseline_1core == "auto" and world == 1 and
                                               args.code in ("ligero", "encode", "sdig-encode")):
            O.lib().of_set_threads(1)
            cpu1_s, oroot1, sample1 = wl.cpu_baseline(O)
            out["cpu_baseline_1core"] = {"value": wl.units / cpu1_s, "unit": wl.unit, "cores": 1, "kind": "port",
                                         "sample": f"{sample1}: one run on 1 thread ({cpu1_s:.2f} s)"}
            if oroot1 is not None and root is not None:
                out["parity_root_vs_oracle"] = out.get("parity_root_vs_oracle", True) and oroot1 == root
    cv = getattr(wl, "cpu_verify", None)
    if cv and "verify" in out:
        out["verify"]["cpu_ms"] = cv[-1][0]
        out["verify"]["parity_vs_oracle"] = bool(all(a for _, a, _ in cv) and gev is not None and
                                                 np.array_equal(np.asarray(cv[-1][2]).reshape(-1),
                                                                np.asarray(gev).reshape(-1)))
    if rank == 0 and want_cpu and getattr(wl, "parity", None):
        out.update(wl.parity(O))
    if rank == 0 and want_cpu:
        flags = [out[k] for k in ("parity_root_vs_oracle", "parity_vs_oracle", "parity_eval_vs_oracle",
                                  "parity_cols_vs_oracle") if k in out]
        if "parity_vs_oracle" in out.get("verify", {}):
            flags.append(out["verify"]["parity_vs_oracle"])
        out["parity_ok"] = bool(steps_agree and flags and all(f is True for f in flags))
    return out


if __name__ == "__main__":
    main()
