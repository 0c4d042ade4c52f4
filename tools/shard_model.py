"""shard_model.py -- expected throughput of the row-sharded cfg3 line (bench.py --gpus N, the driver's
K = 20, W = 5) for N = 1, 2, 4, 8, from the pipelined driver's schedule and measured per-step costs:
strong (K commitments at every N) and weak (the bench's default: K steps of N commitments).

The schedule (csrc/shard_native.cpp make_sched, replayed here and checked against the library's
own lcpc_sharded_p2p_schedule in tests/test_shard_schedule.py): polynomial k's stage s goes out in
tick k + off[s], off = [0 (chaining values), 1 (subtrees), 3 (tensor 0), 4 (partials 0),
4 + L (tensor 1), 5 + L (partials 1), 5 + 3L (column indices), 6 + 3L (columns)] for cfg3's two
degree tests, lag L = max(5, 2 + G).  A run of K polynomials takes K + 6 + 3L ticks.

Time model (one run of K steps):
  T(G, K) = fill + K * tick(G) + chain
  tick(G) = max(gpu / G + xchg(G), host(G))   the steady state: one polynomial enters per tick
  chain   = the last polynomial after its commit: three serial transcript absorptions (the
            Merlin transcript of its proof, one rank) plus the folds, gathers and the proof's
            assembly; its lag ticks run meanwhile (a tick that waits on nothing is host-only)
  fill    = the first polynomial's encode (AHEAD ticks are launched before it is needed)
Inputs, all measured on one MI355X (profiles/):
  gpu   = 1.15 ms: one cfg3 commit + open of GPU work at the replicas' steady state
          (r03_commit_fifo_ab.json: commits complete every 1.15 ms; r03_timeline_k20_replicas.json)
  absorb = 1.15 ms per round (32768 records x 35 ns, r02_transcript_bench.txt)
  host  = 0.06 ms per tick at one rank (r03_sharded_k20_host_timeline_split.csv: tick_run_group +
          tick_submit), 0.10 ms assumed at G > 1 (one RCCL group of 2 (G - 1) sends / receives per
          exchange: not measured on a multi-GPU node)
  xchg  = the tick's exchange bytes over xGMI: the chaining-value all-to-all (7/8 of 2 MiB per rank
          at G = 8) at 7 links x ~50 GB/s per direction (an assumption, MI355X_MICROARCH xGMI)
"""
import json
import math
import sys

GPU_MS = 1.15
ABSORB_MS = 1.15
HOST_MS_1 = 0.06
HOST_MS_G = 0.10
XGMI_GBS = 7 * 50.0
K_DEFAULT = 20
N_ELEMS = 1 << 24
N_ROWS, N_COLS, WB = 512, 65536, 16


def lag_of(G, lag=0):
    return lag if lag else max(5, 2 + G)


def offsets(ndt, G, lag=0):
    L = lag_of(G, lag)
    rounds = max(ndt, 1)
    off = [0, 1, 3, 4]
    for _ in range(1, rounds):
        off += [off[-1] + L, off[-1] + L + 1]
    off.append(off[-1] + (2 if ndt else 1) * L)  # column indices
    off.append(off[-1] + 1)                       # columns
    return off


def n_ticks(K, ndt, G, lag=0):
    return K + offsets(ndt, G, lag)[-1]


def cv_bytes_per_rank(G):
    """chaining values a rank sends per polynomial: its chunks' values of the other ranks' blocks"""
    n_chunks = -(-(32 + N_ROWS * WB) // 1024)
    return (G - 1) / G * (n_chunks / G) * N_COLS * 32


def predict(G, K=K_DEFAULT, lag=0):
    host = HOST_MS_1 if G == 1 else HOST_MS_G
    xchg = 0.0 if G == 1 else cv_bytes_per_rank(G) / (XGMI_GBS * 1e6)
    tick = max(GPU_MS / G + xchg, host)
    L = lag_of(G, lag)
    # the lag must cover one absorption: L ticks of the steady state >= absorb (else the tensor
    # broadcast of the next round waits, and the pipeline stalls on the transcript every round)
    stall = max(0.0, ABSORB_MS - L * tick)
    chain = 3 * ABSORB_MS + 0.35 + (4 * xchg if G > 1 else 0.0)
    fill = GPU_MS / G
    T = fill + K * (tick + stall) + chain
    return {"G": G, "K": K, "lag": L, "ticks": n_ticks(K, 2, G, lag), "tick_ms": tick, "lag_covers_absorb":
            L * tick >= ABSORB_MS, "chain_ms": chain, "run_ms": T, "ms_per_step": T / K,
            "G_elements_per_s": K * N_ELEMS / (T * 1e-3) / 1e9}


def main():
    """strong: K commitments at every N (bench.py --sharded-scaling strong); weak (the bench's
    default): K steps of N commitments, each row-sharded over all N ranks"""
    K = int(sys.argv[1]) if len(sys.argv) > 1 else K_DEFAULT
    base = predict(1, K)["G_elements_per_s"]
    out = {}
    for scaling in ("strong", "weak"):
        rows = [predict(G, K if scaling == "strong" else K * G) for G in (1, 2, 4, 8)]
        for r in rows:
            r["speedup_vs_1"] = r["G_elements_per_s"] / base
            r["efficiency"] = r["speedup_vs_1"] / r["G"]
        out[scaling] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
