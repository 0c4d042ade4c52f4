"""CPU: the RCCL exchange groups of the pipelined row-sharded driver match across ranks.

lcpc_sharded_p2p_schedule (include/lcpc_mi.h) returns, for one rank, the exact ncclSend /
ncclRecv list run_group issues in every group of lcpc_sharded_commit_prove_many.  RCCL pairs the
sends p -> q and the receives on q from p of one group in issue order, so the multi-rank path is
deadlock-free and moves the right bytes iff, in every tick, p's sends to q and q's receives from
p are the same sequence of sizes.  Checked here for 2, 4 and 8 ranks at cfg3 (Ft127 2^24:
512 x 32768 -> 65536, 309 opens, 2 degree tests) and at ragged shapes, without a GPU.  The
exchanges replace nothing in the reference (its rows never leave one host,
lcpc-2d/src/lib.rs:677-682, 736-815); the byte counts are checked against that layout.
"""
import collections
import ctypes as C

import pytest

from lcpc_proof_of_storage_amd import _native

FT63, FT127, FT255 = 0, 1, 3
WB = {FT63: 8, FT127: 16, FT255: 32}


def schedule(fid, n_rows, np_, nc, ndt, nco, G, rank, n_polys, lag=0):
    lib = _native.load()
    n = C.c_size_t()
    assert lib.lcpc_sharded_p2p_schedule(fid, n_rows, np_, nc, ndt, nco, G, rank, n_polys, lag, None, 0,
                                         C.byref(n)) in (0, 30)
    buf = (_native.P2pRecord * max(n.value, 1))()
    rc = lib.lcpc_sharded_p2p_schedule(fid, n_rows, np_, nc, ndt, nco, G, rank, n_polys, lag, buf, n.value,
                                       C.byref(n))
    assert rc == 0, _native.last_error()
    return [(r.tick, r.pos, r.poly, r.stage, bool(r.is_send), r.peer, r.bytes) for r in buf[:n.value]]


def rows_of(fid, n_rows, G):
    lib = _native.load()
    out = []
    for g in range(G):
        r0, nr = C.c_size_t(), C.c_size_t()
        assert lib.lcpc_sharded_rows(fid, n_rows, G, g, C.byref(r0), C.byref(nr)) == 0
        out.append((r0.value, nr.value))
    return out


def check_matching(fid, n_rows, np_, nc, ndt, nco, G, n_polys, lag=0):
    sched = [schedule(fid, n_rows, np_, nc, ndt, nco, G, g, n_polys, lag) for g in range(G)]
    sends = collections.defaultdict(list)  # (tick, p, q) -> [(poly, stage, bytes)]
    recvs = collections.defaultdict(list)
    for g, recs in enumerate(sched):
        last = (-1, -1)
        for tick, pos, poly, stage, is_send, peer, nbytes in recs:
            assert (tick, pos) > last, "records out of group order"
            last = (tick, pos)
            assert 0 <= peer < G and peer != g and nbytes > 0
            if is_send:
                sends[(tick, g, peer)].append((poly, stage, nbytes))
            else:
                recvs[(tick, peer, g)].append((poly, stage, nbytes))
    assert set(sends) == set(recvs), "a tick has sends without matching receives (or the reverse)"
    for key in sends:
        assert sends[key] == recvs[key], f"tick {key[0]}: {key[1]}->{key[2]} sends {sends[key]} vs recvs {recvs[key]}"
    return sched


def stage_bytes(sched, stage, poly=0):
    """bytes rank g sends / receives in (poly, stage)"""
    out = []
    for recs in sched:
        s = sum(r[6] for r in recs if r[2] == poly and r[3] == stage and r[4])
        v = sum(r[6] for r in recs if r[2] == poly and r[3] == stage and not r[4])
        out.append((s, v))
    return out


@pytest.mark.parametrize("G", [2, 4, 8])
def test_cfg3_groups_match(G):
    n_rows, np_, nc, ndt, nco = 512, 32768, 65536, 2, 309
    sched = check_matching(FT127, n_rows, np_, nc, ndt, nco, G, n_polys=20)
    wb = WB[FT127]
    rows = rows_of(FT127, n_rows, G)
    n_chunks = -(-(32 + n_rows * wb) // 1024)
    B = nc // G
    # stage 0: rank g sends its chunks' chaining values of block k to rank k (32 B per column)
    for g, (sb, rb) in enumerate(stage_bytes(sched, 0)):
        nch_g = (g + 1) * n_chunks // G - g * n_chunks // G
        assert sb == (G - 1) * nch_g * B * 32
        assert rb == (n_chunks - nch_g) * B * 32
    # stage 1: all-gather of the (2B - 1)-digest subtrees
    for sb, rb in stage_bytes(sched, 1):
        assert sb == rb == (G - 1) * (2 * B - 1) * 32
    # poly 0's root is rank 0: tensor broadcasts (n_rows elements), then its partial sums
    # (2 tensors in round 0, 1 after), then the column indices and column pieces
    rounds = max(ndt, 1)
    for r in range(rounds):
        bc = stage_bytes(sched, 2 + 2 * r)
        assert bc[0] == ((G - 1) * n_rows * wb, 0) and all(x == (0, n_rows * wb) for x in bc[1:])
        nt = 2 if r == 0 else 1
        ga = stage_bytes(sched, 3 + 2 * r)
        assert ga[0] == (0, (G - 1) * nt * np_ * wb) and all(x == (nt * np_ * wb, 0) for x in ga[1:])
    idx = stage_bytes(sched, 2 + 2 * rounds)
    assert idx[0] == ((G - 1) * nco * 8, 0)
    cols = stage_bytes(sched, 3 + 2 * rounds)
    assert cols[0][1] == nco * (n_rows - rows[0][1]) * wb
    assert all(cols[g] == (nco * rows[g][1] * wb, 0) for g in range(1, G))


@pytest.mark.parametrize("fid,n_rows,np_,nc,ndt,nco,G", [
    (FT127, 37, 64, 128, 2, 7, 4),   # ragged rows: some ranks' row shards differ in size
    (FT127, 3, 16, 32, 1, 5, 4),     # fewer rows than ranks: empty shards
    (FT63, 100, 128, 256, 3, 11, 8),
    (FT255, 9, 64, 128, 0, 4, 2),    # no degree tests: round 0 is the evaluation alone
    (2, 700, 256, 512, 2, 9, 4),     # Ft191: 24-byte elements, cuts every third chunk
    (FT127, 512, 32768, 65536, 2, 309, 8),
])
@pytest.mark.parametrize("lag", [0, 1, 5])
def test_ragged_groups_match(fid, n_rows, np_, nc, ndt, nco, G, lag):
    check_matching(fid, n_rows, np_, nc, ndt, nco, G, n_polys=7, lag=lag)


def test_every_rank_has_the_same_group_structure():
    G = 4
    sched = [schedule(FT127, 512, 32768, 65536, 2, 309, G, g, 9) for g in range(G)]
    # each tick's (poly, stage) set with traffic is seen by all ranks (an all-to-all / gather
    # stage involves every rank)
    per_rank = [{(r[0], r[2], r[3]) for r in recs} for recs in sched]
    assert per_rank[0] == per_rank[1] == per_rank[2] == per_rank[3]


def test_schedule_rejects_bad_rank_counts():
    lib = _native.load()
    n = C.c_size_t()
    assert lib.lcpc_sharded_p2p_schedule(FT127, 512, 32768, 65536, 2, 309, 3, 0, 4, 0, None, 0, C.byref(n)) != 0
    assert lib.lcpc_sharded_p2p_schedule(FT127, 512, 32768, 65536, 2, 309, 16, 0, 4, 0, None, 0, C.byref(n)) == 30


@pytest.mark.parametrize("fid,wb", [(0, 8), (1, 16), (2, 24), (3, 32)])
@pytest.mark.parametrize("n_rows", [1, 41, 84, 85, 512, 9363])
@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_row_cuts_fall_on_chunk_and_element_boundaries(fid, wb, n_rows, G):
    """lcpc_sharded_rows: the ranks' rows tile [0, n_rows) in order, and every cut is where a
    1 KiB BLAKE3 chunk of the leaf message (32 zero bytes || column) starts on an element
    boundary, so a rank's chunks hold only its own elements (Ft191: 24-byte elements)."""
    rows = rows_of(fid, n_rows, G)
    assert rows[0][0] == 0 and sum(nr for _, nr in rows) == n_rows
    for (r0, nr), (r1, _) in zip(rows, rows[1:]):
        assert r0 + nr == r1
    for r0, _ in rows[1:]:
        if 0 < r0 < n_rows:
            assert (32 + r0 * wb) % 1024 == 0, (r0, wb)


def test_model_offsets_match_the_library_schedule():
    """tools/shard_model.py's tick offsets (the basis of DESIGN §6's expected N = 1/2/4/8 table)
    are the library's: polynomial k's stage s is in tick k + off[s] of lcpc_sharded_p2p_schedule"""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import shard_model
    for G in (2, 4, 8):
        off = shard_model.offsets(2, G)
        recs = schedule(FT127, 512, 32768, 65536, 2, 309, G, 0, 20)
        for k in (0, 7, 19):
            ticks = {}
            for grp, _pos, poly, stage, *_ in recs:
                if poly == k:
                    ticks.setdefault(stage, grp // 2)
            assert ticks == {s: k + off[s] for s in range(len(off))}, (G, k, ticks, off)


def test_ticks_per_proof_bounded_at_eight_ranks():
    """G = 8, cfg3, the driver's K = 20: a polynomial's exchanges span 6 + 3 lag ticks from its
    chaining values to its opened columns (lag = 10: 36), the whole run K + 36 ticks, and lag ticks
    of the steady state still cover one transcript absorption (else every round would stall)"""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import shard_model
    G, K = 8, 20
    recs = schedule(FT127, 512, 32768, 65536, 2, 309, G, 0, K)
    span = {}
    for grp, _pos, poly, _stage, *_ in recs:
        lo, hi = span.get(poly, (grp // 2, grp // 2))
        span[poly] = (min(lo, grp // 2), max(hi, grp // 2))
    assert len(span) == K and all(hi - lo <= 36 for lo, hi in span.values())
    assert max(hi for _, hi in span.values()) + 1 <= K + 36
    p = shard_model.predict(G, K)
    assert p["ticks"] == K + 36 and p["lag_covers_absorb"]
