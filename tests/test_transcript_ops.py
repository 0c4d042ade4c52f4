"""The caller-owned transcript boundary (lcpc_transcript_ops), host side -- no GPU needed.

The reference's prove / verify take the caller's `&mut merlin::Transcript`
(lcpc-2d/src/lib.rs:319-326, 547-556).  lcpc_transcript_from_ops forwards every absorb and
squeeze to the caller's functions.  Here the "caller" is the ORACLE's Merlin restatement
(oracle/of_hash.c, checker only) driven through ctypes callbacks, and the library's own host-side
Fiat-Shamir steps (challenge tensor, field-element absorption, column choice: lib.rs:1056-1062,
1075-1077, 1101-1110) must leave it in exactly the state the library's own transcript reaches.
The full prove / verify over ops is in test_gpu_transcript_ops.py.
"""
import ctypes as C

import numpy as np
import pytest

LABEL_DT, LABEL_PR, LABEL_CO = b"$l//DT", b"$l//PR", b"$l//CO"


class CountingOracleTranscript:
    """the oracle's Merlin transcript, counting the calls it receives"""

    def __init__(self, oracle, label=b"test transcript", batched=True):
        self.t = oracle.Transcript(label)
        self.calls = {"append_message": 0, "append_messages": 0, "challenge_bytes": 0}
        if batched:
            self.append_messages = self._append_messages

    def append_message(self, label, msg):
        self.calls["append_message"] += 1
        self.t.append_message(label, msg)

    def _append_messages(self, label, msgs, msg_len):
        self.calls["append_messages"] += 1
        for i in range(len(msgs) // msg_len):
            self.t.append_message(label, msgs[i * msg_len:(i + 1) * msg_len])

    def challenge_bytes(self, label, n):
        self.calls["challenge_bytes"] += 1
        return self.t.challenge_bytes(label, n)


@pytest.fixture(scope="module")
def lib():
    from lcpc_proof_of_storage_amd import _native as N
    return N.load()


def _lib_transcript(gpu):
    t = gpu.Transcript(b"test transcript")
    t.append_message(b"polycommit", bytes(range(32)))
    return t


@pytest.mark.parametrize("batched", [True, False])
@pytest.mark.parametrize("fid", [0, 1, 2, 3, 4])
def test_challenges_through_ops_match_own_transcript(oracle, lib, fid, batched):
    """challenge tensor -> absorb its repr-free twin (raw message batch) -> column choice, through
    a caller (oracle) transcript and through the library's own: identical draws and end state."""
    import lcpc_proof_of_storage_amd as L
    own = _lib_transcript(L)
    caller = CountingOracleTranscript(oracle, batched=batched)
    caller.append_message(b"polycommit", bytes(range(32)))
    ct = L.CallerTranscript(caller)
    n = 37
    nl = L.limbs(fid)
    for tr in (own, ct):
        tr._out = np.zeros(n * nl, np.uint64)
        assert lib.lcpc_challenge_tensor(tr._h, fid, n, tr._out.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
    assert np.array_equal(own._out, ct._out)
    msgs = bytes((7 * i) & 0xFF for i in range(16 * 50))
    for tr in (own, ct):
        lb = (C.c_uint8 * 6).from_buffer_copy(LABEL_PR)
        mb = (C.c_uint8 * len(msgs)).from_buffer_copy(msgs)
        lib.lcpc_transcript_append_messages(tr._h, lb, 6, mb, 16, 50)
    for tr in (own, ct):
        tr._idx = np.zeros(309, np.uint64)
        assert lib.lcpc_challenge_columns(tr._h, 65536, 309, tr._idx.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
    assert np.array_equal(own._idx, ct._idx)
    assert own.challenge_bytes(b"after", 32) == caller.challenge_bytes(b"after", 32)
    # batched callers get ONE call per message vector; the others one per message
    assert caller.calls["append_messages"] == (1 if batched else 0)
    assert caller.calls["append_message"] == (0 if batched else 50) + 1  # (+ the polycommit prefix)
    assert caller.calls["challenge_bytes"] == 3  # tensor key, column key, "after"


def test_column_choice_matches_oracle_draw(oracle, lib):
    """lcpc_challenge_columns over the oracle's transcript = the oracle's own column draw
    (ChaCha20 + Uniform(0, n_cols) on the "$l//CO" key, lib.rs:1101-1110)."""
    import lcpc_proof_of_storage_amd as L
    a = oracle.Transcript(b"x")
    b = oracle.Transcript(b"x")
    ct = L.CallerTranscript(a)
    got = np.zeros(100, np.uint64)
    assert lib.lcpc_challenge_columns(ct._h, 1000, 100, got.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
    key = b.challenge_bytes(LABEL_CO, 32)
    rng = oracle.ChaCha(seed=key)
    assert list(got) == [rng.uniform(0, 1000) for _ in range(100)]
    assert a.challenge_bytes(b"after", 32) == b.challenge_bytes(b"after", 32)


def test_ops_handle_contract(oracle, lib):
    import lcpc_proof_of_storage_amd as L
    from lcpc_proof_of_storage_amd import _native as N
    ct = L.CallerTranscript(oracle.Transcript(b"x"))
    # no transcript state of its own: clone refuses
    assert not lib.lcpc_transcript_clone(ct._h)
    assert "cannot be cloned" in N.last_error()
    # append_message / challenge_bytes are mandatory
    ops = N.TranscriptOps(None, N.TR_APPEND_FN(), N.TR_APPEND_MANY_FN(), N.TR_CHALLENGE_FN())
    assert not lib.lcpc_transcript_from_ops(C.byref(ops))
    assert not lib.lcpc_transcript_from_ops(None)
    # the per-call entry points refuse missing ops before touching a device
    h = C.c_void_p()
    assert lib.lcpc_prove_ops(None, None, 0, None, C.byref(ops), C.byref(h)) == 30
    assert lib.lcpc_verify_ops(None, None, 0, None, 0, None, None, None, None) == 30
    # the library's own transcript reports no callback status
    own = L.Transcript(b"x")
    assert lib.lcpc_transcript_status(own._h) == 0


def test_failing_callback_fails_the_call(oracle, lib):
    """A callback that raises: the Fiat-Shamir step returns LCPC_ERR_TRANSCRIPT (35), the status
    sticks, and later callbacks are not made (the caller's state is no longer the reference's)."""
    import lcpc_proof_of_storage_amd as L

    class Broken:
        def __init__(self):
            self.n = 0

        def append_message(self, label, msg):
            self.n += 1

        def challenge_bytes(self, label, n):
            raise RuntimeError("caller transcript is gone")

    b = Broken()
    ct = L.CallerTranscript(b)
    out = np.zeros(8 * 2, np.uint64)
    assert lib.lcpc_challenge_tensor(ct._h, 1, 8, out.ctypes.data_as(C.POINTER(C.c_uint64))) == 35
    assert lib.lcpc_transcript_status(ct._h) == 1
    assert isinstance(ct.error, RuntimeError)
    lb = (C.c_uint8 * 6).from_buffer_copy(LABEL_PR)
    lib.lcpc_transcript_append_message(ct._h, lb, 6, lb, 6)
    assert b.n == 0  # nothing forwarded after the failure
    with pytest.raises(RuntimeError):
        ct.reraise(35)

    class WrongLength(Broken):
        def challenge_bytes(self, label, n):
            return b"\x00" * (n - 1)

    ct2 = L.CallerTranscript(WrongLength())
    assert lib.lcpc_challenge_columns(ct2._h, 16, 4, out.ctypes.data_as(C.POINTER(C.c_uint64))) == 35
    assert isinstance(ct2.error, ValueError)


def test_labels_are_the_reference_constants(oracle, lib):
    """Every label the library passes through the ops is one of def_labels!'s literal byte strings
    (lcpc-2d/src/macros.rs:29-36) -- what lets a Rust shim map them back to &'static [u8]."""
    import lcpc_proof_of_storage_amd as L
    seen = set()

    class Recorder(CountingOracleTranscript):
        def append_message(self, label, msg):
            seen.add(label)
            super().append_message(label, msg)

        def _append_messages(self, label, msgs, ml):
            seen.add(label)
            super()._append_messages(label, msgs, ml)

        def challenge_bytes(self, label, n):
            seen.add(label)
            return super().challenge_bytes(label, n)

    ct = L.CallerTranscript(Recorder(oracle))
    out = np.zeros(4 * 2, np.uint64)
    p64 = out.ctypes.data_as(C.POINTER(C.c_uint64))
    assert lib.lcpc_challenge_tensor(ct._h, 1, 4, p64) == 0
    assert lib.lcpc_challenge_columns(ct._h, 64, 4, p64) == 0
    assert seen == {LABEL_DT, LABEL_CO}
