"""IncrementalVerifier's flush policy (the MsgId.piece handler, torrent.ts:183-193) on CPU.

The policy is host logic: flush when `flush_pieces` pieces are pending or the oldest pending piece is
`flush_age_ms` old.  Here the library context is a stand-in that records each tv_verify_list call and
answers with hashlib (the checker), so the policy is tested without a GPU; the GPU flow itself is
tests/test_gpu_paths.py::test_incremental_verifier_flow and ::test_flush_policy_on_the_gpu.
"""
import hashlib

import pytest

from torrent_amd import incremental
from torrent_amd.metainfo import make_info
from torrent_amd.piece import BLOCK_SIZE, PieceMsg


class _ListCtx:
    """tv_ctx stand-in: stage() keeps the bytes, verify_list() hashes them (one call = one flush).  It models
    the library's slot pool (TV_OPT_LIST_SLOTS): a staged piece holds a slot until a flush lists it, and staging
    with every slot taken is an error (TV_ERR_STATE in the library)."""

    def __init__(self, device=0):
        self.bytes = {}
        self.flushes = []
        self.slots = 0
        self.max_held = 0

    def set_option(self, key, value):
        from torrent_amd import _native
        if key == _native.TV_OPT_LIST_SLOTS:
            self.slots = value

    def set_layout(self, total, L, P, first, count):
        self.L = L

    def set_digests(self, raw):
        self.raw = raw

    def stage(self, off, data):
        i = off // self.L
        if self.slots and i not in self.bytes and len(self.bytes) >= self.slots:
            raise RuntimeError("every slot holds a staged piece not yet listed")
        self.bytes[i] = bytes(data)
        self.max_held = max(self.max_held, len(self.bytes))

    def verify_list(self, pieces):
        self.flushes.append(list(pieces))
        out = bytes(int(i in self.bytes and hashlib.sha1(self.bytes[i]).digest() == self.raw[20 * i:20 * i + 20])
                    for i in pieces)
        for i in pieces:
            self.bytes.pop(i, None)
        return out

    def close(self):
        pass


def _torrent(P=40, L=2 * BLOCK_SIZE):
    payload = bytes((k * 7 + 3) & 0xFF for k in range(P * L))
    pieces = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    return make_info(L, pieces, "t.bin", length=P * L), payload


def _blocks(info, payload, i):
    L = info.piece_length
    return [PieceMsg(i, o, payload[i * L + o:i * L + o + BLOCK_SIZE]) for o in range(0, L, BLOCK_SIZE)]


@pytest.fixture
def fake(monkeypatch):
    made = []

    def ctx(device=0):
        c = _ListCtx(device)
        made.append(c)
        return c

    monkeypatch.setattr(incremental._native, "Context", ctx)
    return made


def test_flush_at_k_pending(fake):
    info, payload = _torrent()
    got = []
    v = incremental.IncrementalVerifier(info, flush_pieces=8, flush_age_ms=None, on_verified=lambda i, ok: got.append((i, ok)))
    for i in range(20):
        for m in _blocks(info, payload, i):
            v.on_block(m)
    assert [len(f) for f in fake[0].flushes] == [8, 8]          # two automatic flushes of 8
    assert v.auto_flushes == 2 and got == [(i, True) for i in range(16)]
    assert v.flush() == [(i, True) for i in range(16, 20)]      # the rest, by hand
    assert all(v.bitfield[i >> 3] & (0x80 >> (i & 7)) for i in range(20))


def test_flush_at_age(fake, monkeypatch):
    info, payload = _torrent()
    now = [100.0]
    monkeypatch.setattr(incremental.time, "monotonic", lambda: now[0])
    v = incremental.IncrementalVerifier(info, flush_pieces=None, flush_age_ms=30.0)
    for i in range(3):
        for m in _blocks(info, payload, i):
            v.on_block(m)
        now[0] += 0.010                                         # 10 ms between completed pieces
    assert fake[0].flushes == []                                # the oldest is 30 ms old only now
    assert v.due()
    assert v.poll() == [(0, True), (1, True), (2, True)]        # poll() flushes and hands out
    assert [len(f) for f in fake[0].flushes] == [3]
    # the age bound is also checked on blocks that complete nothing
    for m in _blocks(info, payload, 3):
        v.on_block(m)
    now[0] += 0.031
    v.on_block(_blocks(info, payload, 4)[0])
    assert [len(f) for f in fake[0].flushes] == [3, 1]
    assert v.flush() == [(3, True)]                             # held for the next flush() (no callback)


def test_default_policy_from_the_flush_cost(fake):
    """Defaults: 4,096 pieces; age 10 x the estimated flush cost (one piece's serial SHA-1 at ~0.73 us per
    block, measured), at least 5 ms -- ~30 ms for 256 KiB pieces."""
    info, _ = _torrent(P=8, L=256 << 10)
    v = incremental.IncrementalVerifier(info)
    assert v.flush_pieces == 4096
    assert 29.0 < v.flush_age_ms < 32.0
    small, _ = _torrent(P=8, L=BLOCK_SIZE)
    assert incremental.IncrementalVerifier(small).flush_age_ms == 5.0
    manual = incremental.IncrementalVerifier(info, flush_pieces=None, flush_age_ms=None)
    assert not manual.due()


def test_corrupt_piece_is_reported_by_an_automatic_flush(fake):
    info, payload = _torrent()
    got = {}
    v = incremental.IncrementalVerifier(info, flush_pieces=1, flush_age_ms=None, on_verified=got.__setitem__)
    bad = _blocks(info, payload, 5)
    bad[0] = PieceMsg(5, 0, bytes(b ^ 1 for b in bad[0].block))
    for m in bad:
        v.on_block(m)
    assert got == {5: False} and not (v.bitfield[0] & 0x04)
    for m in _blocks(info, payload, 5):                          # re-received correctly
        v.on_block(m)
    assert got == {5: True} and v.bitfield[0] & 0x04


def test_slot_pool_bounds_the_pending_pieces(fake):
    """slots=3 with the caller flushing (no count or age bound): the verifier never holds more than 3 staged
    pieces; the 4th completed piece first flushes the 3 pending ones (a forced flush), and every piece's result
    is delivered exactly once, in completion order."""
    info, payload = _torrent(P=10)
    seen = []
    v = incremental.IncrementalVerifier(info, flush_pieces=None, flush_age_ms=None, slots=3,
                                        on_verified=lambda i, ok: seen.append((i, ok)))
    for i in range(10):
        for m in _blocks(info, payload, i):
            v.on_block(m)
    seen += v.flush()
    ctx = fake[-1]
    assert ctx.max_held == 3 and v.forced_flushes == 3
    assert [len(f) for f in ctx.flushes] == [3, 3, 3, 1]
    assert seen == [(i, True) for i in range(10)]
    assert v.slots == 3
