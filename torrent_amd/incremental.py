"""Incremental verification on piece completion.

The reference's piece-message handler (torrent.ts:183-193) validates a received block
(validateReceivedBlock, piece.ts:39-65) and writes it through Storage.set (storage.ts:67-87), but
never checks a completed piece: Torrent.bitfield stays all zero (torrent.ts:60).  This class adds
that check with the same inputs:

    v = IncrementalVerifier(info, storage)          # storage: the reference's Storage (optional)
    v.on_block(PieceMsg(index, offset, block))      # per received block; True when the piece is complete
    for index, ok in v.flush():                     # ONE GPU launch (tv_verify_list) for all pending pieces
        if ok: send_have(index)                     # v.bitfield already has the bit (torrent.ts:147-149)

A completed piece's bytes are staged into HBM as soon as its last block arrives; flush() verifies
every pending piece in one list launch.  A piece that fails verification is forgotten (its blocks
may be received again), as a client would re-request it.

Device memory is bounded by the pieces AWAITING verification, not by the torrent: the context is a slot
pool of K = `slots` pieces (TV_OPT_LIST_SLOTS; default the flush count, 4,096), a completed piece takes a
slot when it is staged and gives it back when its flush returns, and when all K slots are taken the next
completed piece first flushes the pending ones.  A 200 GiB torrent of 4 MiB pieces holds K x 4 MiB of HBM.

Flush policy.  A list flush costs about one piece's serial SHA-1 whatever the list length, ~0.73 us per
64-B block: 3.0 ms for 256 KiB pieces, whether 1 or 4,096 of them (3.00 / 3.01 / 3.15 ms for 1 / 64 /
4,096; profiles/r02/latency_twin.json, r03 latency).  Flushing per piece therefore costs ~3 ms of GPU time
per piece; batching is the point.  The verifier flushes by itself when
  * `flush_pieces` pieces are pending (default 4,096: the flush time is still flat there), or
  * the oldest pending piece has waited `flush_age_ms` (default 10 x the flush cost, at least 5 ms: 30 ms
    for 256 KiB pieces), checked on every on_block() and by poll() -- so the GPU spends at most ~10 % of
    its time on flushes while pieces trickle in, and a have-bit is at most ~1.1 x flush_age_ms late.
Results of automatic flushes go to `on_verified(index, ok)` when given, else they are returned by the
next flush() / poll().  flush_pieces=1 restores flush-per-piece; flush_age_ms=None with
flush_pieces=None leaves flushing to the caller.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Tuple

from . import _native
from .metainfo import InfoDict
from .piece import BLOCK_SIZE, PieceMsg, piece_length, validate_received_block

US_PER_BLOCK = 0.73       # list-flush time per 64-B block of one piece (kernel 2.94-2.98 ms / 4,097 blocks)
DEFAULT_FLUSH_PIECES = 4096
_AUTO = object()


def flush_cost_ms(piece_len: int) -> float:
    """Estimated GPU time of one list flush of pieces of `piece_len` bytes: one piece's serial SHA-1."""
    return ((piece_len + 8) // 64 + 1) * US_PER_BLOCK / 1e3 + 0.06


class IncrementalVerifier:
    def __init__(self, info: InfoDict, storage=None, device: int = 0,
                 shard: Optional[Tuple[int, int]] = None, flush_pieces=_AUTO, flush_age_ms=_AUTO,
                 on_verified: Optional[Callable[[int, bool], None]] = None, slots: Optional[int] = None):
        self.info = info
        self.storage = storage
        self.flush_pieces = DEFAULT_FLUSH_PIECES if flush_pieces is _AUTO else flush_pieces
        self.flush_age_ms = (max(5.0, 10 * flush_cost_ms(info.piece_length)) if flush_age_ms is _AUTO
                             else flush_age_ms)
        self.on_verified = on_verified
        self.auto_flushes = 0
        self._oldest = 0.0                # time.monotonic() of the oldest pending piece
        self._results: List[Tuple[int, bool]] = []   # automatic flushes' results not yet handed out
        P = info.n_pieces
        self.first, self.count = shard if shard is not None else (0, P)
        # the slot pool: K pieces of HBM awaiting verification (at least the count bound, so it never forces
        # a flush the policy would not make)
        if slots is None:
            slots = self.flush_pieces if isinstance(self.flush_pieces, int) else DEFAULT_FLUSH_PIECES
        self.slots = max(1, min(int(slots), max(1, self.count)))
        self.forced_flushes = 0
        self.ctx = _native.Context(device)
        self.ctx.set_option(_native.TV_OPT_LIST_SLOTS, self.slots)
        self.ctx.set_layout(info.length, info.piece_length, P, self.first, self.count)
        self.ctx.set_digests(info.pieces_raw)
        self.bitfield = bytearray((P + 7) // 8)        # torrent.ts:60
        self._bufs: Dict[int, bytearray] = {}
        self._have_blocks: Dict[int, set] = {}
        self._pending: List[int] = []
        self._pending_set: set = set()

    def _blocks_in(self, index: int) -> int:
        return -(-piece_length(index, self.info) // BLOCK_SIZE)

    def on_block(self, msg: PieceMsg) -> bool:
        """Handle one received block (torrent.ts:183-193).  Raises ValueError for an invalid block
        (piece.ts:39-65).  Returns True when this block completed its piece."""
        validate_received_block(self.info, msg)
        self._auto_flush()                                # the age bound, checked on every block
        i = msg.index
        if not (self.first <= i < self.first + self.count):
            raise ValueError(f"piece {i} is outside this verifier's shard")
        if self.storage is not None:
            self.storage.set(i * self.info.piece_length + msg.offset, msg.block)
        if self.bitfield[i >> 3] & (0x80 >> (i & 7)):
            return False                                  # already verified
        if i in self._pending_set:
            return False                                  # complete and staged, waiting for flush()
        plen = piece_length(i, self.info)
        if msg.offset >= plen:
            return False
        block = memoryview(msg.block)[:plen - msg.offset]  # never past the piece (L % BLOCK_SIZE != 0)
        buf = self._bufs.get(i)
        if buf is None:
            buf = self._bufs[i] = bytearray(plen)
            self._have_blocks[i] = set()
        buf[msg.offset:msg.offset + len(block)] = block
        blocks = self._have_blocks[i]
        blocks.add(msg.offset // BLOCK_SIZE)
        done = False
        if len(blocks) == self._blocks_in(i):
            if len(self._pending) >= self.slots:          # every slot awaits a flush: make room
                self.forced_flushes += 1
                self._deliver(self._flush_pending())
            self.ctx.stage(i * self.info.piece_length, buf)
            del self._bufs[i], self._have_blocks[i]
            if not self._pending:
                self._oldest = time.monotonic()
            self._pending.append(i)
            self._pending_set.add(i)
            done = True
            self._auto_flush()                            # the count bound
        return done

    def due(self) -> bool:
        """Would the flush policy flush now (enough pieces pending, or the oldest old enough)?"""
        if not self._pending:
            return False
        if self.flush_pieces is not None and len(self._pending) >= self.flush_pieces:
            return True
        return (self.flush_age_ms is not None and
                (time.monotonic() - self._oldest) * 1e3 >= self.flush_age_ms)

    def _deliver(self, res: List[Tuple[int, bool]]) -> None:
        if self.on_verified is not None:
            for i, ok in res:
                self.on_verified(i, ok)
        else:
            self._results.extend(res)

    def _auto_flush(self) -> None:
        if self.due():
            self.auto_flushes += 1
            self._deliver(self._flush_pending())

    def poll(self) -> List[Tuple[int, bool]]:
        """For a client's event loop: flush if the policy says so, and hand out every result the automatic
        flushes have not yet returned."""
        self._auto_flush()
        out, self._results = self._results, []
        return out

    def _flush_pending(self) -> List[Tuple[int, bool]]:
        if not self._pending:
            return []
        pending, self._pending = self._pending, []
        self._pending_set.clear()
        ok = self.ctx.verify_list(pending)
        out = []
        for i, r in zip(pending, ok):
            if r:
                self.bitfield[i >> 3] |= 0x80 >> (i & 7)
            out.append((i, bool(r)))
        return out

    def flush(self) -> List[Tuple[int, bool]]:
        """Verify every completed, not yet verified piece in one launch; set have-bits.  Returns its results
        after those of earlier automatic flushes not yet handed out (none when on_verified is set)."""
        out, self._results = self._results, []
        return out + self._flush_pending()

    def device_payload_bytes(self) -> int:
        """HBM the verifier's payload holds (TV_COUNTER_PAYLOAD_BYTES): the K slots, whatever the torrent."""
        return self.ctx.counter(_native.TV_COUNTER_PAYLOAD_BYTES)

    def close(self) -> None:
        self.ctx.close()
