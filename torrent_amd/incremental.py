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
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from . import _native
from .metainfo import InfoDict
from .piece import BLOCK_SIZE, PieceMsg, piece_length, validate_received_block


class IncrementalVerifier:
    def __init__(self, info: InfoDict, storage=None, device: int = 0,
                 shard: Optional[Tuple[int, int]] = None):
        self.info = info
        self.storage = storage
        P = info.n_pieces
        self.first, self.count = shard if shard is not None else (0, P)
        self.ctx = _native.Context(device)
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
        if len(blocks) == self._blocks_in(i):
            self.ctx.stage(i * self.info.piece_length, buf)
            del self._bufs[i], self._have_blocks[i]
            self._pending.append(i)
            self._pending_set.add(i)
            return True
        return False

    def flush(self) -> List[Tuple[int, bool]]:
        """Verify every completed, not yet verified piece in one launch; set have-bits."""
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

    def close(self) -> None:
        self.ctx.close()
