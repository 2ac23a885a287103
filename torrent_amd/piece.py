"""Piece geometry, mirroring reference piece.ts.

* BLOCK_SIZE = 16 KiB (piece.ts:6).
* piece_length(n, info): `(n === info.pieces.length - 1 && info.length % info.pieceLength)
  || info.pieceLength` (piece.ts:16-19).  The piece count is the DIGEST count, so a torrent
  whose `pieces` string is longer or shorter than ceil(length / pieceLength) keeps the
  reference's behaviour.
* validate_requested_block / validate_received_block raise ValueError with the reference's
  messages (piece.ts:21-65 throw `Error`).
"""
from __future__ import annotations

import json
from dataclasses import dataclass

BLOCK_SIZE = 1024 * 16


@dataclass
class RequestMsg:
    index: int
    offset: int
    length: int


@dataclass
class PieceMsg:
    index: int
    offset: int
    block: bytes


def _stringify(msg) -> str:
    if isinstance(msg, PieceMsg):
        d = {"index": msg.index, "offset": msg.offset, "block": f"[Uint8Array; {len(msg.block)}]"}
    else:
        d = {"index": msg.index, "offset": msg.offset, "length": msg.length}
    return json.dumps(d, separators=(",", ":"))


def piece_length(n: int, info) -> int:
    """piece.ts:16-19."""
    if n == info.n_pieces - 1 and info.length % info.piece_length:
        return info.length % info.piece_length
    return info.piece_length


def piece_offset(n: int, info) -> int:
    """Linear byte offset of piece n in the concatenated file space (torrent.ts:165,186)."""
    return n * info.piece_length


def validate_requested_block(info, msg: RequestMsg) -> None:
    """piece.ts:21-37."""
    if msg.index >= info.n_pieces:
        raise ValueError(f"request message with invalid piece index {_stringify(msg)}")
    req_end = msg.offset + msg.length
    last_len = piece_length(info.n_pieces - 1, info)
    if (msg.index == info.n_pieces - 1 and req_end > last_len) or req_end > info.piece_length:
        raise ValueError(f"request message with invalid block length {_stringify(msg)}")


def validate_received_block(info, msg: PieceMsg) -> None:
    """piece.ts:39-65."""
    if msg.index >= info.n_pieces:
        raise ValueError(f"piece message with invalid piece index {_stringify(msg)}")
    if msg.offset % BLOCK_SIZE != 0:
        raise ValueError(f"piece message with invalid block offset {_stringify(msg)}")
    plen = piece_length(msg.index, info)
    num_blocks = -(-plen // BLOCK_SIZE)
    n_block = msg.offset // BLOCK_SIZE
    if msg.index == info.n_pieces - 1 and n_block == num_blocks - 1:
        last_block = plen % BLOCK_SIZE or BLOCK_SIZE
        if len(msg.block) != last_block:
            raise ValueError(f"piece message with invalid last block length {_stringify(msg)}")
    elif len(msg.block) != BLOCK_SIZE:
        raise ValueError(f"piece message with invalid block length {_stringify(msg)}")
