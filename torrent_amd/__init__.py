"""torrent_amd -- MI355X-native piece verification for rclarey/torrent.

The hot path (bulk SHA-1 of every piece against info.pieces -> have-bitfield) runs in
libtorrent_verify.so (hand-written HIP for gfx950, C ABI in include/torrent_verify.h).
This package is the host-side mirror of the reference's piece/storage/metainfo API
(piece.ts, storage.ts, metainfo.ts) plus the new verify module.
"""
from .bencode import bdecode, bencode  # noqa: F401
from .metainfo import FileInfo, InfoDict, Metainfo, make_info, parse_metainfo, partition  # noqa: F401
from .piece import BLOCK_SIZE, piece_length, validate_received_block, validate_requested_block  # noqa: F401
from .storage import FsStorage, MemoryStorage, Storage, fs_storage  # noqa: F401
from .verify import (context_counters, hash_files, hash_pieces, release_contexts, shard_ranges,  # noqa: F401
                     verify_files, verify_payload, verify_piece, verify_piece_async, verify_pieces,
                     verify_pieces_async, verify_stream)
from .incremental import IncrementalVerifier  # noqa: F401
from .make_torrent import make_torrent  # noqa: F401

__all__ = [
    "bdecode", "bencode", "FileInfo", "InfoDict", "Metainfo", "make_info", "parse_metainfo", "partition",
    "BLOCK_SIZE", "piece_length", "validate_received_block", "validate_requested_block",
    "FsStorage", "MemoryStorage", "Storage", "fs_storage",
    "hash_pieces", "shard_ranges", "verify_files", "verify_payload", "verify_piece", "verify_piece_async",
    "verify_pieces", "verify_pieces_async", "verify_stream", "release_contexts", "context_counters", "hash_files",
    "IncrementalVerifier", "make_torrent",
]
