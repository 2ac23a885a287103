"""Metainfo parsing and digest unpacking, mirroring reference metainfo.ts.

`parse_metainfo(bytes) -> Metainfo | None` follows metainfo.ts:100-148: bdecode, validate,
then `pieces = partition(info.pieces, 20)` (metainfo.ts:111, _bytes.ts:92-99), multi-file
`length = sum(file lengths)` (metainfo.ts:125).  Any error returns None (metainfo.ts:145-147).

For the GPU path the digests are also kept as the contiguous raw byte string (`pieces_raw`),
exactly the buffer the `partition` views point into; that is what crosses the C ABI.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import List, Optional

from .bencode import bdecode, bencode


@dataclass
class FileInfo:
    """metainfo.ts:29-34 MultiFileFields."""
    length: int
    path: List[str]


@dataclass
class InfoDict:
    """metainfo.ts:12-44.  `files` is None for a single-file torrent."""
    piece_length: int
    pieces: List[bytes]
    private: int
    name: str
    length: int
    files: Optional[List[FileInfo]] = None
    pieces_raw: bytes = field(default=b"", repr=False)

    @property
    def n_pieces(self) -> int:
        return len(self.pieces)

    @property
    def is_multi_file(self) -> bool:
        return self.files is not None


@dataclass
class Metainfo:
    info_hash: bytes
    info: InfoDict
    announce: str
    creation_date: Optional[int] = None
    comment: Optional[str] = None
    created_by: Optional[str] = None
    encoding: Optional[str] = None


def partition(arr: bytes, n: int) -> List[bytes]:
    """_bytes.ts:92-99: consecutive n-byte slices; the final slice may be short."""
    return [arr[i:i + n] for i in range(0, len(arr), n)]


def _is_bytes(x) -> bool:
    return isinstance(x, (bytes, bytearray, memoryview))


def _valid_info(info) -> bool:
    # metainfo.ts:62-81 (validateSingleFileInfo / validateMultiFileInfo)
    if not isinstance(info, dict):
        return False
    if not isinstance(info.get("piece length"), int) or not _is_bytes(info.get("pieces")):
        return False
    if "private" in info and not isinstance(info["private"], int):
        return False
    if not _is_bytes(info.get("name")):
        return False
    if isinstance(info.get("length"), int):
        return True
    files = info.get("files")
    if not isinstance(files, list):
        return False
    for f in files:
        if not isinstance(f, dict) or not isinstance(f.get("length"), int):
            return False
        p = f.get("path")
        if not isinstance(p, list) or not all(_is_bytes(x) for x in p):
            return False
    return True


def _valid_metainfo(d) -> bool:
    # metainfo.ts:83-90
    if not isinstance(d, dict) or not _valid_info(d.get("info")) or not _is_bytes(d.get("announce")):
        return False
    if "creation date" in d and not isinstance(d["creation date"], int):
        return False
    for k in ("comment", "created by", "encoding"):
        if k in d and not _is_bytes(d[k]):
            return False
    return True


def _text(b) -> str:
    return bytes(b).decode("utf-8", "replace")


def info_from_decoded(info: dict) -> InfoDict:
    pieces_raw = bytes(info["pieces"])
    common = dict(
        piece_length=info["piece length"],
        pieces=partition(pieces_raw, 20),
        private=1 if info.get("private") == 1 else 0,
        name=_text(info["name"]),
        pieces_raw=pieces_raw,
    )
    if "files" in info:
        files = [FileInfo(length=f["length"], path=[_text(x) for x in f["path"]]) for f in info["files"]]
        return InfoDict(files=files, length=sum(f.length for f in files), **common)
    return InfoDict(length=info["length"], **common)


def parse_metainfo(data: bytes) -> Optional[Metainfo]:
    """metainfo.ts:100-148.  Returns None on any parse/validation error."""
    try:
        decoded = bdecode(data)
        if not _valid_metainfo(decoded):
            return None
        info = info_from_decoded(decoded["info"])
        return Metainfo(
            announce=_text(decoded["announce"]),
            creation_date=decoded.get("creation date"),
            comment=_text(decoded["comment"]) if "comment" in decoded else None,
            created_by=_text(decoded["created by"]) if "created by" in decoded else None,
            encoding=_text(decoded["encoding"]) if "encoding" in decoded else None,
            info=info,
            # metainfo.ts:141-143: SHA-1 of the re-bencoded info dict.  One serial hash
            # per torrent: stays on the host.
            info_hash=hashlib.sha1(bencode(decoded["info"])).digest(),
        )
    except Exception:
        return None


def make_info(piece_length: int, pieces_raw: bytes, name: str, length: int | None = None,
              files: Optional[List[FileInfo]] = None, private: int = 0) -> InfoDict:
    """Build an InfoDict directly (synthetic layouts, tests)."""
    if files is not None:
        length = sum(f.length for f in files)
    return InfoDict(piece_length=piece_length, pieces=partition(pieces_raw, 20), private=private,
                    name=name, length=int(length or 0), files=files, pieces_raw=bytes(pieces_raw))


def encode_metainfo(info: InfoDict, announce: str = "http://example.com/announce",
                    comment: str | None = None, created_by: str | None = None) -> bytes:
    """Write a .torrent with an explicit piece length (make_torrent.ts cannot: its piece length
    is forced by make_torrent.ts:17-21)."""
    d: dict = {"announce": announce, "comment": comment, "created by": created_by, "encoding": "UTF-8"}
    if info.files is not None:
        d["info"] = {"files": [{"length": f.length, "path": list(f.path)} for f in info.files],
                     "name": info.name, "piece length": info.piece_length,
                     "pieces": info.pieces_raw, "private": info.private}
    else:
        d["info"] = {"length": info.length, "name": info.name, "piece length": info.piece_length,
                     "pieces": info.pieces_raw, "private": info.private}
    return bencode(d)
