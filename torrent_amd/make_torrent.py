"""Creation mode: a mirror of the reference's tools/make_torrent.ts with the
per-piece SHA-1 (`hashAndStore` -> crypto.subtle.digest, make_torrent.ts:28-31) done on the GPU.

make_torrent(path, tracker, comment=None, creation_date=None) -> bytes of the .torrent, built exactly
as makeTorrent (make_torrent.ts:115-188) builds it:
* piece length 2^clamp(floor(log2(size / 1000)), 15, 20) (make_torrent.ts:17-21) unless given;
* top-level keys in insertion order: announce, comment, created by, creation date, encoding, info
  (bencode.ts writes objects in insertion order, skipping undefined values);
* single file: info = {length, name, piece length, pieces, private: 0};
  directory:   info = {files: [{length, path}], name, piece length, pieces, private: 0};
* the reference quirk of a directory whose total size is below one piece: its only piece is never
  hashed (make_torrent.ts:71,103) and its digest stays 20 zero bytes -- mirrored.
File order for a directory follows collectFiles (make_torrent.ts:35-60): a depth-first walk with an
explicit stack over the directory listing order; `files=` fixes the order explicitly.
"""
from __future__ import annotations

import math
import os
import time
from typing import List, Optional

from .bencode import bencode
from .metainfo import FileInfo, make_info
from .verify import hash_files

CREATED_BY = "https://github.com/rclarey/torrent/blob/master/tools/make_torrent.ts"


def piece_length_for(size: int) -> int:
    """make_torrent.ts:17-21."""
    if size <= 0:
        return 1 << 15
    return 2 ** min(20, max(15, math.floor(math.log2(size / 1000))))


def collect_files(initial_dir: str) -> List[FileInfo]:
    """make_torrent.ts:35-60: stack-based walk; directory entries in listing order."""
    out: List[FileInfo] = []
    dirs = [initial_dir]
    while dirs:
        d = dirs.pop()
        for entry in os.scandir(d):
            p = os.path.join(d, entry.name)
            if entry.is_dir():
                dirs.append(p)
            else:
                out.append(FileInfo(length=os.stat(p).st_size,
                                    path=os.path.relpath(p, initial_dir).split(os.sep)))
    return out


def make_torrent(path: str, tracker: str, comment: Optional[str] = None,
                 creation_date: Optional[int] = None, piece_length: Optional[int] = None,
                 files: Optional[List[FileInfo]] = None, devices=None) -> bytes:
    """makeTorrent(path, tracker, comment) (make_torrent.ts:115-188), digests on the GPU."""
    path = os.path.abspath(path)
    name = os.path.basename(path)
    common = {
        "announce": tracker,
        "comment": comment,
        "created by": CREATED_BY,
        "creation date": int(time.time()) if creation_date is None else creation_date,
        "encoding": "UTF-8",
    }
    if os.path.isdir(path):
        files = collect_files(path) if files is None else files
        size = sum(f.length for f in files)
        L = piece_length or piece_length_for(size)
        n_pieces = -(-size // L)
        geom = make_info(L, bytes(20 * n_pieces), name, files=files)
        if n_pieces == 1 and size < L:
            pieces = bytes(20)                    # never hashed by the reference (quirk)
        else:
            pieces = hash_files(geom, path, devices=devices)
        info = {"files": [{"length": f.length, "path": list(f.path)} for f in files], "name": name,
                "piece length": L, "pieces": pieces, "private": 0}
    else:
        size = os.stat(path).st_size
        L = piece_length or piece_length_for(size)
        n_pieces = -(-size // L)
        geom = make_info(L, bytes(20 * n_pieces), name, length=size)
        pieces = hash_files(geom, os.path.dirname(path), devices=devices)
        info = {"length": size, "name": name, "piece length": L, "pieces": pieces, "private": 0}
    return bencode({**common, "info": info})


def main(argv=None) -> int:
    """CLI of make_torrent.ts:190-250: make_torrent [-c <comment>] -t <tracker url> <target>."""
    import sys
    args = list(sys.argv[1:] if argv is None else argv)
    usage = ("\nmake_torrent\nmake a .torrent file for a given file or directory of files\n\nUSAGE:\n"
             "\tmake_torrent [-c <comment>] -t <tracker url> <target>\n\nOPTIONS:\n"
             "\t--help\t\tPrints this message\n\t-c <comment>\tAdd the provided comment to the .torrent file\n")
    if len(args) not in (3, 5) or "--help" in args:
        print(usage)
        return 0
    comment = tracker = target = None
    i = 0
    while i < len(args):
        if args[i] == "-c" and i + 1 < len(args):
            comment, i = args[i + 1], i + 2
        elif args[i] == "-t" and i + 1 < len(args):
            tracker, i = args[i + 1], i + 2
        elif i == len(args) - 1 and os.path.exists(args[i]):
            target, i = args[i], i + 1
        else:
            print(f'file "{args[i]}" does not exist' if i == len(args) - 1 else usage)
            return 0
    if tracker is None or target is None:
        print(usage)
        return 0
    name = os.path.basename(os.path.abspath(target))
    print(f"making .torrent file for {name}")
    data = make_torrent(target, tracker, comment)
    with open(f"{name}.torrent", "wb") as f:
        f.write(data)
    print(f"output -> {name}.torrent")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
