#!/usr/bin/env python3
"""Regenerate the committed golden fixtures (data only) under tests/golden/.

* kats.json      FIPS 180-4 / NIST SHA-1 known answers (digests computed with hashlib and
                 checked against the published values listed here).
* refdata.json   recipes that reconstruct the payloads of the reference's own fixtures
                 test_data/singlefile.torrent and test_data/multifile.torrent (copied verbatim
                 into this directory as data).  Found by SURVEY.md 0.4: every digest matches.
* layouts.json   seeded synthetic layouts (multi-file with zero-length / tiny files, pieces
                 spanning files, short final piece, corrupted pieces, missing files) with the
                 expected have-bitfield computed by hashlib (independent of the oracle).
Run:  python3 tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.layouts import LAYOUTS, build_layout  # noqa: E402

PUBLISHED = {  # FIPS 180-2 Appendix A / NIST examples
    "abc": "a9993e364706816aba3e25717850c26c9cd0d89d",
    "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq": "84983e441c3bd26ebaae4aa1f95129e5e54670f1",
    "a*1000000": "34aa973cd4c4daa4f61eeb2bdbad27316534016f",
    "": "da39a3ee5e6b4b0d3255bfef95601890afd80709",
}


def kats():
    out = []
    for name, text, rep in [("empty", "", 1), ("abc", "abc", 1),
                            ("448-bit", "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq", 1),
                            ("million-a", "a", 1000000),
                            ("896-bit", "abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu", 1),
                            ("55-bytes", "x" * 55, 1), ("56-bytes", "x" * 56, 1), ("64-bytes", "x" * 64, 1)]:
        d = hashlib.sha1(text.encode() * rep).hexdigest()
        key = "a*1000000" if name == "million-a" else text
        if key in PUBLISHED:
            assert PUBLISHED[key] == d, name
        out.append({"name": name, "text": text, "repeat": rep, "sha1": d})
    return out


def refdata():
    return {
        "singlefile": {"piece_length": 262144, "n_pieces": 1706, "last_len": 180224,
                       "files": [{"path": "singlefile.txt", "pattern": "0\n", "length": 447135744}]},
        "multifile": {"piece_length": 524288, "n_pieces": 1855, "last_len": 253952,
                      "boundary_pieces": [852],
                      "files": [{"path": "file1.txt", "pattern": "0\n", "length": 447135744},
                                {"path": "dir/file2.txt", "pattern": "7\n", "length": 525148160}]},
    }


def layouts():
    out = []
    for spec in LAYOUTS:
        lay = build_layout(spec)
        P, L = lay["n_pieces"], spec["piece_length"]
        bf = bytearray((P + 7) // 8)
        for i in range(P):
            data = lay["read_piece"](i)
            if data is not None and len(lay["pieces"][i]) == 20 and hashlib.sha1(data).digest() == lay["pieces"][i]:
                bf[i >> 3] |= 0x80 >> (i & 7)
        out.append({"name": spec["name"], "n_pieces": P, "total_length": lay["total_length"],
                    "corrupted": lay["corrupted"], "expected_bitfield": bf.hex(),
                    "pieces_sha1": hashlib.sha1(lay["pieces_raw"]).hexdigest()})
    return out


if __name__ == "__main__":
    for name, fn in [("kats.json", kats), ("refdata.json", refdata), ("layouts.json", layouts)]:
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fn(), f, indent=1)
        print("wrote", name)
