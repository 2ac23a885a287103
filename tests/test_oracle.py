"""Pin the CPU oracle against the reference's own golden vectors.

* FIPS 180-4 known answers (and hashlib, an independent SHA-1).
* The reference fixtures test_data/singlefile.torrent and multifile.torrent were produced by
  the reference's SHA-1 path (tools/make_torrent.ts:28-31; `created by` pinned at
  metainfo_test.ts:21,43).  Their payloads are reconstructed from tests/golden/refdata.json
  and EVERY digest (1706 + 1855) must match -- including the short final pieces and the
  multi-file piece #852 that spans file1.txt -> dir/file2.txt.
"""
import hashlib
import json
import os

import pytest

from torrent_amd.metainfo import parse_metainfo

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


def _refdata():
    with open(os.path.join(GOLDEN, "refdata.json")) as f:
        return json.load(f)


def _payload(files):
    return b"".join(f["pattern"].encode() * (f["length"] // len(f["pattern"])) for f in files)


@pytest.fixture(params=["scalar", "sha-ni"])
def impl(request, oracle):
    """Run a test under each compression of the oracle: the scalar FIPS restatement and the
    SHA-NI path the bench's cpu_baseline uses."""
    if not oracle.set_impl(request.param):
        pytest.skip(f"host lacks {request.param}")
    yield request.param
    oracle.set_impl("best")


def test_fips_kats(oracle, impl):
    kats = json.loads(_load("kats.json"))
    assert len(kats) >= 5
    for k in kats:
        msg = k["text"].encode() * k["repeat"]
        assert oracle.sha1(msg).hex() == k["sha1"], k["name"]
        assert hashlib.sha1(msg).hexdigest() == k["sha1"]


def test_oracle_vs_hashlib_random(oracle, impl):
    import random
    rng = random.Random(0)
    for n in list(range(0, 200)) + [1000, 4095, 4096, 65537]:
        m = bytes(rng.randrange(256) for _ in range(n))
        assert oracle.sha1(m) == hashlib.sha1(m).digest()


@pytest.mark.parametrize("name", ["singlefile", "multifile"])
def test_reference_fixture_digests(oracle, impl, name):
    """All digests of the reference's own .torrent fixtures reproduce from the reconstructed
    payload (parity with the reference's SHA-1 path is pinned here)."""
    meta = parse_metainfo(_load(f"{name}.torrent"))
    info = meta.info
    rd = _refdata()[name]
    files = rd["files"]
    if info.files is None:
        assert len(files) == 1 and files[0]["length"] == info.length
    else:
        assert [f.length for f in info.files] == [f["length"] for f in files]
        assert ["/".join(f.path) for f in info.files] == [f["path"] for f in files]
    payload = _payload(files)
    assert len(payload) == info.length
    P, L = info.n_pieces, info.piece_length
    assert P == rd["n_pieces"] and L == rd["piece_length"]
    got = oracle.hash_pieces(payload, info.length, L, P, threads=8)
    assert got == info.pieces_raw  # every digest, in order
    # the bitfield path: all ones, spare bits 0
    bf = oracle.verify_linear(payload, info.length, L, info.pieces_raw)
    assert bf == bytes([0xFF] * (P // 8) + ([(0xFF00 >> (P % 8)) & 0xFF] if P % 8 else []))
    # spot-check with hashlib, including the short last piece and (multifile) the boundary piece
    for i in [0, P // 2, P - 1] + rd.get("boundary_pieces", []):
        n = oracle.piece_len(i, P, info.length, L)
        assert n == rd["last_len"] if i == P - 1 else n == L
        assert hashlib.sha1(payload[i * L:i * L + n]).digest() == info.pieces[i]


def test_reference_fixture_corruptions(oracle):
    """Flip-variants of the singlefile fixture: a flipped payload bit clears exactly that
    piece's bit (piece 0, a middle piece, and the short last piece)."""
    meta = parse_metainfo(_load("singlefile.torrent"))
    info = meta.info
    payload = bytearray(_payload(_refdata()["singlefile"]["files"]))
    P, L = info.n_pieces, info.piece_length
    flips = [0, 852, P - 1]
    for i in flips:
        payload[i * L + 7] ^= 0x20
    bf = oracle.verify_linear(payload, info.length, L, info.pieces_raw)
    for i in range(P):
        bit = (bf[i >> 3] >> (7 - (i & 7))) & 1
        assert bit == (0 if i in flips else 1), i


def test_piece_len_rule(oracle):
    # piece.ts:16-19 uses the DIGEST count, not ceil(length / pieceLength)
    assert oracle.piece_len(9, 10, 10 * 4096, 4096) == 4096
    assert oracle.piece_len(9, 10, 9 * 4096 + 5, 4096) == 5
    assert oracle.piece_len(3, 10, 9 * 4096 + 5, 4096) == 4096
    assert oracle.piece_len(11, 12, 10 * 4096 + 3, 4096) == 3


def test_synthetic_generator_definition(oracle):
    """byte(o) = byte (o & 7) of splitmix64(seed, o >> 3): check against a Python restatement."""
    def splitmix(seed, idx):
        m = (1 << 64) - 1
        z = (seed + (idx + 1) * 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        return z ^ (z >> 31)
    got = oracle.synth_fill(42, 13, 50)
    exp = bytes((splitmix(42, o >> 3) >> (8 * (o & 7))) & 0xFF for o in range(13, 63))
    assert bytes(got) == exp
    d = oracle.synth_piece_digests(42, 10000, 4096, 3, threads=2)
    full = oracle.synth_fill(42, 0, 10000)
    assert d == b"".join(hashlib.sha1(bytes(full[i:i + 4096])).digest() for i in range(0, 10000, 4096))


def test_numpy_generator_equals_the_oracles(oracle):
    """tests/synth.py (the numpy generator and hashlib digests the tools and bench.py generate inputs with, so they
    call nothing under oracle/) gives the oracle's bytes at aligned and unaligned offsets, across its 16 MiB
    chunks and threads, and the oracle's piece digests."""
    import random
    from tests import synth
    rng = random.Random(5)
    for seed in (0, 3, 2**64 - 1, 12345678901234567):
        for off, n in [(0, 0), (0, 1), (7, 9), (13, 50), (8, 64), (rng.randrange(1 << 40), rng.randrange(1, 5000))]:
            assert bytes(synth.fill(seed, off, n)) == bytes(oracle.synth_fill(seed, off, n)), (seed, off, n)
    big = (16 << 20) * 2 + 12345
    assert bytes(synth.fill(9, 5, big, threads=4)) == bytes(oracle.synth_fill(9, 5, big))
    assert synth.piece_digests(42, 10000, 4096, 3, threads=2) == oracle.synth_piece_digests(42, 10000, 4096, 3)
    buf = oracle.synth_fill(7, 0, 70000)
    assert synth.hash_pieces(buf, 16384, 5) == oracle.hash_pieces(buf, 70000, 16384, 5)
