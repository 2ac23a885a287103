"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle on the same seeded inputs.

Bar: bit-exact digests and bitfields.  Oracle = oracle/sha1_oracle.c (pinned against the
reference's test_data digests in tests/test_oracle.py).
"""
import hashlib
import random

import pytest

pytestmark = pytest.mark.gpu

# lane (3-deep ring of single-block loads), split, twin, and 101 = the lane kernel with pair loads (TV_OPT_LANE_PAIRS:
# the auto rule picks pairs only at >= 256 x CUs pieces, so both lane forms are forced here)
KERNELS = [1, 2, 4, 101]


def _ctx(native, kernel=0):
    c = native.Context(0)
    c.set_option(native.TV_OPT_KERNEL, 1 if kernel == 101 else kernel)
    if kernel in (1, 101):
        c.set_option(native.TV_OPT_LANE_PAIRS, 1 if kernel == 101 else 2)
    return c


@pytest.mark.parametrize("kernel", KERNELS)
def test_hash_lengths_all_tail_cases(native, oracle, kernel):
    """One piece per length: every len % 64 residue near the padding edges, 0..300 bytes, and
    multi-block pieces.  Digest must equal hashlib / oracle."""
    lengths = list(range(1, 140)) + [183, 191, 192, 255, 256, 257, 1000, 4095, 4096, 4097, 65536 + 55]
    with _ctx(native, kernel) as ctx:
        for n in lengths:
            data = oracle.synth_fill(n + 1, 0, n)
            ctx.set_layout(n, max(n, 1), 1)
            ctx.stage(0, data)
            got = ctx.hash()
            assert got == hashlib.sha1(bytes(data)).digest(), n


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("L,P,last", [(4096, 300, 4096), (4096, 300, 1), (16384, 129, 9000),
                                      (65536, 64, 65536 - 9), (1 << 20, 70, 123457), (64, 1000, 55),
                                      # the short last piece's dedicated group at every boundary: alone
                                      # (no main group), right after a full wave / split workgroup /
                                      # 256-thread lane workgroup, and sharing an output word
                                      (16384, 1, 1000), (4096, 2, 17), (4096, 65, 100), (4096, 129, 4095),
                                      (4096, 257, 3), (4096, 200, 2048)])
def test_verify_matches_oracle(native, oracle, kernel, L, P, last):
    total = L * (P - 1) + last
    payload = oracle.synth_fill(L + P, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    rng = random.Random(L * 7 + P)
    # corrupt ~3% of pieces: payload bit flips and digest bit flips, always incl. first and last
    bad = sorted(set([0, P - 1] + rng.sample(range(P), max(1, P // 33))))
    for i in bad:
        if rng.random() < 0.5:
            n = last if i == P - 1 else L
            payload[i * L + rng.randrange(n)] ^= 1 << rng.randrange(8)
        else:
            pieces[20 * i + rng.randrange(20)] ^= 1 << rng.randrange(8)
    expect = oracle.verify_linear(payload, total, L, bytes(pieces))
    with _ctx(native, kernel) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload)
        got = ctx.verify()
        assert got == expect
        # hash mode agrees with the oracle on the corrupted payload
        assert ctx.hash() == oracle.hash_pieces(payload, total, L, P)
    for i in bad:
        assert not (got[i >> 3] >> (7 - (i & 7))) & 1


def test_kernels_agree_and_avail_mask(native, oracle):
    L, P = 8192, 515
    total = L * (P - 1) + 77
    payload = oracle.synth_fill(99, 0, total)
    pieces = oracle.hash_pieces(payload, total, L, P)
    rng = random.Random(3)
    avail = bytearray(rng.randrange(256) for _ in range((P + 7) // 8))
    expect = oracle.verify_linear(payload, total, L, pieces, bytes(avail))
    outs = []
    # + 2 pairs per workgroup (split, twin), the twin SIMD-placement probe shapes, twin CU-packed (pack 1),
    # twin without companion workgroups (pack 2) and with companions reading all 32 pieces (pack 3)
    for k, pairs, pack in [(k, 0, 0) for k in KERNELS] + [(2, 2, 0), (4, 2, 0), (4, 3, 0), (4, 4, 0), (4, 5, 0),
                                                          (4, 0, 1), (4, 0, 2), (4, 0, 3)]:
        with _ctx(native, k) as ctx:
            ctx.set_option(native.TV_OPT_SPLIT_PAIRS, pairs)
            ctx.set_option(native.TV_OPT_TWIN_PACK, pack & 1 if pack != 3 else 0)
            ctx.set_option(native.TV_OPT_TWIN_FILL, 0 if pack == 2 else 1)
            ctx.set_option(native.TV_OPT_TWIN_FILL_READS, 1 if pack == 3 else 0)
            ctx.set_layout(total, L, P)
            ctx.set_digests(pieces)
            ctx.stage(0, payload)
            outs.append(ctx.verify(bytes(avail)))
            assert ctx.hash() == pieces, (k, pairs, pack)
    assert all(o == expect for o in outs)


def test_ragged_digest_string_and_extra_pieces(native, oracle):
    """pieces.byteLength % 20 != 0 -> the short final slice never matches (_bytes.ts:94-96);
    more digests than ceil(length/L) -> the extra pieces are unreadable (bit 0)."""
    L = 4096
    total = 10 * L
    payload = oracle.synth_fill(5, 0, total)
    good = oracle.hash_pieces(payload, total, L, 10)
    # ragged: 9 full digests + 7 bytes of the 10th
    ragged = good[:9 * 20 + 7]
    with _ctx(native) as ctx:
        ctx.set_layout(total, L, 10)
        ctx.set_digests(ragged)
        ctx.stage(0, payload)
        got = ctx.verify()
    assert got == oracle.verify_linear(payload, total, L, ragged) == bytes([0xFF, 0x80])
    # 12 digests for 10 pieces of data: pieces 10, 11 unreadable; piece 11 is the "last" piece
    extra = good + hashlib.sha1(b"x").digest() * 2
    with _ctx(native) as ctx:
        ctx.set_layout(total, L, 12)
        ctx.set_digests(extra)
        ctx.stage(0, payload)
        got = ctx.verify()
    assert got == oracle.verify_linear(payload, total, L, extra) == bytes([0xFF, 0xC0])


@pytest.mark.parametrize("kernel", KERNELS)
def test_shards_concatenate(native, oracle, kernel):
    """Sharded verification (the multi-GPU decomposition, run here shard by shard on one GPU)
    concatenates to the single-shard bitfield."""
    from torrent_amd.verify import shard_ranges
    L, P = 2048, 1003
    total = L * (P - 1) + 5
    payload = oracle.synth_fill(17, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    for i in range(0, P, 37):
        pieces[20 * i] ^= 0xFF
    expect = oracle.verify_linear(payload, total, L, bytes(pieces))
    out = bytearray((P + 7) // 8)
    for first, count in shard_ranges(P, 8):
        with _ctx(native, kernel) as ctx:
            ctx.set_layout(total, L, P, first, count)
            ctx.set_digests(bytes(pieces))
            ctx.stage(0, payload)  # bytes outside the shard are ignored
            sl = ctx.verify()
        out[first // 8:first // 8 + len(sl)] = sl
    assert bytes(out) == expect


@pytest.mark.parametrize("L", [65536, 65539])      # 65,539: no row of the 2D column copies is dword-aligned
@pytest.mark.parametrize("chunk", [0, 64, 4096, 65536])
@pytest.mark.parametrize("kernel", KERNELS)
def test_stream_from_host_matches(native, oracle, chunk, kernel, L):
    P = 97
    total = L * (P - 1) + 4321
    payload = oracle.synth_fill(23, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    payload[3 * L + 100] ^= 0x10
    pieces[20 * 50 + 3] ^= 0x01
    expect = oracle.verify_linear(payload, total, L, bytes(pieces))
    with _ctx(native, kernel) as ctx:
        ctx.set_option(native.TV_OPT_STREAM_CHUNK, chunk)
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        assert ctx.verify_host(payload) == expect
        # truncated source: pieces whose bytes extend past the end are unreadable
        cut = 40 * L + 5
        avail = bytearray((P + 7) // 8)
        for i in range(P):
            n = 4321 if i == P - 1 else L
            if i * L + n <= cut:
                avail[i >> 3] |= 0x80 >> (i & 7)
        assert ctx.verify_host(memoryview(payload)[:cut]) == oracle.verify_linear(
            payload, total, L, bytes(pieces), bytes(avail))
        # page-locked source: 2D column copies straight from it (src pitch L)
        hb = native.PinnedBuffer(total)
        try:
            hb.mv[:] = payload
            assert ctx.verify_host(hb.mv) == expect
        finally:
            hb.close()


def test_fill_synthetic_matches_oracle(native, oracle):
    L, P = 4096, 40
    total = L * P
    with _ctx(native) as ctx:
        ctx.set_layout(total, L, P, 8, 16)
        ctx.fill_synthetic(77)
        got = ctx.hash()
    assert got == oracle.synth_piece_digests(77, total, L, P, 8, 16)


def _bits(bf, P):
    return [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("L,P,last", [
    (1, 100, 1),                         # one-byte pieces: every piece is a single padded block
    (100, 1000, 37),                     # piece length not a multiple of 64, 2-block pieces
    (1000, 333, 999),                    # odd length, short last piece one byte shorter
    (16 << 20, 5, (16 << 20) - 3),       # large pieces (16 MiB; 262,144 blocks each)
    (96 << 20, 2, (5 << 20) + 1),        # pieces larger than a 64 MiB staging-ring slot (chunked stage)
])
def test_edge_geometries(native, oracle, kernel, L, P, last):
    """Extreme piece geometries: tiny, unaligned and very large pieces.  Verify, hash and the
    incremental list kernel all equal the oracle; corrupted pieces (first, last, one inside) fail."""
    total = L * (P - 1) + last
    payload = oracle.synth_fill(L ^ P, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P, threads=8))
    bad = sorted({0, P // 2, P - 1})
    for i in bad:
        pieces[20 * i + 19] ^= 0x80
    expect = oracle.verify_linear(payload, total, L, bytes(pieces))
    assert [i for i, b in enumerate(_bits(expect, P)) if not b] == bad
    with _ctx(native, kernel) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload)
        assert ctx.verify() == expect
        assert ctx.hash() == oracle.hash_pieces(payload, total, L, P, threads=8)
        order = list(range(P))[::-1]
        assert list(ctx.verify_list(order)) == [_bits(expect, P)[i] for i in order]


def test_empty_and_zero_length_torrents(native, oracle):
    """P = 0 (an empty `pieces` string): empty bitfield, no digests (torrent.ts:60 allocates
    ceil(0/8) bytes).  length 0 with one digest: piece 0 has length L (piece.ts:16-19: 0 % L is
    falsy) and lies past the end of the data, so it is unreadable -> bit 0 (storage.ts:130-136)."""
    with _ctx(native) as ctx:
        ctx.set_layout(0, 16384, 0)
        ctx.set_digests(b"")
        assert ctx.verify() == b""
        assert ctx.hash() == b""
        assert ctx.verify_host(b"") == b""
    empty_digest = hashlib.sha1(b"").digest()
    expect = oracle.verify_linear(b"", 0, 16384, empty_digest)
    assert expect == b"\x00"
    for k in KERNELS:
        with _ctx(native, k) as ctx:
            ctx.set_layout(0, 16384, 1)
            ctx.set_digests(empty_digest)
            assert ctx.verify() == expect
            assert ctx.verify_host(b"") == expect


def test_geometry_that_overflows_offsets_is_rejected(native):
    """Piece offsets i*L and digest offsets 20*i are 64-bit: a geometry whose offsets would wrap is an
    argument error (thrown, like piece.ts:22-64's validation), not a silent wrong read.  The context
    stays usable afterwards."""
    with _ctx(native) as ctx:
        for total, L, P, first, count in [
            (0, 1 << 30, (1 << 34) + 8, (1 << 34), 8),    # i*L wraps past 2^64
            (0, 64, (1 << 62), (1 << 62) - 8, 8),         # 20*i wraps
            (0, 1 << 36, 1 << 30, 0, (1 << 30) - 8),      # 2^30 pieces of 64 GiB: offsets and shard bytes wrap
        ]:
            with pytest.raises(native.NativeError, match="overflows"):
                ctx.set_layout(total, L, P, first, count)
        ctx.set_layout(100, 64, 2)
        ctx.set_digests(hashlib.sha1(bytes(64)).digest() + hashlib.sha1(bytes(36)).digest())
        ctx.stage(0, bytes(100))
        assert ctx.verify() == b"\xc0"


@pytest.mark.parametrize("L,P,last", [(4096, 1, 4096), (4096, 1, 1000), (8192, 40, 8192), (8192, 40, 77),
                                      (65536, 33, 65536), (1 << 20, 20, 5)])
def test_twin_companions_exact(native, oracle, L, P, last):
    """Twin companion workgroups (TV_OPT_TWIN_FILL, default on) re-hash main pieces and must write nothing:
    with a handful of pieces nearly the whole 2 x CUs grid is companions.  Verify (corrupted digests, an
    availability mask), creation mode and the list path equal the oracle with companions on and off, reading
    one piece or all 32 of the workgroup they copy."""
    total = L * (P - 1) + last
    payload = oracle.synth_fill(P * 7 + 1, 0, total)
    good = oracle.hash_pieces(payload, total, L, P)
    pieces = bytearray(good)
    bad = {0, P // 2, P - 1}
    for i in bad:
        pieces[20 * i + 3] ^= 0x20
    avail = bytearray(b"\xff" * ((P + 7) // 8))
    if P > 2:
        avail[0] &= 0xBF                       # piece 1 unavailable
    expect = oracle.verify_linear(payload, total, L, bytes(pieces), bytes(avail))
    lst = [P - 1, 0, P // 2, P - 1] + list(range(P))
    # companions on (1; 2 also on short lists), with either read mode, and off
    for fill, reads in [(1, 0), (1, 1), (2, 0), (2, 1), (0, 0)]:
        with _ctx(native, 4) as ctx:
            ctx.set_option(native.TV_OPT_TWIN_FILL, fill)
            ctx.set_option(native.TV_OPT_TWIN_FILL_READS, reads)
            ctx.set_layout(total, L, P)
            ctx.stage(0, payload)
            assert ctx.hash() == good, fill
            ctx.set_digests(bytes(pieces))
            assert ctx.verify(bytes(avail)) == expect, fill
            assert ctx.last_kernel()[0] == 4
            assert list(ctx.verify_list(lst)) == [0 if i in bad else 1 for i in lst], fill
