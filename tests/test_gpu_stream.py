"""GPU parity of the streamed verify (tv_stream_*: the bounded pinned ring of BASELINE config 5) against the
CPU oracle.  The resume flow it serves: Client.add -> Storage -> bitfield -> sendBitfield
(reference client.ts:53-67, torrent.ts:56-60,101); the digest is make_torrent.ts:28-31's SHA-1.

Bar: bit-exact bitfields.  Geometry: 4 MiB pieces (cfg5's L) with a short last piece, several columns and
several ring requests per column, page-locked and pageable sources, the caller-filled slot, the library's
host generator, unreadable pieces, concurrent contexts, and the state machine's error paths."""
import threading

import pytest

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _bits(bf, n):
    return [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(n)]


def _column(L, count, chunk):
    """The library's column width (tv_stream.hip stream_column): TV_OPT_STREAM_CHUNK, or the widest power of
    two from 64 KiB up to L whose column of every piece stays <= 512 MiB; at most one 64 MiB slot."""
    C = chunk
    if not C:
        C = 64 << 10
        while C * 2 <= L and C * 2 * count <= 512 * MiB:
            C *= 2
    C = min(C // 64 * 64, -(-L // 64) * 64)
    return max(64, min(C, 64 * MiB))


def _stream(native, ctx, fill, avail=None, unreadable=()):
    """Drive one stream: fill(req) fills or commits each request; returns (bitfield, requests)."""
    ctx.stream_begin(avail)
    reqs = 0
    while True:
        req = ctx.stream_next()
        if not req.rows:
            break
        for i in unreadable:
            if req.piece <= i < req.piece + req.rows and req.offset == 0:
                ctx.stream_unreadable(i)
        fill(req)
        reqs += 1
    return ctx.stream_end(), reqs


@pytest.fixture(scope="module")
def cfg5_small(oracle):
    """65 pieces of 4 MiB (the last one 1 MiB + 13 bytes), synthetic payload, 3 corrupted digests and 2
    corrupted payload bytes; expected bitfield from the oracle."""
    L, P = 4 * MiB, 65
    total = L * (P - 1) + MiB + 13
    payload = oracle.synth_fill(5, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P, threads=8))
    for i in (0, 31, P - 1):
        pieces[20 * i + 7] ^= 0x20
    payload[17 * L + 4 * MiB - 1] ^= 0x01          # last byte of piece 17
    payload[(P - 1) * L + MiB + 12] ^= 0x80         # last byte of the short last piece (digest already bad)
    payload[40 * L] ^= 0x02                         # first byte of piece 40
    expect = oracle.verify_linear(payload, total, L, bytes(pieces))
    assert [i for i, b in enumerate(_bits(expect, P)) if not b] == [0, 17, 31, 40, P - 1]
    return dict(L=L, P=P, total=total, payload=payload, pieces=bytes(pieces), expect=expect)


@pytest.mark.parametrize("chunk", [0, MiB, 3 * 65536])   # auto (one 4 MiB column, 16-row requests), 4 and 22 columns
@pytest.mark.parametrize("source", ["slot", "pageable", "pinned"])
def test_stream_4mib_pieces(native, oracle, cfg5_small, source, chunk):
    """Rows filled by the caller into the lent pinned slot, copied from pageable memory, or DMA'd straight
    from a page-locked buffer (tv_stream_commit_from, src pitch L): the bitfield equals the oracle's."""
    d = cfg5_small
    L, P, total, payload = d["L"], d["P"], d["total"], d["payload"]
    pb = None
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_RESIDENT, 0)
        ctx.set_option(native.TV_OPT_STREAM_CHUNK, chunk)
        ctx.set_layout(total, L, P)
        ctx.set_digests(d["pieces"])
        if source == "pinned":
            pb = native.PinnedBuffer(total)
            pb.mv[:] = payload
        src = pb.mv if pb is not None else payload

        def fill(req):
            base = req.piece * L + req.offset
            if source == "slot":
                slot = ctx.stream_slot(req)
                for q in range(req.rows):
                    n = ctx.row_bytes(req, q)
                    slot[q * req.width:q * req.width + n] = payload[base + q * L:base + q * L + n]
                slot.release()
                ctx.stream_commit(req)
            else:
                ctx.stream_commit_from(req, src, L, base)

        try:
            bf, reqs = _stream(native, ctx, fill)
            assert bf == d["expect"]
            kernel, launches = ctx.last_kernel()
            C = _column(L, P, chunk)
            assert launches == -(-L // C)
            assert reqs == launches * -(-P // max(1, (64 * MiB) // C))
            with pytest.raises(native.NativeError, match="TV_OPT_RESIDENT"):
                ctx.verify()                              # no resident payload in a streamed-only ctx
        finally:
            if pb is not None:
                pb.close()


def test_stream_generated_and_unreadable(native, oracle):
    """The library's host generator fills the slots (tv_stream_fill_synthetic = tv_fill_synthetic's bytes):
    with the oracle's digests every piece verifies except corrupted digests, pieces reported unreadable
    (Storage.get -> null) and pieces masked by the caller's avail bits."""
    L, P = 4 * MiB, 70
    total = L * (P - 1) + 3 * MiB
    dig = bytearray(oracle.synth_piece_digests(8, total, L, P, threads=8))
    bad = {2, 65}
    for i in bad:
        dig[20 * i + 19] ^= 1
    avail = bytearray(b"\xff" * ((P + 7) // 8))
    avail[1] &= 0xEF                                  # piece 11 masked
    avail[-1] &= (0xFF00 >> (P % 8)) & 0xFF
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_RESIDENT, 0)
        ctx.set_option(native.TV_OPT_STREAM_CHUNK, 2 * MiB)
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(dig))

        def fill(req):
            ctx.stream_fill_synthetic(req, 8)
            ctx.stream_commit(req)

        bf, _ = _stream(native, ctx, fill, avail=bytes(avail), unreadable=(0, 33, P - 1))
    zeros = {i for i, b in enumerate(_bits(bf, P)) if not b}
    assert zeros == bad | {11, 0, 33, P - 1}


def test_stream_shards_on_concurrent_contexts(native, oracle):
    """Four contexts streaming four shards at once from four host threads (the per-GPU producers of an
    N-GPU resume check, here all on GPU 0): the concatenated slices equal the oracle's bitfield."""
    from torrent_amd.verify import shard_ranges
    L, P = MiB, 203
    total = L * (P - 1) + 777
    dig = bytearray(oracle.synth_piece_digests(12, total, L, P, threads=8))
    for i in range(0, P, 29):
        dig[20 * i] ^= 0x40
    expect = bytearray((P + 7) // 8)
    for i in range(P):
        if i % 29:
            expect[i >> 3] |= 0x80 >> (i & 7)
    ranges = shard_ranges(P, 4)
    out = [None] * 4
    errs = []

    def run(s, first, count):
        try:
            with native.Context(0) as ctx:
                ctx.set_option(native.TV_OPT_RESIDENT, 0)
                ctx.set_option(native.TV_OPT_STREAM_CHUNK, 128 << 10)
                ctx.set_layout(total, L, P, first, count)
                ctx.set_digests(bytes(dig))

                def fill(req):
                    ctx.stream_fill_synthetic(req, 12)
                    ctx.stream_commit(req)

                out[s], _ = _stream(native, ctx, fill)
        except Exception as e:  # reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(s, f, n)) for s, (f, n) in enumerate(ranges)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    got = bytearray((P + 7) // 8)
    for (first, count), sl in zip(ranges, out):
        got[first // 8:first // 8 + len(sl)] = sl
    assert got == expect


def test_verify_stream_through_storage(native, oracle):
    """verify_stream(info, storage.get): each row is one Storage.get (storage.ts:50-65) into the lent slot.
    The reference's multifile fixture (2 files, piece #852 spanning them, short final piece) verifies in
    full; truncating file 2 makes exactly the pieces touching its missing tail 0."""
    import json
    import os
    from torrent_amd import MemoryStorage, Storage, parse_metainfo, verify_stream
    golden = os.path.join(os.path.dirname(__file__), "golden")
    info = parse_metainfo(open(os.path.join(golden, "multifile.torrent"), "rb").read()).info
    rd = json.load(open(os.path.join(golden, "refdata.json")))["multifile"]
    parts = [f["pattern"].encode() * (f["length"] // len(f["pattern"])) for f in rd["files"]]
    mem = MemoryStorage({tuple(info.files[0].path): parts[0], tuple(info.files[1].path): parts[1]})
    st = Storage(mem, info, os.getcwd())
    P, L = info.n_pieces, info.piece_length
    full = bytes(b"\xff" * (P // 8) + bytes([(0xFF00 >> (P % 8)) & 0xFF]))
    assert bytes(verify_stream(info, st.get)) == full
    assert bytes(verify_stream(info, st.get, devices=[0, 0, 0])) == full
    cut = 1000
    mem.files[tuple(info.files[1].path)] = mem.files[tuple(info.files[1].path)][:cut]
    bf = verify_stream(info, Storage(mem, info, os.getcwd()).get, chunk=128 << 10)
    n0 = info.files[0].length
    for i in range(P):
        end = i * L + (info.length % L if i == P - 1 else L)
        assert _bits(bf, P)[i] == (1 if end <= n0 + cut else 0), i


def test_stream_state_errors_and_abort(native, oracle):
    """The state machine: next before begin, a second next with a request outstanding, a commit of a stale
    request, an early end (aborts), resident calls during a stream; tv_stream_abort leaves the ctx usable,
    and an empty shard completes at once."""
    L, P = 65536, 40
    total = L * P
    payload = oracle.synth_fill(3, 0, total)
    pieces = oracle.hash_pieces(payload, total, L, P)
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(pieces)
        with pytest.raises(native.NativeError, match="tv_stream_begin"):
            ctx.stream_next()
        ctx.stream_begin()
        with pytest.raises(native.NativeError, match="stream is active"):
            ctx.verify()
        req = ctx.stream_next()
        with pytest.raises(native.NativeError, match="outstanding"):
            ctx.stream_next()
        stale = native.StreamReq.from_buffer_copy(req)
        stale.seq += 5
        with pytest.raises(native.NativeError, match="does not match"):
            ctx.stream_commit(stale)
        with pytest.raises(native.NativeError, match="before its last column"):
            ctx.stream_end()                          # aborts
        ctx.stream_begin()
        ctx.stream_next()
        ctx.stream_abort()
        ctx.stage(0, payload)                         # usable again, resident path
        assert ctx.verify() == b"\xff" * 5
        # the stream path after the resident one, then the resident one again
        ctx.stream_begin()
        while True:
            req = ctx.stream_next()
            if not req.rows:
                break
            ctx.stream_commit_from(req, payload, L, req.piece * L + req.offset)
        assert ctx.stream_end() == b"\xff" * 5
        assert ctx.verify() == b"\xff" * 5
        # an empty shard: the first next reports completion
        ctx.set_layout(total, L, P, P, 0)
        ctx.set_digests(pieces)
        ctx.stream_begin()
        assert ctx.stream_next().rows == 0
        assert ctx.stream_end() == b""


@pytest.mark.parametrize("pieces_per_window", [64, 128])
def test_stream_whole_piece_rows_in_windows(native, oracle, pieces_per_window):
    """TV_OPT_STREAM_ROWS: every request row is a whole piece (offset 0, width = the piece length), so a
    Storage reader is asked once per piece; the shard is hashed in windows of 64 / 128 pieces (the budget
    halves bound each chunk buffer), 300 pieces of 16 KiB + 5 B (odd length) with a short last piece and
    unreadable pieces: bit-exact against the oracle, and the reads equal the pieces."""
    from torrent_amd import make_info, verify_stream
    L, P = 16384 + 5, 300
    total = L * (P - 1) + 777
    payload = bytes(oracle.synth_fill(41, 0, total))
    pieces = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    for i in (3, 64, 200):
        pieces[20 * i] ^= 1
    expect = _bits(oracle.verify_linear(bytearray(payload), total, L, bytes(pieces)), P)
    pitch = -(-L // 64) * 64 + 256
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_RESIDENT, 0)
        ctx.set_option(native.TV_OPT_STREAM_ROWS, 1)
        ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, 2 * pieces_per_window * pitch + 2 * 256)
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        seen, unreadable = [], {10, 299, 130}

        def fill(req):
            assert req.offset == 0 and req.width == L
            slot = ctx.stream_slot(req)
            for q in range(req.rows):
                i = req.piece + q
                n = ctx.row_bytes(req, q)
                seen.append(i)
                if i not in unreadable:
                    slot[q * req.width:q * req.width + n] = payload[i * L:i * L + n]
            slot.release()
            ctx.stream_commit(req)

        bf, reqs = _stream(native, ctx, fill, unreadable=unreadable)
        assert sorted(seen) == list(range(P))
        assert ctx.last_kernel()[1] == -(-P // pieces_per_window)      # one launch per window
        want = [0 if i in unreadable else b for i, b in enumerate(expect)]
        assert _bits(bf, P) == want
    # the host function: one read per piece
    info = make_info(L, bytes(pieces), "t", length=total)
    calls = []

    def read(off, n):
        calls.append((off, n))
        return payload[off:off + n]

    assert _bits(verify_stream(info, read), P) == expect
    assert len(calls) == P and all(off % L == 0 for off, _ in calls)
