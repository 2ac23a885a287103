"""Seeded random layouts through every host path on the HIP library, against the reference's semantics.

For each seed a torrent is drawn with a random piece length (powers of two and odd lengths, some not a
multiple of 64), 1-40 files with zero-length, tiny and piece-boundary-aligned files, missing and truncated
files on disk, corrupted pieces, and sometimes a ragged digest string or more digests than data.  The
expected bit of piece i follows the reference exactly: Storage.get(i * L, pieceLength(i)) over the on-disk
files (storage.ts:50-65, 89-137; the Python mirror, pinned by tests/test_host_mirror.py) is non-null and its
SHA-1 (hashlib, the checker) equals slice i of info.pieces (metainfo.ts:111, _bytes.ts:92-99).  The GPU
bitfields of verify_pieces (Storage.get reads), verify_payload (resident and streamed), verify_stream
(bounded ring) and verify_files (files on disk, tv_stage_files) must all equal it, on one and on three
shards."""
import hashlib
import random

import pytest

SEEDS = list(range(48))


def _draw(seed):
    from torrent_amd.metainfo import FileInfo, make_info
    rng = random.Random(1000 + seed)
    L = rng.choice([64, 100, 1000, 4096, 16384 + 7, 65536, 262144])
    n_files = rng.choice([1, 1, 2, 5, 17, 40])
    target = rng.randrange(L // 2 + 1, min(60 * L, 3 << 20))
    sizes = []
    while sum(sizes) < target and len(sizes) < n_files:
        kind = rng.random()
        if kind < 0.15:
            sizes.append(0)
        elif kind < 0.3:
            sizes.append(rng.randrange(1, 64))
        elif kind < 0.45:                          # end the file exactly on a piece boundary
            pos = sum(sizes)
            sizes.append((-pos) % L or L)
        else:
            sizes.append(rng.randrange(1, 4 * L))
    if sum(sizes) == 0:
        sizes.append(L + 3)
    total = sum(sizes)
    P = -(-total // L)
    payload = bytearray(rng.randbytes(total))
    digests = bytearray(b"".join(hashlib.sha1(bytes(payload[i * L:(i + 1) * L])).digest() for i in range(P)))
    for i in rng.sample(range(P), max(1, P // 10)):            # corrupted data
        payload[i * L + rng.randrange(min(L, total - i * L))] ^= 1 << rng.randrange(8)
    extra = rng.random() < 0.2
    if extra:                                                   # more digests than data: those pieces null
        digests += bytes(rng.getrandbits(8) for _ in range(20 * rng.randrange(1, 9)))
    if rng.random() < 0.2:                                      # ragged digest string: last slice short
        digests = digests[:-rng.randrange(1, 20)]
    single = len(sizes) == 1 and rng.random() < 0.5
    files = None if single else [FileInfo(s, [f"s{k % 3}", f"f{k}.bin"]) for k, s in enumerate(sizes)]
    info = make_info(L, bytes(digests), "t.bin", files=files, length=total)
    # on disk: some files missing, some truncated
    missing, short = set(), {}
    for k, s in enumerate(sizes):
        r = rng.random()
        if r < 0.08:
            missing.add(k)
        elif r < 0.14 and s > 0:
            short[k] = rng.randrange(s)
    return info, bytes(payload), sizes, missing, short, single


def _disk(info, payload, sizes, missing, short, single):
    """{path tuple: bytes} as on disk (missing files absent, short ones truncated)."""
    out, o = {}, 0
    for k, s in enumerate(sizes):
        if k not in missing:
            key = (info.name,) if single else tuple(info.files[k].path)
            out[key] = payload[o:o + short.get(k, s)]
        o += s
    return out


def _expected(info, storage):
    from torrent_amd.piece import piece_length
    P, L = info.n_pieces, info.piece_length
    bits = []
    for i in range(P):
        got = storage.get(i * L, piece_length(i, info))
        d = info.pieces_raw[20 * i:20 * i + 20]
        bits.append(int(got is not None and len(d) == 20 and hashlib.sha1(bytes(got)).digest() == d))
    return bits


def _bits(bf, n):
    return [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_layouts_every_host_path(native, tmp_path, monkeypatch, seed):
    import shutil
    from torrent_amd import MemoryStorage, Storage, verify_files, verify_payload, verify_pieces, verify_stream
    from torrent_amd.piece import piece_length
    from torrent_amd.storage import fs_storage
    info, payload, sizes, missing, short, single = _draw(seed)
    P, L = info.n_pieces, info.piece_length
    monkeypatch.chdir(tmp_path)
    disk = _disk(info, payload, sizes, missing, short, single)
    # in memory: Storage paths are [*dir, name] / [*dir, *file.path] (storage.ts:99-114)
    mem = MemoryStorage()
    st = Storage(mem, info, str(tmp_path / "dl"))
    mem.files = {tuple(st.dir_path) + k: bytearray(v) for k, v in disk.items()}
    want = _expected(info, st)
    # on disk, for verify_files; its expectation is fsStorage.get's (a zero-length file in a missing
    # directory does not open), taken on a copy because that get creates files
    for root in ("dl", "ref"):
        for k, data in disk.items():
            p = tmp_path.joinpath(root, *k)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
    want_fs = _expected(info, Storage(fs_storage, info, str(tmp_path / "ref")))
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)          # absent when no file was written or created
    # the linear payload's availability as Storage.get sees it (verify_payload takes one buffer)
    avail = bytearray((P + 7) // 8)
    for i in range(P):
        if st.get(i * L, piece_length(i, info)) is not None:
            avail[i >> 3] |= 0x80 >> (i & 7)
    lin = payload[:info.length]
    before = sorted(str(x) for x in (tmp_path / "dl").rglob("*"))
    for devices in ([0], [0, 0, 0]):
        assert _bits(verify_pieces(info, st, devices=devices), P) == want, ("pieces", seed, devices)
        assert _bits(verify_payload(info, lin, devices=devices, avail=bytes(avail)), P) == want, ("payload", seed)
        assert _bits(verify_payload(info, lin, devices=devices, resident=False, avail=bytes(avail)), P) == want, \
            ("payload streamed", seed)
        assert _bits(verify_stream(info, st.get, devices=devices), P) == want, ("stream", seed, devices)
        assert _bits(verify_files(info, str(tmp_path / "dl"), devices=devices, threads=3), P) == want_fs, \
            ("files", seed, devices)
    # the Storage paths' reader dispatch (runs of pieces per thread) at its extremes: in the calling thread, and
    # more threads than a small batch has pieces
    for devices, threads in (([0], 1), ([0, 0], 16)):
        assert _bits(verify_pieces(info, st, devices=devices, threads=threads), P) == want, ("pieces", seed, threads)
        assert _bits(verify_stream(info, st.get, devices=devices, threads=threads), P) == want, ("stream", seed, threads)
    assert sorted(str(x) for x in (tmp_path / "dl").rglob("*")) == before      # verify_files created nothing


def test_fuzz_layouts_cover_the_edge_cases():
    """The seeds above draw every edge case at least once (CPU-only check of the generator)."""
    seen = set()
    for seed in SEEDS:
        info, payload, sizes, missing, short, single = _draw(seed)
        L = info.piece_length
        seen.add("odd_L" if L % 64 else "L64")
        seen |= {"zero_file"} if 0 in sizes else set()
        seen |= {"missing"} if missing else set()
        seen |= {"short"} if short else set()
        seen |= {"single"} if single else {"multi"}
        seen |= {"ragged"} if len(info.pieces_raw) % 20 else set()
        seen |= {"extra_digests"} if len(info.pieces_raw) // 20 > -(-info.length // L) else set()
        seen |= {"short_last"} if info.length % L else set()
        ends, o = [], 0
        for s in sizes:
            o += s
            ends.append(o)
        seen |= {"boundary_file"} if any(e % L == 0 and 0 < e < info.length for e in ends) else set()
    assert {"odd_L", "L64", "zero_file", "missing", "short", "single", "multi", "ragged", "extra_digests",
            "short_last", "boundary_file"} <= seen, seen


@pytest.mark.parametrize("seed", SEEDS)
def test_random_layouts_files_plan_on_cpu(tmp_path, monkeypatch, seed):
    """verify_files' staging plan for every seed on CPU (the library's read and recovery rules restated in
    tests/test_host_mirror._ImageCtx): readable bits equal Storage(fs_storage).get's per piece (on a copy,
    since that get creates files) over 1 and 3 shards, and every readable piece's bytes are staged."""
    import shutil
    from tests.test_host_mirror import _ImageCtx
    from torrent_amd import Storage, verify
    from torrent_amd.piece import piece_length
    from torrent_amd.storage import fs_storage
    info, payload, sizes, missing, short, single = _draw(seed)
    P, L, total = info.n_pieces, info.piece_length, info.length
    monkeypatch.chdir(tmp_path)
    for root in ("dl", "ref"):
        for k, data in _disk(info, payload, sizes, missing, short, single).items():
            p = tmp_path.joinpath(root, *k)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
    ref = Storage(fs_storage, info, str(tmp_path / "ref"))
    want = [ref.get(i * L, piece_length(i, info)) is not None for i in range(P)]
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)
    st = Storage(fs_storage, info, str(tmp_path / "dl"))
    for n in (1, 3):
        got = []
        for first, count in verify.shard_ranges(P, n):
            if not count:
                continue
            last = first + count - 1
            hi = min(total, last * L + piece_length(last, info))
            ctx = _ImageCtx(total, first * L, hi, L)
            bits = ctx.avail(verify._files_shard(ctx, info, st, first, count, threads=2), first, count)
            got += bits
            for j, ok in enumerate(bits):
                a = (first + j) * L
                if ok:
                    assert ctx.img[a:a + piece_length(first + j, info)] == payload[a:a + piece_length(first + j, info)]
        assert got == want, (seed, n)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:12])
def test_random_layouts_incremental_hash_and_piece(native, seed):
    """The same seeded torrents through the per-piece paths: IncrementalVerifier fed every data piece's
    blocks in random order with duplicates, a corrupted block later re-sent intact, and a random flush
    policy (f1, torrent.ts:183-193); verify_piece on random pieces; hash_pieces (creation, f3) of the
    linear payload.  Expected: hashlib over the same bytes (the reference's crypto.subtle.digest)."""
    from torrent_amd import hash_pieces, verify_piece
    from torrent_amd.incremental import IncrementalVerifier
    from torrent_amd.piece import BLOCK_SIZE, PieceMsg, piece_length
    info, payload, sizes, missing, short, single = _draw(seed)
    P, L, total = info.n_pieces, info.piece_length, info.length
    rng = random.Random(seed)
    data_pieces = [i for i in range(P) if i * L + piece_length(i, info) <= total]
    truth = {i: hashlib.sha1(payload[i * L:i * L + piece_length(i, info)]).digest()
             == info.pieces_raw[20 * i:20 * i + 20] for i in data_pieces}
    # creation: the linear payload's pieces string
    n_data = -(-total // L)
    assert hash_pieces(payload, L) == b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest()
                                               for i in range(n_data))
    # one piece at a time
    for i in rng.sample(data_pieces, min(4, len(data_pieces))):
        assert verify_piece(info, i, payload[i * L:i * L + piece_length(i, info)]) is truth[i], (seed, i)
    # incremental
    msgs = []
    for i in data_pieces:
        n = piece_length(i, info)
        for o in range(0, n, BLOCK_SIZE):
            if i == P - 1 and o + BLOCK_SIZE >= n:                  # the torrent's last block: exact length
                blk = payload[i * L + o:i * L + n]
            else:                                                   # every other block is BLOCK_SIZE long
                blk = payload[i * L + o:i * L + o + BLOCK_SIZE]     # (piece.ts:39-65), past the piece if L
                blk += bytes(BLOCK_SIZE - len(blk))                 # % BLOCK_SIZE != 0: the verifier cuts it
            msgs.append(PieceMsg(i, o, blk))
    rng.shuffle(msgs)
    msgs += rng.sample(msgs, len(msgs) // 5)                        # duplicates, some after completion
    bad = None
    if msgs:
        k = rng.randrange(len(msgs))
        m = msgs[k]
        bad = m.index
        msgs[k] = PieceMsg(m.index, m.offset, bytes(b ^ 0x10 for b in m.block))
        msgs.append(m)                                              # the intact block, re-sent at the end
    seen = {}
    v = IncrementalVerifier(info, flush_pieces=rng.choice([1, 7, None]), flush_age_ms=None,
                            on_verified=lambda i, ok: seen.setdefault(i, []).append(ok))
    try:
        for m in msgs:
            v.on_block(m)
        for i, ok in v.flush():
            seen.setdefault(i, []).append(ok)
        # the corrupted piece: verified False once it completed with the bad block; the final intact
        # re-send then completes it again only if its earlier copy had already failed and been flushed
        got = [bool(v.bitfield[i >> 3] & (0x80 >> (i & 7))) for i in range(P)]
        for i in data_pieces:
            results = seen.get(i, [])
            assert results, (seed, i)
            assert results[-1] == got[i], (seed, i, results)
            if i != bad:
                assert results == [truth[i]] or (not truth[i] and all(r is False for r in results)), (seed, i, results)
                assert got[i] == truth[i], (seed, i)
            else:
                assert all(r is False for r in results[:-1]), (seed, i, results)
        assert not any(got[i] for i in range(P) if i not in truth)
    finally:
        v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:12])
def test_random_layouts_wrong_length_reads(native, seed):
    """A storage whose get returns one byte too many for a piece (the reference's Storage.get never does:
    exactly the length asked, or null) makes that piece unreadable in verify_pieces and verify_stream, and
    no other piece moves: the batch buffer keeps every later piece at its place."""
    from torrent_amd import MemoryStorage, Storage, verify_pieces, verify_stream
    info, payload, sizes, missing, short, single = _draw(seed)
    P = info.n_pieces
    mem = MemoryStorage()
    st = Storage(mem, info, "/dl")
    mem.files = {tuple(st.dir_path) + k: bytearray(v) for k, v in _disk(info, payload, sizes, missing, short,
                                                                         single).items()}
    want = _expected(info, st)
    rng = random.Random(seed)
    wrong = rng.randrange(P)
    L = info.piece_length

    class Longer:
        def get(self, offset, length):
            data = st.get(offset, length)
            return None if data is None else (bytes(data) + b"\x5a" if offset // L == wrong else data)

    want[wrong] = 0
    for devices in ([0], [0, 0, 0]):
        assert _bits(verify_pieces(info, Longer(), devices=devices), P) == want, (seed, devices)
        assert _bits(verify_stream(info, Longer().get, devices=devices), P) == want, (seed, devices)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_layouts_file_table(native, tmp_path, monkeypatch, seed):
    """tv_stage_file_table (the TS host's verifyFiles: the torrent's file table handed over, the library making
    Storage.get's walk) on the 48 seeded layouts: one shard, three shards and a windowed layout
    (windows of ~3 pieces), long segments forced on some shards -- bits equal fsStorage.get + hashlib's, the per-file
    status names exactly the missing / short files that hold shard bytes, and nothing is created."""
    import shutil
    from torrent_amd import Storage
    from torrent_amd.piece import piece_length
    from torrent_amd.storage import fs_storage
    from torrent_amd.verify import shard_ranges
    info, payload, sizes, missing, short, single = _draw(seed)
    P, L, total = info.n_pieces, info.piece_length, info.length
    monkeypatch.chdir(tmp_path)
    disk = _disk(info, payload, sizes, missing, short, single)
    for root in ("dl", "ref"):
        for k, data in disk.items():
            p = tmp_path.joinpath(root, *k)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
    want = _expected(info, Storage(fs_storage, info, str(tmp_path / "ref")))
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)
    paths = Storage(fs_storage, info, str(tmp_path / "dl")).file_paths()
    lengths = [total] if info.files is None else [f.length for f in info.files]
    before = sorted(str(x) for x in (tmp_path / "dl").rglob("*"))
    stride = -(-L // 64) * 64 + 256
    for n, budget, direct_min in ((1, 0, 32 << 20), (3, 0, 1), (1, native.WIN_BUFS_DEFAULT * (3 * stride + 256), 1)):
        got = []
        for first, count in shard_ranges(P, n):
            if not count:
                continue
            with native.Context(0) as ctx:
                ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, budget)
                ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, direct_min)
                ctx.set_option(native.TV_OPT_FILE_THREADS, 3)
                ctx.set_layout(total, L, P, first, count)
                ctx.set_digests(info.pieces_raw)
                status = ctx.stage_file_table(lengths, paths)
                assert len(status) == len(paths)
                # pieces whose bytes run past the data (more digests than data): unreadable, as the hosts mark them
                avail = bytearray(b"\xff" * ((count + 7) // 8))
                for j in range(count):
                    i = first + j
                    if i * L + piece_length(i, info) > total:
                        avail[j >> 3] &= ~(0x80 >> (j & 7)) & 0xFF
                bits = ctx.verify(bytes(avail))
                got += _bits(bits, count)
                # the per-file status: a failure only for files absent or short that hold bytes of this shard
                lo, hi = first * L, min(total, (first + count - 1) * L + piece_length(first + count - 1, info))
                o = 0
                for k, s in enumerate(sizes):
                    holds = s > 0 and o < hi and o + s > lo
                    bad = k in missing or (k in short and short[k] < min(s, hi - o))
                    if holds:
                        assert status[k] == (native.TV_ERR_IO if bad else 0), (seed, n, k)
                    elif s > 0 and (o + s < lo or o >= hi):   # (a file ending at lo has a zero-length segment)
                        assert status[k] == 0, (seed, n, k)
                    o += s
        assert got == want, (seed, n, budget)
    assert sorted(str(x) for x in (tmp_path / "dl").rglob("*")) == before      # nothing created


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_layouts_streamed_files(native, tmp_path, monkeypatch, seed):
    """verify_files through the bounded ring from the files (tv_stream_file_table: the library's readers fill each
    column's rows, walking the file table per row) on the 48 seeded layouts: one and three shards, the library's
    column width and columns sized to a budget of a few pieces (64-byte columns at the smallest) -- bits equal
    fsStorage.get + hashlib's, nothing created."""
    import shutil
    from torrent_amd import Storage, verify_files
    from torrent_amd.storage import fs_storage
    info, payload, sizes, missing, short, single = _draw(seed)
    P, L = info.n_pieces, info.piece_length
    monkeypatch.chdir(tmp_path)
    disk = _disk(info, payload, sizes, missing, short, single)
    for root in ("dl", "ref"):
        for k, data in disk.items():
            p = tmp_path.joinpath(root, *k)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
    want = _expected(info, Storage(fs_storage, info, str(tmp_path / "ref")))
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)
    before = sorted(str(x) for x in (tmp_path / "dl").rglob("*"))
    for devices, budget in (([0], None), ([0, 0, 0], None), ([0], 2 * (3 * L + 4096)), ([0, 0], 1)):
        bf = verify_files(info, str(tmp_path / "dl"), devices=devices, threads=3, budget=budget, stream=True)
        assert _bits(bf, P) == want, (seed, devices, budget)
    assert sorted(str(x) for x in (tmp_path / "dl").rglob("*")) == before


@pytest.mark.gpu
def test_streamed_files_windows_of_columns(native, tmp_path, monkeypatch):
    """tv_stream_file_table's geometry under a device budget: windows of 2,048 pieces, each hashed in columns as wide
    as the budget allows (tv_stream.hip), on a 5,000-piece torrent of 4 KiB pieces with a short last piece, a
    zero-length file, a truncated and a missing file and corrupted pieces -- 1,024-byte columns (3 windows x 4
    columns), 64-byte columns (3 x 64), whole pieces in one window (no budget), an explicit TV_OPT_STREAM_CHUNK
    (columns across the shard), on one and two shards: bits equal fsStorage.get + hashlib's."""
    import shutil
    from torrent_amd import Storage, verify_files
    from torrent_amd.metainfo import FileInfo, make_info
    from torrent_amd.storage import fs_storage
    from torrent_amd.verify import shard_ranges
    rng = random.Random(77)
    L, P = 4096, 5000
    total = P * L - 1234
    payload = bytearray(rng.randbytes(total))
    digests = b"".join(hashlib.sha1(bytes(payload[i * L:(i + 1) * L])).digest() for i in range(P))
    for i in (0, 63, 64, 2047, 2048, 2049, 4095, 4096, P - 1):     # corrupted around the window and word edges
        payload[min(total - 1, i * L + rng.randrange(L))] ^= 0x5A
    sizes = [3 * L + 17, 0, 2000 * L, 1111 * L - 17, 700 * L + 5, 0]
    sizes.append(total - sum(sizes))
    names = [f"f{k}.bin" for k in range(len(sizes))]
    info = make_info(L, digests, "t", files=[FileInfo(n, ["s", nm]) for n, nm in zip(sizes, names)], length=total)
    monkeypatch.chdir(tmp_path)
    for root in ("dl", "ref"):
        (tmp_path / root / "s").mkdir(parents=True)
        o = 0
        for n, nm in zip(sizes, names):
            data = bytes(payload[o:o + n])
            o += n
            if nm == "f4.bin":
                continue                                               # missing
            if nm == "f3.bin":
                data = data[:len(data) - 3000]                         # short
            (tmp_path / root / "s" / nm).write_bytes(data)
    want = _expected(info, Storage(fs_storage, info, str(tmp_path / "ref")))
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)
    assert 0 < sum(want) < P
    before = sorted(str(x) for x in (tmp_path / "dl").rglob("*"))
    half = 2048 * (1024 + 256) + 256
    for devices in ([0], [0, 0]):
        for budget in (2 * half, 1, None):
            bf = verify_files(info, str(tmp_path / "dl"), devices=devices, threads=4, budget=budget, stream=True)
            assert _bits(bf, P) == want, (devices, budget)
    # the geometry: units = windows x columns (tv_last_kernel's launch count)
    paths = Storage(fs_storage, info, str(tmp_path / "dl")).file_paths()
    for budget, chunk, units in ((2 * half, 0, 3 * 4), (1, 0, 3 * 64), (0, 0, 1), (0, 1024, 4)):
        got = []
        for first, count in shard_ranges(P, 1):
            with native.Context(0) as ctx:
                ctx.set_option(native.TV_OPT_RESIDENT, 0)
                ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, budget)
                ctx.set_option(native.TV_OPT_STREAM_CHUNK, chunk)
                ctx.set_layout(total, L, P, first, count)
                ctx.set_digests(info.pieces_raw)
                ctx.set_option(native.TV_OPT_FILE_THREADS, 4)
                bits, status = ctx.stream_file_table(sizes, paths)
                assert ctx.last_kernel()[1] == units, (budget, chunk)
                assert [k for k, s in enumerate(status) if s] == [3, 4], (budget, chunk)
                got += _bits(bits, count)
        assert got == want, (budget, chunk)
    assert sorted(str(x) for x in (tmp_path / "dl").rglob("*")) == before
