"""Cold-cache staging from files: long segments whose bytes are not in the page cache are read
with O_DIRECT into the pinned ring (TV_OPT_FILE_ODIRECT; 4 KiB-rounded requests, the bytes at slot + fo % 4096).
Checked on files evicted from the page cache (tools/fsutil.py: fsync + DONTNEED, re-checked with mincore): sizes
that are not multiples of 4 KiB, file offsets that do and do not agree with the linear offsets mod 4 (the latter
read buffered), a short last piece, corrupted pieces, and a file shorter than its segment -- every bitfield equal
to Storage(fs_storage).get + hashlib's, with O_DIRECT on, off, and refused by the filesystem (fault injection:
the file falls back to buffered reads, never to unreadable pieces)."""
import errno
import hashlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu


def _bits(bf, n):
    return [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(n)]


@pytest.mark.parametrize("bounce", [0, 2, 4])   # the ring path / the bounce path (2: the default)
@pytest.mark.parametrize("odirect", [1, 0, 2])
def test_cold_files_exact(native, oracle, tmp_path, odirect, bounce):
    import fsutil
    from torrent_amd import FileInfo, Storage, make_info, verify_files
    from torrent_amd.storage import fs_storage
    from torrent_amd.verify import _context
    MiB = 1 << 20
    L = MiB
    sizes = [40 * MiB + 4093, 37 * MiB + 2, 50 * MiB + 12345, 33 * MiB]   # (file 1 starts at 40 MiB + 4093: not 0 mod 4)
    total = sum(sizes)
    P = -(-total // L)
    payload = bytearray(oracle.synth_fill(55, 0, total))
    digests = bytearray(b"".join(hashlib.sha1(bytes(payload[i * L:min(total, (i + 1) * L)])).digest() for i in range(P)))
    for i in (3, 77, P - 1):
        digests[20 * i + 1] ^= 0x20
    files, paths, o = [], [], 0
    for k, n in enumerate(sizes):
        p = tmp_path / f"f{k}.bin"
        data = payload[o:o + n]
        if k == 2:
            data = data[:n - 5 * MiB]          # shorter than its segment: its tail pieces read as null
        p.write_bytes(bytes(data))
        files.append(FileInfo(n, [f"f{k}.bin"]))
        paths.append(str(p))
        o += n
    info = make_info(L, bytes(digests), "cold", files=files, length=total)
    want_st = Storage(fs_storage, info, str(tmp_path))
    want = [0] * P
    for i in range(P):
        n = min(L, total - i * L)
        b = want_st.get(i * L, n)
        want[i] = int(b is not None and hashlib.sha1(b).digest() == bytes(digests[20 * i:20 * i + 20]))
    with _context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_ODIRECT, odirect)
        ctx.set_option(native.TV_OPT_FILE_BOUNCE, bounce)   # (readers per lane into 4 MiB bounce buffers)
        ctx._reset_file_clock()
    # warm (just written): read through the page cache, never O_DIRECT (an overlay /tmp once made warm files look
    # cold to cachestat and sent them to the disk at a third of the speed)
    assert fsutil.resident(paths) > 0.99
    cwd = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        assert _bits(verify_files(info, str(tmp_path)), P) == want
    finally:
        os.chdir(cwd)
    with _context(0) as ctx:
        assert ctx._file_clock()["bytes_odirect"] == 0
        ctx._reset_file_clock()
    assert fsutil.drop_cache(paths) <= 0.01
    try:
        cwd = os.getcwd()
        os.chdir(str(tmp_path))
        try:
            bf = verify_files(info, str(tmp_path))
        finally:
            os.chdir(cwd)
        with _context(0) as ctx:
            clock = ctx._file_clock()
    finally:
        with _context(0) as ctx:
            ctx.set_option(native.TV_OPT_FILE_ODIRECT, 1)
            ctx.set_option(native.TV_OPT_FILE_BOUNCE, native.FILE_BOUNCE_DEFAULT)
    assert _bits(bf, P) == want
    if odirect == 1:
        assert clock["bytes_odirect"] > 0, clock      # (the cold chunks whose offsets agree mod 4 went O_DIRECT)
        assert clock["bytes_odirect"] < clock["bytes_read"]   # (and the others buffered)
        assert clock["odirect_fallbacks"] == 0 and clock["odirect_errno"] == 0, clock   # (no read was refused)
    else:   # off, or (2) every O_DIRECT read refused: the same bits through the buffered fallback
        assert clock["bytes_odirect"] == 0
        if odirect == 2:   # (the refusal is counted, with its errno: EINVAL, as a filesystem without O_DIRECT)
            assert clock["odirect_fallbacks"] > 0 and clock["odirect_errno"] == errno.EINVAL, clock
        else:
            assert clock["odirect_fallbacks"] == 0, clock


@pytest.mark.parametrize("seed", list(range(24)))
def test_random_layouts_cold_long_path(native, tmp_path, monkeypatch, seed):
    """The seeded random layouts of tests/test_gpu_fuzz.py (zero-length, tiny, boundary-aligned, missing and
    truncated files, odd piece lengths, ragged digests) with every non-empty segment forced onto the long-segment
    path (direct_min = 1 byte: units dealt to both staging lanes) on a page cache dropped first, so the units go
    O_DIRECT wherever the file and linear offsets agree mod 4: bits equal fsStorage.get + hashlib's."""
    import shutil
    import fsutil
    from tests.test_gpu_fuzz import _disk, _draw, _expected
    from torrent_amd import Storage, verify_files
    from torrent_amd.storage import fs_storage
    info, payload, sizes, missing, short, single = _draw(seed)
    P = info.n_pieces
    monkeypatch.chdir(tmp_path)
    disk = _disk(info, payload, sizes, missing, short, single)
    paths = []
    for root in ("dl", "ref"):
        for k, data in disk.items():
            p = tmp_path.joinpath(root, *k)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
            if root == "dl":
                paths.append(str(p))
    want_fs = _expected(info, Storage(fs_storage, info, str(tmp_path / "ref")))
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)
    stride = -(-info.piece_length // 64) * 64 + 256
    # whole shards on one and three devices, then a windowed layout (a budget of ~3 pieces per window: the lanes
    # stage window by window, each window hashed while the next stages)
    from torrent_amd.verify import _context
    for devices, budget, bounce in (([0], None, 2), ([0, 0, 0], None, 2), ([0], None, 0), ([0], None, 4),
                                    ([0], native.WIN_BUFS_DEFAULT * (3 * stride + 256), 0)):
        if paths:
            assert fsutil.drop_cache(paths) <= 0.01
        with _context(0) as ctx:
            ctx.set_option(native.TV_OPT_FILE_BOUNCE, bounce)
        try:
            bf = verify_files(info, str(tmp_path / "dl"), devices=devices, threads=4, direct_min=1, budget=budget,
                              stream=False)
        finally:
            with _context(0) as ctx:
                ctx.set_option(native.TV_OPT_FILE_BOUNCE, native.FILE_BOUNCE_DEFAULT)
        assert _bits(bf, P) == want_fs, (seed, devices, budget, bounce)


@pytest.mark.parametrize("bounce", [0, 3])
def test_cold_file_end_stays_o_direct(native, oracle, tmp_path, bounce):
    """A cold file whose size is not a multiple of 4 KiB: the O_DIRECT request for its last chunk runs past the end
    of the file and comes back short.  That read is complete (the bytes asked for are in) and must not be continued
    (a next request would start off a 4 KiB boundary and be refused, sending the chunk through the buffered fallback
    a second time): every byte is counted as read O_DIRECT, and the bits are exact."""
    import fsutil
    from torrent_amd import FileInfo, make_info, verify_files
    from torrent_amd.verify import _context
    MiB = 1 << 20
    L = MiB
    total = 150 * MiB + 4097                      # three 64 MiB-ish ring chunks, the last one ragged
    P = -(-total // L)
    payload = bytes(oracle.synth_fill(57, 0, total))
    digests = bytearray(b"".join(hashlib.sha1(payload[i * L:min(total, (i + 1) * L)]).digest() for i in range(P)))
    digests[20 * (P - 1)] ^= 1
    f = tmp_path / "one.bin"
    f.write_bytes(payload)
    info = make_info(L, bytes(digests), "one", files=[FileInfo(total, ["one.bin"])], length=total)
    assert fsutil.drop_cache([str(f)]) <= 0.01
    with _context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_ODIRECT, 1)
        ctx.set_option(native.TV_OPT_FILE_BOUNCE, bounce)
        ctx._reset_file_clock()
    cwd = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        bf = verify_files(info, str(tmp_path))
    finally:
        os.chdir(cwd)
        with _context(0) as ctx:
            ctx.set_option(native.TV_OPT_FILE_BOUNCE, native.FILE_BOUNCE_DEFAULT)
    with _context(0) as ctx:
        clock = ctx._file_clock()
    assert _bits(bf, P) == [1] * (P - 1) + [0]
    assert clock["bytes_odirect"] == clock["bytes_read"] == total, clock
    assert clock["odirect_fallbacks"] == 0, clock


@pytest.mark.parametrize("odirect", [1, 0, 2])
def test_cold_files_streamed(native, oracle, tmp_path, odirect):
    """verify_files through the bounded ring (tv_stream_file_table, stream=True) on files evicted from the page cache:
    a file whose pages are mostly not cached at its open is read O_DIRECT, rows straight into the ring slot where the
    file offset, the row and its length are 4 KiB-aligned (file 0) and through a reader's aligned scratch where not
    (file 1 starts at 40 MiB + 4093), a short file ending mid-row -- every bitfield equal to Storage(fs_storage).get +
    hashlib's; warm files are never read O_DIRECT, and a refused O_DIRECT read (fault injection) falls back to
    buffered reads of that file, counted."""
    import fsutil
    from torrent_amd import FileInfo, Storage, make_info, verify_files
    from torrent_amd.storage import fs_storage
    from torrent_amd.verify import _context
    MiB = 1 << 20
    L = MiB
    sizes = [40 * MiB + 4093, 37 * MiB + 2, 50 * MiB + 12345, 33 * MiB]
    total = sum(sizes)
    P = -(-total // L)
    payload = bytearray(oracle.synth_fill(56, 0, total))
    digests = bytearray(b"".join(hashlib.sha1(bytes(payload[i * L:min(total, (i + 1) * L)])).digest() for i in range(P)))
    for i in (0, 41, P - 1):
        digests[20 * i + 7] ^= 0x04
    files, paths, o = [], [], 0
    for k, n in enumerate(sizes):
        p = tmp_path / f"f{k}.bin"
        data = payload[o:o + n]
        if k == 2:
            data = data[:n - 5 * MiB - 777]     # short: its tail pieces read as null
        p.write_bytes(bytes(data))
        files.append(FileInfo(n, [f"f{k}.bin"]))
        paths.append(str(p))
        o += n
    info = make_info(L, bytes(digests), "cold", files=files, length=total)
    st = Storage(fs_storage, info, str(tmp_path))
    want = [0] * P
    for i in range(P):
        b = st.get(i * L, min(L, total - i * L))
        want[i] = int(b is not None and hashlib.sha1(b).digest() == bytes(digests[20 * i:20 * i + 20]))
    budget = 2 * (P * (256 * 1024 + 256) + 256)      # 256 KiB columns: 4 per piece
    with _context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_ODIRECT, odirect)
    cwd = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        for cold in (False, True):
            if cold:
                assert fsutil.drop_cache(paths) <= 0.01
            else:
                assert fsutil.resident(paths) > 0.99
            with _context(0) as ctx:
                ctx._reset_file_clock()
            bf = verify_files(info, str(tmp_path), threads=4, budget=budget, stream=True)
            with _context(0) as ctx:
                clock = ctx._file_clock()
                assert ctx.last_kernel()[1] == 4                 # one window, four columns
            assert _bits(bf, P) == want, (cold, odirect)
            if cold and odirect == 1:
                assert 0 < clock["bytes_odirect"] == clock["bytes_read"], clock
                assert clock["odirect_fallbacks"] == 0, clock
            else:
                assert clock["bytes_odirect"] == 0, clock
                if cold and odirect == 2:
                    assert clock["odirect_fallbacks"] > 0 and clock["odirect_errno"] == errno.EINVAL, clock
                else:
                    assert clock["odirect_fallbacks"] == 0, clock
        if odirect:   # a cold shard in windows of 64 pieces: 3 windows (64 + 64 + 32) x 2 columns of 640 KiB
            with _context(0) as ctx:
                ctx.set_option(native.TV_OPT_STREAM_COLD_WINDOW, 64)
            assert fsutil.drop_cache(paths) <= 0.01
            bf = verify_files(info, str(tmp_path), threads=4, budget=budget, stream=True)
            with _context(0) as ctx:
                assert ctx.last_kernel()[1] == 6
            assert _bits(bf, P) == want, ("cold windows", odirect)
    finally:
        os.chdir(cwd)
        with _context(0) as ctx:
            ctx.set_option(native.TV_OPT_FILE_ODIRECT, 1)
            ctx.set_option(native.TV_OPT_STREAM_COLD_WINDOW, 0)
