"""How the library opens files, and what a failed segment's mark lasts for.

* Creation mode (hash_files / make_torrent) opens its sources read-only, as make_torrent.ts:78 does
  (Deno.open's default), so a torrent can be made from files the process may not write; verify_files keeps
  fsStorage.get's read + write open (storage.ts:28-32,158), so there an unwritable file reads as null.
* A piece marked unreadable by a failed tv_stage_file(s) is readable again once a later call on the same
  layout stages all its bytes (the file was repaired).
"""
import hashlib
import os

import pytest

pytestmark = pytest.mark.gpu


def _tree(tmp_path, sizes, seed=5):
    import random
    rng = random.Random(seed)
    root = tmp_path / "src"
    root.mkdir()
    data = []
    for k, n in enumerate(sizes):
        b = rng.randbytes(n)
        (root / f"f{k}.bin").write_bytes(b)
        data.append(b)
    return root, data


@pytest.mark.skipif(os.geteuid() == 0, reason="root may open any file read + write; the GPU box runs as a user")
@pytest.mark.parametrize("direct_min", [None, 0])
def test_creation_from_files_the_process_cannot_write(native, tmp_path, direct_min):
    """chmod 444 sources: hash_files (both staging paths: the reader pool, and the windowed page-cache path
    with direct_min=0) and make_torrent give hashlib's pieces; verify_files over the same files reports the
    pieces of the unwritable file 0, exactly as Storage(fs_storage).get's read + write open fails there."""
    from torrent_amd import Storage, fs_storage, hash_files, make_info, make_torrent, parse_metainfo, verify_files
    from torrent_amd.metainfo import FileInfo
    from torrent_amd.piece import piece_length
    L = 32768
    root, data = _tree(tmp_path, [100_000, 70_000, 5])
    lin = b"".join(data)
    P = -(-len(lin) // L)
    want = b"".join(hashlib.sha1(lin[i * L:(i + 1) * L]).digest() for i in range(P))
    files = [FileInfo(len(d), [f"f{k}.bin"]) for k, d in enumerate(data)]
    os.chmod(root / "f1.bin", 0o444)
    try:
        geom = make_info(L, bytes(20 * P), "src", files=files)
        assert hash_files(geom, str(root), direct_min=direct_min) == want
        meta = parse_metainfo(make_torrent(str(root), "http://t/announce", piece_length=L, files=files))
        assert meta.info.pieces_raw == want
        info = make_info(L, want, "src", files=files)
        got = verify_files(info, str(root), direct_min=direct_min)
        st = Storage(fs_storage, info, str(root))
        for i in range(P):
            readable = st.get(i * L, piece_length(i, info)) is not None
            assert ((got[i >> 3] >> (7 - (i & 7))) & 1) == int(readable), i
        assert not all((got[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P))   # f1's pieces: 0
    finally:
        os.chmod(root / "f1.bin", 0o644)


def test_open_mode_option(native, tmp_path):
    """TV_OPT_OPEN_RW round-trips and tv_stage_file honours it for a missing zero-length segment: creatable
    (read + write, fsStorage.get would create it) vs not openable (read-only, make_torrent's open fails)."""
    with native.Context(0) as ctx:
        assert ctx.get_option(native.TV_OPT_OPEN_RW) == 1
        ctx.set_layout(100, 100, 1)
        assert ctx.stage_file(str(tmp_path / "absent.bin"), 0, 0, 0) is True
        ctx.set_option(native.TV_OPT_OPEN_RW, 0)
        assert ctx.get_option(native.TV_OPT_OPEN_RW) == 0
        assert ctx.stage_file(str(tmp_path / "absent.bin"), 0, 0, 0) is False
        assert not (tmp_path / "absent.bin").exists()
        with pytest.raises(native.NativeError):
            ctx.set_option(native.TV_OPT_OPEN_RW, 2)


@pytest.mark.parametrize("windowed", [False, True])
def test_restaged_file_clears_the_unreadable_mark(native, oracle, tmp_path, windowed):
    """A file missing at the first tv_stage_file marks its pieces 0; once it is written and staged again into
    the same layout (no tv_set_layout between) its whole pieces verify 1 -- through tv_stage_file and through
    tv_stage_files (whose segments' union covers a piece that spans two files)."""
    L, P = 4096, 24
    total = L * P
    payload = bytes(oracle.synth_fill(9, 0, total))
    pieces = oracle.hash_pieces(bytearray(payload), total, L, P)
    a, b = tmp_path / "a.bin", tmp_path / "b.bin"
    cut = 10 * L + 100                       # piece 10 spans a and b
    a.write_bytes(payload[:cut])
    with native.Context(0) as ctx:
        if windowed:                         # windows of 4 pieces: every stage is a new pass
            ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, native.WIN_BUFS_DEFAULT * (4 * (L + 256) + 256))
        ctx.set_layout(total, L, P)
        ctx.set_digests(pieces)
        assert ctx.stage_file(str(a), 0, 0, cut)
        assert ctx.stage_file(str(b), 0, cut, total - cut) is False      # missing: pieces 10.. marked
        bf = ctx.verify()
        assert [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)] == [1] * 10 + [0] * 14
        b.write_bytes(payload[cut:])
        assert ctx.stage_file(str(a), 0, 0, cut)
        assert ctx.stage_file(str(b), 0, cut, total - cut)
        bf = ctx.verify()
        # piece 10 is covered by neither call alone: its mark (from b) stays; 11.. are whole in b
        assert [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)] == [1] * 10 + [0] + [1] * 13
        st = ctx.stage_files([str(a), str(b)], [0, 0], [0, cut], [cut, total - cut])
        assert st == [native.TV_OK, native.TV_OK]
        bf = ctx.verify()
        assert [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)] == [1] * P
