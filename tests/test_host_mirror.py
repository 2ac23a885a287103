"""Host-side mirror of the reference interfaces (CPU only): metainfo.ts, piece.ts, storage.ts.

Ports of the reference's own test cases (metainfo_test.ts, storage_test.ts) plus the
file-to-piece mapping quirks the device offset table relies on.
"""
import os
import random

import pytest

from torrent_amd.bencode import bdecode as _bdecode, bencode as _bencode
from torrent_amd.metainfo import encode_metainfo, make_info, parse_metainfo, partition, FileInfo
from torrent_amd.piece import (BLOCK_SIZE, PieceMsg, RequestMsg, piece_length, validate_received_block,
                               validate_requested_block)
from torrent_amd.storage import FsStorage, MemoryStorage, Storage
from torrent_amd.verify import shard_ranges

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


# ---- metainfo_test.ts ------------------------------------------------------------------

def test_parse_single_file():  # metainfo_test.ts:11-30
    m = parse_metainfo(_load("singlefile.torrent"))
    assert m is not None
    assert m.comment == "comment" and m.announce == "http://example.com/announce"
    assert m.encoding == "UTF-8"
    assert m.created_by == "https://github.com/rclarey/torrent/blob/master/tools/make_torrent.ts"
    assert m.creation_date == 1602023427
    i = m.info
    assert (i.piece_length, i.name, i.length, len(i.pieces), i.private) == (262144, "singlefile.txt", 447135744, 1706, 0)
    assert all(len(p) == 20 for p in i.pieces) and b"".join(i.pieces) == i.pieces_raw


def test_parse_multi_file():  # metainfo_test.ts:32-59
    m = parse_metainfo(_load("multifile.torrent"))
    i = m.info
    assert m.creation_date == 1599690859
    assert (i.piece_length, i.name, len(i.pieces), i.private, len(i.files)) == (524288, "multifile", 1855, 0, 2)
    assert i.files[0].length == 447135744 and "/".join(i.files[0].path) == "file1.txt"
    assert i.files[1].length == 525148160 and "/".join(i.files[1].path) == "dir/file2.txt"
    assert i.length == 447135744 + 525148160  # metainfo.ts:125


def test_parse_minimal_extra_missing():  # metainfo_test.ts:61-111
    m = parse_metainfo(_load("minimal.torrent"))
    assert m is not None and m.info.private == 0 and m.comment is None and m.created_by is None
    assert parse_metainfo(_load("extra.torrent")) is not None
    assert parse_metainfo(_load("missing.torrent")) is None
    assert parse_metainfo(b"not bencode") is None


def test_bencode_roundtrip_and_insertion_order():
    d = {"b": 1, "a": [b"x", "y", {"z": -3}], "skip": None}
    enc = _bencode(d)
    assert enc == b"d1:bi1e1:al1:x1:yd1:zi-3eeee"  # insertion order, None skipped (bencode.ts:56-64)
    dec = _bdecode(enc)
    assert dec["b"] == 1 and bytes(dec["a"][0]) == b"x" and dec["a"][2]["z"] == -3
    with pytest.raises(ValueError):
        _bdecode(b"i12")


def test_encode_metainfo_roundtrip():
    info = make_info(1 << 20, bytes(range(40)), "x", files=[FileInfo(5, ["a"]), FileInfo(7, ["d", "b"])])
    m = parse_metainfo(encode_metainfo(info))
    assert m.info.piece_length == 1 << 20 and m.info.length == 12 and m.info.pieces_raw == bytes(range(40))
    assert [f.path for f in m.info.files] == [["a"], ["d", "b"]]


def test_partition_ragged():  # _bytes.ts:92-99
    assert [len(x) for x in partition(bytes(47), 20)] == [20, 20, 7]
    assert partition(b"", 20) == []


# ---- piece.ts -----------------------------------------------------------------------------

def test_piece_length_rule():
    info = make_info(4096, bytes(20 * 10), "x", length=9 * 4096 + 5)
    assert piece_length(9, info) == 5 and piece_length(8, info) == 4096
    info2 = make_info(4096, bytes(20 * 10), "x", length=10 * 4096)
    assert piece_length(9, info2) == 4096


def test_validate_blocks():
    info = make_info(2 * BLOCK_SIZE, bytes(20 * 3), "x", length=2 * 2 * BLOCK_SIZE + 100)
    validate_requested_block(info, RequestMsg(0, 0, BLOCK_SIZE))
    with pytest.raises(ValueError, match="invalid piece index"):
        validate_requested_block(info, RequestMsg(3, 0, 1))
    with pytest.raises(ValueError, match="invalid block length"):
        validate_requested_block(info, RequestMsg(2, 0, 101))
    validate_received_block(info, PieceMsg(2, 0, bytes(100)))
    with pytest.raises(ValueError, match="invalid block offset"):
        validate_received_block(info, PieceMsg(0, 5, bytes(BLOCK_SIZE)))
    with pytest.raises(ValueError, match="invalid last block length"):
        validate_received_block(info, PieceMsg(2, 0, bytes(99)))
    with pytest.raises(ValueError, match="invalid block length"):
        validate_received_block(info, PieceMsg(0, 0, bytes(7)))


# ---- storage_test.ts -------------------------------------------------------------------------

BASE_MULTI = make_info(32 * 1024, bytes(20), "__test", files=[FileInfo(16 * 1024 + 10, ["__test1.txt"]),
                                                              FileInfo(16 * 1024 - 11, ["__test2.txt"])])


class Recorder:
    def __init__(self, results):
        self.calls = []
        self.results = list(results)

    def get(self, path, offset, length):
        self.calls.append((list(path), offset, length))
        return self.results.pop(0)

    def set(self, path, offset, data):
        self.calls.append((list(path), offset, bytes(data)))
        return True

    def exists(self, path):
        return True


def test_storage_get_across_files():  # storage_test.ts:180-204
    vals = os.urandom(16 * 1024 - 1)
    rec = Recorder([vals[:10], vals[10:]])
    st = Storage(rec, BASE_MULTI, os.getcwd())
    assert st.get(16 * 1024, 16 * 1024 - 1) == vals
    assert rec.calls == [(["__test1.txt"], 16 * 1024, 10), (["__test2.txt"], 0, 16 * 1024 - 11)]


def test_storage_get_inside_one_file():  # storage_test.ts:161-178
    vals = os.urandom(16 * 1024)
    rec = Recorder([vals])
    st = Storage(rec, BASE_MULTI, os.getcwd())
    assert st.get(0, 16 * 1024) == vals
    assert rec.calls == [(["__test1.txt"], 0, 16 * 1024)]


def test_storage_fails_if_method_fails():  # storage_test.ts:206-228
    st = Storage(Recorder([None]), BASE_MULTI, os.getcwd())
    assert st.get(0, 10) is None

    class Boom(Recorder):
        def get(self, *a):
            raise RuntimeError("x")
    assert Storage(Boom([]), BASE_MULTI, os.getcwd()).get(0, 10) is None


def test_storage_get_short_and_long_method_results():
    """storage.ts:51,57-58: a StorageMethod.get that returns FEWER bytes than asked fills the front of its slice
    of the zeroed Uint8Array (slice.set(got)) and the get succeeds; MORE bytes make slice.set throw a RangeError,
    which findAndDo's catch turns into false (:130-133): null.  (no reference fixture pins this, so
    the expectation is the reference's code read as written.)"""
    vals = os.urandom(16 * 1024)
    # inside one file
    st = Storage(Recorder([vals[:100]]), BASE_MULTI, os.getcwd())
    assert st.get(0, 1000) == vals[:100] + bytes(900)
    assert Storage(Recorder([vals[:1001]]), BASE_MULTI, os.getcwd()).get(0, 1000) is None
    assert Storage(Recorder([b""]), BASE_MULTI, os.getcwd()).get(0, 10) == bytes(10)   # (an empty array is truthy)
    # across files: each segment's slice is filled from its own front
    rec = Recorder([vals[:4], vals[10:20]])
    got = Storage(rec, BASE_MULTI, os.getcwd()).get(16 * 1024, 30)
    assert got == vals[:4] + bytes(6) + vals[10:20] + bytes(10)
    assert Storage(Recorder([vals[:11], vals[:5]]), BASE_MULTI, os.getcwd()).get(16 * 1024, 30) is None


def test_storage_set_across_files_and_dedupe():  # storage_test.ts:313-335, storage.ts:67-87
    rec = Recorder([])
    st = Storage(rec, BASE_MULTI, os.getcwd())
    data = os.urandom(16 * 1024 - 1)
    assert st.set(16 * 1024, data)
    assert rec.calls == [(["__test1.txt"], 16 * 1024, data[:10]), (["__test2.txt"], 0, data[10:])]
    assert st.set(16 * 1024, data) and len(rec.calls) == 2  # same block: not written again


def test_segments_quirks():
    # zero-length segment at an exact boundary (storage.ts:109-110); past the end -> None (:136)
    info = make_info(8, bytes(20), "t", files=[FileInfo(8, ["a"]), FileInfo(0, ["z"]), FileInfo(8, ["b"])])
    st = Storage(MemoryStorage(), info, os.getcwd())
    assert st.segments(8, 8) == [(["a"], 8, 0, 0), (["z"], 0, 0, 0), (["b"], 0, 8, 0)]
    assert st.segments(12, 8) is None
    single = make_info(8, bytes(20), "s.bin", length=8)
    assert Storage(MemoryStorage(), single, os.path.join(os.getcwd(), "dl")).segments(3, 4) == [(["dl", "s.bin"], 3, 4, 0)]


def test_zero_length_segments_equal_the_walk():
    """Storage.zero_length_segments lists exactly the zero-length entries of segments(i*L, len_i) over every
    piece of a range (storage.ts:109-110: `fileEnd >= offset` at a piece start, and zero-length files), with
    the file offset the walk gives them, on random layouts full of zero-length files and exact boundaries."""
    rng = random.Random(5)
    for trial in range(60):
        L = rng.choice([16, 64, 100])
        sizes = [rng.choice([0, 0, 1, L, 2 * L, rng.randint(0, 3 * L)]) for _ in range(rng.randint(1, 25))]
        if sum(sizes) == 0:
            sizes.append(L + 3)
        total = sum(sizes)
        P = -(-total // L)
        info = make_info(L, bytes(20 * P), "t", files=[FileInfo(n, [f"f{k}"]) for k, n in enumerate(sizes)])
        st = Storage(MemoryStorage(), info, "/tmp/seg")
        first = rng.randrange(P)
        count = rng.randint(1, P - first)
        want = []
        for i in range(first, first + count):
            for path, foff, n, s0 in st.segments(i * L, piece_length(i, info)) or ():
                if n == 0:
                    want.append((int(path[-1][1:]), foff, i * L + s0))
        hi = (first + count - 1) * L + piece_length(first + count - 1, info)
        k, fo, lin = st.zero_length_segments(first * L, hi - first * L, L)
        assert sorted(zip(k.tolist(), fo.tolist(), lin.tolist())) == sorted(want), (trial, sizes, first, count)
        assert all(first <= x // L < first + count for x in lin.tolist())


@pytest.mark.parametrize("dir_path", ["/tmp/seg", "/", "", "/tmp/seg/"])
def test_segment_arrays_equal_the_walk(dir_path):
    """Storage.segment_arrays (the vectorised walk verify_files stages from) equals segments() minus
    its zero-length entries, with the same None cases, on random layouts full of zero-length and tiny
    files and random (offset, length) ranges, including past-the-end ones; file_paths() equals
    os.path.join of each segment's path."""
    import random
    rnd = random.Random(11)
    d = dir_path or os.getcwd()
    for _ in range(300):
        sizes = [rnd.choice([0, 0, 1, 5, 64, 100, 4096]) for _ in range(rnd.randrange(1, 12))]
        total = sum(sizes)
        if total == 0:
            continue
        info = make_info(64, bytes(20 * (-(-total // 64))), "t",
                         files=[FileInfo(n, [f"d{k % 3}", f"f{k}"]) for k, n in enumerate(sizes)])
        st = Storage(MemoryStorage(), info, d)
        paths = st.file_paths()
        for _ in range(20):
            off, ln = rnd.randrange(0, total + 3), rnd.randrange(0, total + 3)
            walk, arrs = st.segments(off, ln), st.segment_arrays(off, ln)
            if walk is None:
                assert arrs is None, (sizes, off, ln)
                continue
            assert arrs is not None, (sizes, off, ln)
            want = [(os.path.join(*p), fo, n, s0) for p, fo, n, s0 in walk if n > 0]
            assert [(paths[k], int(fo), int(n), int(s0)) for k, fo, n, s0 in zip(*arrs)] == want
    single = make_info(8, bytes(20), "s.bin", length=8)
    st = Storage(MemoryStorage(), single, os.path.join(os.getcwd(), "dl"))
    k, fo, n, s0 = st.segment_arrays(3, 4)
    assert (st.file_paths()[int(k[0])], int(fo[0]), int(n[0]), int(s0[0])) == (os.path.join("dl", "s.bin"), 3, 4, 0)


def test_fs_storage(tmp_path):  # storage_test.ts:41-62
    p = tmp_path / "__test.txt"
    p.write_bytes(bytes([1, 2, 3, 4, 5, 6, 7, 8]))
    fs = FsStorage()
    assert list(fs.get([str(p)], 2, 4)) == [3, 4, 5, 6]
    assert fs.get([str(p)], 7, 4) is None                 # reading fails (EOF)
    missing = tmp_path / "nope.txt"
    assert fs.get([str(missing)], 2, 4) is None           # doesn't exist ...
    assert missing.exists()                               # ... but is created (OPEN_OPTIONS create: true)
    assert fs.set([str(tmp_path / "d" / "x.bin")], 3, b"abc") and (tmp_path / "d" / "x.bin").read_bytes() == b"\0\0\0abc"
    assert fs.exists([str(p)]) and not fs.exists([str(tmp_path / "zz")])


def test_fs_storage_fault_injection(tmp_path, monkeypatch):
    """storage_test.ts:96-108 patches Deno.FsFile.prototype.seek to throw: get -> null, set ->
    false.  Here the positional read/write itself throws.  verify_files uses its own preads and
    turns the same failure into an unreadable piece (bit 0)."""
    import torrent_amd.storage as S
    p = tmp_path / "f.bin"
    p.write_bytes(b"x" * 64)

    def boom(*a, **k):
        raise OSError(5, "injected I/O error")

    monkeypatch.setattr(S.os, "pread", boom)
    monkeypatch.setattr(S.os, "pwrite", boom)
    fs = S.FsStorage()
    assert fs.get([str(p)], 0, 8) is None
    assert fs.set([str(p)], 0, b"abc") is False
    info = make_info(32, bytes(40), "f.bin", length=64)
    st = Storage(fs, info, str(tmp_path))
    assert st.get(0, 32) is None and st.set(0, b"y" * 16) is False


def test_layout_segments_agree_with_storage(oracle):
    """The seeded multi-file layouts: Storage.get over a MemoryStorage of the on-disk files
    returns exactly the layout's expected piece bytes (including missing / short files)."""
    from tests.layouts import LAYOUTS, build_layout
    for spec in LAYOUTS:
        if spec.get("big"):
            continue
        lay = build_layout(spec)
        info = lay["info"]
        st = Storage(MemoryStorage(lay["disk_files"]()), info, os.getcwd())
        for i in range(lay["n_pieces"]):
            got = st.get(i * info.piece_length, piece_length(i, info))
            exp = lay["read_piece"](i)
            assert (got is None) == (exp is None), (spec["name"], i)
            if got is not None:
                assert bytes(got) == exp


def test_golden_layout_bitfields_match_oracle(oracle):
    """The committed expected bitfields (hashlib) equal the oracle on the regenerated layouts."""
    import hashlib
    import json
    from tests.layouts import build_layout, by_name
    for rec in json.load(open(os.path.join(GOLDEN, "layouts.json"))):
        if rec["name"] == "cfg3":
            continue  # 2.6 GB: covered by the GPU test
        lay = build_layout(by_name(rec["name"]))
        assert hashlib.sha1(lay["pieces_raw"]).hexdigest() == rec["pieces_sha1"]
        bf = oracle.verify_linear(lay["payload"], lay["total_length"], lay["info"].piece_length,
                                  lay["pieces_raw"], lay["avail"])
        assert bf.hex() == rec["expected_bitfield"], rec["name"]


def test_shard_ranges_byte_aligned():
    for P in [0, 1, 7, 8, 9, 1706, 51200, 16384]:
        for n in [1, 2, 3, 4, 8]:
            rs = shard_ranges(P, n)
            assert len(rs) == n
            assert sum(c for _, c in rs) == P
            pos = 0
            for f, c in rs:
                assert f == pos and (f % 8 == 0 or c == 0)
                pos += c


@pytest.mark.parametrize("name", ["singlefile", "multifile"])
def test_info_hash_is_sha1_of_the_original_info_bytes(name):
    """f4 (metainfo.ts:141-143): infoHash = SHA-1(bencode(decoded.info)).  Re-encoding in
    insertion order reproduces the .torrent's own info bytes, so the hash equals SHA-1 of the
    info slice of the file (what every BitTorrent peer and tracker uses)."""
    import hashlib
    data = _load(f"{name}.torrent")
    m = parse_metainfo(data)
    start = data.index(b"4:info") + len(b"4:info")
    assert data.endswith(b"e")
    raw_info = data[start:-1]                       # "info" is the last key of the top-level dict
    assert _bencode(_bdecode(raw_info)) == raw_info
    assert m.info_hash == hashlib.sha1(raw_info).digest()


def _fs_openable(path: str) -> bool:
    """Would fsStorage.get's Deno.open(path, {read, write, create}) succeed (storage.ts:28-32,158)?  Without
    creating anything: an existing non-directory with read + write access, or a missing file in an existing,
    writable directory.  (The CPU stand-in's copy of tv_core.hip fs_openable.)"""
    import stat
    try:
        st = os.stat(path)
    except FileNotFoundError:
        parent = os.path.dirname(path) or "."
        return os.path.isdir(parent) and os.access(parent, os.W_OK | os.X_OK)
    except OSError:
        return False
    return not stat.S_ISDIR(st.st_mode) and os.access(path, os.R_OK | os.W_OK)


class _ImageCtx:
    """Stand-in for a tv_ctx on CPU: tv_stage_files writes into a linear image of the shard, so
    verify_files' staging plan (the storage.ts segment mapping, one batched call) is checked without a GPU.
    Files are read the way the library reads them, and a failed segment is handled as tv_files.hip
    recover_segment does (restated): the whole pieces of the file's readable prefix are staged, the pieces
    from the first unreadable byte to the segment's end are marked (`bad`, linear piece indices), and a
    failed zero-length segment marks its piece."""

    def __init__(self, total, lo, hi, L):
        self.img = bytearray(total)
        self.written = bytearray(total)
        self.lo, self.hi, self.L = lo, hi, L
        self.calls = 0
        self.bad = set()

    def _mark(self, a, b):
        if a == b:
            if self.lo <= a < self.hi:
                self.bad.add(a // self.L)
            return
        a, b = max(a, self.lo), min(b, self.hi)
        self.bad |= set(range(a // self.L, (b - 1) // self.L + 1)) if b > a else set()

    def avail(self, host_bits, first, count):
        """The bits tv_verify applies: the host's availability and not the marked pieces."""
        return [bool((host_bits[j >> 3] >> (7 - (j & 7))) & 1) and first + j not in self.bad for j in range(count)]

    def set_option(self, key, value):
        pass

    def _put(self, off, data):
        a, b = max(off, self.lo), min(off + len(data), self.hi)
        if b > a:
            self.img[a:b] = data[a - off:b - off]
            for k in range(a, b):
                assert not self.written[k], f"byte {k} staged twice"
                self.written[k] = 1

    def stage_files(self, paths, file_offsets, linear_offsets, lens):
        self.calls += 1
        out = []
        for path, foff, off, n in zip(paths, file_offsets, linear_offsets, lens):
            foff, off, n = int(foff), int(off), int(n)
            if n == 0:   # the library's zero-length rule (tv_core.hip fs_openable), restated
                ok = _fs_openable(path)
                out.append(0 if ok else -5)
                if not ok:
                    self._mark(off, off)
                continue
            data = b""
            if _fs_openable(path) and os.path.isfile(path):
                with open(path, "rb") as f:
                    f.seek(foff)
                    data = f.read(n)
            if len(data) == n:
                self._put(off, data)
                out.append(0)
                continue
            r = max(0, (off + len(data)) // self.L * self.L - off)    # the prefix's whole pieces
            self._put(off, data[:r])
            self._mark(off + r, off + n)
            out.append(-5)
        return out


@pytest.mark.parametrize("layout", ["missing_and_short", "multi_zero_tiny", "single_short_last"])
def test_files_shard_staging_plan(tmp_path, monkeypatch, layout):
    """verify_files' staging plan on CPU: one tv_stage_files call per shard stages every readable byte
    of the shard exactly once at its linear offset, and the availability bits are exactly the pieces
    whose bytes are all on disk (storage.ts:150-172 null -> 0), over 3 shards."""
    from tests.layouts import build_layout, by_name
    from torrent_amd import verify
    from torrent_amd.storage import Storage, fs_storage

    lay = build_layout(by_name(layout))
    info = lay["info"]
    for path, data in lay["disk_files"]().items():
        p = tmp_path.joinpath(*path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
    monkeypatch.chdir(tmp_path)
    st = Storage(fs_storage, info, str(tmp_path))
    L, P, total = info.piece_length, info.n_pieces, info.length
    for first, count in verify.shard_ranges(P, 3):
        if not count:
            continue
        hi = (first + count - 1) * L + (total % L if first + count == P and total % L else L)
        ctx = _ImageCtx(total, first * L, hi, L)
        avail = ctx.avail(verify._files_shard(ctx, info, st, first, count, threads=4), first, count)
        assert ctx.calls == 1
        for j in range(count):
            i = first + j
            want = (lay["avail"][i >> 3] >> (7 - (i & 7))) & 1
            assert avail[j] == want, (layout, i)
            if want:
                a, b = i * L, min(total, (i + 1) * L)
                assert ctx.img[a:b] == lay["payload"][a:b], (layout, i)
                assert all(ctx.written[a:b]), (layout, i)


def test_cli_usage_without_a_gpu(capsys):
    """Both command lines print their usage on bad arguments without touching the library."""
    from torrent_amd.__main__ import main as verify_main
    from torrent_amd.make_torrent import main as make_main
    assert verify_main([]) == 2 and "python -m torrent_amd verify" in capsys.readouterr().out
    assert make_main(["--help"]) == 0 and "make_torrent [-c <comment>] -t <tracker url> <target>" in capsys.readouterr().out


def test_files_shard_zero_length_segments_match_fs_storage(tmp_path, monkeypatch):
    """Zero-length segments (storage.ts:109-110 `fileEnd >= offset`; zero-length files) are still opened by
    fsStorage.get (storage.ts:158): a directory in a zero-length file's place, or a zero-length file in a
    missing directory, makes the piece null; a missing zero-length file in an existing directory is
    created there and reads fine.  verify_files' plan gives the same bits as Storage(fs_storage).get per
    piece (run on a copy of the tree, since that get creates files), without creating any file itself."""
    import shutil
    from torrent_amd import verify
    from torrent_amd.storage import Storage, fs_storage

    L = 4096
    names = [("a",), ("z_dir",), ("b",), ("nodir", "z"), ("c",), ("z_missing",), ("d",), ("z_ok",), ("e",)]
    sizes = [3 * L, 0, 2 * L + 100, 0, L - 100, 0, 2 * L, 0, L + 7]   # a, b end exactly on piece starts
    payload = bytes((k * 13 + 1) & 0xFF for k in range(sum(sizes)))
    P = -(-len(payload) // L)
    info = make_info(L, bytes(20 * P), "t", files=[FileInfo(n, list(p)) for n, p in zip(sizes, names)])
    root = tmp_path / "t0"
    off = 0
    for n, p in zip(sizes, names):
        q = root.joinpath(*p)
        if p == ("z_dir",):
            q.mkdir(parents=True)
        elif p in (("nodir", "z"), ("z_missing",)):
            pass                                                   # missing (nodir/ does not exist)
        else:
            q.parent.mkdir(parents=True, exist_ok=True)
            q.write_bytes(payload[off:off + n])
        off += n
    ref_root = tmp_path / "t1"
    shutil.copytree(root, ref_root)
    monkeypatch.chdir(tmp_path)
    ref = Storage(fs_storage, info, str(ref_root))
    expect = [ref.get(i * L, piece_length(i, info)) is not None for i in range(P)]
    assert not all(expect) and any(expect)
    before = sorted(str(x) for x in root.rglob("*"))
    st = Storage(fs_storage, info, str(root))
    got = []
    for first, count in verify.shard_ranges(P, 2):
        if not count:
            continue
        hi = (first + count - 1) * L + piece_length(first + count - 1, info)
        ctx = _ImageCtx(info.length, first * L, hi, L)
        got += ctx.avail(verify._files_shard(ctx, info, st, first, count, threads=2), first, count)
    assert got == expect
    assert sorted(str(x) for x in root.rglob("*")) == before      # nothing created


def test_file_paths_equal_os_path_join():
    """Storage.file_paths' fast join equals os.path.join(*dir, *path) (fsStorage.get's join, storage.ts:153)
    for every kind of part: empty, absolute, containing separators."""
    cases = [["a"], ["a", "b"], ["", "a"], ["a", ""], ["/abs"], ["a", "/b"], ["a", "", "b"], ["a/b"], ["a//b"],
             ["a/"], ["x", "y", "z"]]
    for d in ["/tmp/x", "/", "rel/dir", ".", "/tmp/x/"]:
        info = make_info(4096, bytes(20), "t", files=[FileInfo(1, c) for c in cases])
        st = Storage(FsStorage(), info, d)
        assert st.file_paths() == [os.path.join(*st.dir_path, *c) for c in cases], d


def test_chunked_map_keeps_order_and_splits_into_runs():
    """verify._chunked_map (the Storage paths' reader dispatch): results in index order for any run count, one pool
    task per contiguous run (never per index), and in the calling thread without a pool."""
    from concurrent.futures import ThreadPoolExecutor
    import threading
    from torrent_amd import verify

    seen = []

    def fn(q):
        seen.append((q, threading.get_ident()))
        return q * q

    assert verify._chunked_map(None, fn, 5, 4) == [0, 1, 4, 9, 16]
    assert {t for _, t in seen} == {threading.get_ident()}
    with ThreadPoolExecutor(4) as pool:
        for n, parts in [(0, 4), (1, 4), (3, 4), (10, 4), (17, 3), (100, 1), (7, 16)]:
            seen.clear()
            assert verify._chunked_map(pool, fn, n, parts) == [q * q for q in range(n)], (n, parts)
            # each run is handled by one thread, in order: indices of one thread are consecutive and ascending
            by_thread = {}
            for q, t in seen:
                by_thread.setdefault(t, []).append(q)
            for qs in by_thread.values():
                assert qs == sorted(qs)
    assert verify._STORAGE_THREADS == 4
