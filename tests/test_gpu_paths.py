"""GPU parity through the host-side API (verify_pieces / verify_payload / verify_piece / hash_pieces)
on the reference's own fixtures, the seeded multi-file layouts (incl. BASELINE config 3) and a
full-size config-2 run checked through size-independent properties."""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


def _ref_payload(name):
    rd = json.load(open(os.path.join(GOLDEN, "refdata.json")))[name]
    return b"".join(f["pattern"].encode() * (f["length"] // len(f["pattern"])) for f in rd["files"])


def _all_ones(P):
    b = bytearray(b"\xff" * (P // 8))
    if P % 8:
        b.append((0xFF00 >> (P % 8)) & 0xFF)
    return bytes(b)


@pytest.mark.parametrize("name", ["singlefile", "multifile"])
@pytest.mark.parametrize("resident", [True, False])
def test_reference_fixtures_on_gpu(native, name, resident):
    """The reference's test_data digests (produced by its own SHA-1 path) verify on the GPU:
    all 1706 / 1855 pieces, including the short final piece and the file-spanning piece #852."""
    from torrent_amd import parse_metainfo, verify_payload
    info = parse_metainfo(_load(f"{name}.torrent")).info
    payload = bytearray(_ref_payload(name))
    P = info.n_pieces
    assert bytes(verify_payload(info, payload, resident=resident)) == _all_ones(P)
    flips = [0, 852, P - 1]
    for i in flips:
        payload[i * info.piece_length + 3] ^= 0x01
    bf = verify_payload(info, payload, resident=resident)
    for i in range(P):
        assert ((bf[i >> 3] >> (7 - (i & 7))) & 1) == (0 if i in flips else 1), i


def test_reference_multifile_through_storage(native):
    """verify_pieces(info, Storage(...)) -- the reference-shaped API over its StorageMethod plugin --
    on the multifile fixture (two files, piece #852 spans them)."""
    from torrent_amd import MemoryStorage, Storage, parse_metainfo, verify_pieces
    info = parse_metainfo(_load("multifile.torrent")).info
    payload = _ref_payload("multifile")
    n0 = info.files[0].length
    mem = MemoryStorage({tuple(info.files[0].path): payload[:n0], tuple(info.files[1].path): payload[n0:]})
    st = Storage(mem, info, os.getcwd())
    assert bytes(verify_pieces(info, st)) == _all_ones(info.n_pieces)
    # truncate file 2 (a short file on disk): pieces touching the missing tail are unreadable -> 0
    mem.files[tuple(info.files[1].path)] = mem.files[tuple(info.files[1].path)][:1000]
    bf = verify_pieces(info, Storage(mem, info, os.getcwd()))
    L = info.piece_length
    for i in range(info.n_pieces):
        end = i * L + (info.length % L if i == info.n_pieces - 1 else L)
        readable = end <= n0 + 1000
        assert ((bf[i >> 3] >> (7 - (i & 7))) & 1) == (1 if readable else 0), i


@pytest.mark.parametrize("layout", ["single_short_last", "multi_zero_tiny", "many_tiny_span",
                                    "missing_and_short", "exact_multiple", "cfg1", "cfg3"])
def test_golden_layouts_on_gpu(native, layout):
    """Seeded layouts: GPU bitfield == committed expected bitfield (hashlib-computed)."""
    from tests.layouts import build_layout, by_name
    from torrent_amd import verify_payload
    rec = {r["name"]: r for r in json.load(open(os.path.join(GOLDEN, "layouts.json")))}[layout]
    lay = build_layout(by_name(layout))
    assert hashlib.sha1(lay["pieces_raw"]).hexdigest() == rec["pieces_sha1"]
    bf = verify_payload(lay["info"], lay["payload"], avail=lay["avail"])
    assert bytes(bf).hex() == rec["expected_bitfield"]
    for i in lay["corrupted"]:
        assert not (bf[i >> 3] >> (7 - (i & 7))) & 1


@pytest.mark.parametrize("layout", ["multi_zero_tiny", "missing_and_short"])
def test_layout_through_fs_storage(native, tmp_path, layout):
    """Real files on disk through fs_storage (missing / truncated files included)."""
    from tests.layouts import build_layout, by_name
    from torrent_amd import Storage, fs_storage, verify_pieces
    rec = {r["name"]: r for r in json.load(open(os.path.join(GOLDEN, "layouts.json")))}[layout]
    lay = build_layout(by_name(layout))
    for path, data in lay["disk_files"]().items():
        p = tmp_path.joinpath(*path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        bf = verify_pieces(lay["info"], Storage(fs_storage, lay["info"], str(tmp_path)))
    finally:
        os.chdir(cwd)
    assert bytes(bf).hex() == rec["expected_bitfield"]


def test_creation_mode_matches_reference_digests(native):
    """hash_pieces (GPU creation mode, make_torrent.ts:147-173) reproduces info.pieces."""
    from torrent_amd import hash_pieces, parse_metainfo
    info = parse_metainfo(_load("multifile.torrent")).info
    assert hash_pieces(_ref_payload("multifile"), info.piece_length) == info.pieces_raw


def test_verify_piece_api(native):
    from torrent_amd import parse_metainfo, verify_piece
    info = parse_metainfo(_load("singlefile.torrent")).info
    payload = _ref_payload("singlefile")
    L, P = info.piece_length, info.n_pieces
    assert verify_piece(info, 0, payload[:L])
    assert verify_piece(info, P - 1, payload[(P - 1) * L:])          # short final piece
    assert not verify_piece(info, 1, payload[:L - 1])                # wrong length
    bad = bytearray(payload[:L]); bad[5] ^= 1
    assert not verify_piece(info, 0, bad)
    with pytest.raises(ValueError):
        verify_piece(info, P, b"x")


def test_multi_device_api_on_one_gpu(native, oracle):
    """devices=[0, 0, 0]: three shards on the same GPU, concatenated (the multi-GPU host path)."""
    from torrent_amd import make_info, verify_payload
    L, P = 8192, 300
    total = L * (P - 1) + 4000
    payload = oracle.synth_fill(31, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    for i in (5, 150, 299):
        pieces[20 * i] ^= 2
    info = make_info(L, bytes(pieces), "x", length=total)
    exp = oracle.verify_linear(payload, total, L, bytes(pieces))
    assert bytes(verify_payload(info, payload, devices=[0, 0, 0])) == exp


@pytest.mark.parametrize("P,ndev", [(1, 2), (9, 4), (50, 8), (3, 8)])
def test_small_torrents_on_many_devices(native, oracle, tmp_path, P, ndev):
    """Fewer pieces than 8 x devices: shard_ranges gives trailing EMPTY shards starting at a piece that need
    not be a multiple of 8 (P = 1 on 2 devices, 9 on 4, 50 on 8).  Every entry point (verify_payload resident
    and streamed from host, verify_stream, verify_pieces over a Storage, verify_files from disk, hash_pieces)
    returns the oracle's bits / digests, like the single-device call."""
    from torrent_amd import (MemoryStorage, Storage, hash_pieces, make_info, shard_ranges, verify_files,
                             verify_payload, verify_pieces, verify_stream)
    assert any(c == 0 and f % 8 for f, c in shard_ranges(P, ndev)) or P == 3
    L = 4096
    total = L * (P - 1) + 1000
    payload = oracle.synth_fill(P * 7 + ndev, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    pieces[20 * (P - 1)] ^= 1                      # the last piece fails
    info = make_info(L, bytes(pieces), "small.bin", length=total)
    expect = oracle.verify_linear(payload, total, L, bytes(pieces))
    devs = [0] * ndev
    assert bytes(verify_payload(info, payload, devices=devs)) == expect
    assert bytes(verify_payload(info, payload, devices=devs, resident=False)) == expect
    assert bytes(verify_stream(info, lambda o, n: bytes(payload[o:o + n]), devices=devs)) == expect
    mem = MemoryStorage({("small.bin",): bytes(payload)})
    assert bytes(verify_pieces(info, Storage(mem, info, os.getcwd()), devices=devs)) == expect
    (tmp_path / "small.bin").write_bytes(bytes(payload))
    assert bytes(verify_files(info, str(tmp_path), devices=devs)) == expect
    assert hash_pieces(bytes(payload), L, devices=devs) == oracle.hash_pieces(payload, total, L, P)


def test_full_size_cfg2_oracle_ground_truth(native, oracle):
    """BASELINE config 2 at full size (16 GiB, 16,384 x 1 MiB, HBM-resident) against the ORACLE on every
    piece: the CPU oracle hashes the whole synthetic torrent on the host's cores (the reference's SHA-1
    path, make_torrent.ts:28-31); the GPU's creation-mode digests equal it byte for byte, and verify with
    the oracle's digests (1 % corrupted) gives exactly the oracle's bitfield with every kernel."""
    L, P = 1 << 20, 16384
    total = L * P
    truth = oracle.synth_piece_digests(2, total, L, P, threads=_threads())
    bad = set(range(3, P, 97))
    d2 = bytearray(truth)
    for i in bad:
        d2[20 * i + 19] ^= 0x80
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.fill_synthetic(2)
        assert ctx.hash() == truth
        ctx.set_digests(bytes(d2))
        for k in (1, 2, 4):
            ctx.set_option(native.TV_OPT_KERNEL, k)
            bf = ctx.verify()
            assert ctx.last_kernel()[0] == k
            assert {i for i in range(P) if not (bf[i >> 3] >> (7 - (i & 7))) & 1} == bad, k


def _threads():
    try:
        import bench
        return bench.cpu_share()["cores"]
    except Exception:
        return 8


def test_full_size_cfg4_oracle_ground_truth(native, oracle):
    """BASELINE config 4 at its largest single-GPU size: 200 GiB, 51,200 x 4 MiB pieces resident in HBM
    (linear offsets to 214,748,364,800), against the ORACLE's digests of all 51,200 pieces: creation mode
    equals them; verify with them (1 % corrupted) is exact with the lane, split and twin kernels; and the 8-GPU
    shard geometry of the same torrent (the last shard, pieces [44800, 51200), at linear offsets > 187 GB)
    hashes and verifies to the oracle's slice."""
    from torrent_amd import release_contexts, shard_ranges
    release_contexts()  # no cached context may hold HBM while 200 GiB is resident
    L, P = 4 << 20, 51200
    total = L * P
    truth = oracle.synth_piece_digests(4, total, L, P, threads=_threads())
    bad = set(range(5, P, 100)) | {P - 1}
    d2 = bytearray(truth)
    for i in bad:
        d2[20 * i] ^= 0x01
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.fill_synthetic(4)
        assert ctx.hash() == truth
        assert ctx.last_kernel()[0] == 1      # auto at 51,200 pieces: lane
        ctx.set_digests(bytes(d2))
        for k in (1, 2, 4):
            ctx.set_option(native.TV_OPT_KERNEL, k)
            bf = ctx.verify()
            assert ctx.last_kernel()[0] == k
            got = {i for i in range(P) if not (bf[i >> 3] >> (7 - (i & 7))) & 1}
            assert got == bad, (k, sorted(got ^ bad)[:10])
        ctx.set_option(native.TV_OPT_KERNEL, 1)
        ctx.set_option(native.TV_OPT_LANE_PAIRS, 1)        # the lane kernel's pair loads (auto picks them >= 65,536)
        bf = ctx.verify()
        got = {i for i in range(P) if not (bf[i >> 3] >> (7 - (i & 7))) & 1}
        assert got == bad, ("lane pairs", sorted(got ^ bad)[:10])
    first, count = shard_ranges(P, 8)[7]
    assert (first, count) == (44800, 6400)
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P, first, count)
        ctx.fill_synthetic(4)
        assert ctx.hash() == truth[20 * first:20 * (first + count)]
        ctx.set_digests(bytes(d2))
        bf = ctx.verify()
        for j in range(count):
            assert ((bf[j >> 3] >> (7 - (j & 7))) & 1) == (0 if first + j in bad else 1), j


def test_read_back_and_pinned_stream(native, oracle):
    """tv_read returns exactly the staged linear bytes (incl. a short last piece and a shard
    window), and tv_verify_host from a pinned (tv_host_alloc) source matches the oracle."""
    L, P = 65536, 130
    total = L * (P - 1) + 12345
    payload = oracle.synth_fill(41, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    pieces[20 * 77] ^= 1
    payload[5 * L + 9] ^= 4
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P, 8, 120)
        ctx.stage(0, payload)
        out = bytearray(total)
        ctx.read(0, out)
        lo, hi = 8 * L, 128 * L
        assert out[lo:hi] == payload[lo:hi] and out[:lo] == bytes(lo)
        part = bytearray(1000)
        ctx.read(9 * L - 500, part)
        assert part == payload[9 * L - 500:9 * L + 500]
    exp = oracle.verify_linear(payload, total, L, bytes(pieces))
    with native.Context(0) as ctx, native.PinnedBuffer(total) as pb:
        pb.mv[:] = payload
        ctx.set_option(native.TV_OPT_STREAM_CHUNK, 16384)
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        assert ctx.verify_host(pb.mv) == exp
        assert ctx.last_kernel()[1] == 4  # 64 KiB pieces in 16 KiB columns


@pytest.mark.parametrize("kernel", [0, 1, 2, 4])
def test_verify_list_matches_oracle(native, oracle, kernel):
    """tv_verify_list (auto / lane list kernel / split and twin kernels in list mode): arbitrary order,
    duplicates, the short last piece in any lane position, corrupted pieces, a shard offset;
    > 256 entries (several workgroups)."""
    import random
    L, P = 16384, 700
    total = L * (P - 1) + 333
    payload = oracle.synth_fill(55, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    bad = {3, 64, 65, 400, P - 1}
    for i in bad:
        pieces[20 * i + 1] ^= 0x40
    rng = random.Random(5)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_KERNEL, kernel)
        ctx.set_layout(total, L, P, 8, P - 8)
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload)
        lst = [rng.randrange(8, P) for _ in range(600)] + [P - 1, P - 1, 8, 9]
        rng.shuffle(lst)
        got = ctx.verify_list(lst)
        assert ctx.last_kernel()[0] == (kernel or 4)
        assert list(got) == [0 if i in bad else 1 for i in lst]
        with pytest.raises(native.NativeError):
            ctx.verify_list([0])          # outside the shard
        # only the last piece (a wave whose every lane is the short piece)
        assert ctx.verify_list([P - 1] * 70) == bytes(70)
        pieces[20 * (P - 1) + 1] ^= 0x40
        ctx.set_digests(bytes(pieces))
        assert ctx.verify_list([P - 1] * 70) == b"\x01" * 70


def test_incremental_verifier_flow(native, oracle):
    """Blocks arrive in random order through the reference-shaped handler; completed pieces are
    verified in batches; a corrupted block yields a 0 and the piece can be re-received."""
    import random
    from torrent_amd import MemoryStorage, Storage, make_info
    from torrent_amd.incremental import IncrementalVerifier
    from torrent_amd.piece import BLOCK_SIZE, PieceMsg
    L, P = 4 * BLOCK_SIZE, 37
    total = L * (P - 1) + BLOCK_SIZE + 100       # last piece: 2 blocks, the second short
    payload = bytes(oracle.synth_fill(77, 0, total))
    info = make_info(L, oracle.hash_pieces(payload, total, L, P), "t.bin", length=total)
    st = Storage(MemoryStorage(), info, os.getcwd())
    v = IncrementalVerifier(info, st)
    msgs = []
    for i in range(P):
        n = L if i < P - 1 else total - (P - 1) * L
        for off in range(0, n, BLOCK_SIZE):
            msgs.append(PieceMsg(i, off, payload[i * L + off:i * L + min(n, off + BLOCK_SIZE)]))
    rng = random.Random(9)
    rng.shuffle(msgs)
    corrupt = msgs[10]
    msgs[10] = PieceMsg(corrupt.index, corrupt.offset, bytes(b ^ 1 for b in corrupt.block))
    results = {}
    for k, m in enumerate(msgs):
        v.on_block(m)
        if k % 25 == 0:
            results.update(dict(v.flush()))
    results.update(dict(v.flush()))
    assert results[corrupt.index] is False
    assert all(ok for i, ok in results.items() if i != corrupt.index) and len(results) == P
    # re-receive the corrupted piece correctly
    i = corrupt.index
    n = L if i < P - 1 else total - (P - 1) * L
    for off in range(0, n, BLOCK_SIZE):
        v.on_block(PieceMsg(i, off, payload[i * L + off:i * L + min(n, off + BLOCK_SIZE)]))
    assert v.flush() == [(i, True)]
    assert bytes(v.bitfield) == bytes(b"\xff" * (P // 8) + bytes([(0xFF00 >> (P % 8)) & 0xFF]))
    assert st.get(0, total) is not None   # blocks also went through Storage.set
    v.close()


@pytest.mark.parametrize("layout", ["multi_zero_tiny", "missing_and_short", "single_short_last", "cfg1"])
def test_verify_files_resume_from_disk(native, tmp_path, layout):
    """verify_files (f2 resume from disk: one tv_stage_files call per shard) gives the same bits as the
    committed expectation and as verify_pieces over fs_storage, whichever path the segments take."""
    from tests.layouts import build_layout, by_name
    from torrent_amd import verify_files
    rec = {r["name"]: r for r in json.load(open(os.path.join(GOLDEN, "layouts.json")))}[layout]
    lay = build_layout(by_name(layout))
    for path, data in lay["disk_files"]().items():
        p = tmp_path.joinpath(*path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
    before = sorted(str(x) for x in tmp_path.rglob("*"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        # default: every segment is short, so all go through the reader pool; 2 shards on GPU 0
        bf = verify_files(lay["info"], str(tmp_path), devices=[0, 0])
        # one reader thread
        bf2 = verify_files(lay["info"], str(tmp_path), threads=1)
        # every non-empty file segment through the tv_stage_file path (page-cache DMA), 2 shards
        bf3 = verify_files(lay["info"], str(tmp_path), devices=[0, 0], direct_min=0)
        # a mix: segments >= 3 KiB take the tv_stage_file path, the rest the reader pool
        bf4 = verify_files(lay["info"], str(tmp_path), direct_min=3072)
    finally:
        os.chdir(cwd)
    assert bytes(bf).hex() == rec["expected_bitfield"]
    assert bytes(bf2).hex() == rec["expected_bitfield"]
    assert bytes(bf3).hex() == rec["expected_bitfield"]
    assert bytes(bf4).hex() == rec["expected_bitfield"]
    assert sorted(str(x) for x in tmp_path.rglob("*")) == before   # no files created


@pytest.mark.parametrize("direct", [1, 0])
def test_stage_file_windows_offsets_and_failures(native, oracle, tmp_path, direct):
    """tv_stage_file: the torrent bytes sit at an unaligned offset inside the file; windows of
    200,000 bytes (not a page multiple) over a shard window [8, 128) of 130 pieces with a short last
    piece; registered page-cache DMA (direct=1) and the pinned-ring copy (direct=0) stage the same
    bytes.  A short or missing file returns False and stages no byte of a piece it cannot complete (the
    library marks those pieces unreadable: tv_verify reports them 0 though their bytes are right); len 0
    needs no file."""
    L, P = 65536, 130
    total = L * (P - 1) + 12345
    payload = oracle.synth_fill(77, 0, total)
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    pieces[20 * 40 + 5] ^= 2
    prefix = 12345
    f = tmp_path / "blob.bin"
    f.write_bytes(b"\xaa" * prefix + bytes(payload))
    short = tmp_path / "short.bin"
    short.write_bytes(b"\x01" * 1000)
    exp = oracle.verify_linear(payload, total, L, bytes(pieces))
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_DIRECT, direct)
        ctx.set_option(native.TV_OPT_FILE_CHUNK, 200000)
        assert ctx.get_option(native.TV_OPT_FILE_CHUNK) == 200000
        ctx.set_layout(total, L, P, 8, 122)
        ctx.set_digests(bytes(pieces))
        assert ctx.stage_file(str(f), prefix, 0, total)
        out = bytearray(total)
        ctx.read(0, out)
        assert out[8 * L:] == payload[8 * L:] and out[:8 * L] == bytes(8 * L)
        bf = ctx.verify()
        want = bytearray((122 + 7) // 8)
        for j in range(122):
            i = 8 + j
            if (exp[i >> 3] >> (7 - (i & 7))) & 1:
                want[j >> 3] |= 0x80 >> (j & 7)
        assert bf == bytes(want)
        # failures: nothing is staged, False is returned (fsStorage.get -> null), no file is created
        assert not ctx.stage_file(str(short), 0, 9 * L, 2000)
        assert not ctx.stage_file(str(tmp_path / "missing.bin"), 0, 9 * L, 10)
        assert not (tmp_path / "missing.bin").exists()
        assert ctx.stage_file(str(tmp_path / "missing.bin"), 0, 9 * L, 0)
        ctx.read(0, out)
        assert out[8 * L:] == payload[8 * L:]
        bf = ctx.verify()
        assert not (bf[0] >> 6) & 1 and bf[0] >> 7 == want[0] >> 7     # piece 9 marked, piece 8 as before
        # a range partly outside the shard: only the shard's bytes are staged
        ctx.stage_file(str(short), 0, 8 * L - 500, 1000)
        ctx.read(0, out)
        assert out[8 * L:8 * L + 500] == b"\x01" * 500 and out[8 * L + 500:] == payload[8 * L + 500:]


@pytest.mark.parametrize("concurrent", [1, 0])
@pytest.mark.parametrize("direct_min", [1 << 62, 0])
def test_stage_files_long_unaligned_and_gapped(native, oracle, tmp_path, direct_min, concurrent):
    """tv_stage_files edge cases, read back byte for byte: a 150 MiB segment (longer than a 64 MiB
    staging slot: split into slot parts and 4 MiB read parts) at a file offset of 3 (never congruent
    with its linear offset mod 4), segments given out of linear order with a gap between them, one
    reaching past the shard's end, a zero-length one for a missing file, and a directory (TV_ERR_IO).
    direct_min = 2^62: all through the reader pool; 0: all through the tv_stage_file path (with
    TV_OPT_FILE_CONCURRENT the 150 MiB segment on the calling thread's lane, the others - the
    directory's TV_ERR_IO among them - on the helper's)."""
    L, P = 1 << 20, 160
    total = L * P
    payload = oracle.synth_fill(91, 0, total)
    (tmp_path / "big.bin").write_bytes(b"xyz" + bytes(payload[:150 * L]))
    (tmp_path / "tail.bin").write_bytes(bytes(payload[150 * L + 5:]))
    (tmp_path / "dir").mkdir()
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, direct_min)
        ctx.set_option(native.TV_OPT_FILE_CONCURRENT, concurrent)
        assert ctx.get_option(native.TV_OPT_FILE_CONCURRENT) == concurrent
        ctx.set_layout(total, L, P, 0, 152)                 # shard: pieces [0, 152)
        st = ctx.stage_files([str(tmp_path / "tail.bin"), str(tmp_path / "big.bin"),
                              str(tmp_path / "missing.bin"), str(tmp_path / "dir")],
                             [0, 3, 0, 0], [150 * L + 5, 0, 17, 150 * L], [total - 150 * L - 5, 150 * L, 0, 5])
        assert st == [0, 0, 0, native.TV_ERR_IO]
        out = bytearray(total)
        ctx.read(0, out)
    assert out[:150 * L] == payload[:150 * L]               # the long segment
    assert out[150 * L + 5:152 * L] == payload[150 * L + 5:152 * L]   # clipped at the shard's end
    assert not (tmp_path / "missing.bin").exists()


@pytest.mark.parametrize("direct", [1, 0])
def test_stage_files_two_lanes_many_segments(native, oracle, tmp_path, direct):
    """Two staging lanes under load: 40 files of ragged sizes at file offsets 0-3 (so the lanes' copies
    are aligned, head/tail split or routed through each lane's own ring), an odd piece length (no
    whole-piece row is dword-aligned), 64 KiB windows, half the segments long enough for the
    tv_stage_file path, staged in one call with and without TV_OPT_FILE_CONCURRENT; every byte read
    back and the verify bitfield all ones."""
    import random
    rnd = random.Random(5)
    L, P = 65539, 700
    total = L * P - 1234
    payload = oracle.synth_fill(17, 0, total)
    cuts = sorted(rnd.sample(range(1, total), 39))
    bounds = [0] + cuts + [total]
    paths, fos, lins, lens = [], [], [], []
    for k in range(40):
        a, b = bounds[k], bounds[k + 1]
        pre = rnd.randrange(4)
        path = tmp_path / f"s{k:02d}.bin"
        path.write_bytes(bytes(pre) + bytes(payload[a:b]))
        paths.append(str(path)); fos.append(pre); lins.append(a); lens.append(b - a)
    order = list(range(40))
    rnd.shuffle(order)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_DIRECT, direct)
        ctx.set_option(native.TV_OPT_FILE_CHUNK, 64 << 10)
        ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, sorted(lens)[20])
        ctx.set_layout(total, L, P)
        ctx.set_digests(oracle.hash_pieces(payload, total, L, P))
        for conc in (1, 0):
            ctx.set_option(native.TV_OPT_FILE_CONCURRENT, conc)
            ctx.fill_synthetic(99)                                  # overwrite what the last round staged
            st = ctx.stage_files([paths[k] for k in order], [fos[k] for k in order],
                                 [lins[k] for k in order], [lens[k] for k in order])
            assert st == [0] * 40
            out = bytearray(total)
            ctx.read(0, out)
            assert out == payload, conc
            bf = ctx.verify()
            assert all(bf[i >> 3] >> (7 - (i & 7)) & 1 for i in range(P)), conc


@pytest.mark.parametrize("direct_min", [1 << 62, 0])
def test_stage_files_odd_piece_length_ring_sources(native, oracle, tmp_path, direct_min):
    """Ring-slot sources at an odd piece length.  The packed reads of the reader pool (direct_min = 2^62)
    and the pread windows of tv_stage_file (direct_min = 0, direct DMA off) sit in ring slots at their
    LINEAR offset's alignment mod 4, which is not the device destination's when L % 4 != 0.  Such
    sources must be DMA'd as they lie: re-bouncing them through the ring took the ring's next slots,
    which after three takes is the slot being read (a race; the two-lane test caught it once).  300
    ragged segments put several hundred unaligned piece fragments into one slot."""
    import random
    rnd = random.Random(11)
    L, P = 16387, 300
    total = L * P - 77
    payload = oracle.synth_fill(23, 0, total)
    bounds = [0] + sorted(rnd.sample(range(1, total), 299)) + [total]
    paths, fos, lins, lens = [], [], [], []
    for k in range(300):
        a, b = bounds[k], bounds[k + 1]
        pre = rnd.randrange(4)
        path = tmp_path / f"o{k:03d}.bin"
        path.write_bytes(bytes(pre) + bytes(payload[a:b]))
        paths.append(str(path)); fos.append(pre); lins.append(a); lens.append(b - a)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_FILE_DIRECT, 0)
        ctx.set_option(native.TV_OPT_FILE_CHUNK, 64 << 10)
        ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, direct_min)
        ctx.set_layout(total, L, P)
        ctx.set_digests(oracle.hash_pieces(payload, total, L, P))
        for rep in range(3):
            ctx.fill_synthetic(50 + rep)
            st = ctx.stage_files(paths, fos, lins, lens)
            assert st == [0] * 300
            out = bytearray(total)
            ctx.read(0, out)
            assert out == payload, rep
            bf = ctx.verify()
            assert all(bf[i >> 3] >> (7 - (i & 7)) & 1 for i in range(P)), rep


def test_verify_files_reference_singlefile(native, tmp_path):
    from torrent_amd import parse_metainfo, verify_files
    info = parse_metainfo(_load("singlefile.torrent")).info
    (tmp_path / info.name).write_bytes(_ref_payload("singlefile"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        bf = verify_files(info, str(tmp_path))
    finally:
        os.chdir(cwd)
    assert bytes(bf) == _all_ones(info.n_pieces)


def test_cli_make_torrent_then_verify(native, tmp_path):
    """The two command lines end to end in fresh processes: `python -m torrent_amd.make_torrent -c ... -t
    ... <file>` (make_torrent.ts:190-250) writes <name>.torrent in the working directory, and
    `python -m torrent_amd verify <torrent> <dir>` reports every piece verified (exit 0); after a one-byte
    corruption it reports the bad piece (exit 1) and the bitfield hex shows which."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    data = bytes((i * 7 + 3) & 0xFF for i in range(3_000_001))   # 3 MB: 32 KiB pieces by make_torrent.ts:17-21
    (tmp_path / "payload.bin").write_bytes(data)
    r = subprocess.run([sys.executable, "-m", "torrent_amd.make_torrent", "-c", "cli test", "-t",
                        "http://tracker.example/announce", "payload.bin"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "output -> payload.bin.torrent" in r.stdout, r.stdout + r.stderr
    from torrent_amd import parse_metainfo
    meta = parse_metainfo((tmp_path / "payload.bin.torrent").read_bytes())
    L, P = meta.info.piece_length, meta.info.n_pieces
    assert L == 1 << 15 and P == -(-len(data) // L) and meta.comment == "cli test"
    assert meta.info.pieces[5] == hashlib.sha1(data[5 * L:6 * L]).digest()
    cmd = [sys.executable, "-m", "torrent_amd", "verify", str(tmp_path / "payload.bin.torrent"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and f"{P}/{P} pieces verified" in r.stdout, r.stdout + r.stderr
    bad = bytearray(data)
    bad[40 * L + 9] ^= 0x20
    (tmp_path / "payload.bin").write_bytes(bytes(bad))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and f"{P - 1}/{P} pieces verified" in r.stdout, r.stdout + r.stderr
    bf = bytes.fromhex(r.stdout.strip().splitlines()[-1])
    assert [i for i in range(P) if not (bf[i >> 3] >> (7 - (i & 7))) & 1] == [40]


@pytest.mark.parametrize("name", ["singlefile", "multifile"])
def test_make_torrent_reproduces_reference_fixture_bytes(native, tmp_path, name):
    """Creation mode end to end: make_torrent on the reconstructed payload (same comment, tracker,
    creation date and file order as the reference's run) reproduces the reference's own
    test_data .torrent byte for byte -- every GPU digest plus the bencode layout of make_torrent.ts."""
    from torrent_amd import parse_metainfo
    from torrent_amd.make_torrent import make_torrent
    ref = _load(f"{name}.torrent")
    meta = parse_metainfo(ref)
    rd = json.load(open(os.path.join(GOLDEN, "refdata.json")))[name]
    if name == "singlefile":
        p = tmp_path / "singlefile.txt"
        p.write_bytes(_ref_payload(name))
        files = None
    else:
        p = tmp_path / "multifile"
        for f in rd["files"]:
            q = p.joinpath(*f["path"].split("/"))
            q.parent.mkdir(parents=True, exist_ok=True)
            q.write_bytes(f["pattern"].encode() * (f["length"] // len(f["pattern"])))
        files = meta.info.files
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        out = make_torrent(str(p), meta.announce, comment=meta.comment, creation_date=meta.creation_date,
                           files=files)
    finally:
        os.chdir(cwd)
    assert out == ref


def test_make_torrent_small_directory_quirk(native, tmp_path):
    """make_torrent.ts never hashes the single piece of a directory smaller than one piece."""
    from torrent_amd import parse_metainfo
    from torrent_amd.make_torrent import make_torrent
    d = tmp_path / "small"
    d.mkdir()
    (d / "a.txt").write_bytes(b"hello")
    out = parse_metainfo(make_torrent(str(d), "http://t/announce", creation_date=1))
    assert out.info.pieces_raw == bytes(20) and out.info.piece_length == 1 << 15


def test_c_consumer_full_path(native, tmp_path):
    """tests/c/abi_consumer.c on the GPU: verify / hash / verify_list / verify_host (pageable and
    pinned) / read-back on the reference's conventions, and two contexts on two host threads."""
    import subprocess
    from tests.test_abi import build_c_consumer
    exe = build_c_consumer(tmp_path)
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_concurrent_calls_do_not_interleave(native, oracle):
    """Many verify_pieces / verify_piece / hash_pieces calls at once (threads via the asyncio
    wrappers) share the cached per-device contexts; each job holds its context for its whole
    set_layout -> stage -> verify sequence, so every result is exact."""
    import asyncio
    from torrent_amd import (MemoryStorage, Storage, hash_pieces, make_info, release_contexts,
                             verify_piece_async, verify_pieces_async)
    jobs = []
    for k in range(6):
        L, P = 4096 * (k + 1), 40 + 13 * k
        total = L * (P - 1) + 1 + k
        payload = bytes(oracle.synth_fill(100 + k, 0, total))
        pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
        pieces[20 * (k * 5) + 1] ^= 1
        info = make_info(L, bytes(pieces), f"t{k}", length=total)
        st = MemoryStorage()
        st.files[(f"t{k}",)] = bytearray(payload)
        jobs.append((info, Storage(st, info, os.getcwd()), payload, oracle.verify_linear(payload, total, L, bytes(pieces))))

    async def main():
        coros = []
        for info, storage, payload, _ in jobs:
            coros.append(verify_pieces_async(info, storage, devices=[0, 0]))
            coros.append(verify_piece_async(info, 1, payload[info.piece_length:2 * info.piece_length]))
        return await asyncio.gather(*coros)

    out = asyncio.run(main())
    for n, (info, _, payload, expect) in enumerate(jobs):
        assert bytes(out[2 * n]) == expect
        assert out[2 * n + 1] is bool((expect[0] >> 6) & 1)
        assert hash_pieces(payload, info.piece_length) == oracle.hash_pieces(
            payload, info.length, info.piece_length, info.n_pieces)
    release_contexts()


def test_verify_files_read_faults_are_unreadable_pieces(native, tmp_path):
    """Read faults (the storage_test.ts:96-108 idea, applied to verify_files' own reads): a path that
    opens but cannot be read (a directory where a file should be: EISDIR) and a missing file make the
    pieces they touch unreadable (bit 0); a file one byte short makes only the piece holding its last byte
    unreadable, since Storage.get reads piece by piece (storage.ts:50-65,150-172) -- never an exception,
    through both the reader pool and the tv_stage_file path, with the same bits as Storage(fs_storage).get.
    tv_stage_files reports each as TV_ERR_IO, and the library itself marks the pieces (no host clearing)."""
    import hashlib as _h
    from torrent_amd import FileInfo, make_info, verify_files
    L = 4096
    sizes = [5 * L + 100, 3 * L, 4 * L + 7, 2 * L, 6 * L]         # files f0 .. f4
    payload = bytes((i * 7 + 3) & 0xFF for i in range(sum(sizes)))
    total = len(payload)
    P = -(-total // L)
    pieces = b"".join(_h.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    info = make_info(L, pieces, "t", files=[FileInfo(n, [f"f{k}"]) for k, n in enumerate(sizes)])
    starts = [sum(sizes[:k]) for k in range(len(sizes) + 1)]
    (tmp_path / "f0").write_bytes(payload[starts[0]:starts[1]])
    (tmp_path / "f1").mkdir()                                      # a directory: open ok, read fails
    (tmp_path / "f2").write_bytes(payload[starts[2]:starts[3] - 1])  # one byte short
    (tmp_path / "f4").write_bytes(payload[starts[4]:starts[5]])       # f3 missing
    bad = {(starts[3] - 1) // L}                                      # f2's last byte
    for k in (1, 3):
        bad |= set(range(starts[k] // L, (starts[k + 1] - 1) // L + 1))
    assert not bad & set(range(9, 12))                               # f2's whole pieces stay readable
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        for dmin in (None, 0):
            bf = verify_files(info, str(tmp_path), direct_min=dmin)
            bits = [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)]
            assert bits == [0 if i in bad else 1 for i in range(P)], dmin
    finally:
        os.chdir(cwd)
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(pieces)
        st = ctx.stage_files([str(tmp_path / f"f{k}") for k in range(5)], [0] * 5, starts[:5], sizes)
        assert st == [0, native.TV_ERR_IO, native.TV_ERR_IO, native.TV_ERR_IO, 0]
        bf = ctx.verify()                                            # no availability from the host
        assert [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(P)] == [0 if i in bad else 1 for i in range(P)]


@pytest.mark.parametrize("concurrent", [1, 0])
def test_ring_leases_keep_rebounced_ring_sources_exact(native, oracle, tmp_path, concurrent):
    """The staging ring's invariant, checked deterministically: a slot stays LENT from take_slot until the
    event after its last queued copy is recorded, and take_slot never hands out a lent slot.
    TV_OPT_DEBUG_REBOUNCE puts back the bounce of ring-resident sources that once raced (the bounce took the
    ring's next slots, and the third take was the slot being read, overwriting bytes still to be DMA'd).
    With leases the bounce skips the source slot, so every byte reads back exact whatever the DMA timing:
    an odd piece length (no staged fragment is dword-congruent, so every fragment bounces), 300 ragged
    segments through the reader pool's packed slots on lane 0 and windowed preads on lane 1."""
    import random
    rnd = random.Random(13)
    L, P = 65539, 300
    total = L * P - 91
    payload = oracle.synth_fill(29, 0, total)
    bounds = [0] + sorted(rnd.sample(range(1, total), 299)) + [total]
    paths, fos, lins, lens = [], [], [], []
    for k in range(300):
        a, b = bounds[k], bounds[k + 1]
        pre = rnd.randrange(4)
        path = tmp_path / f"r{k:03d}.bin"
        path.write_bytes(bytes(pre) + bytes(payload[a:b]))
        paths.append(str(path)); fos.append(pre); lins.append(a); lens.append(b - a)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_DEBUG_REBOUNCE, 1)
        assert ctx.get_option(native.TV_OPT_DEBUG_REBOUNCE) == 1
        ctx.set_option(native.TV_OPT_FILE_DIRECT, 0)
        ctx.set_option(native.TV_OPT_FILE_CHUNK, 64 << 10)
        ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, sorted(lens)[150])  # half the segments on lane 1
        ctx.set_option(native.TV_OPT_FILE_CONCURRENT, concurrent)
        ctx.set_layout(total, L, P)
        ctx.set_digests(oracle.hash_pieces(payload, total, L, P))
        ctx.fill_synthetic(77)
        assert ctx.stage_files(paths, fos, lins, lens) == [0] * 300
        out = bytearray(total)
        ctx.read(0, out)
        assert out == payload
        bf = ctx.verify()
        assert all(bf[i >> 3] >> (7 - (i & 7)) & 1 for i in range(P))
        # pageable tv_stage through the ring with the bounce on, at an odd source alignment
        ctx.fill_synthetic(78)
        src = bytearray(3) + payload
        ctx.stage(0, memoryview(src)[3:])
        ctx.read(0, out)
        assert out == payload


def test_set_layout_reuses_allocations_across_geometries(native, oracle):
    """One context through a sequence of geometries (verify_piece-sized, bigger, smaller, empty, a shard,
    the stream path between them): tv_set_layout keeps the allocations that fit, and no stale digest,
    availability bit or payload byte of an earlier geometry leaks into a later result."""
    cases = [(262144, 1, 262144, 0, 1), (262144, 1, 1000, 0, 1), (4096, 300, 17, 8, 200), (4096, 10, 4096, 0, 10),
             (65536, 3, 100, 0, 3), (1 << 20, 0, 0, 0, 0), (262144, 1, 262144, 0, 1), (8192, 600, 8192, 0, 600),
             (4096, 2, 5, 0, 2)]
    with native.Context(0) as ctx:
        for n, (L, P, last, first, count) in enumerate(cases):
            total = L * (P - 1) + last if P else 0
            payload = oracle.synth_fill(200 + n, 0, total)
            pieces = bytearray(oracle.hash_pieces(payload, total, L, P)) if P else bytearray()
            if P:
                pieces[20 * (P // 2) + 1] ^= 4
            exp = oracle.verify_linear(payload, total, L, bytes(pieces)) if P else b""
            want = bytearray((count + 7) // 8)
            for j in range(count):
                i = first + j
                if (exp[i >> 3] >> (7 - (i & 7))) & 1:
                    want[j >> 3] |= 0x80 >> (j & 7)
            ctx.set_layout(total, L, P, first, count)
            ctx.set_digests(bytes(pieces))
            if total:
                ctx.stage(0, payload)
            assert ctx.verify() == bytes(want), n
            assert ctx.verify_host(memoryview(payload)[first * L:]) == bytes(want), n
            if count:
                assert ctx.verify_list(list(range(first, first + count))) == bytes(
                    (want[j >> 3] >> (7 - (j & 7))) & 1 for j in range(count)), n
