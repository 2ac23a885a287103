"""Windowed layouts: every bulk path on a shard larger than the device budget (TV_OPT_RESIDENT_BUDGET).

The budget is forced down to a few MiB (a few pieces per window) and every result must equal the one the
reference's semantics give, exactly as without a budget: the reference's test_data fixtures (all 1706 / 1855
digests), the seeded golden layouts incl. BASELINE config 3 (10,000 files), the 48 seeded fuzz layouts on
one and three shards, and BASELINE config 2 at full size against the oracle.  The payload the context holds
(TV_COUNTER_PAYLOAD_BYTES) stays within the budget, and a shard that fits is not windowed.
"""
import hashlib
import json
import os
import random

import pytest

from tests.test_gpu_fuzz import SEEDS, _bits, _disk, _draw, _expected

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _stride(L):
    return -(-L // 64) * 64 + 256


def _budget(L, pieces_per_window, bufs=None):
    """A budget whose windows hold `pieces_per_window` pieces (the default count of window buffers of them,
    tv_plan.h kWinBufsDefault, or `bufs`)."""
    from torrent_amd import _native
    return (bufs or _native.WIN_BUFS_DEFAULT) * (pieces_per_window * _stride(L) + 256)


def _check_windowed(budget, expect_windowed=True):
    """Every cached bulk context (slot >= 0) last laid out under `budget` holds at most `budget` bytes of
    payload, and (expect_windowed) at least one of them is windowed."""
    from torrent_amd.verify import context_counters
    seen = [c for (dev, slot), c in context_counters().items() if slot >= 0 and c["budget"] == budget]
    assert seen
    for c in seen:
        assert c["payload_bytes"] <= budget, c
    if expect_windowed:
        assert any(c["window_pieces"] >= 1 for c in seen), seen


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["singlefile", "multifile"])
def test_reference_fixtures_windowed(native, name):
    """The reference's test_data torrents (digests produced by its own SHA-1 path, make_torrent.ts:28-31) with
    8 MiB budgets: 447 / 972 MB payloads in windows of 15 / 7 pieces, resident staging, Storage reads and
    creation mode; the three flipped pieces (#0, the file-spanning #852, the short last) and nothing else fail."""
    from torrent_amd import MemoryStorage, Storage, hash_pieces, parse_metainfo, verify_payload, verify_pieces
    from tests.test_gpu_paths import _all_ones, _load, _ref_payload
    info = parse_metainfo(_load(f"{name}.torrent")).info
    payload = bytearray(_ref_payload(name))
    P, L = info.n_pieces, info.piece_length
    budget = 8 << 20
    assert bytes(verify_payload(info, payload, budget=budget, resident=True)) == _all_ones(P)
    _check_windowed(budget)
    assert bytes(verify_payload(info, payload, budget=budget)) == _all_ones(P)     # (default: streamed here)
    assert hash_pieces(bytes(payload), L, budget=budget) == info.pieces_raw
    flips = [0, 852, P - 1]
    for i in flips:
        payload[i * L + 3] ^= 0x01
    want = bytearray(_all_ones(P))
    for i in flips:
        want[i >> 3] &= ~(0x80 >> (i & 7)) & 0xFF
    for devices in ([0], [0, 0, 0]):
        assert bytes(verify_payload(info, payload, devices=devices, budget=budget,
                                    resident=True)) == bytes(want), devices
        assert bytes(verify_payload(info, payload, devices=devices, budget=budget)) == bytes(want), (devices, "auto")
    if name == "multifile":
        n0 = info.files[0].length
        mem = MemoryStorage({tuple(info.files[0].path): bytes(payload[:n0]),
                             tuple(info.files[1].path): bytes(payload[n0:])})
        assert bytes(verify_pieces(info, Storage(mem, info, os.getcwd()), budget=budget)) == bytes(want)
        _check_windowed(budget)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["single_short_last", "multi_zero_tiny", "many_tiny_span", "missing_and_short",
                                    "exact_multiple", "cfg1", "cfg3"])
def test_golden_layouts_windowed(native, layout, tmp_path, monkeypatch):
    """The committed expected bitfields of the seeded layouts (hashlib-computed), windowed: resident staging
    (verify_payload), file staging (verify_files over the files on disk, 10,000 of them for cfg3) and
    creation mode (hash_pieces), with windows of 1-16 pieces, on one and three shards."""
    from tests.layouts import build_layout, by_name
    from torrent_amd import hash_pieces, verify_files, verify_payload
    rec = {r["name"]: r for r in json.load(open(os.path.join(GOLDEN, "layouts.json")))}[layout]
    lay = build_layout(by_name(layout))
    info, L = lay["info"], lay["info"].piece_length
    rng = random.Random(layout)
    sizes = [1, 3, 16] if info.n_pieces < 1000 else [16, 64]    # (a window kernel costs one piece's SHA-1)
    for devices in ([0], [0, 0, 0]):
        budget = _budget(L, rng.choice(sizes))
        assert bytes(verify_payload(info, lay["payload"], avail=lay["avail"], devices=devices, budget=budget,
                                    resident=True)).hex() == rec["expected_bitfield"], (devices, budget)
        _check_windowed(budget, expect_windowed=devices == [0] and info.n_pieces * _stride(L) + 256 > budget)
        # the default: streamed windows x columns within the budget (tv_verify_host) when the shard exceeds it
        assert bytes(verify_payload(info, lay["payload"], avail=lay["avail"], devices=devices,
                                    budget=budget)).hex() == rec["expected_bitfield"], (devices, budget, "auto")
    monkeypatch.chdir(tmp_path)
    for path, data in lay["disk_files"]().items():
        p = tmp_path.joinpath("dl", *path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
    for devices in ([0], [0, 0, 0]):
        budget = _budget(L, rng.choice([2, 5, 16] if info.n_pieces < 1000 else [16, 64]))
        assert bytes(verify_files(info, str(tmp_path / "dl"), devices=devices, threads=4, budget=budget,
                                  stream=False)).hex() == rec["expected_bitfield"], (devices, budget)
        _check_windowed(budget, expect_windowed=devices == [0] and info.n_pieces * _stride(L) + 256 > budget)
        # the same budget as the default chooses it (columns through the ring where windows would lose: _stream_wins)
        assert bytes(verify_files(info, str(tmp_path / "dl"), devices=devices, threads=4,
                                  budget=budget)).hex() == rec["expected_bitfield"], (devices, budget, "auto")
    clean = hashlib.sha1(lay["pieces_raw"]).hexdigest()
    assert clean == rec["pieces_sha1"]
    if not lay["corrupted"]:
        assert hash_pieces(bytes(lay["payload"]), L, budget=_budget(L, 2)) == lay["pieces_raw"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_layouts_windowed(native, tmp_path, monkeypatch, seed):
    """The 48 seeded fuzz layouts (tests/test_gpu_fuzz.py: odd piece lengths, zero-length / tiny / boundary
    files, missing and short files, ragged digests, extra digests) through verify_pieces, verify_payload and
    verify_files with windows of 1-5 pieces, on one and three shards: the bits equal Storage.get + hashlib's."""
    from torrent_amd import MemoryStorage, Storage, verify_files, verify_payload, verify_pieces
    from torrent_amd.piece import piece_length
    from torrent_amd.storage import fs_storage
    import shutil
    info, payload, sizes, missing, short, single = _draw(seed)
    P, L = info.n_pieces, info.piece_length
    monkeypatch.chdir(tmp_path)
    disk = _disk(info, payload, sizes, missing, short, single)
    mem = MemoryStorage()
    st = Storage(mem, info, str(tmp_path / "dl"))
    mem.files = {tuple(st.dir_path) + k: bytearray(v) for k, v in disk.items()}
    want = _expected(info, st)
    for root in ("dl", "ref"):
        for k, data in disk.items():
            p = tmp_path.joinpath(root, *k)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
    want_fs = _expected(info, Storage(fs_storage, info, str(tmp_path / "ref")))
    shutil.rmtree(tmp_path / "ref", ignore_errors=True)
    avail = bytearray((P + 7) // 8)
    for i in range(P):
        if st.get(i * L, piece_length(i, info)) is not None:
            avail[i >> 3] |= 0x80 >> (i & 7)
    rng = random.Random(seed)
    for devices in ([0], [0, 0, 0]):
        budget = _budget(L, rng.choice([1, 2, 3, 5]))
        assert _bits(verify_pieces(info, st, devices=devices, budget=budget), P) == want, ("pieces", devices, budget)
        assert _bits(verify_payload(info, payload[:info.length], devices=devices, avail=bytes(avail),
                                    budget=budget, resident=True), P) == want, ("payload", devices, budget)
        assert _bits(verify_payload(info, payload[:info.length], devices=devices, avail=bytes(avail),
                                    budget=budget), P) == want, ("payload auto", devices, budget)
        assert _bits(verify_files(info, str(tmp_path / "dl"), devices=devices, threads=3, budget=budget, stream=False),
                     P) == want_fs, ("files", devices, budget)
        _check_windowed(budget, expect_windowed=False)


@pytest.mark.gpu
def test_full_size_cfg2_windowed_against_the_oracle(native, oracle):
    """BASELINE config 2 at full size (16 GiB, 16,384 x 1 MiB) under a 3 GiB budget: windows of 1,472 pieces,
    filled on the device; creation mode equals the ORACLE's digests of every piece and verify (1 % corrupted
    digests) gives exactly the oracle's bitfield, with every kernel choice; the payload held is <= the budget."""
    from tests.test_gpu_paths import _threads
    L, P = 1 << 20, 16384
    total = L * P
    truth = oracle.synth_piece_digests(2, total, L, P, threads=_threads())
    bad = set(range(7, P, 101)) | {P - 1}
    d2 = bytearray(truth)
    for i in bad:
        d2[20 * i + 7] ^= 0x10
    budget = 3 << 30
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, budget)
        for k in (0, 1, 2, 4):
            ctx.set_option(native.TV_OPT_KERNEL, k)
            ctx.set_layout(total, L, P)
            W = ctx.counter(native.TV_COUNTER_WINDOW_PIECES)
            assert 0 < W < P and ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) <= budget
            ctx.fill_synthetic(2)
            assert ctx.hash() == truth, k
            assert ctx.counter(native.TV_COUNTER_WINDOWS) == -(-P // W)
            ctx.set_digests(bytes(d2))
            ctx.fill_synthetic(2)                       # a second pass over the same layout
            bf = ctx.verify()
            got = {i for i in range(P) if not (bf[i >> 3] >> (7 - (i & 7))) & 1}
            assert got == bad, (k, sorted(got ^ bad)[:10])
            assert ctx.last_timing()[0] > 0


@pytest.mark.gpu
def test_windowed_rules(native, oracle):
    """The windowed layout's contract (include/torrent_verify.h, tv_set_layout): staging ascends (bytes of a
    window already hashed this pass are TV_ERR_STATE and change nothing), pieces never staged are 0 / zero
    digests, tv_read reads the open window only, tv_verify_list is refused, a repeated verify reuses the pass,
    staging after it starts a new pass; and a shard that fits the budget stays whole (window counter 0)."""
    L, P = 4096, 100
    total = L * (P - 1) + 1234
    payload = bytes(oracle.synth_fill(77, 0, total))
    pieces = oracle.hash_pieces(bytearray(payload), total, L, P)
    stride = _stride(L)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, P * stride + 256)      # fits exactly: not windowed
        ctx.set_layout(total, L, P)
        assert ctx.counter(native.TV_COUNTER_WINDOW_PIECES) == 0
        ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, _budget(L, 7))
        ctx.set_layout(total, L, P)
        assert ctx.counter(native.TV_COUNTER_WINDOW_PIECES) == 7
        assert ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) == _budget(L, 7)
        assert ctx.counter(native.TV_COUNTER_WINDOW_BUFS) == native.WIN_BUFS_DEFAULT
        assert ctx.counter(native.TV_COUNTER_WINDOW_STREAMS) == native.WIN_BUFS_DEFAULT - 1
        ctx.set_digests(pieces)
        ctx.stage(0, payload[:30 * L])                  # windows 0-4 (pieces 0-29)
        out = bytearray(L)
        ctx.read(28 * L, out)                           # window 4 is open
        assert bytes(out) == payload[28 * L:29 * L]
        with pytest.raises(native.NativeError) as e:
            ctx.read(0, out)                            # window 0 was hashed
        assert e.value.code == native.TV_ERR_STATE
        with pytest.raises(native.NativeError) as e:
            ctx.stage(3 * L, payload[3 * L:4 * L])      # descending: refused
        assert e.value.code == native.TV_ERR_STATE and "ascending" in str(e.value)
        with pytest.raises(native.NativeError) as e:
            ctx.verify_list([0])
        assert e.value.code == native.TV_ERR_STATE
        ctx.stage(56 * L, payload[56 * L:])             # windows 8.. (pieces 35-55 never staged)
        bf = ctx.verify()
        want = [0 if 30 <= i < 56 else 1 for i in range(P)]
        assert _bits(bf, P) == want
        assert ctx.counter(native.TV_COUNTER_WINDOWS) == 5 + 7       # windows 0-4 and 8-14
        assert ctx.verify() == bf                       # the same pass
        digests = ctx.hash()
        for i in range(P):
            d = digests[20 * i:20 * i + 20]
            if 35 <= i < 56:                            # windows 5-7: never opened, zero digests
                assert d == bytes(20), i
            elif 30 <= i < 35:                          # window 4's unstaged pieces: a stale buffer's bytes
                assert d != pieces[20 * i:20 * i + 20], i
            else:
                assert d == pieces[20 * i:20 * i + 20], i
        ctx.stage(0, payload)                           # a new pass: everything
        assert _bits(ctx.verify(), P) == [1] * P
        assert _bits(ctx.verify(bytes([0x7F]) + b"\xff" * ((P + 7) // 8 - 1)), P) == [0] + [1] * (P - 1)


@pytest.mark.gpu
@pytest.mark.parametrize("windowed", [False, True])
def test_stage_many_equals_stage_calls(native, windowed):
    """tv_stage_many (the TS verifyPieces' hand-over of a batch of separate piece buffers) stages exactly what the
    same tv_stage calls in order stage: pieces of a ragged layout with a short last piece, some missing, each its
    own buffer (pageable and page-locked, odd addresses), on a whole-shard and a windowed layout; the bitfield
    equals hashlib's, a NULL source with bytes is TV_ERR_ARG, and n = 0 is a no-op."""
    import ctypes
    from torrent_amd import _native as N
    L, P = 40000, 37
    total = L * (P - 1) + 1234
    rng = random.Random(11)
    payload = bytes(rng.randrange(256) for _ in range(total))
    digests = bytearray(b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P)))
    for i in (4, 20):
        digests[20 * i] ^= 1
    missing = {7, 8, 30}
    with N.Context(0) as ctx, N.PinnedBuffer(2 * L + 8) as pin:
        if windowed:
            ctx.set_option(N.TV_OPT_RESIDENT_BUDGET, _budget(L, 5))
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(digests))
        parts = []
        for i in range(P):
            if i in missing:
                continue
            chunk = payload[i * L:min(total, (i + 1) * L)]
            if i % 9 == 3:      # a page-locked source at an odd address
                pin.mv[1:1 + len(chunk)] = chunk
                parts.append((i * L, pin.mv[1:1 + len(chunk)]))
                ctx.stage_many(parts)   # (the pinned buffer is reused: hand over what uses it now)
                parts = []
            else:
                parts.append((i * L, bytearray(b"\x00" + chunk)[1:]))   # a pageable copy of its own
        ctx.stage_many(parts)
        ctx.stage_many([])
        if windowed:
            assert ctx.counter(N.TV_COUNTER_WINDOW_PIECES) >= 1
        avail = bytearray((P + 7) // 8)
        for i in range(P):
            if i not in missing:
                avail[i >> 3] |= 0x80 >> (i & 7)
        bf = ctx.verify(bytes(avail))
        want = [0 if (i in missing or i in (4, 20)) else 1 for i in range(P)]
        assert _bits(bf, P) == want
        L_ = ctx._L
        offs, srcs, lens = (ctypes.c_uint64 * 1)(0), (ctypes.c_uint64 * 1)(0), (ctypes.c_uint64 * 1)(16)
        assert L_.tv_stage_many(ctx._h, 1, offs, srcs, lens) == N.TV_ERR_ARG


@pytest.mark.gpu
def test_unstaged_windows_never_verify_against_zero_digests(native, oracle):
    """the windows a pass never opens get all-zero digest rows; a torrent whose expected digest for
    such a piece is 20 zero bytes must still read 0 there (the piece was never staged: Storage.get would have
    given nothing), with or without caller availability bits, while the staged pieces verify."""
    L, P = 4096, 60
    total = L * P
    payload = bytes(oracle.synth_fill(78, 0, total))
    pieces = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    for i in (20, 21, 35):                          # crafted: zero digests for pieces of never-staged windows
        pieces[20 * i:20 * i + 20] = bytes(20)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, _budget(L, 7))
        ctx.set_layout(total, L, P)
        assert ctx.counter(native.TV_COUNTER_WINDOW_PIECES) == 7
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload[:14 * L])              # windows 0-1
        ctx.stage(42 * L, payload[42 * L:])          # windows 6-8 (pieces 14-41 never staged)
        want = [1 if (i < 14 or i >= 42) else 0 for i in range(P)]
        assert _bits(ctx.verify(), P) == want
        assert _bits(ctx.verify(b"\xff" * ((P + 7) // 8)), P) == want
        ctx.stage(0, payload)                        # a new pass stages everything: the crafted pieces now fail
        want = [0 if i in (20, 21, 35) else 1 for i in range(P)]
        assert _bits(ctx.verify(), P) == want


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["ascending", "shuffled"])
@pytest.mark.parametrize("big", [False, True])
def test_stage_many_packs_small_buffers(native, oracle, order, big):
    """tv_stage_many packs short pageable buffers into ring slots (many per slot, one DMA per run of adjacent
    bytes): ~150 MiB cut into buffers of 1 B .. 900 KiB at odd addresses, sub-piece and across piece boundaries,
    with (big) or without a few 16-20 MiB buffers (staged unpacked) among them -- without, the buffers are dealt to
    both staging lanes -- handed over in one call in ascending or shuffled order; every piece verifies (bitfield =
    hashlib's), and the corrupted ones do not."""
    from torrent_amd import _native as N
    L = 1 << 16
    total = 200 * (1 << 20) + 4321
    P = -(-total // L)
    payload = bytes(oracle.synth_fill(91, 0, total))
    digests = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    for i in (0, 777, P - 1):
        digests[20 * i + 3] ^= 0x40
    rng = random.Random(5)
    cuts, o = [], 0
    while o < total:
        n = rng.choice([rng.randrange(1, 64), rng.randrange(64, 70000), rng.randrange(70000, 900 * 1024),
                        rng.randrange(16 << 20, 20 << 20) if (big and rng.random() < 0.05) else rng.randrange(1, 5000)])
        n = min(n, total - o)
        cuts.append((o, n))
        o += n
    if order == "shuffled":
        rng.shuffle(cuts)
    keep = []
    parts = []
    for off, n in cuts:
        b = bytearray(b"\x00" * (1 + off % 3) + payload[off:off + n])
        keep.append(b)
        parts.append((off, memoryview(b)[1 + off % 3:]))
    with N.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(digests))
        ctx.stage_many(parts)
        bf = ctx.verify()
    want = [0 if i in (0, 777, P - 1) else 1 for i in range(P)]
    assert _bits(bf, P) == want


@pytest.mark.gpu
def test_stage_ranges_of_one_buffer(native, oracle):
    """_native.Context.stage_ranges (tv_stage_many over ranges of one host buffer, addresses computed with numpy):
    a payload staged as its file table's ranges -- zero-length and tiny files, ranges across piece boundaries --
    verifies as the whole payload does."""
    import numpy as np
    from torrent_amd import _native as N
    L = 1 << 15
    rng = random.Random(9)
    sizes = [rng.choice([0, rng.randrange(1, 64), rng.randrange(64, 3 * L)]) for _ in range(3000)]
    total = sum(sizes)
    P = -(-total // L)
    payload = bytes(oracle.synth_fill(33, 0, total))
    digests = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    digests[20 * 5] ^= 1
    starts = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    with N.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(digests))
        ctx.stage_ranges(payload, starts, starts, np.asarray(sizes, dtype=np.uint64))
        bf = ctx.verify()
        with pytest.raises(ValueError):
            ctx.stage_ranges(payload, [0], [total - 3], [4])
        with pytest.raises(ValueError):       # an offset that wraps when added (-1 as uint64) is refused too
            ctx.stage_ranges(payload, [0], np.array([-1], dtype=np.int64), [2])
    assert _bits(bf, P) == [0 if i == 5 else 1 for i in range(P)]


@pytest.mark.gpu
@pytest.mark.parametrize("bufs,streams", [(1, 0), (2, 0), (2, 1), (3, 0), (4, 0), (4, 1), (4, 2), (8, 0), (8, 4)])
def test_window_buffers_and_hash_streams(native, oracle, bufs, streams):
    """Windows hashed side by side (TV_OPT_WIN_BUFS buffers, TV_OPT_WIN_STREAMS hash streams)
    give the bits and digests of one buffer at a time: a ragged 203-piece shard with a short last piece and
    corrupted digests, staged in one call and in uneven calls (some pieces twice, a gap), filled by the device
    generator, verified and hashed -- every combination equal to the oracle, and the payload within the budget."""
    L, P = 8192, 203
    total = L * (P - 1) + 777
    payload = bytes(oracle.synth_fill(91, 0, total))
    pieces = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    clean = bytes(pieces)
    for i in (0, 17, 64, 150, P - 1):
        pieces[20 * i + 5] ^= 0x40
    want = [0 if i in (0, 17, 64, 150, P - 1) else 1 for i in range(P)]
    budget = _budget(L, 9, bufs)
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_WIN_BUFS, bufs)
        ctx.set_option(native.TV_OPT_WIN_STREAMS, streams)
        ctx.set_option(native.TV_OPT_RESIDENT_BUDGET, budget)
        ctx.set_layout(total, L, P)
        assert ctx.counter(native.TV_COUNTER_WINDOW_PIECES) == 9
        assert ctx.counter(native.TV_COUNTER_WINDOW_BUFS) == bufs
        assert ctx.counter(native.TV_COUNTER_WINDOW_STREAMS) == (streams or max(1, min(4, bufs - 1)))
        assert ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) <= budget
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload)
        assert _bits(ctx.verify(), P) == want
        assert ctx.counter(native.TV_COUNTER_WINDOWS) == -(-P // 9)
        ctx.stage(0, payload)                        # a new pass: the hash of every piece
        assert ctx.hash() == clean
        # uneven calls: pieces 0-40 in ragged parts, 41-59 never staged, the rest in one call
        for a, b in ((0, 5 * L + 3), (5 * L + 3, 5 * L + 4), (5 * L + 4, 41 * L)):
            ctx.stage(a, payload[a:b])
        ctx.stage(60 * L, payload[60 * L:])
        assert _bits(ctx.verify(), P) == [0 if 41 <= i < 60 else w for i, w in enumerate(want)]
        ctx.fill_synthetic(5)                        # the device generator fills every window
        synth = bytes(oracle.synth_fill(5, 0, total))
        assert ctx.hash() == bytes(oracle.hash_pieces(bytearray(synth), total, L, P))
