"""GPU tests of the round-3 boundary rules: zero-length segments checked behind the ABI (tv_stage_files),
allocation reuse and release (tv_set_layout, tv_get_counter), verify_piece's own context, the f1 flush
policy on the HIP path, and list flushes without companion workgroups."""
import hashlib
import os
import shutil

import pytest

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _bits(bf, n):
    return [(bf[i >> 3] >> (7 - (i & 7))) & 1 for i in range(n)]


def test_verify_files_zero_length_segments_match_fs_storage(native, tmp_path, monkeypatch):
    """Storage.get's zero-length segments (storage.ts:109-110: a file ending where a piece starts, a
    zero-length file inside a piece) go to tv_stage_files, which reports TV_ERR_IO where fsStorage.get's open
    (storage.ts:158) would fail: a directory in a zero-length file's place, or a zero-length file in a
    missing directory.  verify_files gives, piece for piece, the bits of Storage(fs_storage).get + SHA-1
    (run on a copy of the tree: that get creates files), and creates nothing itself."""
    from torrent_amd import make_info, verify_files
    from torrent_amd.metainfo import FileInfo
    from torrent_amd.piece import piece_length
    from torrent_amd.storage import Storage, fs_storage

    L = 4096
    names = [("a",), ("z_dir",), ("b",), ("nodir", "z"), ("c",), ("z_missing",), ("d",), ("z_ok",), ("e",)]
    sizes = [3 * L, 0, 2 * L + 100, 0, L - 100, 0, 2 * L, 0, L + 7]   # a, b end exactly on piece starts
    payload = bytes((k * 13 + 1) & 0xFF for k in range(sum(sizes)))
    P = -(-len(payload) // L)
    digests = bytearray(b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P)))
    digests[20 * 5] ^= 1                                          # one corrupted digest too
    info = make_info(L, bytes(digests), "t", files=[FileInfo(n, list(p)) for n, p in zip(sizes, names)])
    root = tmp_path / "t0"
    off = 0
    for n, p in zip(sizes, names):
        q = root.joinpath(*p)
        if p == ("z_dir",):
            q.mkdir(parents=True)
        elif p not in (("nodir", "z"), ("z_missing",)):
            q.parent.mkdir(parents=True, exist_ok=True)
            q.write_bytes(payload[off:off + n])
        off += n
    ref_root = tmp_path / "t1"
    shutil.copytree(root, ref_root)
    monkeypatch.chdir(tmp_path)
    ref = Storage(fs_storage, info, str(ref_root))
    expect = []
    for i in range(P):
        got = ref.get(i * L, piece_length(i, info))
        expect.append(int(got is not None and hashlib.sha1(got).digest() == bytes(digests[20 * i:20 * i + 20])))
    assert 0 < sum(expect) < P - 1
    before = sorted(str(x) for x in root.rglob("*"))
    for devices in ([0], [0, 0]):
        assert _bits(verify_files(info, str(root), devices=devices, threads=2), P) == expect, devices
    assert sorted(str(x) for x in root.rglob("*")) == before     # nothing created


def test_streamed_layout_after_a_resident_one_has_no_payload(native):
    """A layout set with TV_OPT_RESIDENT = 0 after a smaller resident one: the resident calls fail with
    TV_ERR_STATE (never run on the old, too-small buffer), and the payload is released."""
    with native.Context(0) as ctx:
        ctx.set_layout(64 * 1024, 4096, 16)                     # small resident layout
        ctx.set_digests(bytes(20 * 16))
        assert ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) > 0
        ctx.set_option(native.TV_OPT_RESIDENT, 0)
        ctx.set_layout(64 * MiB, MiB, 64)                       # larger, streamed-only
        ctx.set_digests(bytes(20 * 64))
        assert ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) == 0
        for call in (ctx.verify, ctx.hash, lambda: ctx.stage(0, b"x" * 100), lambda: ctx.fill_synthetic(1),
                     lambda: ctx.read(0, bytearray(100)), lambda: ctx.verify_list([3])):
            with pytest.raises(native.NativeError) as e:
                call()
            assert e.value.code == native.TV_ERR_STATE


def test_chunk_buffers_are_released_for_a_resident_layout(native, oracle):
    """The streamed path's two device chunk buffers are not kept beside a resident payload, and a streamed
    layout that fits them reuses them."""
    from torrent_amd import make_info, verify_payload, verify_stream
    L, P = MiB, 96
    payload = bytes(oracle.synth_fill(3, 0, L * P))
    info = make_info(L, oracle.hash_pieces(payload, L * P, L, P), "t", length=L * P)
    read = lambda off, n: payload[off:off + n]                      # noqa: E731
    from torrent_amd import verify as V
    V.release_contexts()
    assert verify_stream(info, read) == b"\xff" * (P // 8)
    c0 = V.context_counters()[(0, 0)]
    assert c0["payload_bytes"] == 0 and c0["device_bytes"] >= 2 * P * MiB
    assert verify_stream(info, read) == b"\xff" * (P // 8)        # same geometry: chunks reused
    c1 = V.context_counters()[(0, 0)]
    assert c1["device_allocs"] == c0["device_allocs"]
    assert verify_payload(info, payload) == b"\xff" * (P // 8)    # resident: chunks released first
    c2 = V.context_counters()[(0, 0)]
    assert c2["payload_bytes"] >= L * P
    assert c2["device_bytes"] < c2["payload_bytes"] + 64 * MiB
    V.release_contexts()


def test_piece_calls_do_not_evict_the_bulk_payload(native, oracle):
    """verify_piece runs on its own cached context: a 1 GiB verify_payload interleaved with 100 verify_piece
    calls allocates its resident payload once (library counter), and so does verify_piece."""
    from torrent_amd import make_info, verify_payload, verify_piece
    from torrent_amd import verify as V
    L, P = 4 * MiB, 256
    payload = bytes(oracle.synth_fill(21, 0, L * P))
    pieces = bytearray(oracle.hash_pieces(payload, L * P, L, P))
    pieces[20 * 7] ^= 1
    info = make_info(L, bytes(pieces), "t", length=L * P)
    want = bytearray(b"\xff" * (P // 8))
    want[0] &= ~0x01 & 0xFF
    V.release_contexts()
    for rnd in range(4):
        assert verify_payload(info, payload) == want
        for k in range(25):
            i = (rnd * 25 + k) * 2 % P
            assert verify_piece(info, i, payload[i * L:(i + 1) * L]) is (i != 7)
    cnt = V.context_counters()
    assert cnt[(0, 0)]["payload_allocs"] == 1, cnt
    assert cnt[(0, V._PIECE_SLOT)]["payload_allocs"] == 1, cnt
    assert cnt[(0, 0)]["payload_bytes"] >= L * P
    V.release_contexts()


def test_flush_policy_on_the_gpu(native, oracle):
    """IncrementalVerifier flushes by itself at K pending pieces (tv_verify_list launches counted through
    the callback), and the results match the oracle, a corrupted block included."""
    import random
    from torrent_amd import make_info
    from torrent_amd.incremental import IncrementalVerifier
    from torrent_amd.piece import BLOCK_SIZE, PieceMsg
    L, P = 2 * BLOCK_SIZE, 61
    total = L * (P - 1) + 777
    payload = bytes(oracle.synth_fill(5, 0, total))
    info = make_info(L, oracle.hash_pieces(payload, total, L, P), "t.bin", length=total)
    got = {}
    v = IncrementalVerifier(info, flush_pieces=8, flush_age_ms=None, on_verified=got.__setitem__)
    msgs = []
    for i in range(P):
        n = L if i < P - 1 else total - (P - 1) * L
        msgs += [PieceMsg(i, o, payload[i * L + o:i * L + min(n, o + BLOCK_SIZE)]) for o in range(0, n, BLOCK_SIZE)]
    random.Random(3).shuffle(msgs)
    bad = msgs[4]
    msgs[4] = PieceMsg(bad.index, bad.offset, bytes(b ^ 0x20 for b in bad.block))
    for m in msgs:
        v.on_block(m)
    assert v.auto_flushes == P // 8 and len(got) == 8 * (P // 8)
    for i, ok in v.flush():
        got[i] = ok
    assert got == {i: i != bad.index for i in range(P)}
    v.close()


@pytest.mark.parametrize("n", [1, 5, 64, 300])
def test_short_lists_run_without_companions(native, oracle, n):
    """tv_verify_list with fewer pieces than one twin workgroup holds launches no companion workgroups
    (they would all re-hash the same few pieces); results are exact either way."""
    L, P = 256 << 10, 512
    total = L * P
    payload = bytes(oracle.synth_fill(9, 0, total))
    pieces = bytearray(oracle.hash_pieces(payload, total, L, P))
    pieces[20 * 3 + 2] ^= 1
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload)
        lst = [(3 + 7 * k) % P for k in range(n)]
        assert list(ctx.verify_list(lst)) == [int(i != 3) for i in lst]
        assert ctx.last_kernel()[0] == native.KERNEL_TWIN
        assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == -(-n // 32)      # the real grid only
        ctx.set_option(native.TV_OPT_TWIN_FILL, 2)                                  # companions forced
        assert list(ctx.verify_list(lst)) == [int(i != 3) for i in lst]
        assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == 2 * _cus()


def _cus():
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_int(0)
    assert hip.hipDeviceGetAttribute(ctypes.byref(n), 63, 0) == 0     # hipDeviceAttributeMultiprocessorCount
    return n.value


def test_long_lists_keep_companions(native, oracle):
    """A list that gives every CU a twin workgroup (>= 32 x CUs pieces) keeps its companions (2 x CUs
    workgroups), as resident launches do."""
    cus = _cus()
    L, P = 16 << 10, 32 * cus
    total = L * P
    with native.Context(0) as ctx:
        ctx.set_layout(total, L, P)
        ctx.fill_synthetic(4)
        d = bytearray(ctx.hash())
        d[20 * 9] ^= 1
        ctx.set_digests(bytes(d))
        lst = list(range(P))
        assert list(ctx.verify_list(lst)) == [int(i != 9) for i in lst]
        assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == 2 * cus


def test_failed_segment_marks_last_until_the_next_layout(native, tmp_path):
    """A file segment the library could not read whole marks, inside the library, exactly the pieces
    Storage.get would return null for: a 10-piece file 3 pieces + 5 bytes long keeps pieces 0-2 (staged from
    the file's prefix) and loses 3-9.  The marks hold for tv_verify (no availability from the host) and for
    tv_verify_list, end for the pieces a later call stages whole (the bytes were repaired: ADVICE r03), and
    all end with the next tv_set_layout."""
    L, P = 4096, 10
    payload = bytes((k * 29 + 7) & 0xFF for k in range(L * P))
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    f = tmp_path / "short.bin"
    f.write_bytes(payload[:3 * L + 5])
    with native.Context(0) as ctx:
        ctx.set_layout(L * P, L, P)
        ctx.set_digests(digests)
        ctx.stage(0, payload)                                       # every byte right before the file read
        assert ctx.stage_files([str(f)], [0], [0], [L * P]) == [native.TV_ERR_IO]
        want = [1, 1, 1] + [0] * 7
        assert _bits(ctx.verify(), P) == want
        assert list(ctx.verify_list(list(range(P)))) == want
        ctx.stage(0, payload[:5 * L + 7])                           # pieces 0-4 staged whole: unmarked
        assert _bits(ctx.verify(), P) == [1] * 5 + [0] * 5
        assert not ctx.stage_file(str(tmp_path / "absent.bin"), 0, 0, L)   # a missing file marks piece 0
        assert _bits(ctx.verify(), P) == [0] + [1] * 4 + [0] * 5
        ctx.set_layout(L * P, L, P)                                 # a new layout clears them
        ctx.set_digests(digests)
        ctx.stage(0, payload)
        assert _bits(ctx.verify(), P) == [1] * P


def test_hash_files_refuses_a_short_or_missing_file(native, tmp_path):
    """Creation from disk (f3, make_torrent.ts:62-113) hashes the files concatenated in order, and raises
    instead of hashing a file that is short or missing -- the library's recovery keeps a short file's whole
    pieces readable for verification, so hash_files checks the statuses, not the availability bits."""
    from torrent_amd.metainfo import FileInfo, make_info
    from torrent_amd.verify import hash_files
    L = 4096
    sizes = [5 * L + 11, 0, 3 * L, 2 * L + 9]
    payload = bytes((k * 31 + 5) & 0xFF for k in range(sum(sizes)))
    P = -(-len(payload) // L)
    want = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    info = make_info(L, bytes(20 * P), "t", files=[FileInfo(n, [f"f{k}"]) for k, n in enumerate(sizes)])
    off = 0
    for k, n in enumerate(sizes):
        (tmp_path / f"f{k}").write_bytes(payload[off:off + n])
        off += n
    for devices in ([0], [0, 0]):
        assert hash_files(info, str(tmp_path), devices=devices) == want
    (tmp_path / "f2").write_bytes(payload[sizes[0]:sizes[0] + 3 * L - 1])     # one byte short
    with pytest.raises(FileNotFoundError):
        hash_files(info, str(tmp_path))
    (tmp_path / "f2").unlink()
    with pytest.raises(FileNotFoundError):
        hash_files(info, str(tmp_path), devices=[0, 0])


def test_numa_binding_places_the_ring_and_keeps_results(native, tmp_path):
    """TV_OPT_NUMA_BIND (default on): the ctx knows its GPU's NUMA node (sysfs numa_node of the GPU's PCI
    function), allocates its pinned ring there, and the bits of a files staging are the same bound and
    unbound (the binding moves the library's threads, nothing else)."""
    import ctypes
    L, P = 65536, 40
    payload = bytes((k * 11 + 3) & 0xFF for k in range(L * P - 777))
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    f = tmp_path / "t.bin"
    f.write_bytes(payload)
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    assert hip.hipDeviceGetPCIBusId(buf, 64, 0) == 0
    try:
        sys_node = int(open(f"/sys/bus/pci/devices/{buf.value.decode().lower()}/numa_node").read())
    except OSError:
        sys_node = -1
    results = []
    for bind in (1, 0):
        with native.Context(0) as ctx:
            assert ctx.get_option(native.TV_OPT_NUMA_BIND) == 1
            node = ctx.counter(native.TV_COUNTER_NUMA_NODE)
            assert node == (sys_node if sys_node >= 0 else 2 ** 64 - 1)
            ctx.set_option(native.TV_OPT_NUMA_BIND, bind)
            ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, 1 << 62)          # every segment via the readers
            ctx.set_layout(len(payload), L, P)
            ctx.set_digests(digests)
            assert ctx.counter(native.TV_COUNTER_RING_NODE) == 2 ** 64 - 1    # no ring yet
            segs = [(0, 5 * L + 9), (5 * L + 9, 17 * L), (22 * L + 9, len(payload) - 22 * L - 9)]
            st = ctx.stage_files([str(f)] * 3, [a for a, _ in segs], [a for a, _ in segs], [n for _, n in segs])
            assert st == [0, 0, 0]
            if bind and sys_node >= 0:
                assert ctx.counter(native.TV_COUNTER_RING_NODE) == sys_node
            results.append(bytes(ctx.verify()))
    assert results[0] == results[1] and _bits(results[0], P) == [1] * P


def test_contexts_release_threads_and_memory(native, tmp_path):
    """tv_destroy releases everything a ctx took: 30 create / stage-from-files / verify / destroy cycles (each
    ctx spins up two pinned rings, its reader pool and the staging helper lane) leave the process's thread
    count, the device's free memory and the resident set where they started."""
    import ctypes
    L, P = 65536, 64
    payload = bytes((k * 7 + 1) & 0xFF for k in range(L * P))
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(P))
    files = []
    for k in range(4):
        f = tmp_path / f"f{k}"
        f.write_bytes(payload[k * 16 * L:(k + 1) * 16 * L])
        files.append(str(f))
    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()

    def state():
        assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
        rss = next(int(line.split()[1]) for line in open("/proc/self/status") if line.startswith("VmRSS:")) << 10
        return len(os.listdir("/proc/self/task")), free.value, rss

    def cycle():
        with native.Context(0) as ctx:
            ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, 8 * L)       # two lanes: helper thread + readers
            ctx.set_layout(L * P, L, P)
            ctx.set_digests(digests)
            assert ctx.stage_files(files, [0] * 4, [k * 16 * L for k in range(4)], [16 * L] * 4) == [0] * 4
            assert _bits(ctx.verify(), P) == [1] * P

    cycle()                                                          # runtime-level first-use allocations
    threads0, free0, rss0 = state()
    for _ in range(30):
        cycle()
    threads1, free1, rss1 = state()
    assert threads1 <= threads0, (threads0, threads1)
    assert free1 >= free0 - (64 << 20), (free0, free1)               # no device memory left behind
    assert rss1 <= rss0 + (256 << 20), (rss0, rss1)                  # nor pinned rings (384 MiB a ctx)


@pytest.mark.gpu
def test_companions_stand_down_on_a_shared_gpu(native, oracle):
    """TV_OPT_TWIN_FILL = 1 (auto): while another process holds >= 1 GiB of the GPU's memory (the kernel driver's
    per-process accounting, /sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>), a twin launch with fewer than 2 x CUs
    workgroups runs its real grid only -- the companions would take CUs the other process may be using; once it has
    gone they are back.  3 keeps them regardless.  The bits are the same every time."""
    import subprocess
    import sys
    import time
    L, P = 1 << 16, 64 * 32            # 64 twin workgroups: fewer than 2 per CU
    payload = bytes(oracle.synth_fill(61, 0, L * P))
    pieces = bytearray(oracle.hash_pieces(bytearray(payload), L * P, L, P))
    pieces[20 * 9] ^= 1
    cus = _cus()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with native.Context(0) as ctx:
        if ctx.counter(native.TV_COUNTER_KFD_GPU_ID) == 0:
            pytest.skip("the kernel driver's process accounting is not readable here")
        ctx.set_option(native.TV_OPT_KERNEL, native.KERNEL_TWIN)
        ctx.set_layout(L * P, L, P)
        ctx.set_digests(bytes(pieces))
        ctx.stage(0, payload)
        for _ in range(10):       # (a process an earlier test started may still be letting go of the GPU)
            if ctx.counter(native.TV_COUNTER_COTENANT_VRAM) < (1 << 30):
                break
            time.sleep(1.1)
        else:
            pytest.skip("another process holds >= 1 GiB of this GPU: the 'alone' half cannot run here")
        want = ctx.verify()
        assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == 2 * cus          # alone: companions
        child = subprocess.Popen(
            [sys.executable, "-c",
             "import sys; sys.path.insert(0, %r)\n"
             "from torrent_amd import _native\n"
             "c = _native.Context(0)\n"
             "c.set_layout(2 << 30, 1 << 20, 2048)\n"         # ~2 GiB of resident payload
             "c.fill_synthetic(1)\n"
             "print('ready', flush=True)\n"
             "sys.stdin.read()\n" % root],
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        try:
            assert child.stdout.readline().strip() == "ready"
            time.sleep(1.1)                                  # (the library re-reads the accounting once a second)
            assert ctx.counter(native.TV_COUNTER_COTENANT_VRAM) >= (1 << 30)
            assert ctx.verify() == want
            assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == P // 32    # the real grid only
            ctx.set_option(native.TV_OPT_TWIN_FILL, 3)
            assert ctx.verify() == want
            assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == 2 * cus    # forced on
            ctx.set_option(native.TV_OPT_TWIN_FILL, 1)
        finally:
            child.stdin.close()
            child.wait(timeout=60)
        time.sleep(1.1)
        assert ctx.verify() == want
        assert ctx.counter(native.TV_COUNTER_LAST_WORKGROUPS) == 2 * cus          # alone again


def test_verify_files_name_with_a_nul_reads_as_null(native, tmp_path, monkeypatch):
    """A file name holding a NUL cannot be opened (Deno.open throws inside fsStorage.get's try, so the reference's
    piece is null, storage.ts:157-170): verify_files reports its pieces 0 -- no exception -- and the pieces of the
    other files as their bytes say."""
    from torrent_amd import make_info, verify_files
    from torrent_amd.metainfo import FileInfo
    L = 4096
    payload = bytes((j * 7 + 3) & 0xFF for j in range(3 * L))
    # a: piece 0; the NUL name: 100 bytes of piece 1; c: the rest of piece 1 and piece 2 (the NUL name does not end
    # on piece 2's start, where Storage.get's walk would open it again with 0 bytes and null piece 2 as well)
    sizes, names = [L, 100, 2 * L - 100], [["a.bin"], ["bad\0name"], ["c.bin"]]
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(3))
    info = make_info(L, digests, "t", files=[FileInfo(n, p) for n, p in zip(sizes, names)])
    (tmp_path / "a.bin").write_bytes(payload[:L])
    (tmp_path / "c.bin").write_bytes(payload[L + 100:])
    monkeypatch.chdir(tmp_path)
    assert _bits(verify_files(info, str(tmp_path)), 3) == [1, 0, 1]


@pytest.mark.gpu
def test_verify_files_fifo_in_the_table_reads_as_null(native, tmp_path, monkeypatch):
    """A named pipe where the table has a 2 MiB file: fsStorage.get opens it (read + write: no block) and its seek
    fails, so the reference's pieces over it are null.  Every file path -- staged in windows or whole, streamed in
    columns (whose residency sample opens files nonblocking and samples only regular files) -- reports them 0 without
    blocking, and the other pieces as their bytes say."""
    from torrent_amd import make_info, verify_files
    from torrent_amd.metainfo import FileInfo
    MiB = 1 << 20
    L = MiB
    payload = bytes((j * 13 + 5) & 0xFF for j in range(5 * L))
    sizes, names = [2 * L, 2 * L, L], [["a.bin"], ["p.fifo"], ["c.bin"]]
    digests = b"".join(hashlib.sha1(payload[i * L:(i + 1) * L]).digest() for i in range(5))
    info = make_info(L, digests, "t", files=[FileInfo(n, p) for n, p in zip(sizes, names)])
    (tmp_path / "a.bin").write_bytes(payload[:2 * L])
    os.mkfifo(tmp_path / "p.fifo")
    (tmp_path / "c.bin").write_bytes(payload[4 * L:])
    monkeypatch.chdir(tmp_path)
    for kw in ({}, {"stream": False, "budget": 2 * (L + 256) * 3}, {"stream": True, "budget": 1 << 24},
               {"stream": True}):
        assert _bits(verify_files(info, str(tmp_path), threads=2, **kw), 5) == [1, 1, 0, 0, 1], kw
