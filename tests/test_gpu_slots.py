"""Incremental verify over a slot pool (TV_OPT_LIST_SLOTS; SURVEY 8f row f1, torrent.ts:183-193).

Only the pieces awaiting verification hold device memory: K slots, whatever the torrent.  Checked at the ABI
(slot taking and freeing, the K + 1st piece refused, unstaged pieces 0, duplicates, the short last piece
listed among full ones) and through IncrementalVerifier on BASELINE config 4's geometry (200 GiB of 51,200
x 4 MiB pieces) holding K x stride of payload, against hashlib.
"""
import hashlib
import random

import pytest

pytestmark = pytest.mark.gpu


def test_slot_pool_abi(native, oracle):
    L, P = 4096, 40
    total = L * (P - 1) + 333                          # short last piece
    payload = bytes(oracle.synth_fill(21, 0, total))
    pieces = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    pieces[20 * 7] ^= 1                                 # piece 7 fails
    stride = L + 256

    def data(i):
        return payload[i * L:min(total, (i + 1) * L)]

    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_LIST_SLOTS, 4)
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        assert ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) == 4 * stride + 256
        for i in (39, 7, 3, 12):                        # the short last piece among them
            ctx.stage(i * L, data(i))
        assert ctx.counter(native.TV_COUNTER_SLOTS_USED) == 4
        with pytest.raises(native.NativeError) as e:
            ctx.stage(5 * L, data(5))                   # the 5th piece: no slot
        assert e.value.code == native.TV_ERR_STATE
        ctx.stage(3 * L, data(3))                       # re-staging a piece keeps its slot
        out = bytearray(L)
        ctx.read(12 * L, out)
        assert bytes(out) == data(12)
        ok = ctx.verify_list([3, 39, 7, 12, 3, 20])     # duplicates; 20 was never staged
        assert list(ok) == [1, 1, 0, 1, 1, 0]
        assert ctx.counter(native.TV_COUNTER_SLOTS_USED) == 0
        assert list(ctx.verify_list([3])) == [0]       # its slot was freed: never staged since
        order = list(range(P))
        random.Random(3).shuffle(order)
        for k in range(0, P, 4):                        # every piece, four at a time, in random order
            batch = order[k:k + 4]
            for i in batch:
                ctx.stage(i * L, data(i))
            assert list(ctx.verify_list(batch)) == [int(i != 7) for i in batch]
        with pytest.raises(native.NativeError) as e:
            ctx.verify()
        assert e.value.code == native.TV_ERR_STATE
        with pytest.raises(native.NativeError):
            ctx.hash()
        ctx.set_option(native.TV_OPT_LIST_SLOTS, 0)     # back to the resident shard
        ctx.set_layout(total, L, P)
        assert ctx.counter(native.TV_COUNTER_PAYLOAD_BYTES) == P * stride + 256


def test_incremental_verifier_on_cfg4_geometry_holds_k_slots(native, oracle):
    """IncrementalVerifier over the 200 GiB / 51,200 x 4 MiB torrent of BASELINE config 4 with K = 8 slots:
    blocks of 24 scattered pieces arrive interleaved in random order (with re-sends), two pieces corrupted; the
    device payload stays K x stride (32 MiB, not 200 GiB), forced flushes make room, every result equals
    hashlib's and the have-bits follow."""
    from torrent_amd import make_info
    from torrent_amd.incremental import IncrementalVerifier
    from torrent_amd.piece import BLOCK_SIZE, PieceMsg
    L, P = 4 << 20, 51200
    total = L * P
    rng = random.Random(4)
    chosen = sorted(rng.sample(range(P), 23) + [P - 1])
    datas = {i: bytes(oracle.synth_fill(4, i * L, L)) for i in chosen}
    digests = bytearray(rng.randbytes(20 * P))
    for i in chosen:
        digests[20 * i:20 * i + 20] = hashlib.sha1(datas[i]).digest()
    bad = set(rng.sample(chosen, 2))
    info = make_info(L, bytes(digests), "cfg4.bin", length=total)
    msgs = []
    for i in chosen:
        d = bytearray(datas[i])
        if i in bad:
            d[rng.randrange(L)] ^= 0x20
        msgs += [PieceMsg(i, o, bytes(d[o:o + BLOCK_SIZE])) for o in range(0, L, BLOCK_SIZE)]
    rng.shuffle(msgs)
    msgs += rng.sample(msgs, 50)
    seen = {}
    v = IncrementalVerifier(info, flush_pieces=None, flush_age_ms=None, slots=8,
                            on_verified=lambda i, ok: seen.setdefault(i, []).append(ok))
    try:
        assert v.device_payload_bytes() == 8 * (L + 256) + 256
        for m in msgs:
            v.on_block(m)
        for i, ok in v.flush():
            seen.setdefault(i, []).append(ok)
        assert v.forced_flushes >= 2
        assert v.device_payload_bytes() == 8 * (L + 256) + 256
        for i in chosen:
            assert seen[i][0] == (i not in bad), i
            assert bool(v.bitfield[i >> 3] & (0x80 >> (i & 7))) == (i not in bad)
        assert sum(bin(b).count("1") for b in v.bitfield) == len(chosen) - len(bad)
    finally:
        v.close()


def test_stage_files_on_a_slot_pool_with_two_lanes(native, oracle, tmp_path):
    """tv_stage_files deals long segments to two staging lanes (a helper thread on lane 1), and on a
    slot pool both lanes take slots for their pieces (piece_dst) at once: every staged piece must get a slot of its
    own, none lost or given twice.  Two files of long segments (>= TV_OPT_FILE_DIRECT_MIN) cut into many units;
    the pool holds every piece; verify_list reads each piece's own bytes."""
    L = 1 << 16
    per_file = 96                                    # pieces per file: 6 MiB each
    P = 2 * per_file
    total = L * P
    payload = bytes(oracle.synth_fill(31, 0, total))
    pieces = bytearray(oracle.hash_pieces(bytearray(payload), total, L, P))
    pieces[20 * 50] ^= 1
    paths = []
    for k in range(2):
        p = tmp_path / f"f{k}.bin"
        p.write_bytes(payload[k * per_file * L:(k + 1) * per_file * L])
        paths.append(str(p))
    with native.Context(0) as ctx:
        ctx.set_option(native.TV_OPT_LIST_SLOTS, P)
        ctx.set_option(native.TV_OPT_FILE_DIRECT_MIN, 1 << 20)
        ctx.set_option(native.TV_OPT_FILE_CHUNK, 1 << 20)     # 16 units over the two lanes
        ctx.set_option(native.TV_OPT_FILE_CONCURRENT, 1)
        ctx.set_layout(total, L, P)
        ctx.set_digests(bytes(pieces))
        for rep in range(3):
            st = ctx.stage_files(paths, [0, 0], [0, per_file * L], [per_file * L, per_file * L])
            assert list(st) == [native.TV_OK, native.TV_OK]
            assert ctx.counter(native.TV_COUNTER_SLOTS_USED) == P
            order = list(range(P))
            random.Random(rep).shuffle(order)
            ok = ctx.verify_list(order)
            assert list(ok) == [int(i != 50) for i in order]
            assert ctx.counter(native.TV_COUNTER_SLOTS_USED) == 0
