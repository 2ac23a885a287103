"""N>1 path on CPU: world_size-2 gloo processes, each verifying its 8-aligned piece shard.

This is the multi-GPU decomposition of bench.py / verify.shard_ranges: contiguous shards,
no data-path collective, bitfield slices concatenated by byte position; torch.distributed only for
barrier / max-over-ranks timing / correctness sum (bench._max, bench._sum).  The per-shard verify
here is the CPU oracle (the checker), since this container has no GPU; the GPU shard path itself is
tests/test_gpu_parity.py::test_shards_concatenate.
"""
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    import bench
    from oracle import oracle as O
    from torrent_amd.verify import shard_ranges
    dist, r, w, _ = bench._dist()
    assert (r, w) == (rank, ws)
    L, P = 4096, 203
    total = L * (P - 1) + 999
    payload = O.synth_fill(9, 0, total)
    pieces = bytearray(O.hash_pieces(payload, total, L, P))
    for i in range(0, P, 17):
        pieces[20 * i + 3] ^= 1
    first, count = shard_ranges(P, w)[r]
    assert first % 8 == 0 or count == 0       # an empty trailing shard may start anywhere
    full = O.verify_linear(payload, total, L, bytes(pieces))
    # shard-local verify: bits of pieces [first, first+count) (oracle as the stand-in worker)
    sl = bytearray((count + 7) // 8)
    for j in range(count):
        i = first + j
        if (full[i >> 3] >> (7 - (i & 7))) & 1:
            sl[j >> 3] |= 0x80 >> (j & 7)
    bench._barrier(dist)
    t = bench._max(dist, float(r + 1))
    ok = bench._sum(dist, 1.0)
    gathered = [None] * w
    dist.all_gather_object(gathered, (first, bytes(sl)))
    out = bytearray((P + 7) // 8)
    for f, b in gathered:
        out[f // 8:f // 8 + len(b)] = b
    placement = bench.rank_placement(dist, w, r, r, bench.pick_device(r, 1), 1)
    q.put((r, t, ok, bytes(out) == full, placement))
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 4, 8])
def test_gloo_two_ranks_shard_and_reduce(ws):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, t, ok, match, placement in res:
        assert t == float(ws)      # max over ranks
        assert ok == float(ws)     # sum over ranks
        assert match               # concatenated slices == single-shard bitfield
        # every rank sees every rank's placement (gathered over gloo), in rank order
        assert [p["rank"] for p in placement] == list(range(ws))
        assert all(p["device"] == 0 and p["local_rank"] == p["rank"] for p in placement)


def test_device_placement_rule():
    """bench.pick_device: LOCAL_RANK on a node where each rank sees all GPUs; 0 when the launcher gives each
    rank one GPU (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES); ranks wrap round on fewer GPUs (rehearsals)."""
    import bench
    assert [bench.pick_device(r, 8) for r in range(8)] == list(range(8))
    assert [bench.pick_device(r, 1) for r in range(8)] == [0] * 8
    assert [bench.pick_device(r, 4) for r in range(8)] == [0, 1, 2, 3, 0, 1, 2, 3]
    assert bench.pick_device(3, 0) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_two_ranks_on_the_hip_path(scaling):
    """The N>1 path itself, on one GPU: `torch.distributed.run --nproc-per-node 2 bench.py` (gloo barriers,
    max-over-ranks time), each rank verifying its shard of one torrent through the HIP library against the
    oracle's digests -- strong-scaled (the torrent's pieces split over the ranks) and weak-scaled (each rank its
    own whole-size shard of an N-times larger torrent, the default `value`); rank 0 prints one valid JSON line
    with an exact bitfield."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--workload", "tiny", "--" + scaling, "--steps", "3", "--warmup", "1", "--no-cfg4", "--e2e-steps", "0",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["scaling"] == scaling and rec["bitfield_exact"] is True
    assert "cfg4" in rec["scaling_note"] and rec["roofline"]["aggregate_piece_ceiling"] > 0
    if scaling == "strong":
        assert rec["config"]["total_pieces"] == 1000 and rec["config"]["pieces_per_gpu"] == 504
    else:
        assert rec["config"]["total_pieces"] == 2000 and rec["config"]["pieces_per_gpu"] == 1000


def test_aggregate_piece_ceiling_follows_the_shards():
    """bench.aggregate_piece_ceiling (what BASELINE configs[3], the 200 GiB cfg4 torrent sharded
    over N GPUs, can reach at most): the sum over verify.shard_ranges(51200, N) of each shard's piece ceiling under
    the kernel the library picks for it -- the lane kernel on one GPU (51,200 pieces saturate R_valu's cap), the
    twin kernel on 6,400-piece shards at N = 8 -- for N = 1, 2, 4, 8."""
    import bench
    from torrent_amd.verify import shard_ranges
    for n in (1, 2, 4, 8):
        shards = [c for _, c in shard_ranges(51200, n) if c]
        assert sum(shards) == 51200 and len(shards) == n
        want = sum(bench.piece_ceiling(bench.kernel_for(c), c) for c in shards)
        assert bench.aggregate_piece_ceiling("cfg4", n) == pytest.approx(want)
    assert [bench.kernel_for(c) for c in (6400, 12800, 16384, 16385, 25600, 32768, 32769, 51200)] == \
        [4, 4, 4, 2, 2, 2, 1, 1]
    one = bench.aggregate_piece_ceiling("cfg4", 1)
    assert one == pytest.approx(min(bench.VALU_PEAK_GBPS, bench.piece_ceiling(1, 51200)))
    eight = bench.aggregate_piece_ceiling("cfg4", 8)
    assert eight == pytest.approx(8 * bench.piece_ceiling(4, 6400))
    assert 4000 < eight < 5000     # piece-bound past one GPU (flat at ~4.2-4.5 TB/s measured)
