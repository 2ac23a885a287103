#!/usr/bin/env python3
"""Benchmark: verified GB/s of SHA-1 piece verification, HBM-resident (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2|cfg4|suppl|p262k] [--weak|--strong]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`value` (the timed workload): BASELINE configs[1] = cfg2, a 16 GiB synthetic single-file torrent in 16,384 pieces
of 1 MiB, HBM-resident on one MI355X; at N > 1 weak-scaled (the pieces are independent units, sharded with no
data-path collective): an N x 16 GiB torrent of N x 16,384 pieces, rank r verifying its contiguous 16 GiB shard,
so the driver's 1 -> 8 curve is one configuration.  `--workload cfg4 --strong` times BASELINE configs[3] instead.
  One step = one tv_verify of the rank's whole resident shard (availability bits up, the verify kernel,
  the bitfield slice down).  W untimed steps, then exactly K steps between a barrier + device synchronize
  on both sides; time = max over ranks; value = bytes of all ranks' shards x K / time.

Expected values are the CPU ORACLE's (oracle/sha1_oracle.c, pinned by the reference's own test_data
digests): the rank's whole shard is hashed on the host's cores before the timed region and 1 % of the
digests are corrupted, so `bitfield_exact` means "equal, on every piece, to the oracle's bitfield".

Legs reported beside `value` (never as it):
  * cfg4: BASELINE configs[3], ONE 200 GiB torrent in 51,200 pieces of 4 MiB, strong-scaled: rank r verifies
    the contiguous 8-aligned shard shard_ranges(51200, N)[r] (the bitfield slices are whole bytes and
    concatenate); at N = 1 the whole torrent on one GPU.  Piece-bound past one GPU.
  * e2e_cfg5: BASELINE configs[4], the end-to-end resume check: the cfg4 torrent streamed from host memory
    over PCIe through the library's BOUNDED pinned ring (tv_stream_*; 3 x 64 MiB per GPU, no resident
    payload, no whole-shard host buffer), each rank its shard.  `generated`: the bytes are produced by the
    host generator into the ring slots inside the timed region; `pinned_pool`: rows are DMA'd straight
    from a 1 GiB page-locked pool of pre-generated pieces (the torrent is that pool repeated), i.e. the
    PCIe path without the producer.
  * cfg3 (N = 1): BASELINE configs[2], the multi-file torrent (10,000 files, 256 KiB pieces spanning files, short
    final piece, 1 % corrupted) staged file by file, resident verify at the live clock + one-shot wall clock.
  * piece_saturated (N = 1): 65,536 x 256 KiB pieces (SURVEY 8d suppl.) against the VALU roofline.
  * cpu_baseline (rank 0, N = 1): the oracle (C port of the per-piece SHA-1 path, SHA-NI) on the host's
    allowed cores: a bounded sample of the cfg2 workload, BASELINE configs[0] (cfg1) as its own entry, the
    1-core figure, and the full-shard ground-truth pass.

The roofline object is for the verify kernel: algorithmic bytes per launch (the shard's payload bytes,
SURVEY.md 8d: each payload byte read once) / the average kernel duration from HIP events recorded on the
library's compute stream around each launch, against min(HBM peak, the measured SHA-1 VALU roofline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from torrent_amd import _native  # noqa: E402  (load the HIP library before torch)
from torrent_amd.verify import shard_ranges  # noqa: E402
from torrent_amd._cpu import cpu_share  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# SHA-1 VALU roofline from the measured SIMD cost per wave64 instruction (tools/ubench_simd.hip,
# profiles/r01/ubench_simd.log): v_alignbit / v_add3 / v_perm 4 cycles (half rate), v_bitop3 / VOP2 2
# cycles (full rate).  Minimal mix per 64-B block: 224 alignbit + 160 add3 + 16 perm (400 x 4) + 144
# bitop3 + 64 xor + 5 add (213 x 2) = 2,026 SIMD cycles per 64 lanes.
CLOCK_HZ = 2.4e9
SIMD_CYC_PER_BLOCK = 400 * 4 + 213 * 2
VALU_PEAK_GBPS = 1024 * 64 * 64 * CLOCK_HZ / SIMD_CYC_PER_BLOCK / 1e9
ROOF_PEAK_GBPS = min(HBM_PEAK_GBPS, VALU_PEAK_GBPS)
VALU_DERIVATION = (
    "R_valu = 1024 SIMDs x 64 lanes x 64 B x 2.4 GHz / 2,026 SIMD cycles per block. 2,026 = the minimal "
    "gfx950 SHA-1 mix per 64-B block at the per-op SIMD costs measured by tools/ubench_simd.hip "
    "(profiles/r01/ubench_simd.log): 400 half-rate ops x 4 cyc (224 v_alignbit_b32 rotates, 160 v_add3_u32, "
    "16 v_perm_b32 byte swaps) + 213 full-rate ops x 2 cyc (144 v_bitop3_b32, 64 v_xor_b32, 5 v_add_u32). "
    "MI355X_MICROARCH.md gives 2-cycle full-rate wave64 VALU for every op, which would make it 1,226 cycles "
    "and R_valu 8.2 TB/s (> HBM); the ubench measures v_alignbit/v_add3/v_perm at 4.06-4.25 cycles, half "
    "rate, so the binding roofline is R_valu, not HBM")
# Cycles per VALU instruction of a lone wave: 4.07 for 8-byte VOP3 ops in a long loop body, 4.09 for the
# SHA-1 round mix (tools/ubench_fetch.hip, profiles/r01/ubench_fetch.log); the wave64 cadence is 4.
LONE_WAVE_CYC = 4.07
SERIAL_INSTR = {1: 613, 2: 405, 4: 405}  # per-block serial VALU stream: lane kernel / split and twin rounds waves
KERNEL_NAMES = {1: "lane", 2: "split", 4: "twin"}


def piece_ceiling(kernel: int, count: int) -> float:
    """GB/s if every piece advanced at its kernel's serial SHA-1 stream's lone-wave rate (count pieces x
    64 B per block / (serial instructions per block x 4.07 cycles)), capped at R_valu."""
    rate = 64 * CLOCK_HZ / (SERIAL_INSTR.get(kernel, SERIAL_INSTR[1]) * LONE_WAVE_CYC)   # B/s per piece
    return min(VALU_PEAK_GBPS, count * rate / 1e9)

def kernel_for(count: int, cus: int = 256) -> int:
    """The library's automatic kernel for a resident launch of `count` full pieces (tv_core.hip choose_kernel_n):
    twin while its 32-piece workgroups number <= 2 per CU, split up to 32,768 pieces, the lane kernel beyond."""
    if (count + 31) // 32 <= 2 * cus:
        return 4
    return 2 if count <= 32768 else 1


def aggregate_piece_ceiling(workload: str, n_gpus: int, cus: int = 256) -> float:
    """What a STRONG-scaled resident workload (one torrent, shard_ranges over n_gpus) can reach at most in all:
    the sum over ranks of each shard's piece-parallelism ceiling under the kernel the library picks for it."""
    _, P, _, _ = WORKLOADS[workload]
    return sum(piece_ceiling(kernel_for(c, cus), c) for _, c in shard_ranges(P, n_gpus) if c)


# one page-locked 1 GiB host -> HBM copy on a gpurun box (tools/pcie_probe.py, profiles/r02/pcie_ceiling.json)
PCIE_H2D_GBPS = 57.6

MiB = 1 << 20
WORKLOADS = {
    # name: (piece_length, pieces (per GPU for weak, whole torrent for strong), seed, description)
    "cfg1": (256 << 10, 256, 1, "cfg1: 64 MiB synthetic single file, 256 KiB pieces (256 pieces)"),
    "cfg2": (MiB, 16384, 2, "cfg2: 16 GiB synthetic single-file torrent, 1 MiB pieces (16384 pieces), HBM-resident"),
    "cfg4": (4 * MiB, 51200, 4, "cfg4: 200 GiB synthetic single-file torrent, 4 MiB pieces (51200 pieces), HBM-resident"),
    "suppl": (256 << 10, 65536, 6, "suppl: 16 GiB, 256 KiB pieces (65536 pieces), HBM-resident"),
    "p262k": (64 << 10, 262144, 7, "p262k: 16 GiB, 64 KiB pieces (262144 pieces), HBM-resident (VALU-saturating)"),
    "tiny": (64 << 10, 1000, 9, "tiny: 62.5 MiB, 64 KiB pieces (1000 pieces) -- multi-rank rehearsals and tests only"),
}
POOL_PIECES = 256          # e2e pinned_pool: 256 x 4 MiB = 1 GiB page-locked pool
E2E_CHUNK = 256 << 10      # e2e column width: one 64 MiB ring request = 256 rows = the whole pool


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist
        # gloo prints its "connected to N peer ranks" banner on fd 1 from C++: send it to stderr, so the
        # bench's stdout carries exactly one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", init_method="env://")
            dist.barrier()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        return dist, rank, ws, local
    return None, 0, 1, 0


def _barrier(dist):
    if dist is not None:
        dist.barrier()


def _max(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def pick_device(local_rank: int, visible: int) -> int:
    """HIP device of a rank: LOCAL_RANK when the rank sees every GPU of the node, 0 when the launcher made
    one GPU visible per rank (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES), and ranks wrap round when there
    are more ranks than GPUs (rehearsals on one GPU)."""
    return local_rank % max(1, visible)


def _pci_bus_id(device: int) -> str:
    """PCI bus id of HIP device `device` (hipDeviceGetPCIBusId), to tell physical GPUs apart across ranks."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) == 0:
            return buf.value.decode()
    except OSError:
        pass
    return f"unknown-{device}"


def rank_placement(dist, ws: int, rank: int, local: int, device: int, ndev: int) -> list:
    """Every rank's (rank, LOCAL_RANK, device, PCI bus id, visibility variables), gathered on all ranks."""
    me = {"rank": rank, "local_rank": local, "device": device, "visible_devices": ndev,
          "pci_bus_id": _pci_bus_id(device), "host": os.uname().nodename,
          **{k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
             if os.environ.get(k) is not None}}
    if dist is None:
        return [me]
    out = [None] * ws
    dist.all_gather_object(out, me)
    return out


def _device_sync(ctx, device: int) -> None:
    ctx.synchronize()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize(device)
    except Exception:
        pass


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _corrupt(dig: bytearray, count: int, salt: int) -> set:
    """Corrupt 1 % of a shard's digests (every 100th piece, plus its last) -> the pieces expected to fail."""
    bad = set(range(salt % 100, count, 100)) | {count - 1}
    for j in bad:
        dig[20 * j + 7] ^= 0x10
    return bad


def _expected_bits(count: int, bad: set) -> bytes:
    out = bytearray(b"\xff" * ((count + 7) // 8))
    if count % 8:
        out[-1] = (0xFF00 >> (count % 8)) & 0xFF
    for j in bad:
        out[j >> 3] &= ~(0x80 >> (j & 7)) & 0xFF
    return bytes(out)


def ground_truth(seed: int, total: int, L: int, P: int, first: int, count: int, threads: int) -> tuple:
    """The oracle's digests of the shard's synthetic pieces (generated and hashed on `threads` host cores;
    outside every timed region) and the seconds it took."""
    from oracle import oracle as O
    O.set_impl("best")
    t0 = time.perf_counter()
    d = O.synth_piece_digests(seed, total, L, P, first, count, threads=threads)
    return d, time.perf_counter() - t0


def _traffic(workload: str, bytes_per_launch: int) -> tuple:
    """(HBM bytes per launch, note) from profiles/traffic_<workload>.json (PMC passes, corrected as the MI355X guide
    prescribes), when it was measured on this launch geometry AND on this build of the library (its build_id is
    the source id compiled into the library the bench loaded); else (None, why not)."""
    tpath = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if not os.path.exists(tpath):
        return None, f"no PMC record ({os.path.relpath(tpath, ROOT)})"
    try:
        rec = json.load(open(tpath))
    except Exception as exc:
        return None, f"unreadable PMC record: {exc}"
    if rec.get("payload_bytes_per_launch") != bytes_per_launch:
        return None, "the PMC record is of another launch geometry"
    lib_id = _native.build_id()
    if rec.get("build_id") != lib_id:
        return None, (f"the PMC record was measured on build {rec.get('build_id')}, the library timed is build "
                      f"{lib_id}: re-measure (tools/gpu_r05_pmc.sh)")
    return rec.get("hbm_bytes_per_launch"), (f"{os.path.relpath(tpath, ROOT)}: PMC passes on build {lib_id}, "
                                             f"{rec.get('method', '')[:160]}")


def resident_leg(dist, ws: int, rank: int, device: int, workload: str, strong: bool, steps: int, warmup: int,
                 kernel_opt: int, threads: int, want_digests: bool = False) -> dict:
    """One resident workload on every rank: synthetic payload filled in HBM by the device generator, oracle
    digests with 1 % corrupted, W + K timed verify steps.  Every rank runs it (barriers inside)."""
    L, n, seed, desc = WORKLOADS[workload]
    if strong:
        P = n
        first, count = shard_ranges(P, ws)[rank]
    else:
        P = n * ws
        first, count = rank * n, n
    total = L * P
    t_leg = time.perf_counter()
    dig, gt_s = ground_truth(seed, total, L, P, first, count, threads)
    t_setup = time.perf_counter()
    ctx = _native.Context(device)
    try:
        ctx.set_option(_native.TV_OPT_KERNEL, kernel_opt)
        ctx.set_clock_probe(True)   # workgroup 0 samples the shader clock it runs at
        ctx.set_layout(total, L, P, first, count)
        # a resident step re-hashes the whole shard: the layout must hold it whole (a windowed layout, for a
        # shard above the device budget, would hash once per pass and make repeated verifies compares)
        if ctx.counter(_native.TV_COUNTER_WINDOW_PIECES):
            raise RuntimeError(f"{workload}: the shard does not fit the device budget "
                               f"({ctx.counter(_native.TV_COUNTER_BUDGET)} B); the resident bench needs it whole")
        ctx.fill_synthetic(seed)
        creation_exact = ctx.hash() == dig            # creation mode (make_torrent.ts:28-31) at full size
        d2 = bytearray(dig)
        bad = _corrupt(d2, count, seed)
        pieces = bytearray(20 * P)
        pieces[20 * first:20 * (first + count)] = d2
        ctx.set_digests(bytes(pieces))
        expect = _expected_bits(count, bad)
        # torch's device context is created by the first _device_sync (~1.5 s, GPU idle): do that before the
        # warmup, so the warmup -- not the first timed steps -- brings the shader clock back up
        _device_sync(ctx, device)
        t_warm = time.perf_counter()
        for _ in range(warmup):
            ctx.verify()
        _device_sync(ctx, device)
        t_warm_end = time.perf_counter()
        _barrier(dist)
        kernel_ms = []
        t0 = time.perf_counter()
        for _ in range(steps):
            bf = ctx.verify()
            kernel_ms.append(ctx.last_timing()[0])
        _device_sync(ctx, device)
        t1 = time.perf_counter()
        _barrier(dist)
        kernel, _ = ctx.last_kernel()
        clock_ghz = ctx.last_clock_khz() / 1e6   # (after the timed region: it syncs)
        grid = ctx.counter(_native.TV_COUNTER_LAST_WORKGROUPS)
        cotenant = ctx.counter(_native.TV_COUNTER_COTENANT_VRAM)
    finally:
        ctx.close()
    t_end = time.perf_counter()
    elapsed = _max(dist, t1 - t0)
    exact = _sum(dist, 1.0 if (bf == expect and creation_exact) else 0.0) == ws
    avg = sum(kernel_ms) / len(kernel_ms)
    bytes_rank = L * count
    bytes_all = _sum(dist, float(bytes_rank))
    achieved = bytes_rank / (avg / 1e3) / 1e9
    ceiling = piece_ceiling(kernel, count)
    ceiling_all = _sum(dist, ceiling)   # every rank's shard at its own kernel's piece ceiling
    if strong:
        what = desc.split(" (")[0] + f" ({P} pieces in all, {ws} shard(s), strong scaling)"
    elif ws > 1:
        what = desc + f"; per GPU: one {ws}-shard torrent of {P} pieces, each rank its {n}-piece shard (weak scaling)"
    else:
        what = desc
    out = {"workload": what,
           "piece_length": L, "total_pieces": P, "pieces_per_gpu": count, "bytes_per_gpu": bytes_rank,
           "value": round(bytes_all * steps / elapsed / 1e9, 2), "unit": "GB/s", "steps": steps, "warmup": warmup,
           "ms_per_step": round(elapsed * 1e3 / steps, 3), "scaling": "strong" if strong else "weak",
           "kernel": KERNEL_NAMES.get(kernel, str(kernel)), "kernel_ms_avg": round(avg, 3),
           "kernel_ms_median": round(sorted(kernel_ms)[len(kernel_ms) // 2], 3),
           "kernel_ms_min_max": [round(min(kernel_ms), 3), round(max(kernel_ms), 3)],
           "kernel_ms_max_over_ranks": round(_max(dist, avg), 3), "achieved": round(achieved, 1),
           "piece_parallelism_ceiling": round(ceiling, 1), "frac_of_piece_ceiling": round(achieved / ceiling, 4),
           "frac_of_valu_peak": round(achieved / VALU_PEAK_GBPS, 4),
           "aggregate_piece_ceiling": round(ceiling_all, 1),
           "frac_of_aggregate_piece_ceiling": round(bytes_all * steps / elapsed / 1e9 / ceiling_all, 4),
           "aggregate_note": "the sum over ranks of each rank's shard piece ceiling (its kernel's serial SHA-1 rate "
                             "x its pieces): the most this configuration can verify per second on these GPUs; "
                             "frac_of_aggregate_piece_ceiling = value / it",
           "clock_ghz": round(clock_ghz, 3) if clock_ghz else None,
           "frac_of_valu_peak_at_clock": round(achieved / (VALU_PEAK_GBPS * clock_ghz / (CLOCK_HZ / 1e9)), 4)
           if clock_ghz else None,
           "clock_note": "shader clock of the last timed launch (its workgroup 0's shader-counter ticks over 100 MHz "
                         "real-time ticks, TV_OPT_CLOCK_PROBE); R_valu is quoted at 2.4 GHz, "
                         "frac_of_valu_peak_at_clock rescales it to this clock",
           "workgroups": grid, "cotenant_vram_max_over_ranks": int(_max(dist, float(cotenant))),
           "grid_note": "workgroups of the last launch (twin with fewer than 2 per CU: companions fill it to 2 x CUs "
                        "unless other processes hold >= 1 GiB of the GPU, cotenant_vram: KFD accounting)",
           "bitfield_exact": exact, "expected": "oracle digests of every piece, 1 % corrupted",
           "ground_truth_s": round(gt_s, 2), "ground_truth_threads": threads,
           "phase_s": {"ground_truth": round(gt_s, 2), "setup": round(t_warm - t_setup, 2),
                       "warmup": round(t_warm_end - t_warm, 3), "timed": round(t1 - t0, 3),
                       "leg": round(t_end - t_leg, 2), "leg_max_over_ranks": round(_max(dist, t_end - t_leg), 2),
                       "note": "this rank's wall seconds; setup = context, layout, device fill, creation-mode "
                               "hash check and digests"}}
    if want_digests:
        out["_digests"] = dig
        out["_first"] = first
    return out


def producer_rate(ctx, seed: int, seconds: float = 1.0) -> float:
    """GB/s of the host generator alone (tv_stream_fill_synthetic into one lent ring slot, no DMA), on the
    ctx's TV_OPT_FILE_THREADS threads.  Every rank runs it at the same time, so the sum over ranks is what
    the node's CPU share generates with this per-rank budget."""
    ctx.stream_begin()
    try:
        req = ctx.stream_next()
        nbytes = req.rows * req.width
        reps, t0 = 0, time.perf_counter()
        while True:
            ctx.stream_fill_synthetic(req, seed)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return nbytes * reps / el / 1e9
    finally:
        ctx.stream_abort()


def e2e_cfg5(dist, ws: int, rank: int, device: int, steps: int, threads: int, shard_digests=None,
             share: dict = None, physical_gpus: int = 1) -> dict:
    """BASELINE configs[4]: the cfg4 torrent (200 GiB, 51,200 x 4 MiB) streamed host -> PCIe -> HBM through the
    library's bounded pinned ring (tv_stream_*), each rank its shard_ranges shard, no resident payload."""
    from oracle import oracle as O
    L, P, seed, _ = WORKLOADS["cfg4"]
    total = L * P
    first, count = shard_ranges(P, ws)[rank]
    if shard_digests is None:
        shard_digests, _ = ground_truth(seed, total, L, P, first, count, threads)
    d2 = bytearray(shard_digests)
    bad = _corrupt(d2, count, 5)
    pieces = bytearray(20 * P)
    pieces[20 * first:20 * (first + count)] = d2
    expect = _expected_bits(count, bad)
    out = {"workload": "cfg5: the cfg4 torrent (200 GiB, 51200 x 4 MiB) streamed from host memory over PCIe "
                       "through the bounded pinned ring, copy/compute overlapped, no resident payload",
           "piece_length": L, "total_pieces": P, "pieces_per_gpu": count, "bytes_per_gpu": L * count, "ranks": ws,
           "ring_bytes_per_gpu": _native.TV_STREAM_RING_SLOTS * _native.TV_STREAM_SLOT_BYTES,
           "column_bytes": E2E_CHUNK, "unit": "GB/s", "steps": steps}
    ctx = _native.Context(device)
    pool = None
    try:
        ctx.set_option(_native.TV_OPT_RESIDENT, 0)
        ctx.set_option(_native.TV_OPT_STREAM_CHUNK, E2E_CHUNK)
        # generator threads: 8 of a 16-core share generate at ~100 GB/s (tools/pcie_probe.py) and more do not
        # raise the streamed rate (tools/e2e_gen_probe.py); a rank with a smaller share (several ranks on one
        # node's quota) generates on all of its cores -- the calling thread is one of them and otherwise only
        # waits for slots
        gen_threads = max(1, min(8, threads))
        ctx.set_option(_native.TV_OPT_FILE_THREADS, gen_threads)
        ctx.set_layout(total, L, P, first, count)
        ctx.set_digests(bytes(pieces))
        t_gen = time.perf_counter()
        _barrier(dist)
        gen_alone = producer_rate(ctx, seed)
        gen_alone_all = _sum(dist, gen_alone)
        t_gen_end = time.perf_counter()

        phase = {"next_s": 0.0, "fill_commit_s": 0.0}

        def run(fill) -> tuple:
            ctx.stream_begin()
            reqs = 0
            while True:
                t0 = time.perf_counter()
                req = ctx.stream_next()
                t1 = time.perf_counter()
                phase["next_s"] += t1 - t0
                if not req.rows:
                    break
                fill(req)
                phase["fill_commit_s"] += time.perf_counter() - t1
                reqs += 1
            return ctx.stream_end(), reqs

        def gen(req):
            ctx.stream_fill_synthetic(req, seed)
            ctx.stream_commit(req)

        # warm the ring and the chunk buffers (first allocation) outside the timed region
        ctx.stream_begin()
        for _ in range(2):
            gen(ctx.stream_next())
        ctx.stream_abort()

        def timed(fill):
            _barrier(dist)
            t0 = time.perf_counter()
            for _ in range(steps):
                bf, reqs = run(fill)
            t1 = time.perf_counter()
            _barrier(dist)
            return bf, reqs, _max(dist, t1 - t0)

        phase.update(next_s=0.0, fill_commit_s=0.0)
        t_g0 = time.perf_counter()
        bf, reqs, el = timed(gen)
        t_g1 = time.perf_counter()
        gen_phase = {k: round(v, 3) for k, v in phase.items()}
        ok = _sum(dist, 1.0 if bf == expect else 0.0) == ws
        out["generated"] = {"value": round(total * steps / el / 1e9, 2), "ms_per_step": round(el * 1e3 / steps, 1),
                            "bitfield_exact": ok, "requests_per_step": reqs, "rank0_phase_s": gen_phase,
                            "producer": f"host generator (tv_stream_fill_synthetic, {gen_threads} threads) writing "
                                        "the bytes into the ring slots inside the timed region"}
        # pinned_pool: the torrent is a 1 GiB page-locked pool of 256 pieces repeated; rows DMA'd from it
        t_p0 = time.perf_counter()
        pool = _native.PinnedBuffer(POOL_PIECES * L)
        from tests import synth   # (inputs and their hashlib digests; the oracle runs only as the ground truth)
        synth.fill_into(pool.mv, seed + 100, 0, threads=threads)
        pool_dig = synth.hash_pieces(pool.mv, L, POOL_PIECES, threads=threads)
        dp = bytearray(20 * P)
        for j in range(count):
            k = j % POOL_PIECES
            dp[20 * (first + j):20 * (first + j + 1)] = pool_dig[20 * k:20 * k + 20]
        bad2 = _corrupt(memoryview(dp)[20 * first:20 * (first + count)], count, 7)
        ctx.set_digests(bytes(dp))

        def from_pool(req):
            ctx.stream_commit_from(req, pool.mv, L, ((req.piece - first) % POOL_PIECES) * L + req.offset)

        phase.update(next_s=0.0, fill_commit_s=0.0)
        t_p1 = time.perf_counter()
        bf, reqs, el = timed(from_pool)
        t_p2 = time.perf_counter()
        pool_phase = {k: round(v, 3) for k, v in phase.items()}
        ok = _sum(dist, 1.0 if bf == _expected_bits(count, bad2) else 0.0) == ws
        out["pinned_pool"] = {"value": round(total * steps / el / 1e9, 2), "ms_per_step": round(el * 1e3 / steps, 1),
                              "bitfield_exact": ok, "requests_per_step": reqs, "rank0_phase_s": pool_phase,
                              "producer": f"rows DMA'd straight from a {POOL_PIECES * L >> 20} MiB page-locked pool "
                                          f"(piece first+j = pool piece j % {POOL_PIECES})"}
        out["bitfield_exact"] = out["generated"]["bitfield_exact"] and ok
        out["kernel"] = KERNEL_NAMES.get(ctx.last_kernel()[0], "?")
        # what bounds the generated figure: the producer (the node's generator rate at this per-rank thread
        # budget, measured alone on every rank at once) or the PCIe links (PCIE_H2D_GBPS per physical GPU)
        pcie_all = PCIE_H2D_GBPS * physical_gpus
        out["producer"] = {
            "producer_threads": gen_threads, "threads_per_rank": threads,
            "cpu_quota_per_rank": (share or {}).get("cores_per_rank"),
            "cpu_share_node": (share or {}).get("cores"), "cpu_share_source": (share or {}).get("source"),
            "generator_alone_gbps_rank0": round(gen_alone, 1), "generator_alone_gbps_all_ranks": round(gen_alone_all, 1),
            "pcie_h2d_gbps_all_gpus": round(pcie_all, 1), "physical_gpus": physical_gpus,
            "bound": "producer" if gen_alone_all < pcie_all else "pcie",
            "note": "generated is bounded by min(generator_alone_gbps_all_ranks, pcie_h2d_gbps_all_gpus); "
                    "pinned_pool takes the producer out (the PCIe path alone)"}
        # the leg's value is the PCIe path (pinned_pool); the generated figure stays beside it with its bound
        out["value"] = out["pinned_pool"]["value"]
        out["value_is"] = "pinned_pool (PCIe path); generated beside it, bounded as producer.bound says"
        out["phase_s"] = {"producer_probe": round(t_gen_end - t_gen, 2), "generated": round(t_g1 - t_g0, 2),
                          "pool_setup": round(t_p1 - t_p0, 2), "pinned_pool": round(t_p2 - t_p1, 2)}
    finally:
        if pool is not None:
            pool.close()
        ctx.close()
    return out


def cfg3_leg(device: int, steps: int, warmup: int, kernel_opt: int, idle_s: float = 0.5) -> dict:
    """BASELINE configs[2]: the multi-file torrent -- 10,000 files of U[0, 512 KiB] (20 zero-length, 5 under 64 B),
    256 KiB pieces spanning file boundaries, a short final piece, 1 % corrupted (tests/layouts.py "cfg3", the seeded
    generator the parity tests use; expected bits committed in tests/golden/layouts.json).  The payload is built in
    host memory and staged FILE BY FILE (tv_stage_many with one range per file at its linear offset: the
    storage.ts:89-137 walk's segments, zero-length files included), so the file -> piece mapping and the short
    final piece go through the library as a multi-file torrent's would.  Timed: (a) the resident verify, W + K
    steps with the shader clock probed (the value; frac_of_piece_ceiling is also given at the live clock), and
    (b) one-shot calls as a host makes them after `idle_s` of GPU idle: stage every file + verify, wall clock,
    with that call's kernel time and clock."""
    from tests import synth
    from tests.layouts import build_layout, by_name
    t_leg = time.perf_counter()
    spec = by_name("cfg3")
    lay = build_layout(spec, fill=synth.fill)   # (hashlib digests of tests/synth.py's bytes; bits: the golden file)
    info = lay["info"]
    golden = {r["name"]: r for r in json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))}["cfg3"]
    want = bytes.fromhex(golden["expected_bitfield"])
    L, P, total = info.piece_length, info.n_pieces, info.length
    payload = lay["payload"]
    starts, sizes = lay["starts"], lay["sizes"]
    import numpy as np
    # one range of the payload per file, at its linear offset (the file table; zero-length files included)
    seg_lin = np.asarray(starts[:len(sizes)], dtype=np.uint64)
    seg_len = np.asarray(sizes, dtype=np.uint64)

    def stage_files_from_memory():
        ctx.stage_ranges(payload, seg_lin, seg_lin, seg_len)
    t_built = time.perf_counter()
    ctx = _native.Context(device)
    try:
        ctx.set_option(_native.TV_OPT_KERNEL, kernel_opt)
        ctx.set_clock_probe(True)
        ctx.set_layout(total, L, P)
        if ctx.counter(_native.TV_COUNTER_WINDOW_PIECES):
            raise RuntimeError("cfg3: the shard does not fit the device budget")
        ctx.set_digests(info.pieces_raw)
        t0 = time.perf_counter()
        stage_files_from_memory()
        stage_s = time.perf_counter() - t0
        _device_sync(ctx, device)
        for _ in range(warmup):
            ctx.verify()
        _device_sync(ctx, device)
        kernel_ms = []
        t0 = time.perf_counter()
        for _ in range(steps):
            bf = ctx.verify()
            kernel_ms.append(ctx.last_timing()[0])
        _device_sync(ctx, device)
        t1 = time.perf_counter()
        kernel, _ = ctx.last_kernel()
        clock_ghz = ctx.last_clock_khz() / 1e6
        exact = bytes(bf) == want
        # one-shot calls: a host stages every file and verifies, after the GPU idled
        shots = []
        for _ in range(3):
            time.sleep(idle_s)
            t2 = time.perf_counter()
            stage_files_from_memory()
            bf1 = ctx.verify()
            t3 = time.perf_counter()
            shots.append({"wall_ms": round((t3 - t2) * 1e3, 2), "gbps": round(total / (t3 - t2) / 1e9, 2),
                          "kernel_ms": round(ctx.last_timing()[0], 3),
                          "clock_ghz": round(ctx.last_clock_khz() / 1e6, 3), "exact": bytes(bf1) == want})
        exact = exact and all(x["exact"] for x in shots)
    finally:
        ctx.close()
    avg = sum(kernel_ms) / len(kernel_ms)
    achieved = total / (avg / 1e3) / 1e9
    ceiling = piece_ceiling(kernel, P)
    ceiling_at_clock = ceiling * clock_ghz / (CLOCK_HZ / 1e9) if clock_ghz else None
    best = min(shots, key=lambda x: x["wall_ms"])
    return {"workload": "cfg3: multi-file torrent, 10,000 files of U[0, 512 KiB] (20 zero-length, 5 under 64 B), "
                        "256 KiB pieces spanning file boundaries + short final piece, 1 % corrupted; staged file by "
                        "file (one tv_stage_many segment per file), HBM-resident verify",
            "files": len(sizes), "piece_length": L, "total_pieces": P, "bytes": total,
            "short_last_piece": total % L, "corrupted": len(lay["corrupted"]),
            "value": round(total * steps / (t1 - t0) / 1e9, 2), "unit": "GB/s", "steps": steps, "warmup": warmup,
            "ms_per_step": round((t1 - t0) * 1e3 / steps, 3), "kernel": KERNEL_NAMES.get(kernel, str(kernel)),
            "kernel_ms_avg": round(avg, 3), "kernel_ms_median": round(sorted(kernel_ms)[len(kernel_ms) // 2], 3),
            "kernel_ms_min_max": [round(min(kernel_ms), 3), round(max(kernel_ms), 3)], "achieved": round(achieved, 1),
            "piece_parallelism_ceiling": round(ceiling, 1), "frac_of_piece_ceiling": round(achieved / ceiling, 4),
            "clock_ghz": round(clock_ghz, 3) if clock_ghz else None,
            "piece_ceiling_at_clock": round(ceiling_at_clock, 1) if ceiling_at_clock else None,
            "frac_of_piece_ceiling_at_clock": round(achieved / ceiling_at_clock, 4) if ceiling_at_clock else None,
            "bitfield_exact": exact, "expected": "tests/golden/layouts.json cfg3 expected_bitfield (hashlib digests)",
            "one_shot": {"what": f"stage all {len(sizes)} files from pageable host memory + verify, wall clock, "
                                 f"after {idle_s} s of GPU idle (best of {len(shots)})",
                         "best_wall_ms": best["wall_ms"], "best_gbps": best["gbps"], "calls": shots},
            "first_stage_s": round(stage_s, 3),
            "phase_s": {"build_layout": round(t_built - t_leg, 2), "leg": round(time.perf_counter() - t_leg, 2)}}


def cpu_baseline(share: dict, target_s: float = 10.0) -> dict:
    """The CPU oracle (C port of the per-piece SHA-1 path; SHA-NI where the host has it: the reference's
    WebCrypto SHA-1 is native code of that class) on the allowed cores, one piece per task:
    a bounded sample of cfg2 (4 GiB of its pieces, generated once, hashed repeatedly for ~target_s),
    BASELINE configs[0] = cfg1 (64 MiB, 256 x 256 KiB) as its own entry, and the 1-core figures."""
    from oracle import oracle as O
    O.set_impl("best")
    cores = share["cores"]

    def timed(buf, L, n, threads, seconds):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.hash_pieces(buf, n * L, L, n, 0, n, threads=threads)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return n * L * reps / el / 1e9, reps, el

    L2, _, seed2, _ = WORKLOADS["cfg2"]
    n2 = 4096
    buf = O.synth_fill(seed2, 0, n2 * L2)
    gbps, reps, el = timed(buf, L2, n2, cores, target_s)
    one, _, _ = timed(buf, L2, 64, 1, max(1.0, target_s / 5))
    del buf
    L1, n1, seed1, desc1 = WORKLOADS["cfg1"]
    b1 = O.synth_fill(seed1, 0, n1 * L1)
    c1, r1, e1 = timed(b1, L1, n1, cores, max(1.0, target_s / 4))
    c1one, _, _ = timed(b1, L1, n1, 1, max(1.0, target_s / 5))
    return {"value": round(gbps, 3), "unit": "GB/s", "cores": cores, "kind": "port",
            "sample": f"{n2} of cfg2's 1 MiB pieces (4 GiB of the same synthetic payload) hashed {reps} times "
                      f"({el:.1f} s) by oracle/sha1_oracle.c ({O.impl()} SHA-1, one piece per task, {cores} threads)",
            "impl": O.impl(), "per_core": round(one, 3), "cpu_model": _cpu_model(),
            "cores_source": share["source"], "nproc": share["nproc"], "affinity_cpus": share["affinity"],
            "cgroup_quota_cpus": share["cgroup_quota_cpus"], "omp_num_threads": share["omp_num_threads"],
            "cfg1": {"workload": desc1 + ", the reference's CPU SHA-1 path restated (oracle)",
                     "value": round(c1, 3), "unit": "GB/s", "ms_per_verify": round(n1 * L1 / c1 / 1e6, 2),
                     "cores": cores, "reps": r1, "per_core": round(c1one, 3)}}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="timed workload (default: cfg2, weak-scaled at N>1)")
    sc = ap.add_mutually_exclusive_group()
    sc.add_argument("--strong", action="store_true", help="the workload's pieces are the WHOLE torrent, sharded")
    sc.add_argument("--weak", action="store_true", help="the workload's pieces are per GPU")
    ap.add_argument("--kernel", type=int, default=0, help="0 auto, 1 lane, 2 split, 4 twin")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-saturating", action="store_true", help="skip the piece_saturated leg (N=1)")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the cfg4 leg (the 200 GiB torrent, strong-scaled)")
    ap.add_argument("--no-cfg3", action="store_true", help="skip the cfg3 multi-file leg (N=1)")
    ap.add_argument("--e2e-steps", type=int, default=1, help="timed e2e_cfg5 passes (0 = skip the leg)")
    ap.add_argument("--leg-steps", type=int, default=5, help="timed steps of the cfg4 / suppl legs")
    a = ap.parse_args()

    dist, rank, ws, local = _dist()
    ndev = _native.device_count()
    device = pick_device(local, ndev)
    share = cpu_share()
    # the node's allowed cores are shared by the ranks on it (ground truth, generators)
    threads = max(1, share["cores"] // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))
    share["cores_per_rank"] = threads
    placement = rank_placement(dist, ws, rank, local, device, ndev)
    physical = len({p["pci_bus_id"] for p in placement}) if placement else 1
    # `value`: cfg2 at every N, weak-scaled (the units -- pieces -- are independent and sharded with no data-path
    # collective: each rank verifies its own 16 GiB / 16,384-piece shard of an N x 16 GiB torrent), so the 1 -> 8
    # curve is one configuration; cfg4 (BASELINE configs[3], one 200 GiB torrent strong-scaled over the N GPUs) is
    # the `cfg4` leg at every N
    workload = a.workload or "cfg2"
    strong = a.strong

    main_leg = resident_leg(dist, ws, rank, device, workload, strong, a.steps, a.warmup, a.kernel, threads,
                            want_digests=(workload == "cfg4" and strong))
    legs = {}
    cfg4_digests = None
    if workload == "cfg4" and strong:
        cfg4_digests = main_leg.pop("_digests")
        main_leg.pop("_first")
    elif not a.no_cfg4:
        legs["cfg4"] = resident_leg(dist, ws, rank, device, "cfg4", True, a.leg_steps, 1, a.kernel, threads,
                                    want_digests=True)
        cfg4_digests = legs["cfg4"].pop("_digests")
        legs["cfg4"].pop("_first")
    if a.e2e_steps > 0:
        try:
            legs["e2e_cfg5"] = e2e_cfg5(dist, ws, rank, device, a.e2e_steps, threads, cfg4_digests, share,
                                        physical)
        except Exception as exc:  # reported, never fatal to the bench line
            legs["e2e_cfg5"] = {"skipped": f"{type(exc).__name__}: {exc}"}
    cfg4_digests = None
    if ws == 1 and workload == "cfg2" and not a.no_cfg3:
        try:
            # (3 ms launches: 20 warm-up steps bring the shader clock up from the layout build's idle, and 20 timed
            # steps average over its last ramp; rocprofv3 showed 5 timed steps still speeding up in round 5)
            legs["cfg3"] = cfg3_leg(device, max(20, a.leg_steps), 20, a.kernel)
        except Exception as exc:
            legs["cfg3"] = {"skipped": f"{type(exc).__name__}: {exc}"}
    if ws == 1 and workload == "cfg2" and not a.no_saturating:
        try:
            legs["piece_saturated"] = resident_leg(dist, 1, 0, device, "suppl", False, a.leg_steps, 1, a.kernel, threads)
        except Exception as exc:
            legs["piece_saturated"] = {"skipped": f"{type(exc).__name__}: {exc}"}

    if rank == 0:
        bytes_per_gpu = main_leg["bytes_per_gpu"]
        traffic, traffic_note = _traffic(workload, bytes_per_gpu)
        tp = legs.get("piece_saturated")
        if tp and "bytes_per_gpu" in tp:
            tsat, tnote = _traffic("suppl", tp["bytes_per_gpu"])
            tp["traffic_ratio"] = round(tsat / tp["bytes_per_gpu"], 5) if tsat else None
            tp["traffic_source"] = tnote
        achieved = main_leg["achieved"]
        out = {
            "metric": "verified GB/s (SHA-1 pieces, HBM-resident)",
            "value": main_leg["value"],
            "unit": "GB/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": main_leg["ms_per_step"],
            "higher_is_better": True,
            "scaling": main_leg["scaling"],
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device counter-PRNG payload; expected digests from the CPU oracle, 1% corrupted)",
            "config": {"workload": main_leg["workload"], "piece_length": main_leg["piece_length"],
                       "pieces_per_gpu": main_leg["pieces_per_gpu"], "total_pieces": main_leg["total_pieces"],
                       "bytes_per_gpu": bytes_per_gpu, "kernel": main_leg["kernel"],
                       "parallelism": f"piece shards x{ws}, no collective"},
            "bitfield_exact": main_leg["bitfield_exact"],
            "expected": main_leg["expected"],
            "roofline": {"bound": "valu", "achieved": achieved, "peak": round(ROOF_PEAK_GBPS, 1), "unit": "GB/s",
                         "frac": round(achieved / ROOF_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_ratio": round(traffic / bytes_per_gpu, 6) if traffic else None,
                         "traffic_source": traffic_note, "build_id": _native.build_id(),
                         "kernel_ms_avg": main_leg["kernel_ms_avg"], "kernel_ms_median": main_leg["kernel_ms_median"],
                         "kernel_ms_min_max": main_leg["kernel_ms_min_max"],
                         "kernel_ms_max_over_ranks": main_leg["kernel_ms_max_over_ranks"],
                         "algorithmic_bytes_per_launch": bytes_per_gpu,
                         "peak_is": "min(HBM 8000 GB/s, R_valu)", "valu_peak": round(VALU_PEAK_GBPS, 1),
                         "hbm_peak": HBM_PEAK_GBPS, "frac_hbm": round(achieved / HBM_PEAK_GBPS, 4),
                         "piece_parallelism_ceiling": main_leg["piece_parallelism_ceiling"],
                         "frac_of_piece_ceiling": main_leg["frac_of_piece_ceiling"],
                         "aggregate_piece_ceiling": main_leg["aggregate_piece_ceiling"],
                         "frac_of_aggregate_piece_ceiling": main_leg["frac_of_aggregate_piece_ceiling"],
                         "clock_ghz": main_leg["clock_ghz"], "frac_at_clock": main_leg["frac_of_valu_peak_at_clock"],
                         "valu_peak_derivation": VALU_DERIVATION,
                         "note": "SHA-1 is serial per piece, so P pieces per GPU cap the rate at P x 64 B / "
                                 "(serial VALU instr x 4.07 cyc) (piece_parallelism_ceiling; 405 instr for the "
                                 "twin and split rounds waves, 613 for the lane kernel); full R_valu needs >= 65,536 "
                                 "pieces per GPU (piece_saturated)"},
            "ground_truth_s": main_leg["ground_truth_s"],
        }
        out["scaling_note"] = (
            f"value is {workload} {'strong' if strong else 'weak'}-scaled "
            + ("(each GPU verifies its own 16 GiB / 16,384-piece shard of an N x 16 GiB torrent, no collective), "
               if workload == "cfg2" and not strong else "")
            + "so the driver's per-N curve of value is one configuration; BASELINE configs[3] -- ONE 200 GiB torrent "
              "of 51,200 x 4 MiB pieces sharded over the N GPUs -- is the cfg4 leg at every N: read the sharded "
              "curve from cfg4.value against cfg4.aggregate_piece_ceiling (piece-bound past one GPU, "
              f"predicted {round(aggregate_piece_ceiling('cfg4', ws), 1)} GB/s at N = {ws})")
        if "cfg4" in legs and "value" in legs["cfg4"]:
            out["scaling_figure"] = {"workload": "cfg4 (BASELINE configs[3], strong)", "value": legs["cfg4"]["value"],
                                     "aggregate_piece_ceiling": legs["cfg4"]["aggregate_piece_ceiling"],
                                     "frac_of_aggregate_piece_ceiling":
                                         legs["cfg4"]["frac_of_aggregate_piece_ceiling"],
                                     "predicted_aggregate_piece_ceiling":
                                         round(aggregate_piece_ceiling("cfg4", ws), 1)}
        out.update(legs)
        if ws == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(share, a.cpu_seconds)
        out["placement"] = {"ranks": placement, "physical_gpus": physical, "visible_devices": ndev,
                            "rule": "device = LOCAL_RANK % (devices visible to the rank): LOCAL_RANK on a node "
                                    "where every rank sees all GPUs, 0 where the launcher gives each rank one "
                                    "(HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES)"}
        if physical < ws:
            out["placement"]["note"] = (f"{ws} ranks share {physical} physical GPU(s): a rehearsal of the N = {ws} "
                                        "path, not a scaling point")
        out["wall_s"] = round(time.perf_counter() - T_START, 1)
        print(json.dumps(out), flush=True)
    ok = main_leg["bitfield_exact"] and all(v.get("bitfield_exact", True) for v in legs.values())
    if dist is not None:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
