#!/usr/bin/env python3
"""Benchmark: verified GB/s of SHA-1 piece verification, HBM-resident (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2|suppl|cfg4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (default cfg2 = BASELINE.json configs[1]): a synthetic single-file torrent, 16 GiB per
GPU, 1 MiB pieces (16,384 pieces per GPU).  Weak scaling: the torrent has N x 16,384 pieces and
rank r verifies the contiguous shard [r*16384, (r+1)*16384) of it (shard start a multiple of 8 so
its bitfield slice is whole bytes; no data-path collective exists).  The payload is generated in
HBM by the device fill kernel (counter PRNG, the oracle's definition); expected digests are the
GPU's own creation-mode digests, with 1 % of them corrupted so the expected bitfield is known, and
a sample of them is checked against the CPU oracle.

One step = one tv_verify of the rank's whole resident shard (upload availability bits, the verify
kernel, bitfield download).  W untimed steps, then exactly K steps between a barrier +
device synchronize on both sides; the time is the max over ranks.  value = total payload bytes
of all ranks x K / time.

The roofline object is for the verify kernel: algorithmic bytes per launch (the shard's payload
bytes, SURVEY.md 8d: one byte read per payload byte) / the average kernel duration from HIP events
recorded on the library's compute stream around each launch.  The cpu_baseline leg (rank 0, N=1)
times the CPU oracle (a port of the reference's per-piece SHA-1 path) on a bounded sample of the
same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from torrent_amd import _native  # noqa: E402  (load the HIP library before torch)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# SHA-1 VALU roofline from the measured SIMD cost per wave64 instruction (tools/ubench_simd.hip,
# profiles/r01/ubench_simd.log): v_alignbit / v_add3 / v_perm 4 cycles (half rate), v_bitop3 / VOP2 2
# cycles (full rate).  Minimal mix per 64-B block: 224 alignbit + 160 add3 + 16 perm (400 x 4) + 144
# bitop3 + 64 xor + 5 add (213 x 2) = 2,026 SIMD cycles per 64 lanes.
CLOCK_HZ = 2.4e9
SIMD_CYC_PER_BLOCK = 400 * 4 + 213 * 2
VALU_PEAK_GBPS = 1024 * 64 * 64 * CLOCK_HZ / SIMD_CYC_PER_BLOCK / 1e9
# Cycles per VALU instruction of a lone wave: 4.07 for 8-byte VOP3 ops in a long loop body, 4.09 for the
# SHA-1 round mix (tools/ubench_fetch.hip, profiles/r01/ubench_fetch.log); the wave64 cadence is 4.
LONE_WAVE_CYC = 4.07
SERIAL_INSTR = {1: 613, 2: 405}  # per-block serial stream: lane kernel / split rounds wave

WORKLOADS = {
    # name: (piece_length, pieces per GPU, description)
    "cfg2": (1 << 20, 16384, "cfg2: 16 GiB synthetic single-file torrent per GPU, 1 MiB pieces (16384 pieces), HBM-resident"),
    "suppl": (256 << 10, 65536, "suppl: 16 GiB per GPU, 256 KiB pieces (65536 pieces), HBM-resident"),
    "cfg4": (4 << 20, 51200, "cfg4: 200 GiB single-file torrent, 4 MiB pieces (51200 pieces per GPU at N=1), HBM-resident"),
    "p262k": (64 << 10, 262144, "p262k: 16 GiB per GPU, 64 KiB pieces (262144 pieces), HBM-resident (VALU-saturating)"),
}
SEED = 2


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
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


def cpu_baseline(L: int, total: int, P: int, first: int, gpu_digests: bytes, target_s: float = 10.0):
    """Time the CPU oracle (C port of the per-piece SHA-1 path, SHA-NI where the host has it: the
    reference's WebCrypto SHA-1 is native code of that class) on a bounded sample:
    the first `n` pieces of this shard, generated once (not timed), hashed repeatedly for
    ~target_s on all `cores` threads, then ~target_s/5 on one thread (the 1-core figure).  Also
    checks the sample's digests against the GPU's (parity inside the bench)."""
    from oracle import oracle as O
    O.set_impl("best")
    n = max(1, min(256, (256 << 20) // L))
    cores = min(16, len(os.sched_getaffinity(0)))
    buf = O.synth_fill(SEED, first * L, n * L)
    # digests of the sample (piece-relative: a sub-torrent of n pieces of length L)
    d = O.hash_pieces(buf, n * L, L, n, 0, n, threads=cores)
    parity_ok = d == gpu_digests[: 20 * n]

    def timed(threads: int, pieces: int, seconds: float):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.hash_pieces(buf, pieces * L, L, pieces, 0, pieces, threads=threads)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return reps * pieces * L / el / 1e9, reps, el

    gbps, reps, el = timed(cores, n, target_s)
    one, _, _ = timed(1, min(n, 16), max(1.0, target_s / 5))
    return {"value": round(gbps, 3), "unit": "GB/s", "cores": cores, "kind": "port",
            "sample": f"{n} pieces x {L >> 10} KiB of the same synthetic payload hashed {reps} times "
                      f"({el:.1f} s) by oracle/sha1_oracle.c ({O.impl()} SHA-1, one piece per task, "
                      f"{cores} threads)",
            "impl": O.impl(), "per_core": round(one, 3), "cpu_model": _cpu_model(),
            "host_cpus_visible": os.cpu_count(), "parity_vs_gpu": parity_ok}


def saturating_leg(device: int, steps: int = 5) -> dict:
    """The piece-saturated configuration (SURVEY 8d "suppl": 16 GiB, 65,536 x 256 KiB pieces, one
    lane-kernel wave per SIMD) on the same GPU, reported beside `value` (never as it): with enough
    pieces the per-piece serial limit of cfg2 is gone and the kernel runs against the VALU roofline,
    the one the north-star's >= 60 % target is stated for.  1 % corrupted digests; bitfield checked."""
    L, per, desc = WORKLOADS["suppl"]
    ctx = _native.Context(device)
    try:
        ctx.set_layout(L * per, L, per)
        ctx.fill_synthetic(SEED + 4)
        dig = bytearray(ctx.hash())
        bad = set(range(0, per, 100)) | {per - 1}
        for j in bad:
            dig[20 * j + 3] ^= 0x01
        ctx.set_digests(bytes(dig))
        expect = bytearray(b"\xff" * (per // 8))
        for j in bad:
            expect[j >> 3] &= ~(0x80 >> (j & 7)) & 0xFF
        bf = ctx.verify()
        ms = []
        for _ in range(steps):
            bf = ctx.verify()
            ms.append(ctx.last_timing()[0])
        kernel, _ = ctx.last_kernel()
    finally:
        ctx.close()
    avg = sum(ms) / len(ms)
    gbps = L * per / (avg / 1e3) / 1e9
    return {"workload": desc, "kernel": {1: "lane", 2: "split"}.get(kernel, str(kernel)), "steps": steps,
            "kernel_ms_avg": round(avg, 3), "achieved": round(gbps, 1), "unit": "GB/s",
            "valu_peak": round(VALU_PEAK_GBPS, 1), "frac_of_valu_peak": round(gbps / VALU_PEAK_GBPS, 4),
            "bitfield_exact": bf == bytes(expect)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--kernel", type=int, default=0, help="0 auto, 1 lane, 2 split")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-saturating", action="store_true",
                    help="skip the piece-saturated leg (N=1 only: 65,536 x 256 KiB pieces against R_valu)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the workload's piece count is the WHOLE torrent, split into N contiguous "
                         "8-aligned shards (BASELINE config 4: 200 GiB over 2/4/8 GPUs); default is weak scaling")
    ap.add_argument("--e2e-steps", type=int, default=3,
                    help="timed end-to-end passes from pinned host memory over PCIe (0 = skip)")
    a = ap.parse_args()

    dist, rank, ws, local = _dist()
    L, per_gpu, desc = WORKLOADS[a.workload]
    if a.strong:
        from torrent_amd.verify import shard_ranges
        P = per_gpu
        first, per_gpu = shard_ranges(P, ws)[rank]
        desc = desc.split(" per GPU")[0].split(" (")[0] + f" ({P} pieces in all, {ws} shard(s), strong scaling)"
    else:
        P = per_gpu * ws
        first = rank * per_gpu
    total = L * P

    device = local % max(1, _native.device_count())
    ctx = _native.Context(device)
    ctx.set_option(_native.TV_OPT_KERNEL, a.kernel)
    ctx.set_layout(total, L, P, first, per_gpu)
    ctx.fill_synthetic(SEED)
    shard_digests = ctx.hash()                     # creation mode on the resident shard
    # 1 % corrupted digests (every 100th piece, plus the shard's last) -> known expected bitfield
    bad = set(range(0, per_gpu, 100)) | {per_gpu - 1}
    dig = bytearray(shard_digests)
    for j in bad:
        dig[20 * j + 7] ^= 0x10
    pieces = bytearray(20 * P)
    pieces[20 * first:20 * (first + per_gpu)] = dig
    ctx.set_digests(bytes(pieces))
    expect = bytearray(b"\xff" * ((per_gpu + 7) // 8))
    if per_gpu % 8:
        expect[-1] = (0xFF00 >> (per_gpu % 8)) & 0xFF
    for j in bad:
        expect[j >> 3] &= ~(0x80 >> (j & 7)) & 0xFF

    for _ in range(a.warmup):
        bf = ctx.verify()
    _device_sync(ctx, device)
    _barrier(dist)
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        bf = ctx.verify()
        kernel_ms.append(ctx.last_timing()[0])
    _device_sync(ctx, device)
    t1 = time.perf_counter()
    _barrier(dist)
    elapsed = _max(dist, t1 - t0)
    correct = bf == bytes(expect)
    all_correct = _sum(dist, 1.0 if correct else 0.0) == ws
    kernel, _ = ctx.last_kernel()
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    worst_kernel_ms = _max(dist, avg_kernel_ms)

    bytes_per_gpu = L * per_gpu

    # End-to-end leg (reported beside `value`, never as it): the same shard streamed from a pinned
    # host copy over PCIe with copy/compute overlap (tv_verify_host; SURVEY 8d config 5 form).
    e2e = None
    host = None
    if a.e2e_steps > 0:
        try:
            host = _native.PinnedBuffer(bytes_per_gpu)
        except Exception as exc:  # e.g. not enough page-lockable host memory on this node
            e2e = {"skipped": f"pinned host allocation of {bytes_per_gpu} B failed: {exc}"}
        # collective decision: every rank runs the leg (and its barriers) or none does
        if _sum(dist, 1.0 if host is not None else 0.0) < ws:
            if host is not None:
                host.close()
                host = None
            e2e = e2e or {"skipped": "pinned host allocation failed on another rank"}
    if host is not None:
        ctx.read(first * L, host.mv)            # host copy of the resident synthetic payload
        bf2 = ctx.verify_host(host.mv)          # warmup
        _device_sync(ctx, device)
        _barrier(dist)
        e0 = time.perf_counter()
        for _ in range(a.e2e_steps):
            bf2 = ctx.verify_host(host.mv)
        _device_sync(ctx, device)
        e1 = time.perf_counter()
        _barrier(dist)
        e_el = _max(dist, e1 - e0)
        e_ok = _sum(dist, 1.0 if bf2 == bytes(expect) else 0.0) == ws
        e2e = {"value": round(total * a.e2e_steps / e_el / 1e9, 2), "unit": "GB/s",
               "steps": a.e2e_steps, "ms_per_step": round(e_el * 1e3 / a.e2e_steps, 2), "bitfield_exact": e_ok,
               "launches_per_step": ctx.last_kernel()[1],
               "mode": "pinned host -> HBM column stream (2D DMA) overlapped with the verify kernel; PCIe-inclusive"}
        host.close()

    sat = None
    if ws == 1 and a.workload == "cfg2" and not a.no_saturating:
        try:
            sat = saturating_leg(device)
        except Exception as exc:  # reported, never fatal to the bench line
            sat = {"skipped": f"{type(exc).__name__}: {exc}"}

    value = total * a.steps / elapsed / 1e9      # every rank's shard: weak N x per-GPU bytes, strong the whole torrent
    achieved = bytes_per_gpu / (avg_kernel_ms / 1e3) / 1e9
    piece_ceiling = min(VALU_PEAK_GBPS, per_gpu * 64 * CLOCK_HZ / (SERIAL_INSTR.get(kernel, 613) * LONE_WAVE_CYC) / 1e9)

    if rank == 0:
        traffic = None
        tpath = os.path.join(ROOT, "profiles", f"traffic_{a.workload}.json")
        if os.path.exists(tpath):
            try:
                rec = json.load(open(tpath))
                # a per-launch PMC figure applies only to the launch geometry it was measured on
                if rec.get("payload_bytes_per_launch") == bytes_per_gpu:
                    traffic = rec.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "verified GB/s (SHA-1 pieces, HBM-resident)",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if a.strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device counter-PRNG payload; 1% corrupted digests)",
            "config": {"workload": desc, "piece_length": L, "pieces_per_gpu": per_gpu,
                       "total_pieces": P, "bytes_per_gpu": bytes_per_gpu,
                       "kernel": {1: "lane", 2: "split"}.get(kernel, str(kernel)),
                       "parallelism": f"piece shards x{ws}, no collective"},
            "bitfield_exact": all_correct,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel_ms_avg": round(avg_kernel_ms, 3), "kernel_ms_max_over_ranks": round(worst_kernel_ms, 3),
                         "algorithmic_bytes_per_launch": bytes_per_gpu,
                         "valu_peak": round(VALU_PEAK_GBPS, 1),
                         "frac_of_valu_peak": round(achieved / VALU_PEAK_GBPS, 4),
                         "piece_parallelism_ceiling": round(piece_ceiling, 1),
                         "frac_of_piece_ceiling": round(achieved / piece_ceiling, 4),
                         "note": "SHA-1 is VALU-bound on MI355X (valu_peak from measured per-op SIMD costs), not "
                                 "HBM-bound; it is serial per piece, so P pieces cap the rate at P x 64 B / "
                                 "(serial VALU instr x 4.07 cyc) per GPU (piece_parallelism_ceiling)"},
        }
        if sat is not None:
            out["piece_saturated"] = sat
        if e2e is not None:
            out["e2e_pinned_host"] = e2e
        if ws == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(L, total, P, first, shard_digests, a.cpu_seconds)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0 if all_correct and (e2e is None or e2e.get("bitfield_exact", True)) else 1


if __name__ == "__main__":
    sys.exit(main())
