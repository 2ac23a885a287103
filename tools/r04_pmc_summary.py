"""Round-4 summaries of the saturated lane kernel's PMC passes (tools/gpu_r04_pmc.sh) -> profiles/r04/ and the
per-launch traffic files the bench reads (profiles/traffic_<workload>.json).

Counter units (MI355X_MICROARCH.md, PMC section): FETCH_SIZE in KiB and, for 16-B/lane streaming reads on
gfx950, half the bytes actually read (doubled here); TCC_EA0_RDREQ_{32B,64B,128B} count requests of that size
(bytes = 32 x + 64 y + 128 z, with the plain TCC_EA0_RDREQ total as a cross-check); GRBM_GUI_ACTIVE = shader
cycles summed over the 8 XCDs (/ 8 / the dispatch's duration = the clock); SQ_* wave counters in quad-cycles.
The verify dispatches are the bench's `lane_kernel<false>` launches after the creation-mode hash; the PMC runs'
own durations (Start/End_Timestamp) give the clock of that same dispatch.

usage: python tools/r04_pmc_summary.py gpurun_out/r04_pmc profiles/r04
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

WORKLOADS = {"p262k": (64 << 10, 262144), "suppl": (256 << 10, 65536)}


def dispatches(path, match):
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [per[k] for k in sorted(per)]


def mean(xs):
    xs = [x for x in xs if x is not None]
    return sum(xs) / len(xs) if xs else None


def main():
    src, out = sys.argv[1:3]
    os.makedirs(out, exist_ok=True)
    summary = {}
    for w, (L, P) in WORKLOADS.items():
        payload = L * P
        passes = {}
        for i in range(1, 5):
            d = dispatches(os.path.join(src, f"pmc_{w}", f"p{i}"), "lane_kernel<false")
            passes[i] = d[1:] if len(d) > 1 else d      # the verify launches after the first (warm-up) one
        fetch = mean([2 * 1024 * r["FETCH_SIZE"] for r in passes[1]])
        rd = mean([32 * r["TCC_EA0_RDREQ_32B_sum"] + 64 * r["TCC_EA0_RDREQ_64B_sum"] + 128 * r["TCC_EA0_RDREQ_128B_sum"]
                   for r in passes[2]])
        hit = mean([r["TCC_HIT_sum"] / (r["TCC_HIT_sum"] + r["TCC_MISS_sum"]) for r in passes[3]])
        clock = mean([r["GRBM_GUI_ACTIVE"] / 8 / r["_ns"] for r in passes[3]])     # cycles per ns = GHz
        blocks = (L + 8) // 64 + 1
        cyc_block = mean([r["GRBM_GUI_ACTIVE"] / 8 / blocks for r in passes[3]])
        waves = P // 64
        p4 = passes[4]
        per_wave = {k: mean([4 * r[k] / waves / blocks for r in p4]) for k in
                    ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")}
        valu_per_wave_block = mean([r["SQ_INSTS_VALU"] / waves / blocks for r in p4])
        bench = json.load(open(os.path.join(src, f"bench_{w}.json")))
        rec = {
            "workload": bench["config"]["workload"], "kernel": bench["config"]["kernel"],
            "payload_bytes_per_launch": payload,
            "hbm_read_bytes_fetch_size_x2": fetch, "hbm_read_bytes_rdreq": rd,
            "traffic_ratio": fetch / payload, "traffic_ratio_rdreq": rd / payload,
            "l2_hit_rate": hit, "clock_ghz_pmc": clock, "cycles_per_block": cyc_block,
            "per_wave_per_block_cycles": per_wave, "valu_per_wave_per_block": valu_per_wave_block,
            "bench_line": {k: bench["roofline"][k] for k in ("achieved", "frac", "kernel_ms_avg", "clock_ghz",
                                                              "frac_at_clock")},
            "bench_value_gbps": bench["value"],
            "frac_of_valu_peak_at_pmc_clock": bench["roofline"]["achieved"] / (bench["roofline"]["valu_peak"] * clock / 2.4),
            "sources": {"pmc": f"gpurun_out/r04_pmc/pmc_{w}/p1..p4 (tools/gpu_r04_pmc.sh)",
                        "bench": f"profiles/r04/bench_{w}.json"},
        }
        summary[w] = rec
        json.dump({"workload": w, "kernel": "lane", "payload_bytes_per_launch": payload,
                   "hbm_bytes_per_launch": fetch,
                   "method": "rocprofv3 --pmc FETCH_SIZE in its own pass over `bench.py --workload " + w + "` "
                             "(tools/gpu_r04_pmc.sh): 2 x FETCH_SIZE x 1024 bytes per verify dispatch (gfx950 reports "
                             "half the bytes of a 16-B/lane streaming read: MI355X_MICROARCH.md HBM section), mean over "
                             "the verify dispatches after the first; TCC_EA0_RDREQ by size agrees: "
                             f"{rd / payload:.5f} x payload",
                   "source": "profiles/r04/pmc_saturated.json"},
                  open(os.path.join(os.path.dirname(out.rstrip("/")), f"traffic_{w}.json"), "w"), indent=1)
    json.dump(summary, open(os.path.join(out, "pmc_saturated.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
