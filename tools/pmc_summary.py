"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) for the verify kernel dispatches.

usage: python tools/pmc_summary.py gpurun_out/pmc/<tag> <payload_bytes_per_launch> [first_n_dispatches]
Prints per-launch counter means (verify dispatches only: tv_*_kernel<false>) as JSON.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(tag_dir, first_n=None):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(tag_dir, "p*", "*counter_collection.csv"))):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "kernel<false" not in k:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per[d][row["Counter_Name"]] += float(row["Counter_Value"])
        ids = sorted(per, key=lambda x: int(x))
        if first_n:
            ids = ids[:first_n]     # resident verify dispatches come first (warmup + steps)
        for d in ids:
            for c, v in per[d].items():
                vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}


if __name__ == "__main__":
    tag_dir, payload = sys.argv[1], float(sys.argv[2])
    first_n = int(sys.argv[3]) if len(sys.argv) > 3 else None
    m = load(tag_dir, first_n)
    out = {"counters_mean_per_launch": m}
    if "TCC_EA0_RDREQ_32B_sum" in m:
        rd = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + 128 * m.get("TCC_EA0_RDREQ_128B_sum", 0)
        out["rdreq_bytes_by_size"] = rd
        out["rdreq_bytes_over_payload"] = rd / payload
    if "FETCH_SIZE" in m:
        out["fetch_size_bytes"] = m["FETCH_SIZE"] * 1024
        out["fetch_size_x2_over_payload"] = 2 * m["FETCH_SIZE"] * 1024 / payload
    if "TCC_HIT_sum" in m:
        out["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    if "SQ_INSTS_VALU" in m and "SQ_WAVE_CYCLES" in m:
        out["valu_per_wave_cycle"] = m["SQ_INSTS_VALU"] / max(1.0, m["SQ_WAVE_CYCLES"])
    print(json.dumps(out, indent=1))
