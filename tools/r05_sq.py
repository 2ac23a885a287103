"""VALU issue figures of the resident verify kernels from one SQ + GRBM PMC pass (tools/gpu_r05_sq.sh output):
per verify dispatch after the first, VALU instructions per wave per 64-B block, the share of wave time with a VALU
instruction issuing (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, both in quad-cycles), the parked share (SQ_WAIT_ANY),
cycles per block (GRBM_GUI_ACTIVE / 8 XCDs / blocks per piece) and the shader clock (GUI cycles per XCD / kernel
time).  Writes <out>/sq_valu.json with the build id the pass ran on.

    python tools/r05_sq.py gpurun_out/r05_sq profiles/r05
"""
import collections
import csv
import json
import os
import sys

BLOCKS = {"cfg2": (1 << 20) // 64 + 1, "suppl": (256 << 10) // 64 + 1}   # 64-B blocks per piece, padding block incl.


def main():
    src, out = sys.argv[1], sys.argv[2]
    build = open(os.path.join(src, "build_id.txt")).read().strip()
    res = {"build_id": build, "source": src, "method": "rocprofv3 --pmc (8 SQ counters + GRBM_GUI_ACTIVE, one pass) over "
           "`bench.py --workload W --steps 2 --warmup 1` (tools/gpu_r05_sq.sh); SQ_*_CYCLES / SQ_ACTIVE_INST_* / "
           "SQ_WAIT_* in quad-cycles (MI355X_MICROARCH.md), GRBM_GUI_ACTIVE summed over the 8 XCDs"}
    for w, blocks in BLOCKS.items():
        path = os.path.join(src, f"sq_{w}", "p1", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        by = collections.defaultdict(lambda: collections.defaultdict(float))
        meta = {}
        for r in csv.DictReader(open(path)):
            d = int(r["Dispatch_Id"])
            by[d][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[d] = (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        verify = [d for d in sorted(by) if meta[d][0].startswith(("void tv_twin_kernel<false", "void tv_lane_kernel<false",
                                                                   "void tv_split_kernel<false"))]
        rows = []
        for d in verify:
            c = by[d]
            ns = meta[d][2] - meta[d][1]
            gui = c["GRBM_GUI_ACTIVE"] / 8
            rows.append({
                "dispatch": d, "kernel": meta[d][0], "waves": int(c["SQ_WAVES"]),
                "valu_per_wave_block": round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"] / blocks, 1),
                "valu_active_share_of_wave_time": round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4),
                "parked_share_of_wave_time": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
                "issue_stall_share": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
                "cycles_per_block": round(gui / blocks, 1), "kernel_ms_under_profiler": round(ns / 1e6, 3),
                "clock_ghz": round(gui / ns, 3)})
        res[w] = {"blocks_per_piece": blocks, "dispatches": rows}
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "sq_valu.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
