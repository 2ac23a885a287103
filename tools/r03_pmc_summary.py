"""Per-block summaries of the round-3 PMC passes (tools/gpu_r03_profile.sh, tools/gpu_companions_r03.sh) ->
profiles/r03/*.json.  Counter units: GRBM_GUI_ACTIVE = shader cycles summed over the 8 XCDs; SQ_WAVE_CYCLES,
SQ_WAIT_*, SQ_ACTIVE_INST_* = quad-cycles summed over waves (MI355X_MICROARCH.md, rocprofv3 PMC slots and
per-instruction constants); FETCH_SIZE = KiB, half the bytes of a wide streaming read on gfx950 (doubled here).
usage: python tools/r03_pmc_summary.py gpurun_out/r03_prof gpurun_out/r03_comp profiles/r03"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def dispatches(path, match):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return [per[d] for d in sorted(per)]


def mean(rows, k):
    v = [r[k] for r in rows if k in r]
    return sum(v) / len(v) if v else None


def main():
    prof, comp, out = sys.argv[1:4]
    os.makedirs(out, exist_ok=True)
    # split kernel, cfg4 N = 2 shard: 25,600 x 4 MiB (65,537 blocks per piece), 400 workgroups of 2 waves
    blocks, wgs = 65537, 400
    rows = []
    for i in (1, 2, 3):
        d = dispatches(os.path.join(prof, "pmc_split", f"p{i}"), "split_kernel<false")
        rows.append(d[2:])            # after the creation-mode hash and the 2 warm-up verifies
    m = {k: mean(r, k) for r in rows for k in r[0]}
    waves = 2 * wgs
    per_wave_block = lambda q: 4 * q / waves / blocks if q is not None else None   # noqa: E731
    split = {
        "geometry": "cfg4 shard at N = 2: 25,600 x 4 MiB pieces, split kernel, 400 workgroups x {rounds, helper}",
        "timing": json.load(open(os.path.join(prof, "split25600_plain.json"))),
        "cycles_per_block": m["GRBM_GUI_ACTIVE"] / 8 / blocks,
        "per_wave_per_block_cycles": {k: per_wave_block(m[k]) for k in
                                      ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                       "SQ_WAIT_INST_LDS")},
        "per_workgroup_per_block": {"valu": m["SQ_INSTS_VALU"] / wgs / blocks, "lds_instr": m["SQ_INSTS_LDS"] / wgs / blocks,
                                    "salu": m["SQ_INSTS_SALU"] / wgs / blocks, "vmem_rd": m["SQ_INSTS_VMEM_RD"] / wgs / blocks,
                                    "lds_array_cycles": m["SQ_LDS_IDX_ACTIVE"] / wgs / blocks,
                                    "lds_bank_conflict_cycles": m["SQ_LDS_BANK_CONFLICT"] / wgs / blocks},
        "counters_mean_per_launch": m,
    }
    json.dump(split, open(os.path.join(out, "pmc_split_25600.json"), "w"), indent=1)
    # twin at 8,192 (one 2-wave workgroup per CU, companions off) vs 16,384 (two per CU), 1 MiB pieces
    occ = {}
    for p in ("p1", "p2"):
        d = dispatches(os.path.join(prof, "pmc_occ", p), "twin_kernel<false")
        for P, part in ((8192, d[:4]), (16384, d[4:])):
            rec = occ.setdefault(P, {})
            for k in part[0]:
                rec[k] = mean(part[1:], k)
    blocks1 = 16385
    occ_out = {}
    for P, c in occ.items():
        waves = 2 * (P // 32)
        occ_out[str(P)] = {
            "workgroups_per_cu": P // 32 // 256, "cycles_per_block": c["GRBM_GUI_ACTIVE"] / 8 / blocks1,
            "per_wave_per_block_cycles": {k: 4 * c[k] / waves / blocks1 for k in
                                          ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
                                           "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS")},
            "valu_per_wave_per_block": c["SQ_INSTS_VALU"] / waves / blocks1,
            "lds_bank_conflict": c["SQ_LDS_BANK_CONFLICT"], "counters_mean_per_launch": c}
    json.dump(occ_out, open(os.path.join(out, "pmc_twin_occupancy.json"), "w"), indent=1)
    # companions: light (reads 0) / full (reads 1) / off, at 6,400 and 12,800 x 4 MiB
    comp_out = {"times": [json.loads(x) for x in open(os.path.join(comp, "times.jsonl"))]}
    for sh in (8, 4):
        for f, r in ((1, 0), (1, 1), (0, 0)):
            d = dispatches(os.path.join(comp, f"pmc_s{sh}_f{f}_r{r}"), "twin_kernel<false")[1:]
            payload = 51200 // sh * 4 * 2 ** 20
            comp_out[f"pieces_{51200 // sh}_" + {(1, 0): "light", (1, 1): "full", (0, 0): "off"}[(f, r)]] = {
                "hbm_read_over_payload": [round(x["FETCH_SIZE"] * 2048 / payload, 4) for x in d],
                "cycles_per_block": [round(x["GRBM_GUI_ACTIVE"] / 8 / 65537, 1) for x in d]}
    json.dump(comp_out, open(os.path.join(out, "companions_ab.json"), "w"), indent=1)
    print(json.dumps({"split_cycles_per_block": split["cycles_per_block"],
                      "split_per_wave": split["per_wave_per_block_cycles"],
                      "occ": {P: (v["cycles_per_block"], v["per_wave_per_block_cycles"]) for P, v in occ_out.items()}},
                     indent=1))


if __name__ == "__main__":
    main()
