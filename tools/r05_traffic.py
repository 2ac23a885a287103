"""Round-5 HBM traffic per verify launch from rocprofv3 PMC passes (tools/gpu_r05_pmc.sh), written to
profiles/traffic_<workload>.json WITH the build id of the library measured (bench.py attaches
a traffic figure only to the build it was measured on).

Counter units (MI355X_MICROARCH.md, PMC section): FETCH_SIZE in KiB and, for 16-B/lane streaming reads on gfx950,
half the bytes actually read (doubled here); TCC_EA0_RDREQ_{32B,64B,128B} count requests of that size (bytes =
32 x + 64 y + 128 z).  Each counter group ran in its own pass.  The verify dispatches are the bench's resident
verify launches (the kernel named per workload), the first one (warm-up) dropped.

usage: python tools/r05_traffic.py <gpurun_out pmc dir> <profiles/rNN dir> [workload ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {"cfg2": (1 << 20, 16384, "tv_twin_kernel<false"), "suppl": (256 << 10, 65536, "tv_lane_kernel<false")}


def dispatches(path, match):
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith(match) or match in r["Kernel_Name"]:
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [per[k] for k in sorted(per)]


def main():
    src, out = sys.argv[1:3]
    names = sys.argv[3:] or list(WORKLOADS)
    os.makedirs(out, exist_ok=True)
    build = open(os.path.join(src, "build_id.txt")).read().strip()
    for w in names:
        L, P, match = WORKLOADS[w]
        payload = L * P
        p1 = dispatches(os.path.join(src, f"pmc_{w}", "p1"), match)[1:]
        p2 = dispatches(os.path.join(src, f"pmc_{w}", "p2"), match)[1:]
        fetch = [2 * 1024 * r["FETCH_SIZE"] for r in p1]
        rdreq = [32 * r["TCC_EA0_RDREQ_32B_sum"] + 64 * r["TCC_EA0_RDREQ_64B_sum"] + 128 * r["TCC_EA0_RDREQ_128B_sum"]
                 for r in p2]
        rec = {"workload": w, "kernel": match.split("<")[0].replace("tv_", "").replace("_kernel", ""),
               "build_id": build, "payload_bytes_per_launch": payload,
               "hbm_bytes_per_launch": sum(fetch) / len(fetch),
               "traffic_ratio": sum(fetch) / len(fetch) / payload,
               "rdreq_bytes_per_launch": sum(rdreq) / len(rdreq) if rdreq else None,
               "rdreq_ratio": sum(rdreq) / len(rdreq) / payload if rdreq else None,
               "per_dispatch_fetch_x2": fetch, "per_dispatch_rdreq": rdreq,
               "method": f"rocprofv3 --pmc FETCH_SIZE in its own pass over `bench.py --workload {w}` "
                         "(tools/gpu_r05_pmc.sh): 2 x FETCH_SIZE x 1024 bytes per verify dispatch (gfx950 reports half "
                         "the bytes of a 16-B/lane streaming read: MI355X_MICROARCH.md HBM section), mean over the "
                         "verify dispatches after the first; TCC_EA0_RDREQ_{32B,64B,128B} by size in a second pass",
               "source": f"{os.path.relpath(src, ROOT)}/pmc_{w}/p1, p2 -> {os.path.relpath(out, ROOT)}/"}
        json.dump(rec, open(os.path.join(ROOT, "profiles", f"traffic_{w}.json"), "w"), indent=1)
        json.dump(rec, open(os.path.join(out, f"traffic_{w}.json"), "w"), indent=1)
        print(json.dumps({k: v for k, v in rec.items() if not k.startswith("per_")}))


if __name__ == "__main__":
    main()
