#!/bin/bash
# One PMC pass (GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES) over tools/twin_occ_pmc.py, then shader cycles
# per block per twin dispatch (GRBM_GUI_ACTIVE / 8 XCDs / 16,385 blocks).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/occpmc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/occpmc" -o run -- \
    python3 tools/twin_occ_pmc.py > gpurun_out/occpmc.log 2>&1 || { tail gpurun_out/occpmc.log; exit 1; }
cat gpurun_out/occpmc.log
python3 - <<'PY'
import csv, glob
from collections import defaultdict
f = glob.glob("gpurun_out/occpmc/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(f)):
    if "twin_kernel<false" in r["Kernel_Name"]:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for d in sorted(per):
    c = per[d]
    print(d, "cycles/block", round(c["GRBM_GUI_ACTIVE"] / 8 / 16385, 1), {k: v for k, v in c.items()})
PY
