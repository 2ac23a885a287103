#!/bin/bash
# Round 4: lane kernel classic (3-deep ring) vs pair loads (4-deep ring refilled in pairs), interleaved, over piece
# counts from 40,960 to 262,144 (16 GiB per point) and at cfg4's exact geometry (51,200 x 4 MiB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_pairs}
mkdir -p $out
KERNEL=1 GIB=16 REPS=7 timeout -k 10 500 python3 tools/variant_bench.py 40960,51200,65536,131072,262144 base pairs > $out/ab_lane_sweep.jsonl 2>&1 && echo SWEEP_OK &&
KERNEL=1 GIB=200 REPS=5 timeout -k 10 500 python3 tools/variant_bench.py 51200 base pairs > $out/ab_lane_cfg4.jsonl 2>&1 && echo CFG4_OK
rc=$?
python3 - <<'PY'
import json, collections
for f in ("gpurun_out/r04_pairs/ab_lane_sweep.jsonl", "gpurun_out/r04_pairs/ab_lane_cfg4.jsonl"):
    best = collections.defaultdict(list)
    for l in open(f):
        try: r = json.loads(l)
        except Exception: continue
        if "best_ms" in r: best[(r["P"], r["L"], r["variant"])].append((r["best_ms"], r["median_ms"], r["ok"]))
    for k, v in sorted(best.items()): print(k, v)
PY
exit $rc
