#!/bin/bash
# A/B of the lane kernel's steady-state loop shape (TV_LANE_TRIPS 1 vs 0) at cfg4 geometry and 65,536 / 40,960 pieces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/trips_ab
mkdir -p $O
KERNEL=1 REPS=5 GIB=200 timeout -k 10 300 python3 tools/variant_bench.py 51200 trips1 trips0 > $O/cfg4.jsonl 2>&1 &&
KERNEL=1 REPS=5 GIB=16 timeout -k 10 200 python3 tools/variant_bench.py 65536,40960 trips1 trips0 > $O/p16.jsonl 2>&1
rc=$?
cat $O/cfg4.jsonl $O/p16.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('digests_match_first'), d.get('error','')[:300])"
exit $rc
