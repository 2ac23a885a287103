#!/bin/bash
# A/B: split loops with s_sub-borrow loop control (b1) and s_setprio 3 on the rounds wave (p3) vs the shipped build (b0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/borrow_ab
mkdir -p $O
KERNEL=2 REPS=5 GIB=16 timeout -k 10 400 python3 tools/variant_bench.py 16384,25600,32768 b0 b1 p3 > $O/ab.jsonl 2>&1
rc=$?
cat $O/ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('error','')[:300])"
exit $rc
