#!/bin/bash
# A/B: the split helper writes K+W (k0, shipped before) vs W with the rounds wave adding K (k1, TV_GEN_KROUNDS=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/krounds_ab
mkdir -p $O
KERNEL=2 REPS=5 GIB=16 timeout -k 10 400 python3 tools/variant_bench.py 16384,25600,32768 k0 k1 > $O/ab.jsonl 2>&1
rc=$?
cat $O/ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('error','')[:300])"
exit $rc
