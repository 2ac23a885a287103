#!/bin/bash
# Twin kernel A/B at cfg2, 2-wave workgroups (PAIRS=1): the rounds loop with and without its in-loop
# s_nop (TV_GEN_TWIN_NONOP) / when the next block's reads are issued (TV_GEN_TWIN_ISSUE); split on the same library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/twin_ab5
mkdir -p $O
KERNEL=2 PAIRS=1 REPS=5 GIB=16 timeout -k 10 200 python3 tools/variant_bench.py 16384 t3_end > $O/split.jsonl 2>&1 || exit 1
KERNEL=4 PAIRS=1 REPS=7 GIB=16 timeout -k 10 500 python3 tools/variant_bench.py 16384 t3_end t3_mid t3_spread > $O/twin.jsonl 2>&1
rc=$?
cat $O/split.jsonl $O/twin.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('kernel'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('error','')[:300])"
exit $rc
