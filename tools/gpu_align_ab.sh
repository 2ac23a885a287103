#!/bin/bash
# A/B of the lane compression's instruction alignment (tools/gen_sha1_asm.py TV_GEN_PAIRXOR / TV_GEN_ALIGN):
# base = round-2 build, align = block start .p2align 3 only, pair = schedule xors paired + aligned start.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/align_ab
mkdir -p $O
KERNEL=1 REPS=5 GIB=200 timeout -k 10 400 python3 tools/variant_bench.py 51200 base align pair > $O/cfg4.jsonl 2>&1 &&
KERNEL=1 REPS=5 GIB=16 timeout -k 10 300 python3 tools/variant_bench.py 65536,40960 base align pair > $O/p16.jsonl 2>&1
rc=$?
cat $O/cfg4.jsonl $O/p16.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('digests_match_first'), d.get('error','')[:300])"
exit $rc
