#!/bin/bash
# A/B of the split kernel's instruction alignment (tools/gen_sha1_asm.py TV_GEN_HPAIR / TV_GEN_LALIGN).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/split_align_ab
mkdir -p $O
KERNEL=2 REPS=5 GIB=16 timeout -k 10 500 python3 tools/variant_bench.py 16384,25600,32768 s_base s_hpair s_lalign s_both > $O/ab.jsonl 2>&1
rc=$?
cat $O/ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('digests_match_first'), d.get('error','')[:300])"
exit $rc
