#!/bin/bash
# Split kernel A/B (edit the variant names): next block's reads mid-block (TV_GEN_SPLIT_MID=1, s_mid) or all 15 after round 79 (TV_GEN_SPLIT_PRE=1, s_pre),
# 20-quad ring) vs the shipped 15 reads at the block start, at cfg4's N = 2 per-GPU piece count and at cfg2's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/split_pre
mkdir -p $O
KERNEL=2 PAIRS=1 REPS=5 GIB=16 timeout -k 10 500 python3 tools/variant_bench.py 25600,16384 s_base s_pre > $O/ab.jsonl 2>&1
rc=$?
cat $O/ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('kernel'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('digests_match_first'), d.get('error','')[:300])"
exit $rc
