#!/bin/bash
# Twin kernel A/B probes (tools/build_variants.py t_*): helper work classes (HX: wrong digests by design),
# wait placement and next-block reads; split (KERNEL=2) on the same library as the reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/twin_ab
mkdir -p $O
KERNEL=2 REPS=5 GIB=16 timeout -k 10 200 python3 tools/variant_bench.py 16384 t_base > $O/split.jsonl 2>&1 || exit 1
KERNEL=4 REPS=5 GIB=16 timeout -k 10 500 python3 tools/variant_bench.py 16384 t_base t_novalu t_nowrite t_noload t_w5 t_nopre t_w3 > $O/twin.jsonl 2>&1
rc=$?
cat $O/split.jsonl $O/twin.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('kernel'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('error','')[:300])"
exit $rc
