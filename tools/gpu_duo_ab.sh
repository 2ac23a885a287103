set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/duo_ab
KERNEL=4 REPS=3 timeout -k 10 500 python3 tools/variant_bench.py 32768,51200 p0 p1 p2 > gpurun_out/duo_ab/ab.jsonl 2>&1
rc=$?; cat gpurun_out/duo_ab/ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), d.get('best_ms'), d.get('gbps'), d.get('ok'), d.get('digests_match_first'), d.get('error','')[:300])"
exit $rc
