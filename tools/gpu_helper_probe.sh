#!/bin/bash
# Timing-only probes of the split kernel's helper wave (tools/gen_sha1_asm.py TV_GEN_HX): which part of the
# helper's work slows its rounds wave?  hx_novalu / hx_nowrite / hx_noload produce WRONG digests by design.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/helper_probe
mkdir -p $O
KERNEL=2 REPS=5 GIB=16 timeout -k 10 400 python3 tools/variant_bench.py 16384,32768 hx_base hx_novalu hx_nowrite hx_noload > $O/ab.jsonl 2>&1
rc=$?
cat $O/ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('variant'), d.get('P'), round(d.get('best_ms',0),3), round(d.get('median_ms',0),3), d.get('gbps'), d.get('ok'), d.get('error','')[:300])"
exit $rc
