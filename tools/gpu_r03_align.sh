#!/bin/bash
# Twin rounds-loop 64-byte placement A/B at cfg2 (16,384 x 1 MiB): variants built by tools/build_variants.py
# (TV_GEN_TWIN_RALIGN = k puts the loop head at 4 + 8 k mod 64), the round-2 library (r02) and the current
# default (cur), interleaved twice, each in its own process (tools/variant_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03_align
KERNEL=4 GIB=16 REPS=7 timeout -k 10 600 python3 tools/variant_bench.py 16384 ${VARIANTS:-r02 cur r0 r1 r2 r3 r4 r5 r6 r7} > gpurun_out/r03_align/twin_ralign.jsonl 2>&1
rc=$?
cat gpurun_out/r03_align/twin_ralign.jsonl
exit $rc
