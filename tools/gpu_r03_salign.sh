#!/bin/bash
# Split rounds-loop 64-byte placement A/B at cfg4's N = 2 shard geometry (25,600 x 4 MiB = 100 GiB): variants from
# tools/build_variants.py (TV_GEN_SPLIT_RALIGN = k: loop head at 8 k mod 64), interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03_align
KERNEL=2 GIB=100 REPS=5 timeout -k 10 700 python3 tools/variant_bench.py 25600 ${VARIANTS:-scur s0 s1 s2 s3 s4 s5 s6 s7} > gpurun_out/r03_align/split_ralign.jsonl 2>&1
rc=$?
cat gpurun_out/r03_align/split_ralign.jsonl
exit $rc
