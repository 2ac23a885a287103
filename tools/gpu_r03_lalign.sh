#!/bin/bash
# Lane-kernel loop placement A/B at cfg4 on one GPU (51,200 x 4 MiB = 200 GiB): variants lp0..lp15 from
# tools/build_variants.py D_TV_LANE_PAD=k (the raw-block loop's head at 44 + 4 k mod 64), interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03_align
KERNEL=1 GIB=200 REPS=4 timeout -k 10 1000 python3 tools/variant_bench.py 51200 ${VARIANTS:-lp0 lp1 lp2 lp3 lp4 lp5 lp6 lp7 lp8 lp9 lp10 lp11 lp12 lp13 lp14 lp15} > gpurun_out/r03_align/lane_pad.jsonl 2>&1
rc=$?
cat gpurun_out/r03_align/lane_pad.jsonl
exit $rc
