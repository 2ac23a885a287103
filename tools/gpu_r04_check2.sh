#!/bin/bash
# Round 4 check 2: the -m gpu suite on the build with the split helper's mid-block LDS-write wait and the pair-load
# lane loop's aligned byte swaps; lane A/B of the byte swaps (asm vs compiler) at 65,536 / 262,144 pieces; bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${CHECK_OUT:-r04_check2}
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
KERNEL=1 GIB=16 REPS=7 timeout -k 10 400 python3 tools/variant_bench.py 65536,262144 cur bswapc > $out/ab_lane_bswap.jsonl 2>&1 && echo AB_OK &&
KERNEL=1 GIB=16 REPS=7 timeout -k 10 400 python3 tools/variant_bench.py 65536,262144 bswapc cur >> $out/ab_lane_bswap.jsonl 2>&1 && echo AB2_OK &&
timeout -k 10 300 python3 -u bench.py > $out/bench_n1.json 2> $out/bench_n1.err && echo BENCH_OK
