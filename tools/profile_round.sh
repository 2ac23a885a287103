#!/bin/bash
# GPU session: bench line + rocprofv3 kernel-trace/stats summary + counter list.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err && echo BENCH_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/kt" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof/kt_bench.json 2> gpurun_out/prof/kt.err && echo KT_OK &&
timeout -k 10 120 rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1; echo LIST_DONE
cat gpurun_out/bench_cfg2.json
find gpurun_out/prof -name "*stats*" | head
