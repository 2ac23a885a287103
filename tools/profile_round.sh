#!/bin/bash
# GPU session: bench line + rocprofv3 kernel-trace/stats of the same command + PMC traffic passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=${1:-r01}
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err && echo BENCH_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG/kt" -o run -- \
    python3 bench.py --no-cpu-baseline --e2e-steps 0 > gpurun_out/prof_$TAG/kt_bench.json 2> gpurun_out/prof_$TAG/kt.err && echo KT_OK &&
timeout -k 10 600 bash tools/pmc.sh cfg2 0 cfg2_split_$TAG && echo PMC_OK
cat gpurun_out/prof_$TAG/bench.json
