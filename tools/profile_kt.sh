#!/bin/bash
# GPU session: the bench line, then rocprofv3 --kernel-trace --stats of the same bench command
# (no PMC; tools/pmc.sh does the counter passes).  usage: tools/profile_kt.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=${1:-r01}
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err && echo BENCH_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG/kt" -o run -- \
    python3 bench.py --no-cpu-baseline --e2e-steps 0 > gpurun_out/prof_$TAG/kt_bench.json 2> gpurun_out/prof_$TAG/kt.err && echo KT_OK
rc=$?
cat gpurun_out/prof_$TAG/bench.json gpurun_out/prof_$TAG/kt_bench.json
exit $rc
