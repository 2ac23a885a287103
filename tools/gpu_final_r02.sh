#!/bin/bash
# Round-2 final-build GPU session: smoke, the whole -m gpu suite, the default bench line, then rocprofv3
# --kernel-trace --stats of the cfg2 and cfg4 bench commands (their verify-kernel averages back the bench's
# HIP-event kernel_ms_avg).  Each GPU step under its own time limit, chained with &&.
# usage: tools/gpu_final_r02.sh [tag]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 600 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo BENCH_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt_cfg2" -o run -- \
    python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-saturating --no-cfg4 > $O/kt_cfg2.json 2> $O/kt_cfg2.err && echo KT_CFG2_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt_cfg4" -o run -- \
    python3 bench.py --workload cfg4 --strong --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/kt_cfg4.json 2> $O/kt_cfg4.err && echo KT_CFG4_OK
rc=$?
tail -2 $O/smoke.log; tail -2 $O/pytest_gpu.log; cat $O/bench_n1.json
exit $rc
