#!/bin/bash
# Round-3 bench session: the default bench line (N = 1: cfg2 + cfg4 anchor + e2e_cfg5 + piece_saturated + CPU
# baseline), rocprofv3 --kernel-trace --stats of the cfg2 bench command (its average verify-kernel duration must
# agree with the line's HIP-event kernel_ms_avg), and one FETCH_SIZE pass (HBM bytes per cfg2 verify launch).
# Each step under its own time limit; the first failure ends the session.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r03_bench
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo BENCH_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt_cfg2" -o run -- \
    python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-saturating --no-cfg4 > $O/kt_cfg2.json 2> $O/kt_cfg2.err && echo KT_OK &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-saturating --no-cfg4 > $O/pmc_fetch.json 2> $O/pmc_fetch.err && echo PMC_OK
rc=$?
cat $O/bench_n1.json
exit $rc
