#!/bin/bash
# cfg4 on one GPU (200 GiB, 4 MiB pieces, lane kernel): the bench line, then one PMC pass for the clock
# (GRBM_GUI_ACTIVE per dispatch / kernel time) so a kernel time can be read as cycles per block.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/cfg4
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload cfg4 --e2e-steps 0 --no-saturating --no-cpu-baseline --steps 5 --warmup 2 \
    > gpurun_out/cfg4/bench.json 2> gpurun_out/cfg4/bench.err && echo BENCH_OK &&
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/cfg4/pmc" -o run -- \
    python3 bench.py --workload cfg4 --e2e-steps 0 --no-saturating --no-cpu-baseline --steps 3 --warmup 1 \
    > gpurun_out/cfg4/pmc_bench.json 2> gpurun_out/cfg4/pmc.err && echo PMC_OK
rc=$?
cat gpurun_out/cfg4/bench.json | cut -c1-400
exit $rc
