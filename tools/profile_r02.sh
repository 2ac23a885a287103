#!/bin/bash
# Round-2 GPU session: rocprofv3 --kernel-trace --stats of the cfg2 and cfg4 bench lines (their average
# verify-kernel durations must agree with the bench's HIP-event kernel_ms_avg), then a 2-rank rehearsal of
# the N>1 default (cfg4 strong + cfg2_weak + e2e_cfg5) on one GPU.  Each step under its own time limit.
# usage: tools/profile_r02.sh [tag]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt_cfg2" -o run -- \
    python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-saturating --no-cfg4 > $O/kt_cfg2.json 2> $O/kt_cfg2.err && echo KT_CFG2_OK &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt_cfg4" -o run -- \
    python3 bench.py --workload cfg4 --strong --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/kt_cfg4.json 2> $O/kt_cfg4.err && echo KT_CFG4_OK &&
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err && echo N2_OK
rc=$?
cat $O/kt_cfg2.json $O/kt_cfg4.json $O/bench_n2_rehearsal.json
exit $rc
