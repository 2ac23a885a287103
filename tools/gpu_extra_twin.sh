#!/bin/bash
# Final (twin) build, extras: the 2-rank rehearsal of the N>1 default on one GPU (cfg4 strong 25,600 pieces per
# rank = split, cfg2_weak 16,384 per rank = twin, e2e_cfg5 per rank), and cfg3 end to end.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/extra_twin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err && echo N2_OK &&
mkdir -p /tmp/cfg3 && timeout -k 10 300 python3 tools/cfg3_bench.py /tmp/cfg3 > $O/cfg3.log 2>&1 && echo CFG3_OK
rc=$?
cat $O/bench_n2_rehearsal.json; tail -8 $O/cfg3.log
exit $rc
