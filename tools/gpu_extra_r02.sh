#!/bin/bash
# Round-2 final build, second session: PMC passes of the cfg4 lane kernel (cycles per block after the aligned
# compression), the 2-rank rehearsal of the N>1 default on one GPU, and cfg3 end to end.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/extra
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 bash tools/pmc.sh cfg4 1 cfg4_aligned > $O/pmc.log 2>&1 && echo PMC_OK &&
python3 tools/pmc_summary.py gpurun_out/pmc/cfg4_aligned 214748364800 > $O/pmc_cfg4_summary.json 2>&1 &&
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err && echo N2_OK &&
mkdir -p /tmp/cfg3 && timeout -k 10 300 python3 tools/cfg3_bench.py /tmp/cfg3 > $O/cfg3.log 2>&1 && echo CFG3_OK
rc=$?
cat $O/pmc.log; cat $O/pmc_cfg4_summary.json; cat $O/bench_n2_rehearsal.json; tail -8 $O/cfg3.log
exit $rc
