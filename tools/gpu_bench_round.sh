#!/bin/bash
# one GPU session: smoke, parity tests, the bench line at N=1 and a 2-rank rehearsal on one GPU.
# Each GPU step has its own time limit; the steps are chained with && (nothing runs after a failure).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK &&
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
   bench.py --gpus 2 --steps 5 --warmup 2 --no-saturating > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err && echo BENCH_N2_OK
rc=$?
tail -3 gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/bench.err 2>/dev/null
cat gpurun_out/bench.json gpurun_out/bench_n2.json 2>/dev/null
exit $rc
