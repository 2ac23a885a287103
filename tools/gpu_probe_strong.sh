set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q -k "cfg1" --timeout 120 --timeout-method thread > gpurun_out/pytest_cfg1.log 2>&1 && echo CFG1_OK &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
   bench.py --gpus 2 --steps 5 --warmup 2 --strong --e2e-steps 1 > gpurun_out/bench_strong_n2.json 2> gpurun_out/bench_strong_n2.err && echo STRONG_OK
rc=$?
tail -3 gpurun_out/pytest_cfg1.log; cat gpurun_out/bench_strong_n2.json; tail -3 gpurun_out/bench_strong_n2.err
exit $rc
