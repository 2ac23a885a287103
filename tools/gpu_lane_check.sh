set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u tools/quick_bench.py mid > gpurun_out/quick_mid.log 2>&1 && echo QB_OK &&
timeout -k 10 300 python3 bench.py --workload cfg4 --e2e-steps 0 --no-saturating --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_cfg4_next.json 2>/dev/null && echo CFG4_OK
rc=$?
tail -n 2 gpurun_out/pytest_gpu.log; cat gpurun_out/quick_mid.log; cut -c1-420 gpurun_out/bench_cfg4_next.json
exit $rc
