#!/bin/bash
# Twin kernel on one GPU: the parity suite (every kernel, incl. twin = TV_OPT_KERNEL 4), the full-size cfg2
# oracle test, and a split-vs-twin piece-count sweep (16 GiB per point).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_paths.py::test_full_size_cfg2_oracle_ground_truth" -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/twin_parity.log 2>&1 || { tail -40 gpurun_out/twin_parity.log; exit 1; }
tail -3 gpurun_out/twin_parity.log
SWEEP_VARIANTS=split1,twin SWEEP_PS=${SWEEP_PS:-8192,12800,16384,20480,25600} timeout -k 10 300 python -u tools/sweep_pieces.py gpurun_out/sweep_twin.jsonl > gpurun_out/sweep_twin.log 2>&1
cat gpurun_out/sweep_twin.log
