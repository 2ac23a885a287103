#!/bin/bash
# Whole-call time per tv_verify step (tools/step_ab.py) with and without torch's device context in the process
# (bench.py creates it for its synchronize), interleaved 3 times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03_step
for r in 1 2 3; do
  ROUNDS=1 TORCH=0 timeout -k 10 300 python3 tools/step_ab.py cur >> gpurun_out/r03_step/step_torch.jsonl 2>&1 &&
  ROUNDS=1 TORCH=1 timeout -k 10 300 python3 tools/step_ab.py cur >> gpurun_out/r03_step/step_torch.jsonl 2>&1 || exit 1
done
cat gpurun_out/r03_step/step_torch.jsonl
