#!/bin/bash
# Duo kernel first look: SIMD placement probe, kernel parity tests (every kernel), piece-count sweep
# lane / split / duo above 32,768 pieces.  Each GPU step under its own limit, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${1:-duo}
mkdir -p $O
timeout -k 10 60 build/simd_probe > $O/simd_probe.log 2>&1 && echo PROBE_OK && cat $O/simd_probe.log | tail -12 &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/parity.log 2>&1 && echo PARITY_OK && tail -2 $O/parity.log &&
SWEEP_VARIANTS=lane,split1,duo SWEEP_PS=${2:-32768,40960,51200,65536,98304} timeout -k 10 400 python3 tools/sweep_pieces.py $O/sweep.jsonl > $O/sweep.log 2>&1 && echo SWEEP_OK
rc=$?
tail -3 $O/parity.log; tail -8 $O/sweep.log
exit $rc
