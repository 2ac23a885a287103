#!/bin/bash
# Twin companions (TV_OPT_TWIN_FILL, default on): the -m gpu suite, then the piece-count sweep (auto = twin with
# companions below 16,384 pieces) and the occupancy probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/companions
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo TESTS_OK &&
SWEEP_VARIANTS=split1,twin1 SWEEP_PS=4096,6400,8192,12800,16384,20480,25600 timeout -k 10 600 python -u tools/sweep_pieces.py $O/sweep.jsonl > $O/sweep.log 2>&1 && echo SWEEP_OK &&
timeout -k 10 300 python -u tools/twin_occupancy_probe.py > $O/occ.log 2>&1 && echo OCC_OK
rc=$?
tail -2 $O/pytest_gpu.log; tail -10 $O/sweep.log; cat $O/occ.log
exit $rc
