set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u - > gpurun_out/stage_repeat.log 2>&1 <<'PY'
import sys, pytest
fails = 0
for rep in range(6):
    rc = pytest.main(["-q", "-x", "-m", "gpu", "tests/test_gpu_paths.py", "-k", "stage_files or stage_file_windows or resume_from_disk",
                      "-p", "no:cacheprovider"])
    print("REP", rep, "rc", int(rc), flush=True)
    fails += int(rc) != 0
    if rc != 0:
        break
print("FAILS", fails)
sys.exit(1 if fails else 0)
PY
rc=$?
grep "REP\|FAILS\|passed\|failed" gpurun_out/stage_repeat.log
exit $rc
