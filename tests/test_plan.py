"""CPU unit test of the resident payload planner (torrent_amd/csrc/tv_plan.h): tv_set_layout's out-of-memory
retry loop ends for every shape, including pieces larger than the memory left (it looped forever)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_payload_planner_terminates(tmp_path):
    exe = str(tmp_path / "plan_test")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", os.path.join(ROOT, "tests", "c", "plan_test.cpp"),
                           "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
