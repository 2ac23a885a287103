"""CPU unit tests of torrent_amd/csrc/tv_plan.h: the resident payload planner (tv_set_layout's out-of-memory retry loop
ends for every shape, including pieces larger than the memory left; ADVICE r04: it looped forever), a stream's
windows x columns under a device budget (stream_geometry: the documented shapes, and its invariants over a sweep),
and the file table's walk."""
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


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_file_table_walk_equals_the_python_host(tmp_path):
    """tv_stage_file_table's walk (tv_plan.h walk_file_table, run on the CPU by tests/c/walk_main.cpp) hands the
    library the same segments as verify_files' own walk (torrent_amd/verify.py _files_shard over storage.py;
    zero-length ones included) for the 48 seeded random layouts of tests/test_gpu_fuzz.py on 1, 3 and 8 shards --
    so both hosts' plans agree whether the host or the library walks the file table."""
    from tests.test_gpu_fuzz import SEEDS, _draw
    from torrent_amd import verify
    from torrent_amd.piece import piece_length
    from torrent_amd.storage import Storage, fs_storage
    exe = str(tmp_path / "walk_main")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                           os.path.join(ROOT, "tests", "c", "walk_main.cpp"), "-o", exe])

    class Plan:
        def __init__(self):
            self.segments = []

        def set_option(self, key, value):
            pass

        def stage_files(self, paths, fo, lin, lens):
            self.segments += [(p, int(a), int(b), int(c)) for p, a, b, c in zip(paths, fo, lin, lens)]
            return [0] * len(paths)

    checked = 0
    for seed in SEEDS:
        info = _draw(seed)[0]
        P, L = info.n_pieces, info.piece_length
        st = Storage(fs_storage, info, "/plan/dl")
        paths = st.file_paths()
        lengths = [info.length] if info.files is None else [f.length for f in info.files]
        for n in (1, 3, 8):
            for first, count in verify.shard_ranges(P, n):
                if not count:
                    continue
                plan = Plan()
                verify._files_shard(plan, info, st, first, count, threads=1)
                last = first + count - 1
                lo, hi = first * L, min(info.length, last * L + piece_length(last, info))
                inp = f"{len(lengths)} {lo} {hi} {L}\n" + " ".join(map(str, lengths)) + "\n"
                out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
                segs = [tuple(map(int, ln.split())) for ln in out if ln and not ln.startswith("reached")]
                reached = int([ln for ln in out if ln.startswith("reached")][0].split()[1])
                got = sorted((paths[k], fo, lin, ln) for k, fo, lin, ln in segs)
                assert got == sorted(plan.segments), (seed, n, first)
                assert reached >= hi, (seed, n, first)      # (the fuzz tables always cover their torrent)
                checked += 1
    assert checked > 48 * 3
