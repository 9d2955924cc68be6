"""CPU check of the engine's pass rules with the chunk simulator (tools/sim/chunk_sim.cpp).

The simulator replays a stream chunk by chunk the way the engine does -- rank-packed speculation against the frontier,
exact per-invoker validation, commit of the known-to-fit prefix -- and, in modes 7-9, the in-pass re-decisions of
DESIGN.md section 5.1 (one per pass / unlimited / unlimited but a re-decided action's next lane stops the pass, the
shipped rule).  Every lane it commits is compared with the sequential reference replay (oracle/), and every
re-decision that resumes its walk at the speculated step is compared with a walk from the action's cursor: the run
fails on "UNSOUND" or on any resume mismatch.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    d = tmp_path_factory.mktemp("sim")
    exe = str(d / "chunk_sim")
    subprocess.run(["g++", "-O2", "-o", exe, os.path.join(ROOT, "tools", "sim", "chunk_sim.cpp")], check=True,
                   capture_output=True)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sim", "dump_workload.py"), "c2", "40000", str(d)],
                   check=True, capture_output=True)
    return exe, str(d / "c2")


@pytest.mark.parametrize("width,mode", [(192, 5), (192, 7), (192, 8), (192, 9), (392, 9)])
def test_pass_rules_match_the_sequential_replay(sim, width, mode):
    exe, data = sim
    r = subprocess.run([exe, data, str(width), str(mode)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = r.stdout.strip().splitlines()[-1]
    assert "UNSOUND" not in r.stderr and "resume mismatch" not in r.stderr
    assert re.search(r"mismatches=0\b", line), line
    assert re.search(r"resume_bad=0\b", line), line
    if mode >= 7:
        assert int(re.search(r" ext=(\d+)", line).group(1)) > 0, line
