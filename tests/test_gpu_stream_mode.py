"""The resident engine's stream mode (OWGS_SPEC_REPLAY=1: owgs_replay / owgs_replay_device(_span) through
owgs_resident.hip instead of the chunked engine) on the parity suite's stream cases: full-size
streams of every BASELINE config, shared fqn@version keys, pools near capacity, 15k/20k-invoker pools, span replays
with health changes and malformed streams, each bit-exact with the literal oracle.  The switch is read once per
process, so the cases run in a child pytest process (one at a time on the GPU)."""
import os
import re  # noqa: F401
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = ("stream_parity or malformed or large_pool or golden or span or capacity or redecision or activation_batch "
         "or state_overlap")


def test_stream_mode_parity_suite():
    env = dict(os.environ, OWGS_SPEC_REPLAY="1")
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.join(HERE, "test_gpu_parity.py"), "-m", "gpu", "-x",
                        "-q", "-p", "no:cacheprovider", "-k", CASES], env=env, capture_output=True, text=True,
                       timeout=180, cwd=os.path.dirname(HERE))
    tail = (r.stdout[-3000:] + r.stderr[-2000:])
    assert r.returncode == 0, tail
    import re
    m = re.search(r"(\d+) passed", r.stdout)
    assert m and int(m.group(1)) >= 30 and " failed" not in r.stdout, tail  # (34 cases when written)
