"""Invoker health supervision (InvokerSupervision.scala): the CPU oracle against the
hand-derived golden vectors of tests/golden/health_vectors.json (T-ISUP cases + akka timer rules)."""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "health_vectors.json")
CASES = json.load(open(GOLD))


def run_case(pool, case):
    """Feed every batch of a golden case to `pool` (oracle or GPU mirror); assert per-batch status and test actions."""
    for k, bt in enumerate(case["batches"]):
        ev = np.array(bt["events"], dtype=np.int64).reshape(-1, 4)
        pool.events(ev[:, 1], ev[:, 0], ev[:, 2], ev[:, 3], bt["now"])
        st, mem, te, ring, tick = pool.read()
        assert st.tolist() == bt["status"], f"{case['name']} batch {k}: status"
        assert te.tolist() == bt["tests"], f"{case['name']} batch {k}: test actions"
    f = case["final"]
    if "mem" in f:
        assert mem.tolist() == f["mem"]
    if "tick" in f:
        assert tick.tolist() == f["tick"]
    if "ring" in f:
        assert ring.tolist() == f["ring"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_health_golden(case):
    run_case(O.HealthPool(), case)


def test_oracle_health_rejects_bad_batches():
    p = O.HealthPool(start_ms=100)
    with pytest.raises(ValueError):
        p.events([0], [0], [99], [1], 100)          # before the clock
    with pytest.raises(ValueError):
        p.events([0, 0], [0, 0], [200, 150], [1, 1], 300)  # decreasing
    with pytest.raises(ValueError):
        p.events([0], [5], [200], [1], 300)          # unknown kind
    with pytest.raises(ValueError):
        p.events([0], [0], [200], [1], 150)          # now before the last event
    assert p.read()[0].size == 0
