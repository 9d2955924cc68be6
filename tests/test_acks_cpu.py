"""Completion-ack oracle (oracle/owack_oracle.c) against the hand-derived known-answer vectors, and the oracle's
processCompletion flow on CPU.  Vectors: tests/golden/ack_vectors.json (tests/golden/make_ack_golden.py)."""
import json
import os

import numpy as np

import oracle as O
from openwhisk_amd import workload as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def vectors():
    with open(os.path.join(ROOT, "tests", "golden", "ack_vectors.json"), encoding="utf-8") as f:
        return json.load(f)


def test_oracle_parse_matches_known_answers():
    g = vectors()
    msgs = [v["msg"].encode("utf-8") for v in g["vectors"]]
    kind, inst, sy, he, aid = O.parse_acks(msgs, g["health_start_ms"])
    for i, v in enumerate(g["vectors"]):
        assert kind[i] == v["kind"], v["name"]
        if v["kind"] == O.ACK_COMPLETION:
            assert (inst[i], sy[i], he[i]) == (v["instance"], v["syserr"], v["health"]), v["name"]
            assert "%016x%016x" % (aid[i, 0], aid[i, 1]) == v["aid"], v["name"]


def test_workload_messages_are_canonical_completions():
    rng = np.random.default_rng(5)
    aids = W.activation_ids(rng, 50)
    msgs = [W.completion_message(a, i, i % 3 == 0) for i, a in enumerate(aids)]
    kind, inst, sy, he, aid = O.parse_acks(msgs, 1)
    assert np.all(kind == O.ACK_COMPLETION)
    assert inst.tolist() == list(range(50))
    assert sy.tolist() == [int(i % 3 == 0) for i in range(50)]
    assert ["%016x%016x" % tuple(x) for x in aid] == aids
    assert O.parse_acks([W.combined_message(aids[0], 3)], 1)[0][0] == O.ACK_JVM


def test_oracle_completion_flow_releases_slots():
    """CLB:286-345 on the oracle: released once, then no entry; health acks; out-of-range invoker is a no-op."""
    st = O.BalancerState(managed_fraction=1.0, blackbox_fraction=0.0)
    st.update_invokers(np.arange(3), np.full(3, 1024 * 2**20), np.zeros(3, np.uint8))
    a = st.register_action("ns", "ns/a", 0, 256)
    inv, _ = st.publish(a, 0)
    flow = O.AckFlow(st, health_start_ms=77, cap=1 << 8)
    aid = "00000000000000000000000000000abc"
    assert flow.track(aid, a, 5) == (5, 0)
    assert flow.track(aid, a, 6) == (5, 1)  # getOrElseUpdate keeps the first entry
    before = st.permits().copy()
    msgs = [W.completion_message(aid, inv), W.completion_message(aid, inv),
            W.completion_message(aid, inv, tid=("sid_invokerHealth", 77))]
    k, i2, t, f = flow.process_acks(msgs)
    assert k.tolist() == [O.OUT_RELEASED, O.OUT_NOENTRY, O.OUT_HEALTH]
    assert t.tolist() == [5, -1, -1]
    assert st.permits()[inv] == before[inv] + 256
    assert flow.live() == 0
