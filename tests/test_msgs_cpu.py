"""ActivationMessage serialisation + topic fan-out: the CPU oracle against the hand-written
golden messages (tests/golden/msg_vectors.json)."""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "msg_vectors.json")))


def words(hexid):
    return [int(hexid[:16], 16), int(hexid[16:], 16)]


def batch_of(case):
    acts = case["acts"]
    flags = [(a["blocking"] and O.MSG_BLOCKING) | (a["extra"] and O.MSG_EXTRA_LOGGING)
             | (a["content"] is not None and O.MSG_HAS_CONTENT) | (a["cause"] is not None and O.MSG_HAS_CAUSE)
             | (a["trace"] is not None and O.MSG_HAS_TRACE) for a in acts]
    return dict(invoker=[a["invoker"] for a in acts], tmpl=[a["tmpl"] for a in acts],
                aid_words=[words(a["aid"]) for a in acts], tids=[a["tid"] for a in acts],
                tid_start=[a["start"] for a in acts], flags=flags,
                contents=[a["content"] or "" for a in acts], causes=[words(a["cause"] or "0" * 32) for a in acts],
                traces=[a["trace"] or "" for a in acts], n_topics=case["n_topics"])


def check(case, out, off, order, topic):
    msgs = [out[off[j]:off[j + 1]].decode("utf-8") for j in range(len(off) - 1)]
    got = [msgs[topic[k]:topic[k + 1]] for k in range(case["n_topics"])]
    assert got == case["topics"], case["name"]
    for m in msgs:
        json.loads(m)  # every message is valid JSON


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_oracle_msg_golden(case):
    T = GOLD["templates"]
    out, off, order, topic = O.serialize_activations(T["a"], T["b"], GOLD["rci"], **batch_of(case))
    check(case, out, off, order, topic)


def test_oracle_msg_rejects_bad_input():
    T = GOLD["templates"]
    b = batch_of(GOLD["cases"][0])
    with pytest.raises(ValueError):
        O.serialize_activations(T["a"], T["b"], GOLD["rci"], **{**b, "tmpl": [7]})
    with pytest.raises(ValueError):
        O.serialize_activations(T["a"], T["b"], GOLD["rci"], **{**b, "tids": [b"\xc3("]})  # malformed UTF-8
