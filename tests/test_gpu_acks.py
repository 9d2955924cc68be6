"""GPU parity of the completion-ack path (owgs_acks.hip through the C ABI) against the oracle (owack_oracle.c).

Bar: bit-exact outcome codes, invoker instances, tickets, flags, activationSlots size and final slot state.
Parse vectors: tests/golden/ack_vectors.json (hand-derived from the reference, see make_ack_golden.py).
"""
import json
import os
import types

import numpy as np
import pytest

import oracle as O
from openwhisk_amd import GpuShardingContainerPoolBalancer
from openwhisk_amd import workload as W
from openwhisk_amd._lib import ACK_FORCED_NOENTRY, ACK_HEALTH, ACK_NOENTRY, ACK_RELEASED
from openwhisk_amd.balancer import Action

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = 1700000000123


def _vectors():
    with open(os.path.join(ROOT, "tests", "golden", "ack_vectors.json"), encoding="utf-8") as f:
        return json.load(f)


def expected_unresolved(kind, he):
    """Outcome of a parsed message when activationSlots is empty (CLB:320-337)."""
    out = kind.astype(np.int64).copy()
    comp = kind == O.ACK_COMPLETION
    out[comp] = np.where(he[comp] == 1, ACK_HEALTH, ACK_NOENTRY)
    return out


def check_parse(b, msgs):
    kind, inst, sy, he, _ = O.parse_acks(msgs, H)
    gk, gi, gt, gf = b.process_acks(msgs)
    exp = expected_unresolved(kind, he)
    bad = np.nonzero(gk != exp)[0]
    assert len(bad) == 0, [(msgs[i], int(gk[i]), int(exp[i])) for i in bad[:3]]
    comp = kind == O.ACK_COMPLETION
    assert np.array_equal(gi[comp], inst[comp])
    assert np.array_equal(gf & 1, np.where(comp, sy, 0).astype(np.uint8))
    assert np.all(gt == -1)


def test_parse_known_answer_vectors():
    g = _vectors()
    b = GpuShardingContainerPoolBalancer()
    b.set_health_tid(g["health_start_ms"])
    msgs = [v["msg"].encode("utf-8") for v in g["vectors"]]
    gk, gi, _, gf = b.process_acks(msgs)
    for i, v in enumerate(g["vectors"]):
        if v["kind"] == O.ACK_COMPLETION:
            assert gk[i] == (ACK_HEALTH if v["health"] else ACK_NOENTRY), v["name"]
            assert (gi[i], gf[i] & 1) == (v["instance"], v["syserr"]), v["name"]
        else:
            assert gk[i] == v["kind"], v["name"]


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_parse_fuzz_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    base = [v["msg"].encode("utf-8") for v in _vectors()["vectors"]]
    aids = W.activation_ids(rng, 200)
    base += [W.completion_message(a, int(rng.integers(0, 100)), bool(rng.random() < .5)) for a in aids]
    msgs = [W.mutate(rng, base[int(rng.integers(0, len(base)))], int(rng.integers(1, 4))) for _ in range(20000)]
    b = GpuShardingContainerPoolBalancer()
    b.set_health_tid(H)
    check_parse(b, msgs)


def _publish_first_batch(w, zombies=False):
    """GPU and oracle states after the first batch of w's stream (no releases)."""
    n = int(w.stream.acq_off[1])
    s1 = types.SimpleNamespace(acq_off=np.array([0, n]), act=w.stream.act[:n], rel_off=np.array([0, 0]),
                               rel_aid=np.zeros(0, np.int64), seq_base=w.stream.seq_base)
    st = O.state_for(w, zombies=zombies)
    o_inv, _, _ = st.replay(s1)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    g_inv, _, _ = b.replay(s1)
    assert np.array_equal(o_inv, g_inv)
    return b, st, g_inv, w.stream.act[:n]


@pytest.mark.parametrize("name,n,n_inv", [("c4", 60_000, None), ("headline", 120_000, None), ("headline", 300_000, 25_000)])
def test_completion_flow_matches_oracle(name, n, n_inv):
    """track (setupActivation) -> raw acks (processAcknowledgement) -> forced timeouts (processCompletion).  The
    25,000-invoker case is beyond the on-chip image (owgs_limits): its releases go through the large-state engine
    (owgs_seq.hip), which keeps the reference's empty entries literally (the oracle with zombies=True)."""
    w = W.config(name, n_activations=n, **({"n_invokers": n_inv} if n_inv else {}))
    if n_inv:
        import ctypes as C
        from openwhisk_amd import _lib
        mx, ms = C.c_int32(), C.c_int32()
        _lib.lib().owgs_limits(C.byref(mx), C.byref(ms))
        assert len(w.inv_ids) > mx.value
    b, st, inv, act = _publish_first_batch(w, zombies=bool(n_inv))
    b.set_health_tid(H)
    rng = np.random.default_rng(7)
    sched = np.nonzero(inv >= 0)[0]  # publish only tracks scheduled activations (SCPB:290-305)
    aids = W.activation_ids(rng, len(sched))
    flow = O.AckFlow(st, H)
    gt, gx = b.track_activations(aids, act[sched], sched)
    for j, i in enumerate(sched):
        t, x = flow.track(aids[j], int(act[i]), int(i))
        assert (gt[j], gx[j]) == (t, x)
    assert b.activations_live() == flow.live() == len(sched)
    # acks for 80 % of the activations, in random order, with duplicates / unknown / health / garbage mixed in
    part = rng.permutation(len(sched))[: int(0.8 * len(sched))]
    msgs = W.ack_batch(rng, [aids[j] for j in part], inv[sched[part]], H)
    ok, oi, ot, of = flow.process_acks(msgs)
    gk, gi, gtk, gf = b.process_acks(msgs)
    bad = np.nonzero(ok != gk)[0]
    assert len(bad) == 0, [(msgs[i], int(gk[i]), int(ok[i])) for i in bad[:3]]
    assert np.array_equal(ot, gtk)
    assert np.array_equal(of, gf)
    assert (gk == ACK_RELEASED).sum() > 0.7 * len(part)
    assert b.activations_live() == flow.live()
    assert np.array_equal(b.permits(), st.permits())
    # completion-ack timeouts for everything still tracked, plus a few already completed (forced after regular)
    rest = np.setdiff1d(np.arange(len(sched)), part)
    again = part[:50]
    ids = np.concatenate([rest, again])
    kk, tt, ff = b.complete_activations([aids[j] for j in ids], inv[sched[ids]], forced=np.ones(len(ids), np.uint8))
    for q, j in enumerate(ids):
        hi, lo = O.aid_words(aids[j])
        o, t, _, rf = flow.complete(hi, lo, int(inv[sched[j]]), True, False)
        assert (kk[q], tt[q], ff[q] >> 1) == (o, t, O._rel_bits(rf))
    assert set(kk[len(rest):].tolist()) <= {ACK_FORCED_NOENTRY, ACK_RELEASED}
    assert b.activations_live() == flow.live()
    assert np.array_equal(b.permits(), st.permits())
    # the state stays coherent: the next publish batch schedules identically
    a0 = int(w.stream.acq_off[1])
    m = min(int(w.stream.acq_off[2]) - a0, 20000)
    nxt = w.stream.act[a0: a0 + m]
    g2, _ = b.publish(nxt, seq_base=10**9)
    o2 = [st.publish(int(a), 10**9 + k)[0] for k, a in enumerate(nxt)]
    assert g2.tolist() == o2


def test_track_duplicates_in_one_batch_keep_the_first():
    b = GpuShardingContainerPoolBalancer()
    (a,), _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256)])
    aid = ["%032x" % 0xabc] * 5 + ["%032x" % 0xdef]
    t, x = b.track_activations(aid, [a] * 6, [10, 11, 12, 13, 14, 15])
    assert t.tolist() == [10, 10, 10, 10, 10, 15] and x.tolist() == [0, 1, 1, 1, 1, 0]
    t, x = b.track_activations(aid[:1], [a], [99])
    assert (t[0], x[0]) == (10, 1)
    assert b.activations_live() == 2
    with pytest.raises(Exception):
        b.track_activations(["XYZ" * 10 + "ab"], [a], [0])
    assert b.activations_live() == 2  # a malformed batch creates no entry


def test_table_grows_and_rehashes():
    b = GpuShardingContainerPoolBalancer()
    (a,), _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256)])
    rng = np.random.default_rng(3)
    aids = W.activation_ids(rng, 150_000)
    for k in range(0, len(aids), 50_000):
        t, x = b.track_activations(aids[k:k + 50_000], np.full(50_000, a), np.arange(k, k + 50_000))
        assert np.all(x == 0) and np.array_equal(t, np.arange(k, k + 50_000))
    kk, tt, _ = b.complete_activations(aids[::3], np.full(50_000, 99999))
    assert np.all(kk == ACK_RELEASED) and np.array_equal(tt, np.arange(0, 150_000, 3))
    assert b.activations_live() == 100_000
    t, x = b.track_activations(aids[1:20:3], np.full(7, a), np.full(7, -5))
    assert np.all(x == 1) and t.tolist() == list(range(1, 20, 3))
