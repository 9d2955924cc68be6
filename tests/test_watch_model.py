"""The watched-pair rules (tests/watch_model.py, implemented by the engine's owgs_w_* kernels) against the literal
oracle, which creates the reference's empty NestedSemaphore entries on every failed concurrent try
(NestedSemaphore.scala:61-62), on shim-like job sequences with repeated cluster changes (SCPB:561-584) while
concurrent activations are in flight.  CPU only: this pins the rules themselves; tests/test_gpu_shim_sequence.py and
tests/test_gpu_watch.py pin the device path to the same oracle."""
import numpy as np
import pytest

import oracle as O
from watch_model import WatchModel

MB = 1024 * 1024


def _setup(rng, n_inv, n_act, conc_frac, mem_mb):
    ids = np.arange(n_inv, dtype=np.int32)
    mem = np.full(n_inv, mem_mb * MB, np.int64)
    st = np.zeros(n_inv, np.uint8)
    st[rng.choice(n_inv, size=max(1, n_inv // 8), replace=False)] = 1
    o = O.BalancerState(0.75, 0.25, rng_seed=7, zombies=True)
    o.update_invokers(ids, mem, st)
    m = WatchModel(ids, mem, st, 0.75, 0.25, 7)
    acts = []
    n_keys = max(2, n_act // 2)
    lim = {}  # one set of limits per fqn@version
    for a in range(n_act):
        k = int(rng.integers(0, n_keys))  # shared fqn@version keys across invoking namespaces
        if k not in lim:
            lim[k] = (int(rng.integers(2, 5)) if rng.random() < conc_frac else 1, [128, 256, 512][k % 3], k % 7 == 0)
        maxc, amem, bb = lim[k]
        ns, path = f"ns{a}", f"ns{k}/pkg/act{k}"
        oh = o.register_action(ns, path, k, amem, maxc, bb)
        mh = m.register(o.action_hash(oh), k, amem, maxc, bb)
        acts.append((oh, mh))
    return o, m, acts


_STATS = {"resurrected": 0, "nosuch_watched": 0, "z_set": 0}


@pytest.mark.parametrize("seed", range(24))
def test_watch_rules_match_literal_oracle(seed):
    rng = np.random.default_rng(1000 + seed)
    n_inv = int(rng.integers(6, 20))
    o, m, acts = _setup(rng, n_inv, n_act=int(rng.integers(4, 14)), conc_frac=0.6, mem_mb=1024)
    live = []  # (invoker, action) of in-flight activations
    seq = 0
    sizes = [1, 2, 3]
    for step in range(200):
        r = rng.random()
        if r < 0.08:
            s = int(rng.choice(sizes))
            o.update_cluster(s)
            m.update_cluster(s)
            continue
        if r < 0.12:
            st = (rng.random(n_inv) < 0.15).astype(np.uint8)
            o.update_invokers(np.arange(n_inv, dtype=np.int32), np.full(n_inv, 1024 * MB, np.int64), st)
            m.set_status(st)
            continue
        if r < 0.55 and live:  # a release run, random completion order
            k = int(rng.integers(1, min(len(live), 12) + 1))
            idx = rng.choice(len(live), size=k, replace=False)
            run = [live[i] for i in idx]
            live = [x for i, x in enumerate(live) if i not in set(idx.tolist())]
            for inv, (oh, mh) in run:
                fo = O._rel_bits(o.release(inv, oh))
                fm = m.release(inv, mh)
                assert fo == fm, (step, inv)
            continue
        k = int(rng.integers(1, 16))  # a publish run
        for _ in range(k):
            oh, mh = acts[int(rng.integers(0, len(acts)))]
            io, fo = o.publish(oh, seq)
            im, fm = m.publish(mh, seq)
            seq += 1
            assert (io, fo) == (im, fm), (step, seq)
            if io >= 0:
                live.append((io, (oh, mh)))
        m.end_publish_run()
        assert np.array_equal(o.permits(), np.array(m.P, np.int32))
    for k, v in m.stats.items():
        _STATS[k] += v


def test_watch_rules_were_exercised():
    """the sequences above reach every rule: empty entries taking releases, NoSuchElement on watched pairs"""
    assert _STATS["resurrected"] > 0 and _STATS["nosuch_watched"] > 0 and _STATS["z_set"] > 0, _STATS
