"""Invoker health supervision on the GPU (owgs_health.hip) against the CPU oracle
(oracle/owhealth_oracle.c) and the hand-derived golden vectors (tests/golden/health_vectors.json)."""
import numpy as np
import pytest

import oracle as O
from openwhisk_amd import GpuShardingContainerPoolBalancer, OwgsError
from openwhisk_amd.balancer import Action
from test_health_cpu import CASES, run_case

pytestmark = pytest.mark.gpu

MB = 1 << 20


class GpuPool:
    def __init__(self, b=None):
        self.b = b or GpuShardingContainerPoolBalancer()

    def events(self, inv, kind, t, mem, now, apply=False):
        self.b.health_events(inv, kind, t, mem, now, apply=apply)

    def read(self):
        return self.b.health_read()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_health_golden(case):
    run_case(GpuPool(), case)


def random_batches(rng, n_ids, n_batches, per_batch, t0=0, span=30000):
    """Seeded supervision traffic: pings from a growing id range, completions of every result (errors and timeouts
    in bursts so that invokers cross the tolerance), explicit state timeouts, gaps long enough for timeouts and
    Ticks to fire."""
    t = t0
    out = []
    for b in range(n_batches):
        hi = max(1, int(n_ids * (b + 1) / n_batches))
        n = per_batch
        kind = rng.choice(5, size=n, p=[0.35, 0.35, 0.13, 0.13, 0.04]).astype(np.uint8)
        inv = rng.integers(0, hi + hi // 10 + 1, size=n).astype(np.int32)  # some ids never ping
        dt = rng.exponential(span / n, size=n)
        dt[rng.random(n) < 0.002] += 70000   # occasional silence: state timeouts and Ticks
        ts = t + np.cumsum(dt).astype(np.int64)
        mem = (rng.integers(1, 64, size=n) * 256 * MB).astype(np.int64)
        now = int(ts[-1]) + int(rng.integers(0, 20000))
        out.append((inv, kind, ts, mem, now))
        t = now
    return out


def compare(g, o):
    for name, a, b in zip(("status", "mem", "tests", "ring", "tick"), g, o):
        assert np.array_equal(a, b), f"{name} differs at {np.flatnonzero(a != b)[:8]}"


@pytest.mark.parametrize("seed,n_ids,n_batches,per_batch", [(1, 50, 12, 400), (2, 3000, 8, 20000),
                                                            (3, 10000, 4, 250000)])
def test_gpu_health_random_streams(seed, n_ids, n_batches, per_batch):
    rng = np.random.default_rng(seed)
    g, o = GpuPool(), O.HealthPool()
    seen = set()
    for inv, kind, ts, mem, now in random_batches(rng, n_ids, n_batches, per_batch):
        g.events(inv, kind, ts, mem, now)
        o.events(inv, kind, ts, mem, now)
        compare(g.read(), o.read())
        seen |= set(o.read()[0].tolist())
    assert len(seen) >= 3  # the stream exercises several states


def test_gpu_health_timers_only_batches():
    """Batches without events still fire every due timer of every actor (Healthy -> Offline, Ticks)."""
    rng = np.random.default_rng(7)
    g, o = GpuPool(), O.HealthPool()
    inv = np.arange(2000, dtype=np.int32)
    ts = np.sort(rng.integers(0, 5000, size=2000)).astype(np.int64)
    z = np.zeros(2000, np.uint8)
    m = np.full(2000, 1024 * MB, np.int64)
    for p in (g, o):
        p.events(inv, z, ts, m, 5000)
        p.events(inv[::2], np.ones(1000, np.uint8), ts[::2] + 5000, m[::2], 11000)  # half become Healthy
    compare(g.read(), o.read())
    for now in (12000, 14999, 15000, 60000, 130000, 250000):
        g.events([], [], [], [], now)
        o.events([], [], [], [], now)
        compare(g.read(), o.read())


def test_gpu_health_rejects_bad_batches_without_state_change():
    g = GpuPool()
    g.events([3], [0], [100], [MB], 100)
    before = g.read()
    for args in (([0], [0], [99], [MB], 200), ([0, 1], [0, 0], [300, 200], [MB, MB], 400), ([0], [9], [200], [MB], 300),
                 ([-1], [0], [200], [MB], 300), ([0], [0], [200], [MB], 150), ([1 << 24], [0], [200], [MB], 300)):
        with pytest.raises(OwgsError):
            g.events(*args)
        compare(g.read(), before)


def test_gpu_health_apply_feeds_the_scheduler():
    """apply=True: the status vector becomes updateInvokers' input (SCPB:226-227); scheduling then walks only the
    Healthy invokers, bit-exact with the oracle balancer built from the oracle's health vector."""
    rng = np.random.default_rng(11)
    b = GpuShardingContainerPoolBalancer(managed_fraction=0.9, blackbox_fraction=0.1, rng_seed=5)
    g, o = GpuPool(b), O.HealthPool()
    n = 400
    inv = np.arange(n, dtype=np.int32)
    mem = (rng.integers(4, 32, size=n) * 512 * MB).astype(np.int64)
    z = np.zeros(n, np.uint8)
    bad = rng.random(n) < 0.3
    res = np.where(bad, 2, 1).astype(np.uint8)  # 30 % report system errors
    evs = [(inv, z, np.full(n, 10, np.int64), mem, 10),
           (np.repeat(inv, 5), np.repeat(res, 5), np.full(5 * n, 20, np.int64), np.repeat(mem, 5), 20),
           (inv[:50], z[:50], np.full(50, 30, np.int64), mem[:50], 30)]
    for a in evs:
        g.events(*a, apply=True)
        o.events(*a)
    st_o, mem_o = o.read()[:2]
    compare(g.read(), o.read())
    assert (st_o == 0).sum() > 100 and (st_o == 1).sum() > 50
    st = O.BalancerState(managed_fraction=0.9, blackbox_fraction=0.1, rng_seed=5, zombies=False)
    st.update_invokers(np.arange(n, dtype=np.int32), mem_o, st_o)
    assert b.managed_size == st.managed_size and b.blackbox_size == st.blackbox_size
    acts = [Action(f"ns{k}", f"ns{k}/a{k}", "0.0.1", int(rng.choice([128, 256, 512, 1024])), 1, k % 10 == 0)
            for k in range(200)]
    b.register_actions(acts)
    for k, a in enumerate(acts):
        st.register_action(a.namespace, a.path, k, a.mem_mb, a.max_concurrent, a.blackbox)
    seq = rng.integers(0, len(acts), size=5000).astype(np.int32)
    gi, gf = b.publish(seq, seq_base=0)
    oi = [st.publish(int(a), k)[0] for k, a in enumerate(seq)]
    assert gi.tolist() == oi
    assert np.all(st_o[gi[gi >= 0]] == 0)  # only Healthy invokers are chosen
    assert np.array_equal(b.permits(), st.permits())
