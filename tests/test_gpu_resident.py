"""owgs_process_batch through the resident engine (openwhisk_amd/csrc/owgs_resident.hip): the shim's small drained
batches served by one workgroup that keeps the slot state on chip between calls, against the literal oracle driven
one reference call at a time (releaseInvoker SCPB:327-331 via processCompletion CLB:260-346, then publish SCPB:257-290
-> schedule SCPB:398-436 with NestedSemaphore tryAcquireConcurrent / forceAcquireConcurrent NS:32-91).

Every comparison is per call (decisions, overload flags, release flags) and on the final permits; the resident
counters (owgs_resident_stats) show which path served the calls, so a silent fallback to the launch chain fails the
test."""
import time

import numpy as np
import pytest

import oracle as O
from openwhisk_amd import Action, GpuShardingContainerPoolBalancer
from openwhisk_amd import workload as W
from openwhisk_amd.balancer import UNHEALTHY

pytestmark = pytest.mark.gpu
MB = 1024 * 1024


class Shim:
    """The shim's batching thread over one workload: jobs in arrival order (a batch's completions, then its
    publishes), drained `drain` jobs at a time into runs; releases name the invoker of the activation's decision."""

    def __init__(self, w, zombies=True, shadow=False):
        self.w = w
        self.g = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction,
                                                  blackbox_fraction=w.blackbox_fraction, rng_seed=w.rng_seed)
        self.o = O.BalancerState(w.managed_fraction, w.blackbox_fraction, rng_seed=w.rng_seed, zombies=zombies)
        # shadow: the oracle WITHOUT the reference's empty entries, driven alike (its release flags show whether a
        # stream reaches the releases that only those entries explain)
        self.z = O.BalancerState(w.managed_fraction, w.blackbox_fraction, rng_seed=w.rng_seed, zombies=False) \
            if shadow else None
        self.z_rf, self.o_rf = [], []
        for b in (self.g, self.o) + ((self.z,) if self.z else ()):
            (b.update_invokers_arrays if b is self.g else b.update_invokers)(w.inv_ids, w.inv_mem, w.inv_status)
            if w.cluster_size != 1:
                b.update_cluster(w.cluster_size)
        self.gh, _ = self.g.register_actions(w.actions)
        keys = {}
        self.oh = [self.o.register_action(a.namespace, a.path, keys.setdefault(a.key, len(keys)), a.mem_mb,
                                          a.max_concurrent, a.blackbox) for a in w.actions]
        if self.z:
            for a in w.actions:
                self.z.register_action(a.namespace, a.path, keys[a.key], a.mem_mb, a.max_concurrent, a.blackbox)
        s = w.stream
        self.jobs = []
        for b in range(s.n_batches):
            self.jobs += [(0, int(a)) for a in s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]]]
            self.jobs += [(1, i) for i in range(int(s.acq_off[b]), int(s.acq_off[b + 1]))]
        self.pos = 0
        self.seq = 0
        self.dec = np.full(len(s.act), -9, np.int32)
        self.calls = 0

    def done(self):
        return self.pos >= len(self.jobs)

    def call(self, drain):
        """one drained batch through owgs_process_batch, checked against the oracle (which replays the same jobs one
        reference call at a time, so a release may name an activation published earlier in the same drain)"""
        batch = self.jobs[self.pos:self.pos + drain]
        self.pos += len(batch)
        act = self.w.stream.act
        ro, po, ri, ra, pa, pubs, orf, oi = [0], [0], [], [], [], [], [], []
        i = 0
        while i < len(batch):
            while i < len(batch) and batch[i][0] == 0:
                a = batch[i][1]
                i += 1
                if self.dec[a] < 0:  # a failed publish holds no ActivationEntry (CLB:278-279)
                    continue
                ri.append(int(self.dec[a]))
                ra.append(int(self.gh[act[a]]))
                orf.append(O._rel_bits(self.o.release(int(self.dec[a]), self.oh[act[a]])))
                if self.z:
                    self.z_rf.append(O._rel_bits(self.z.release(int(self.dec[a]), self.oh[act[a]])))
                    self.o_rf.append(orf[-1])
            while i < len(batch) and batch[i][0] == 1:
                a = batch[i][1]
                i += 1
                pubs.append(a)
                pa.append(int(self.gh[act[a]]))
                x, f = self.o.publish(self.oh[act[a]], self.seq + len(oi))
                if self.z:
                    self.z.publish(self.oh[act[a]], self.seq + len(oi))
                oi.append((int(x), int(f)))
                self.dec[a] = x
            ro.append(len(ri))
            po.append(len(pa))
        gi, gf, grf = self.g.process_batch(ro, ri, ra, po, pa, seq_base=self.seq)
        self.seq += len(pubs)
        assert grf.tolist() == orf, self.calls
        assert [(int(x), int(f)) for x, f in zip(gi, gf)] == oi, self.calls
        self.calls += 1
        return len(pubs), len(ri)


@pytest.mark.parametrize("cfg,kw", [
    ("headline", dict(n_activations=30_000, n_invokers=1000, n_actions=2000, n_namespaces=200)),
    ("c4", dict(n_activations=30_000)),
    ("c2", dict(n_activations=30_000)),
    ("c3", dict(n_activations=30_000)),
])
def test_resident_small_drains_match_oracle(cfg, kw):
    """Drains of 1..600 jobs (the shim's steady state): every call is served by the resident engine, without a
    relaunch, bit-exact with the oracle; concurrent actions, shared fqn@version keys, unhealthy invokers and overload
    fallbacks included (configs[1..3] and a reduced headline)."""
    w = W.config(cfg, **kw)
    sh = Shim(w)
    rng = np.random.default_rng(7)
    pubs = 0
    while not sh.done():
        n, _ = sh.call(int(rng.integers(1, 601)))
        pubs += n
    st = sh.g.resident_stats()
    assert st["served"] == sh.calls and st["chained"] == 0 and st["refused"] == 0, st
    assert st["launches"] - st["life_exits"] == 1, st  # (relaunches only at the lifetime bound, OWGS_RES_LIFE_US)
    if cfg in ("headline", "c4"):  # (configs with concurrent actions) the helper wave speculated some chunks ahead
        assert st["prespec_chunks"] > 0, st
    assert np.array_equal(sh.g.permits(), sh.o.permits())
    assert sh.g.resident_stats()["alive"] == 0  # permits() stopped it (the state was written back)
    assert pubs == int(w.stream.acq_off[-1])


@pytest.mark.parametrize("cfg,kw", [
    ("headline", dict(n_activations=40_000, n_invokers=1000, n_actions=2000, n_namespaces=200)),
    ("c4", dict(n_activations=40_000)),
])
def test_resident_calls_beyond_the_first_read(cfg, kw):
    """Drains of 900..1024 jobs (up to OWGS_RES_MAX): the call block (4 B per publish, 8 B per release) outgrows the
    engine's first 4 KB read of pinned memory, so the rest of the block is read and the records gathered after it;
    bit-exact with the oracle, every call on the resident engine."""
    w = W.config(cfg, **kw)
    sh = Shim(w)
    rng = np.random.default_rng(11)
    big = 0
    while not sh.done():
        n, r = sh.call(int(rng.integers(900, 1025)))
        big += (4 * n + 8 * r) > 4096
    st = sh.g.resident_stats()
    assert big >= 5, big
    assert st["served"] == sh.calls and st["chained"] == 0 and st["refused"] == 0, st
    assert np.array_equal(sh.g.permits(), sh.o.permits())


def test_resident_interleaved_with_the_chain_and_state_updates():
    """Small drains on the resident engine, large ones (beyond OWGS_RES_MAX) on the launch chain, a health change
    (owgs_update_invokers) and a snapshot read in between: each non-resident entry point stops the engine, which writes
    the state back; the next small call launches it again from that state."""
    w = W.config("headline", n_activations=40_000, n_invokers=800, n_actions=1500, n_namespaces=150)
    sh = Shim(w)
    rng = np.random.default_rng(3)
    k = 0
    while not sh.done():
        k += 1
        if k % 7 == 0:
            sh.call(3000)  # chained
        elif k % 11 == 0:
            st = w.inv_status.copy()
            st[rng.choice(len(st), size=len(st) // 25, replace=False)] = UNHEALTHY
            sh.g.update_invokers_arrays(w.inv_ids, w.inv_mem, st)
            sh.o.update_invokers(w.inv_ids, w.inv_mem, st)
        elif k % 13 == 0:
            assert np.array_equal(sh.g.permits(), sh.o.permits())
        else:
            sh.call(int(rng.integers(1, 400)))
    st = sh.g.resident_stats()
    assert st["chained"] >= 3 and st["served"] >= 20 and st["launches"] >= 5, st
    assert np.array_equal(sh.g.permits(), sh.o.permits())


def test_resident_engine_exits_when_idle_and_relaunches():
    """After 20 ms without a call (OWGS_RES_IDLE_US) the engine writes the state back and exits by itself; the next
    call launches it again and continues from that state."""
    w = W.config("c4", n_activations=6_000)
    sh = Shim(w)
    for _ in range(5):
        sh.call(200)
        time.sleep(0.1)
    st = sh.g.resident_stats()
    assert st["served"] == 5 and st["launches"] - st["life_exits"] == 5, st
    while not sh.done():
        sh.call(300)
    assert np.array_equal(sh.g.permits(), sh.o.permits())


def test_resident_map_beyond_the_primary_table():
    """More live (invoker, fqn) entries than the on-chip primary holds (3,840): new keys go to the HBM overflow, and
    the cleanup between calls keeps the primary's chains short; every call still resident and exact."""
    rng = np.random.default_rng(5)
    n_inv, n_act = 64, 6000
    g = GpuShardingContainerPoolBalancer(managed_fraction=1.0, blackbox_fraction=0.0, rng_seed=9)
    o = O.BalancerState(1.0, 0.0, rng_seed=9, zombies=True)
    ids, mem = np.arange(n_inv, dtype=np.int32), np.full(n_inv, 1 << 40, np.int64)
    g.update_invokers_arrays(ids, mem, np.zeros(n_inv, np.uint8))
    o.update_invokers(ids, mem, np.zeros(n_inv, np.uint8))
    acts = [Action(f"ns{a % 7}", f"ns{a % 7}/p/a{a}", "0.0.1", 128, 2) for a in range(n_act)]
    gh, _ = g.register_actions(acts)
    oh = [o.register_action(a.namespace, a.path, k, a.mem_mb, a.max_concurrent) for k, a in enumerate(acts)]
    live = []  # (invoker, action) of activations in flight
    seq = 0
    for call in range(60):
        nrel = min(len(live), int(rng.integers(0, 200)))
        pick = rng.choice(len(live), size=nrel, replace=False) if nrel else np.zeros(0, int)
        rel = [live[j] for j in sorted(pick)]
        live = [x for j, x in enumerate(live) if j not in set(pick.tolist())]
        pubs = rng.integers(0, n_act, size=int(rng.integers(100, 400)))
        orf = [O._rel_bits(o.release(x, oh[a])) for x, a in rel]
        oi = [o.publish(oh[a], seq + k) for k, a in enumerate(pubs)]
        gi, gf, grf = g.process_batch([0, len(rel)], [x for x, _ in rel], [gh[a] for _, a in rel], [0, len(pubs)],
                                      [gh[a] for a in pubs], seq_base=seq)
        seq += len(pubs)
        assert grf.tolist() == orf, call
        assert [(int(x), int(f)) for x, f in zip(gi, gf)] == oi, call
        live += [(int(x), int(a)) for x, a in zip(gi, pubs) if x >= 0]
    st = g.resident_stats()
    assert st["served"] == 60 and st["chained"] == 0, st
    assert np.array_equal(g.permits(), o.permits())


def test_resident_refuses_releases_beyond_the_permit_range():
    """A call whose releases could push a slot beyond the on-chip permit range (2^29 MB) is refused untouched and
    taken by the launch chain, whose release kernels apply ForcibleSemaphore's bound release by release (FS:48-50)."""
    lim = 2**29
    g = GpuShardingContainerPoolBalancer(managed_fraction=1.0, blackbox_fraction=0.0)
    o = O.BalancerState(1.0, 0.0, zombies=True)
    mem_b = (lim - 300) * MB
    g.update_invokers_arrays(np.array([0], np.int32), np.array([mem_b], np.int64), np.zeros(1, np.uint8))
    o.update_invokers(np.array([0], np.int32), np.array([mem_b], np.int64), np.zeros(1, np.uint8))
    acts = [Action("ns", "ns/c", "0.0.1", 256, 4), Action("ns", "ns/a", "0.0.1", 128, 1)]
    hs, _ = g.register_actions(acts)
    oh = [o.register_action(a.namespace, a.path, k, a.mem_mb, a.max_concurrent, a.blackbox) for k, a in enumerate(acts)]
    gi, gf, _ = g.process_batch([0, 0], [], [], [0, 3], [hs[0]] * 3)
    oi = [o.publish(oh[0], k) for k in range(3)]
    assert [(int(a), int(b)) for a, b in zip(gi, gf)] == oi
    assert g.resident_stats()["served"] == 1
    gi2, gf2, grf = g.process_batch([0, 3], [0, 0, 0], [hs[0]] * 3, [0, 2], [hs[0], hs[1]], seq_base=3)
    orf = [O._rel_bits(o.release(0, oh[0])) for _ in range(3)]
    oi2 = [o.publish(oh[p], 3 + k) for k, p in enumerate([0, 1])]
    assert grf.tolist() == orf
    assert [(int(a), int(b)) for a, b in zip(gi2, gf2)] == oi2
    st = g.resident_stats()
    assert st["refused"] == 1 and st["chained"] == 1, st
    assert g.permits().tolist() == o.permits().tolist()


def _hot_small_pool(seed=11, n_activations=20_000):
    """A few invokers near full, a handful of hot actions (Zipf 1.5), 40 % concurrent ones with small
    maxConcurrent: repeats of one action in a chunk, clashes at one invoker and walks past the speculation's budget are
    the common case, not the exception."""
    return W.generate(name="hot", n_invokers=24, user_memory_mb=2048, n_actions=30, n_namespaces=5, zipf_s=1.5,
                      conc_frac=0.4, conc_range=(2, 4), blackbox_frac=0.2, unhealthy_frac=0.1, shared_frac=0.3,
                      n_activations=n_activations, load=1.05, delay_mean=3.0, seed=seed)


@pytest.mark.parametrize("seed", [11, 12])
def test_resident_speculation_on_hot_small_pools(seed):
    """The resident engine's speculative walks (every decision of a chunk walks against the state at the chunk's
    start; in stream order the prefix whose targets still hold commits at once, repeats of one action take the room
    the earlier ones leave, the first decision that does not hold is decided alone) on the hardest inputs for it:
    bit-exact with the oracle call by call."""
    w = _hot_small_pool(seed)
    sh = Shim(w)
    rng = np.random.default_rng(seed)
    while not sh.done():
        sh.call(int(rng.integers(1, 300)))
    st = sh.g.resident_stats()
    assert st["served"] == sh.calls and st["chained"] == 0, st
    assert st["grouped_decisions"] > 0, st  # decisions committed from speculation
    assert np.array_equal(sh.g.permits(), sh.o.permits())


_BUDGET_SCRIPT = r"""
import sys
sys.path[:0] = [{root!r}, {oracle!r}, {tests!r}]
import numpy as np
import test_gpu_resident as T
for seed in (11, 12):
    w = T._hot_small_pool(seed, n_activations=8_000)
    sh = T.Shim(w)
    rng = np.random.default_rng(seed)
    while not sh.done():
        sh.call(int(rng.integers(1, 200)))
    assert np.array_equal(sh.g.permits(), sh.o.permits())
print("ok")
"""


@pytest.mark.parametrize("budget,split,pre", [("0", "1", "1"), ("1", "1", "1"), ("4", "1", "1"), ("16", "0", "1"),
                                              ("16", "1", "0"), ("4", "1", "0")])
def test_resident_speculation_budgets(budget, split, pre):
    """Walk budgets of 0 (no speculation: decisions one at a time), 1 and 4 steps (most walks unfinished: decided
    alone from where the speculation stopped) give the same decisions, and so does the default budget with the
    concurrent speculation on wave 0 instead of the helper wave (OWGS_RES_SPLIT=0), and without the helper waves'
    speculation of a run's next chunk (OWGS_RES_PRE=0).  The switches are read once per process, so each case runs in
    a child process."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = _BUDGET_SCRIPT.format(root=root, oracle=os.path.join(root, "oracle"), tests=here)
    env = dict(os.environ, OWGS_RES_SPEC=budget, OWGS_RES_SPLIT=split, OWGS_RES_PRE=pre)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_WRAP_SCRIPT = r"""
import sys
sys.path[:0] = [{root!r}, {oracle!r}, {tests!r}]
import numpy as np
import test_gpu_resident as T
from openwhisk_amd import workload as W
w = W.config("c4", n_activations=60_000)
sh = T.Shim(w)
rng = np.random.default_rng(4)
while not sh.done():
    sh.call(int(rng.integers(20, 120)))
st = sh.g.resident_stats()
assert st["served"] == sh.calls and st["chained"] == 0 and st["refused"] == 0, st
assert st["launches"] - st["life_exits"] >= 3, st
assert np.array_equal(sh.g.permits(), sh.o.permits())
print("ok", sh.calls, st["launches"], st["life_exits"])
"""


def test_resident_doorbell_and_cursor_generation_wrap():
    """The doorbell counts calls and the walk-cursor generation counts release runs, both for the life of a context
    (ADVICE r04): a context started just below both limits (OWGS_RES_CALL_BASE, OWGS_RES_GEN_BASE; read once per
    process, so a child process) crosses them -- the library stops the engine before either wraps and the relaunch
    starts both over (the stored cursors cleared) -- and every call stays resident and bit-exact."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = _WRAP_SCRIPT.format(root=root, oracle=os.path.join(root, "oracle"), tests=here)
    env = dict(os.environ, OWGS_RES_CALL_BASE=str(0x7FFFFF00 - 8 - 150), OWGS_RES_GEN_BASE=str(0xFFFFFF00 - 2 - 400),
               OWGS_RES_IDLE_US="2000000", OWGS_RES_LIFE_US="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_SPEC_THEN_CALLS_SCRIPT = r"""
import sys
sys.path[:0] = [{root!r}, {oracle!r}, {tests!r}]
import types
import numpy as np
import test_gpu_resident as T
from openwhisk_amd import workload as W
w = W.config("c2", n_activations=60_000)
s = w.stream
sh = T.Shim(w)
k = s.n_batches // 2
pre = types.SimpleNamespace(n_batches=k, acq_off=s.acq_off[:k + 1], act=s.act[:int(s.acq_off[k])],
                            rel_off=s.rel_off[:k + 1], rel_aid=s.rel_aid[:int(s.rel_off[k])], seq_base=1 << 40)
g_inv, g_fl, g_rf = sh.g.replay(pre)
assert sh.g.stream_mode_stats() is not None  # the replay ran in the resident engine's stream mode
o_inv, o_fl, o_rf = sh.o.replay(pre)
assert np.array_equal(g_inv, o_inv) and np.array_equal(g_fl, o_fl) and np.array_equal(g_rf, o_rf)
rng = np.random.default_rng(6)
while not sh.done():
    sh.call(int(rng.integers(20, 400)))
st = sh.g.resident_stats()
assert st["served"] == sh.calls and st["chained"] == 0, st
assert np.array_equal(sh.g.permits(), sh.o.permits())
print("ok", sh.calls)
"""


def test_stream_mode_replay_then_resident_calls():
    """A stream-mode replay (OWGS_SPEC_REPLAY=1: the resident engine replays whole batches and stores walk cursors
    under generations 1..n) followed by the shim's first owgs_process_batch on the same context: the first resident
    launch must start above every generation already stored, or stale cursors would skip walk steps that fit again
    after later releases.  Every call bit-exact with the oracle; the switch is read once per process, so
    a child process."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = _SPEC_THEN_CALLS_SCRIPT.format(root=root, oracle=os.path.join(root, "oracle"), tests=here)
    env = dict(os.environ, OWGS_SPEC_REPLAY="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_resident_lifetime_bound_and_other_contexts_on_shared_queues():
    """The resident engine holds its stream's hardware queue while it runs, and GPU_MAX_HW_QUEUES (4) makes the
    streams of several contexts share queues: three contexts in one process, each driven by its own thread -- one
    serving small drains on the resident engine without pause, two taking the launch chain (drains beyond OWGS_RES_MAX)
    and device replays -- all finish, every call bit-exact, because the engine exits between calls at its lifetime
    bound (OWGS_RES_LIFE_US, 100 ms) and is relaunched."""
    import threading
    res = {}

    def resident():
        sh = Shim(W.config("c4", n_activations=120_000))
        rng = np.random.default_rng(1)
        while not sh.done():
            sh.call(int(rng.integers(50, 400)))
        res["resident"] = (sh.g.resident_stats(), np.array_equal(sh.g.permits(), sh.o.permits()))

    def chained(name, cfg):
        sh = Shim(W.config(cfg, n_activations=60_000))
        while not sh.done():
            sh.call(3000)
        st = sh.g.resident_stats()
        res[name] = (st, np.array_equal(sh.g.permits(), sh.o.permits()))

    def replays():
        w = W.config("c2", n_activations=200_000)
        o = O.state_for(w)
        g = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction,
                                             blackbox_fraction=w.blackbox_fraction, rng_seed=w.rng_seed)
        g.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
        g.register_actions(w.actions)
        out, fl, rf = g.replay(w.stream)
        oo, of, orf = o.replay(w.stream)
        res["replay"] = (np.array_equal(out, oo) and np.array_equal(fl, of), np.array_equal(g.permits(), o.permits()))

    ts = [threading.Thread(target=resident), threading.Thread(target=chained, args=("chain", "headline")),
          threading.Thread(target=replays)]
    t0 = time.time()
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), f"a context did not finish within 100 s ({time.time() - t0:.1f} s)"
    st, ok = res["resident"]
    assert ok and st["served"] > 100 and st["chained"] == 0, st
    st, ok = res["chain"]
    assert ok and st["chained"] > 0, st
    assert res["replay"] == (True, True)


@pytest.mark.parametrize("cfg,kw,sizes", [
    ("c4", dict(n_activations=60_000), (2, 1)),
    ("headline", dict(n_activations=60_000, n_invokers=1000, n_actions=2000, n_namespaces=200, conc_frac=0.3), (2,)),
    ("hot", None, (2, 3)),
])
def test_resident_serves_watched_pairs_after_membership_changes(cfg, kw, sizes):
    """updateCluster (SCPB:561-584) discards the NestedSemaphore entries of activations still in flight, so their
    releases meet the new state: a present entry takes RS.release(1, true) whatever its operationCount, an absent one
    throws NoSuchElement (NS:103) unless a failed concurrent try left the reference an empty entry (NS:61-62).  The
    resident engine applies these releases and marks the failed tries itself, so the shim's small drains stay on it
    after a membership change: >= 95 % of the calls after the change are resident-served, every call bit-exact with
    the literal oracle, and the oracle without empty entries disagrees (the stream reaches those releases)."""
    w = _hot_small_pool(21, n_activations=30_000) if cfg == "hot" else W.config(cfg, **kw)
    sh = Shim(w, shadow=True)
    rng = np.random.default_rng(17)
    n_jobs = len(sh.jobs)
    at = [int(n_jobs * (k + 1) / (len(sizes) + 2)) for k in range(len(sizes))]
    before = after = 0
    st0 = None
    while not sh.done():
        if at and sh.pos >= at[0]:
            at.pop(0)
            x = sizes[len(sizes) - len(at) - 1]
            for b in (sh.g, sh.o, sh.z):
                b.update_cluster(x)
            if st0 is None:
                st0 = sh.g.resident_stats()
        sh.call(int(rng.integers(1, 600)))
        if st0 is None:
            before += 1
        else:
            after += 1
    st = sh.g.resident_stats()
    served_after = st["served"] - st0["served"]
    assert served_after >= 0.95 * after, (served_after, after, st)
    assert st["watch_calls"] > 0, st
    assert np.array_equal(sh.g.permits(), sh.o.permits())
    assert sh.z_rf != sh.o_rf  # releases only the reference's empty entries explain were reached
