"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle and the reference's golden vectors.

Bar: bit-exact assignment vectors, overload flags, release flags and final slot state.  Run on an MI355X
(pytest -m gpu).  All cases run in this one process.
"""
import numpy as np
import pytest

import oracle as O
from openwhisk_amd import GpuShardingContainerPoolBalancer, InvokerHealth
from openwhisk_amd import workload as W
from openwhisk_amd.balancer import Action, HEALTHY, NONE, OFFLINE, THROW_INDEX, UNHEALTHY

pytestmark = pytest.mark.gpu
MB = 1024 * 1024
ST = {"healthy": HEALTHY, "unhealthy": UNHEALTHY, "offline": OFFLINE}


def gpu(**kw):
    return GpuShardingContainerPoolBalancer(**kw)


def test_device_selftest():
    gpu().selftest()


# ----------------------------------------------------------------------------------------------- hashing
def test_generate_hash_on_gpu_matches_jls():
    names = [("invocationSpace", "testspace/testname"), ("", "polygenelubricants"), ("a", "b"), ("ns", "x" * 300),
             ("guest", "guest/pkg/act"), ("Aa", "BB")]
    b = gpu()
    acts = [Action(ns, p, "0.0.1", 256) for ns, p in names]
    _, h = b.register_actions(acts)
    assert h.tolist() == [O.generate_hash(ns, p) for ns, p in names]
    assert h[1] == -2**31  # Int.MinValue.abs stays negative (SCPB:371)
    w = W.config("headline", n_activations=10)
    b2 = gpu()
    _, h2 = b2.register_actions(w.actions)
    assert h2.tolist() == [O.generate_hash(a.namespace, a.path) for a in w.actions]


# ----------------------------------------------------------------------------------------------- schedule goldens
@pytest.mark.parametrize("name", ["schedule_empty_invokers", "schedule_no_healthy", "schedule_step_then_overload",
                                  "schedule_ignore_unhealthy_offline", "schedule_enough_free_slots",
                                  "schedule_concurrent_actions"])
def test_schedule_golden(golden, name):
    c = golden[name]
    b = gpu(rng_seed=99)
    b.set_slots([c["slots"]["permits"]] * c["slots"]["count"])
    b.set_pool(0, [(i, ST[s]) for i, s in c["invokers"]])
    key = 7
    # one call per batch element; the whole sequence is a single batch with sequential semantics
    calls = c["calls"]
    ids, fl = b.schedule(c["max_concurrent"], key, [x["mem"] for x in calls], [x["index"] for x in calls],
                         [x["step"] for x in calls], seq=np.arange(len(calls)))
    for k, call in enumerate(calls):
        exp = call["expect"]
        if exp is None:
            assert ids[k] == NONE
        else:
            assert [ids[k], bool(fl[k] & 1)] == exp
    # concurrency expectations are checked call by call
    if any("concurrent_permits_after" in x for x in calls):
        b2 = gpu()
        b2.set_slots([c["slots"]["permits"]] * c["slots"]["count"])
        b2.set_pool(0, [(i, ST[s]) for i, s in c["invokers"]])
        for call in calls:
            i2, _ = b2.schedule(c["max_concurrent"], key, call["mem"], call["index"], call["step"])
            cp = call["concurrent_permits_after"]
            assert i2[0] == call["expect"][0]
            assert b2.concurrent_state(cp["invoker"], key)[0] == cp["permits"]
    if "then_overload" in c:
        t = c["then_overload"]
        r, f = b.schedule(c["max_concurrent"], key, t["mem"], t["index"], t["step"], seq=np.arange(t["calls"]))
        assert set(t["ids_contain_all"]) <= set(r.tolist()) <= set(t["ids_subset_of"])
        assert np.all(f & 1)
        # oracle agreement of the random fallback (same counter RNG)
        inv = [(i, ST[s]) for i, s in c["invokers"]]
        slots = O.Slots(c["slots"]["count"], c["slots"]["permits"])
        for call in calls:
            O.schedule(c["max_concurrent"], key, inv, slots, call["mem"], call["index"], call["step"],
                       seq=0, rng_seed=99)
        exp = [O.schedule(c["max_concurrent"], key, inv, slots, t["mem"], t["index"], t["step"], seq=s, rng_seed=99)
               for s in range(t["calls"])]
        assert r.tolist() == [e[0] for e in exp]
    if "final_permits" in c:
        assert b.permits().tolist() == c["final_permits"]


# ----------------------------------------------------------------------------------------------- state goldens
@pytest.mark.parametrize("name", ["state_grow_keep_old", "state_update_cluster", "state_cluster_below_one",
                                  "state_cluster_min_memory"])
def test_state_golden(golden, name):
    c = golden[name]
    b = gpu(managed_fraction=c["managed_fraction"], blackbox_fraction=c["blackbox_fraction"])
    act = None
    for step in c["steps"]:
        if "update_invokers" in step:
            b.update_invokers([InvokerHealth(i, m, ST[s]) for i, m, s in step["update_invokers"]])
        if "try_acquire" in step:
            i, m = step["try_acquire"]
            # NestedSemaphore.tryAcquire(m) on slot i == a schedule() of one maxConcurrent=1 action pinned to i
            b.set_pool(0, [(i, HEALTHY)])
            r, _ = b.schedule(1, 0, m, 0, 1)
            assert r[0] == i
        if "update_cluster" in step:
            b.update_cluster(step["update_cluster"])
        e = step.get("expect", {})
        if "permits" in e:
            assert b.permits().tolist() == e["permits"]
        if "managed_steps" in e:
            assert b.managed_step_sizes == e["managed_steps"]
            assert b.blackbox_step_sizes == e["blackbox_steps"]
        if "managed" in e:
            assert b.managed_size == len(e["managed"]) and b.blackbox_size == len(e["blackbox"])
    del act


def test_state_overlap_sizes(golden):
    c = golden["state_overlap_small_n"]
    bs = {}
    for row in c["rows"][::7]:
        bf = row["bf"]
        b = bs.setdefault(bf, gpu(managed_fraction=1.0 - bf, blackbox_fraction=bf))
        i = row["i"]
        b.update_invokers([InvokerHealth(1, c["user_memory_mb"] * MB)] * i)
        assert b.blackbox_size == row["blackbox_size"]
        assert b.managed_size + b.blackbox_size == row["managed_plus_blackbox"]


# ----------------------------------------------------------------------------------------------- component golden
def test_balancer_activation_batch(golden):
    c = golden["balancer_activation_batch"]
    n_inv = c["n_invokers"]
    for row in c["rows"][::5]:
        b = gpu(managed_fraction=c["managed_fraction"], blackbox_fraction=c["blackbox_fraction"])
        b.update_invokers([InvokerHealth(i, c["invoker_memory_mb"] * MB) for i in range(n_inv)])
        (a,), (h,) = b.register_actions([Action(c["namespace"], c["action_path"], "0.0.1", c["action_memory_mb"],
                                                c["max_concurrent"])])
        key = b.key_id(a)
        steps = b.managed_step_sizes
        home, step = h % n_inv, steps[h % len(steps)]
        inv, fl = b.publish(np.full(row["activations"], a))
        assert np.all(fl == 0)
        nxt = home
        for g in row["groups_in_walk_order"]:
            assert b.concurrent_state(nxt, key) == (g["remaining"], g["count"])
            nxt = (nxt + step) % n_inv
        rf = b.release_invoker(inv, np.full(len(inv), a))
        assert np.all(rf == 0)
        assert b.permits().tolist() == c["after_release"]["permits"]
        assert all(b.concurrent_state(i, key) is None for i in range(n_inv))


# ----------------------------------------------------------------------------------------------- stream parity
def gpu_for(w):
    b = gpu(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction, rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    return b


def check_stream(w, zombies=True):
    st = O.state_for(w, zombies=zombies)
    o_inv, o_fl, o_rf = st.replay(w.stream)
    b = gpu_for(w)
    g_inv, g_fl, g_rf = b.replay(w.stream)
    bad = np.nonzero(o_inv != g_inv)[0]
    assert len(bad) == 0, f"{w.name}: first mismatch at {bad[:5]} oracle={o_inv[bad[:5]]} gpu={g_inv[bad[:5]]}"
    assert np.array_equal(o_fl, g_fl)
    assert np.array_equal(o_rf, g_rf)
    assert np.array_equal(st.permits(), b.permits())
    return b, g_inv, g_fl


@pytest.mark.parametrize("name,n", [("c1", None), ("c2", 200_000), ("c3", 60_000), ("c4", 200_000),
                                    ("headline", 300_000)])
def test_stream_parity(name, n):
    w = W.config(name, n_activations=n)
    check_stream(w)


@pytest.mark.parametrize("kw", [dict(shared_frac=0.6, conc_frac=0.6, n_actions=2000, n_invokers=2000),
                                dict(shared_frac=0.5, conc_frac=0.4, n_actions=500, n_invokers=300, conc_range=(2, 8)),
                                dict(shared_frac=0.3, conc_frac=1.0, n_actions=300, n_invokers=1000,
                                     unhealthy_frac=0.2, load=1.3)])
def test_stream_parity_shared_keys(kw):
    # many fqn@version keys shared by several actions (different walks, one NestedSemaphore entry per invoker):
    # stresses the shared-key validation rule, the kept concurrent speculation and concurrent forced acquires
    w = W.config("headline", n_activations=120_000, **kw)
    check_stream(w)


@pytest.mark.parametrize("kw", [
    # overloaded pools of odd sizes (the blackbox pool starts at an id that is not a multiple of 4): ranks beyond the
    # pool's remaining capacity fail through the capacity scan / cached bound instead of a full walk
    dict(n_invokers=5003, load=1.5, conc_frac=0.0, unhealthy_frac=0.1, blackbox_frac=0.2, n_activations=150_000),
    dict(n_invokers=2999, load=2.0, conc_frac=0.2, unhealthy_frac=0.05, blackbox_frac=0.3, n_activations=100_000,
         cluster_size=3),
    # a slot smaller than most actions (clusterSize 64: 256 MB): rank-0 failures and hot actions running dry
    dict(n_invokers=4001, load=1.1, n_activations=100_000, cluster_size=64),
])
def test_stream_parity_pool_capacity_bounds(kw):
    w = W.config("headline", **kw)
    check_stream(w)


@pytest.mark.parametrize("seed,kw", [
    (11, dict(n_invokers=300, load=1.0, conc_frac=0.0, blackbox_frac=0.0, unhealthy_frac=0.0)),
    (12, dict(n_invokers=257, load=1.3, conc_frac=0.1, blackbox_frac=0.1, unhealthy_frac=0.05)),
    (13, dict(n_invokers=600, load=0.95, conc_frac=0.3, conc_range=(2, 6), shared_frac=0.4)),
    (14, dict(n_invokers=1000, load=1.1, cluster_size=4, zipf_s=1.3)),
])
def test_stream_parity_in_pass_redecisions(seed, kw):
    # small, nearly full pools: most passes stop on a lane whose invoker an earlier lane filled, and the I/O wave
    # re-decides those lanes inside the pass -- many per pass, with fallbacks, hot actions,
    # concurrent lanes and blackbox pools around them
    w = W.config("headline", n_activations=60_000, seed=seed, **kw)
    b, _, _ = check_stream(w)
    if b.stream_mode_stats() is None:  # (the chunked engine's counter; stream mode decides such lanes alone)
        assert b.stats()["redecided"] > 0
    else:
        assert b.stream_mode_stats()["decided_alone"] > 0


def test_engine_specialisation_switch():
    # a context with maxConcurrent == 1 actions only replays on the map-free engine (OWGS_F_*); once a
    # concurrent action is registered, later calls take the engine with the NestedSemaphore map.  Both streams, and
    # the state carried from one to the other, stay bit-exact with the oracle.
    import dataclasses
    w1 = W.config("c2", n_activations=40_000)
    w2 = W.config("c4", n_activations=40_000)
    # (the generators name actions alike: the second set gets its own versions, one set of limits per fqn@version)
    w2 = dataclasses.replace(w2, actions=[dataclasses.replace(a, version="0.0.2") for a in w2.actions])
    assert all(a.max_concurrent == 1 for a in w1.actions) and any(a.max_concurrent > 1 for a in w2.actions)
    keys = {}
    st = O.state_for(w1, slot_keys=keys)
    b = gpu_for(w1)
    for w, stream in ((w1, w1.stream), (w2, dataclasses.replace(w2.stream, act=w2.stream.act + len(w1.actions)))):
        if w is w2:
            for a in w2.actions:
                st.register_action(a.namespace, a.path, keys.setdefault(a.key, len(keys)), a.mem_mb, a.max_concurrent,
                                   a.blackbox)
            b.register_actions(w2.actions)
        o_inv, o_fl, o_rf = st.replay(stream)
        g_inv, g_fl, g_rf = b.replay(stream)
        bad = np.nonzero(o_inv != g_inv)[0]
        assert len(bad) == 0, f"{w.name}: first mismatch at {bad[:5]}"
        assert np.array_equal(o_fl, g_fl) and np.array_equal(o_rf, g_rf)
        assert np.array_equal(st.permits(), b.permits())


def test_malformed_release_stream_fails_loudly():
    # a stream that releases one activation twice (CommonLoadBalancer never does: activationSlots.remove finds no
    # entry the second time, CLB:278-279) is rejected by the release front end (owgs_relpos_kernel's claim of the
    # activation's record) with OWGS_EINVAL; restore() then gives back a balancer that replays a valid stream exactly
    from openwhisk_amd._lib import OwgsError
    w = W.config("c4", n_activations=30_000)
    s = w.stream
    b = gpu_for(w)
    b.snapshot()
    last = s.n_batches - 1
    dup = int(s.rel_aid[s.rel_off[1]])  # released in batch 1, released again in the last batch
    rel_aid = np.insert(s.rel_aid, s.rel_off[last], dup)
    rel_off = s.rel_off.copy()
    rel_off[last + 1:] += 1
    bad = W.Stream(act=s.act, acq_off=s.acq_off, rel_off=rel_off, rel_aid=rel_aid, seq_base=s.seq_base)
    with pytest.raises(OwgsError) as e:
        b.replay(bad)
    assert e.value.code == -22  # OWGS_EINVAL
    b.restore()
    st = O.state_for(w, zombies=True)
    o_inv, o_fl, o_rf = st.replay(s)
    g_inv, g_fl, g_rf = b.replay(s)
    assert np.array_equal(o_inv, g_inv) and np.array_equal(o_fl, g_fl) and np.array_equal(o_rf, g_rf)
    assert np.array_equal(st.permits(), b.permits())


def test_stream_parity_literal_zombie_oracle():
    # the literal oracle (entries created on failed tries, NS:61-62) gives the same answers on valid streams
    w = W.config("c4", n_activations=50_000)
    check_stream(w, zombies=True)


def test_headline_full_size_parity_and_determinism():
    w = W.config("headline")
    b, g1, f1 = check_stream(w)
    b2 = gpu_for(w)
    g2, f2, _ = b2.replay(w.stream)
    assert np.array_equal(g1, g2) and np.array_equal(f1, f2)


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c2_64k"])
def test_baseline_configs_full_size_parity(name):
    # BASELINE.json configs[1..3] at their full sizes (1M activations each), bit-exact with the oracle; c2_64k is
    # configs[1] in SURVEY 8(d)'s literal 64k batches (98 % overload fallbacks)
    check_stream(W.config(name))


def test_c5_shard_full_size_parity():
    # configs[4]: one of 8 controller shards (clusterSize 8) with its full 1M-activation stream
    check_stream(W.config("headline", shard=3, n_shards=8))


@pytest.mark.parametrize("shard,n_shards", [(1, 8), (6, 8), (1, 4)])
def test_cluster_shard_forced_concurrent_cursor(shard, n_shards):
    # regression: a concurrent action forced onto invoker x (fallback) in one chunk, then scheduled again in the next
    # chunk, whose walk cursors were gathered before the forced acquire moved the cursor back to x's step (these
    # shards hit it at activations 670829 / 938326 / 288323 of their full 1M streams)
    check_stream(W.config("headline", shard=shard, n_shards=n_shards), zombies=True)


def test_multi_shard_cluster_parity():
    # C5-style shards: clusterSize 8, each shard its own stream; shard state = 1/8 of every invoker
    for g in (0, 7):
        w = W.config("headline", shard=g, n_shards=8, n_activations=100_000)
        check_stream(w)


# ----------------------------------------------------------------------------------------------- edge cases
def test_no_invokers_is_none():
    b = gpu()
    (a,), _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256)])
    inv, fl = b.publish([a, a])
    assert inv.tolist() == [NONE, NONE]


def test_int_min_hash_throws_like_reference():
    b = gpu()
    b.update_invokers([InvokerHealth(i, 4096 * MB) for i in range(10)])  # managed 9: 2^31 % 9 != 0
    (a,), (h,) = b.register_actions([Action("", "polygenelubricants", "0.0.1", 256)])
    assert h == -2**31
    inv, _ = b.publish([a])
    assert inv[0] == THROW_INDEX
    assert b.permits().tolist() == [4096] * 10


def test_invoker_id_outside_slots_throws():
    b = gpu()
    b.set_slots([10, 10])
    b.set_pool(0, [(0, HEALTHY), (5, HEALTHY)])
    r, _ = b.schedule(1, 0, [10, 10], 0, 1)
    assert r.tolist() == [0, THROW_INDEX]


def test_release_flags():
    b = gpu()
    b.update_invokers([InvokerHealth(i, 1024 * MB) for i in range(4)])
    acts, _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256, 1), Action("ns", "ns/c", "0.0.1", 256, 4)])
    inv, _ = b.publish([acts[1]])
    # unknown concurrent key on another invoker -> NoSuchElementException; out-of-range invoker -> lift no-op;
    # never-scheduled activation -> no entry
    other = (inv[0] + 1) % 4
    rf = b.release_invoker([other, 99, -1, inv[0], inv[0]], [acts[1], acts[0], acts[0], acts[1], acts[1]])
    assert rf.tolist() == [1, 0, 4, 0, 1]
    assert b.permits().tolist() == [1024] * 4


def test_release_overflow_takes_the_ordered_path():
    # a batch where a release can overflow an invoker's permits (FS:48-50) is applied in stream order: exactly the
    # overflowing releases are rejected (flag 2, state unchanged), the others of the batch still apply
    b = gpu()
    b.update_invokers([InvokerHealth(i, 1024 * MB) for i in range(3)])
    acts, _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256, 1)])
    top = 2**31 - 1
    b.set_slots([top - 300, 1000, top - 256])
    rf = b.release_invoker([0, 1, 0, 2, 2], [acts[0]] * 5)
    assert rf.tolist() == [0, 0, 2, 0, 2]
    assert b.permits().tolist() == [top - 44, 1256, top]
    # without overflow risk the same releases take the parallel path
    b.set_slots([1000, 1000, 1000])
    rf = b.release_invoker([0, 1, 0, 2, 2, 7, -1], [acts[0]] * 7)
    assert rf.tolist() == [0, 0, 0, 0, 0, 0, 4]
    assert b.permits().tolist() == [1512, 1256, 1512]


def test_fused_batch_with_release_range_risk_replays_through_the_release_kernels():
    """owgs_process_batch applies a drained batch's releases inside its one engine launch; when they could push a slot
    beyond the engine's permit range (their summed memory, every concurrent release counted as returning its memory)
    the engine stops before touching anything and the call runs again through the per-run release kernels -- the
    release path that flags ForcibleSemaphore's overflow Error release by release (FS:48-50).  Here the bound is
    crossed but the true result is not: decisions, flags and permits are the oracle's."""
    lim = 2**29
    mem_b = (lim - 300) * MB  # one invoker whose slot sits just under the range
    g = gpu(managed_fraction=1.0, blackbox_fraction=0.0)
    o = O.BalancerState(1.0, 0.0, zombies=True)
    g.update_invokers_arrays(np.array([0], np.int32), np.array([mem_b], np.int64), np.zeros(1, np.uint8))
    o.update_invokers(np.array([0], np.int32), np.array([mem_b], np.int64), np.zeros(1, np.uint8))
    acts = [Action("ns", "ns/c", "0.0.1", 256, 4), Action("ns", "ns/a", "0.0.1", 128, 1)]
    hs, _ = g.register_actions(acts)
    oh = [o.register_action(a.namespace, a.path, k, a.mem_mb, a.max_concurrent, a.blackbox) for k, a in enumerate(acts)]
    gi, gf, _ = g.process_batch([0, 0], [], [], [0, 3], [hs[0]] * 3)  # one container, 3 of its 4 slots
    oi = [o.publish(oh[0], k) for k in range(3)]
    assert [(int(a), int(b)) for a, b in zip(gi, gf)] == oi
    assert g.permits().tolist() == o.permits().tolist() == [lim - 556]
    # 3 releases (bound 768 > 556 of room) then 2 publishes: the container empties once (256 back), then a new one
    gi2, gf2, grf = g.process_batch([0, 3], [0, 0, 0], [hs[0]] * 3, [0, 2], [hs[0], hs[1]],
                                    seq=np.arange(3, 5, dtype=np.uint64))
    orf = [O._rel_bits(o.release(0, oh[0])) for _ in range(3)]
    oi2 = [o.publish(oh[p], 3 + k) for k, p in enumerate([0, 1])]
    assert grf.tolist() == orf == [0, 0, 0]
    assert [(int(a), int(b)) for a, b in zip(gi2, gf2)] == oi2
    assert g.permits().tolist() == o.permits().tolist() == [lim - 300 - 256 - 128]


def test_release_after_cluster_change_is_nosuchelement():
    b = gpu()
    b.update_invokers([InvokerHealth(i, 1024 * MB) for i in range(2)])
    (a,), _ = b.register_actions([Action("ns", "ns/c", "0.0.1", 128, 3)])
    inv, _ = b.publish([a])
    b.update_cluster(2)  # throws all state away (SCPB:566-568)
    rf = b.release_invoker(inv, [a])
    assert rf.tolist() == [1]
    assert b.permits().tolist() == [512, 512]


def _large(b):
    """Move a context to the large-state engine the way a deployment would: an action above the on-chip engines'
    maxConcurrent (4095, a 12-bit field; owgs_seq.hip keeps 32-bit fields)."""
    from openwhisk_amd._lib import OwgsError
    b.register_actions([Action("zz", "zz/wide", "0.0.1", 128, 5000)])
    with pytest.raises(OwgsError) as e:  # (snapshots are on-chip only: proof that the context moved)
        b.snapshot()
    assert e.value.code == -34
    return b


def test_large_engine_edge_cases_match_the_on_chip_ones():
    """The reference's edge cases on the large-state engine (small pools, the context moved there by a maxConcurrent
    of 5000): no invokers -> None (SCPB:288-290), the Int.MinValue hash -> IndexOutOfBounds (SCPB:266-268), every
    release flag (NS:103, CLB:278-279, invokerSlots.lift SCPB:329), ForcibleSemaphore's overflow Error (FS:48-50) in
    stream order, and a release after updateCluster (SCPB:566-568) -- the same outcomes as the tests above."""
    b = _large(gpu())
    (a,), _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256)])
    assert b.publish([a, a])[0].tolist() == [NONE, NONE]
    b = _large(gpu())
    b.update_invokers([InvokerHealth(i, 4096 * MB) for i in range(10)])
    (a,), (h,) = b.register_actions([Action("", "polygenelubricants", "0.0.1", 256)])
    assert h == -2**31 and b.publish([a])[0][0] == THROW_INDEX
    assert b.permits().tolist() == [4096] * 10
    b = _large(gpu())
    b.update_invokers([InvokerHealth(i, 1024 * MB) for i in range(4)])
    acts, _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256, 1), Action("ns", "ns/c", "0.0.1", 256, 4)])
    inv, _ = b.publish([acts[1]])
    other = (inv[0] + 1) % 4
    rf = b.release_invoker([other, 99, -1, inv[0], inv[0]], [acts[1], acts[0], acts[0], acts[1], acts[1]])
    assert rf.tolist() == [1, 0, 4, 0, 1]
    assert b.permits().tolist() == [1024] * 4
    top = 2**31 - 1
    b = _large(gpu())
    b.update_invokers_arrays(np.arange(3, dtype=np.int32), np.array([top - 300, 1000, top - 256], np.int64) * MB,
                             np.zeros(3, np.uint8))
    acts, _ = b.register_actions([Action("ns", "ns/a", "0.0.1", 256, 1)])
    rf = b.release_invoker([0, 1, 0, 2, 2], [acts[0]] * 5)
    assert rf.tolist() == [0, 0, 2, 0, 2]
    assert b.permits().tolist() == [top - 44, 1256, top]
    b = _large(gpu())
    b.update_invokers([InvokerHealth(i, 1024 * MB) for i in range(2)])
    (a,), _ = b.register_actions([Action("ns", "ns/c", "0.0.1", 128, 3)])
    inv, _ = b.publish([a])
    b.update_cluster(2)
    assert b.release_invoker(inv, [a]).tolist() == [1]
    assert b.permits().tolist() == [512, 512]


# ----------------------------------------------------------------------------------------------- state updates (§8f-2)
def test_pairwise_coprime_golden_on_gpu(golden):
    b = gpu()
    for x, exp in golden["pairwise_coprime_numbers_until"]["expect"].items():
        assert b.pairwise_coprime_numbers_until(int(x)) == exp


def test_pairwise_coprime_sweep_matches_oracle_fold():
    """owgs_coprime_kernel (sieve + ordered compaction) == the literal greedy fold (SCPB:379-384) for every x."""
    b = gpu()
    xs = list(range(-2, 1300)) + [2310, 4096, 9000, 9001, 10000, 30030, 32767, 65536, 70001, 100003]
    for x in xs:
        assert b.pairwise_coprime_numbers_until(x) == O.pairwise_coprime_numbers_until(x), x
    # the kernel's largest pool (524,287, one LDS bit per number): the fold's closed form, {1} and the primes p <= x
    # with p !| x (owgs_state.hip header), from a numpy sieve -- the literal fold takes minutes at this size
    x = 524_287
    sieve = np.ones(x + 1, bool)
    sieve[:2] = False
    for p in range(2, int(x ** 0.5) + 1):
        if sieve[p]:
            sieve[p * p::p] = False
    exp = [1] + [int(p) for p in np.nonzero(sieve)[0] if x % int(p) != 0]
    assert b.pairwise_coprime_numbers_until(x) == exp
    with pytest.raises(Exception):
        b.pairwise_coprime_numbers_until(1 << 20)


@pytest.mark.parametrize("seed", [1, 2])
def test_update_invokers_and_cluster_on_device_match_oracle(seed):
    """Step sizes, grown slots (old ones kept) and updateCluster's re-created slots, 10k invokers (SCPB:512-584)."""
    rng = np.random.default_rng(seed)
    b = gpu(managed_fraction=0.9, blackbox_fraction=0.1)
    o = O.BalancerState(managed_fraction=0.9, blackbox_fraction=0.1)
    n_steps = [3000, 3000, 10000, 9999, 10000]
    for n in n_steps:
        ids = np.arange(n, dtype=np.int32)
        mem = rng.choice([128, 256, 1000, 2048, 16384, 65536], size=n).astype(np.int64) * MB + rng.integers(0, MB, n)
        st = rng.choice([HEALTHY, UNHEALTHY, OFFLINE], p=[0.9, 0.05, 0.05], size=n).astype(np.uint8)
        b.update_invokers_arrays(ids, mem, st)
        o.update_invokers(ids, mem, st)
        assert b.managed_step_sizes == o.managed_step_sizes
        assert b.blackbox_step_sizes == o.blackbox_step_sizes
        assert np.array_equal(b.permits(), o.permits())
        for size in (3, 8, 64, 1):
            b.update_cluster(size)
            o.update_cluster(size)
            assert np.array_equal(b.permits(), o.permits()), (n, size)


@pytest.mark.parametrize("shard_ids,n_shards,n_act", [((0, 1, 3), 4, 150_000),
                                                      (tuple(range(12)), 16, 20_000)])
def test_multi_shard_single_launch_parity(shard_ids, n_shards, n_act):
    # owgs_replay_device_multi: several controller shards in ONE engine launch (one workgroup each), every shard
    # bit-exact with its own oracle replay; a second launch after restore repeats the results.  3 shards take the
    # kernarg path (owgs_engine_multi_kernel), 12 the argument blocks in HBM (owgs_engine_multi_dev_kernel)
    import torch

    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    shards = []
    for g in shard_ids:
        w = W.config("headline", shard=g, n_shards=n_shards, n_activations=n_act)
        b = gpu_for(w)
        b.snapshot()
        s = w.stream
        d = [t(s.acq_off, np.int64), t(s.act, np.int32), t(s.rel_off, np.int64),
             t(s.rel_aid if len(s.rel_aid) else np.zeros(1), np.int64),
             torch.empty(len(s.act), dtype=torch.int32, device=dev),
             torch.empty(len(s.act), dtype=torch.uint8, device=dev),
             torch.empty(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)]
        io = (s.n_batches, d[0].data_ptr(), d[1].data_ptr(), len(s.act), d[2].data_ptr(), d[3].data_ptr(),
              len(s.rel_aid), s.seq_base, d[4].data_ptr(), d[5].data_ptr(), d[6].data_ptr())
        shards.append((w, b, d, io))
    for rep in range(2):
        for _, b, _, _ in shards:
            b.restore()
        torch.cuda.synchronize()
        GpuShardingContainerPoolBalancer.replay_device_multi([(b, io) for _, b, _, io in shards])
        torch.cuda.synchronize()
        for w, b, d, _ in shards:
            st = O.state_for(w)
            o_inv, o_fl, o_rf = st.replay(w.stream)
            assert np.array_equal(o_inv, d[4].cpu().numpy()), (rep, w.name)
            assert np.array_equal(o_fl, d[5].cpu().numpy())
            assert np.array_equal(o_rf, d[6].cpu().numpy()[: len(o_rf)])
            assert np.array_equal(st.permits(), b.permits())


def test_multi_shard_replay_with_a_shard_on_the_large_state_engine():
    """owgs_replay_device_multi with one shard whose maxConcurrent is beyond the on-chip map's field (> 4,095, so its
    slot state lives on the large-state engine, section 5.7) next to ordinary shards: the call routes every shard through
    its own replay (no shared engine launch can hold the large shard) and each is bit-exact with its oracle (ADVICE
    r05: the large shard used to go through the on-chip engine with its maxConcurrent masked to 12 bits)."""
    import torch

    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    shards = []
    for g, kw in ((0, {}), (1, dict(conc_frac=0.3, conc_range=(4_000, 6_000))), (2, {})):
        w = W.config("headline", shard=g, n_shards=4, n_activations=60_000, n_invokers=2000, **kw)
        b = gpu_for(w)
        s = w.stream
        d = [t(s.acq_off, np.int64), t(s.act, np.int32), t(s.rel_off, np.int64),
             t(s.rel_aid if len(s.rel_aid) else np.zeros(1), np.int64),
             torch.empty(len(s.act), dtype=torch.int32, device=dev),
             torch.empty(len(s.act), dtype=torch.uint8, device=dev),
             torch.empty(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)]
        io = (s.n_batches, d[0].data_ptr(), d[1].data_ptr(), len(s.act), d[2].data_ptr(), d[3].data_ptr(),
              len(s.rel_aid), s.seq_base, d[4].data_ptr(), d[5].data_ptr(), d[6].data_ptr())
        shards.append((w, b, d, io))
    assert max(a.max_concurrent for a in shards[1][0].actions) > 4095
    torch.cuda.synchronize()
    GpuShardingContainerPoolBalancer.replay_device_multi([(b, io) for _, b, _, io in shards])
    torch.cuda.synchronize()
    for w, b, d, _ in shards:
        st = O.state_for(w)
        o_inv, o_fl, o_rf = st.replay(w.stream)
        assert np.array_equal(o_inv, d[4].cpu().numpy()), w.name
        assert np.array_equal(o_fl, d[5].cpu().numpy())
        assert np.array_equal(o_rf, d[6].cpu().numpy()[: len(o_rf)])
        assert np.array_equal(st.permits(), b.permits())


# ----------------------------------------------------------------------------------------------- unbounded map
@pytest.mark.parametrize("kw", [
    # up to 19.5k live (invoker, fqn) entries: most of the map lives in the HBM overflow
    dict(n_activations=150_000, n_invokers=3000, n_actions=12_000, n_namespaces=1200, conc_frac=1.0, conc_range=(2, 2),
         delay_mean=6.0, unhealthy_frac=0.0, blackbox_frac=0.0, zipf_s=0.6),
    # ~6.7k live entries: the primary table fills and spills mid-batch
    dict(n_activations=60_000, n_invokers=3000, n_actions=6000, n_namespaces=600, conc_frac=1.0, conc_range=(2, 3),
         delay_mean=6.0, unhealthy_frac=0.0, blackbox_frac=0.0),
])
def test_concurrency_map_beyond_the_primary_table(kw):
    """The reference keeps one TrieMap entry per (invoker, fqn@version) with no cap (NestedSemaphore.scala:30, 61-62).
    Streams whose live entries exceed the engine's 4096-entry on-chip table continue in the HBM overflow: decisions,
    flags and final permits bit-exact with the oracle, the surviving entries readable (concurrentState), and a
    restore() + second replay repeats everything (the overflow is part of the snapshot)."""
    w = W.config("headline", **kw)
    st = O.state_for(w, zombies=False)  # (entries compared below: the engine keeps no empty ones)
    o_inv, o_fl, o_rf = st.replay(w.stream)
    b = gpu_for(w)
    b.snapshot()
    for rep in range(2):
        if rep:
            b.restore()
        g_inv, g_fl, g_rf = b.replay(w.stream)
        bad = np.nonzero(o_inv != g_inv)[0]
        assert len(bad) == 0, f"rep {rep}: first mismatch at {bad[:5]}"
        assert np.array_equal(o_fl, g_fl) and np.array_equal(o_rf, g_rf)
        assert np.array_equal(st.permits(), b.permits())
    # NestedSemaphore.concurrentState of a sample of the keys that remain
    keys = {}
    for a in w.actions:
        keys.setdefault(a.key, len(keys))
    sl = st.invoker_slots
    rng = np.random.default_rng(0)
    checked = 0
    for inv in rng.choice(len(sl), size=200, replace=False):
        for k in rng.choice(len(keys), size=40, replace=False):
            o = sl[int(inv)].concurrent_state(int(k))
            g = b.concurrent_state(int(inv), int(k))
            assert o == g, (inv, k, o, g)
            checked += o is not None
    assert checked > 0


# ----------------------------------------------------------------------------------------------- large pools
@pytest.mark.parametrize("n_inv", [15_000, 20_000])
def test_large_pool_stream_parity(n_inv):
    """More invoker ids than the wide engine's LDS image holds (~12.9k): the context switches to the narrow geometry
    (7 x 32-lane chunks, owgs_engine_narrow.hip) and stays bit-exact with the oracle (SCPB:512-551 has no cap)."""
    w = W.config("headline", n_invokers=n_inv, n_activations=150_000)
    b, _, _ = check_stream(w)
    st = b.stream_mode_stats()
    assert (b.stats()["passes"] if st is None else st["decisions"]) > 0


def test_rejected_update_leaves_the_context_unchanged():
    """owgs_update_invokers validates the state it would build before changing anything: a pool beyond every engine
    (the on-chip ones, owgs_limits, and the large-state engine's 65,535 pool positions) is refused with OWGS_ERANGE and
    the context keeps scheduling exactly as before (same permits, same pools)."""
    import ctypes as C
    from openwhisk_amd import _lib
    from openwhisk_amd._lib import OwgsError
    mx, ms = C.c_int32(), C.c_int32()
    _lib.lib().owgs_limits(C.byref(mx), C.byref(ms))
    w = W.config("headline", n_invokers=2000, n_activations=40_000)
    b = gpu_for(w)
    before = (b.permits().copy(), b.managed_size, b.blackbox_size, b.cluster_size, b.managed_step_sizes)
    n = 600_000  # managed pool 540,000 positions: beyond every engine (owgs_coprime_max 524,287)
    with pytest.raises(OwgsError) as e:
        b.update_invokers_arrays(np.arange(n, dtype=np.int32), np.full(n, 16384 * MB, np.int64), np.zeros(n, np.uint8))
    assert e.value.code == -34  # OWGS_ERANGE
    after = (b.permits(), b.managed_size, b.blackbox_size, b.cluster_size, b.managed_step_sizes)
    assert np.array_equal(before[0], after[0]) and before[1:] == after[1:]
    st = O.state_for(w, zombies=True)
    o_inv, o_fl, o_rf = st.replay(w.stream)
    g_inv, g_fl, g_rf = b.replay(w.stream)
    assert np.array_equal(o_inv, g_inv) and np.array_equal(o_fl, g_fl) and np.array_equal(o_rf, g_rf)
    assert np.array_equal(st.permits(), b.permits())


# ----------------------------------------------------------------------------------------------- per-batch health
@pytest.mark.parametrize("cluster_at", [None, 3])
def test_span_replay_with_health_changes_matches_oracle(cluster_at):
    """configs[4] cadence on one GPU: before every batch the agreed health vector is applied (owgs_update_health_device
    = updateInvokers, SCPB:512-551) and the batch replays as one owgs_replay_device_span (its releases name activations
    decided by earlier calls).  Bit-exact with the oracle applying the same vectors between batches; one variant also
    changes the cluster size mid-stream (updateCluster, SCPB:561-584: watched pairs)."""
    import torch
    from openwhisk_amd import cluster

    w = W.config("headline", n_activations=250_000, n_invokers=3000, conc_frac=0.3)
    s = w.stream
    sched = cluster.health_schedule(w.inv_status, s.n_batches, churn=0.03)
    b = gpu_for(w)
    st = O.state_for(w, zombies=True)
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    d_act, d_aid = t(s.act, np.int32), t(s.rel_aid, np.int64)
    d_out = torch.full((len(s.act),), -9, dtype=torch.int32, device=dev)
    d_fl = torch.zeros(len(s.act), dtype=torch.uint8, device=dev)
    d_rf = torch.zeros(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)
    d_h = [t(sched[k], np.uint8) for k in range(s.n_batches)]
    n = len(s.act)
    o_inv = np.full(n, -9, np.int32)
    o_fl = np.zeros(n, np.uint8)
    o_rf = np.zeros(max(len(s.rel_aid), 1), np.uint8)
    P = O._ptr
    acq = np.ascontiguousarray(s.acq_off, np.int64)
    rel = np.ascontiguousarray(s.rel_off, np.int64)
    act = np.ascontiguousarray(s.act, np.int32)
    aid = np.ascontiguousarray(s.rel_aid, np.int64)
    for k in range(s.n_batches):
        if k == cluster_at:
            b.update_cluster(2)
            st.update_cluster(2)
        b.update_health_device(len(w.inv_status), d_h[k].data_ptr())
        b.replay_device_span(s.acq_off[k], s.acq_off[k + 1], s.rel_off[k], s.rel_off[k + 1], d_act.data_ptr(),
                             d_aid.data_ptr(), s.seq_base, d_out.data_ptr(), d_fl.data_ptr(), d_rf.data_ptr())
        st.update_invokers(w.inv_ids, w.inv_mem, sched[k])
        O.lib().owo_replay(st.h, 1, P(acq[k:]), P(act), P(rel[k:]), P(aid), int(s.seq_base), P(o_inv), P(o_fl), P(o_rf))
    torch.cuda.synchronize()
    g_inv = d_out.cpu().numpy()
    bad = np.nonzero(g_inv != o_inv)[0]
    assert len(bad) == 0, f"first mismatch at {bad[:5]}"
    assert np.array_equal(d_fl.cpu().numpy(), o_fl)
    assert np.array_equal(d_rf.cpu().numpy()[:len(s.rel_aid)], o_rf[:len(s.rel_aid)])
    assert np.array_equal(b.permits(), st.permits())
    if cluster_at is None:  # the schedule matters: a static-health replay decides differently
        st0 = O.state_for(w, zombies=True)
        assert not np.array_equal(st0.replay(s)[0], o_inv)


@pytest.mark.gpu
def test_health_on_one_stream_replay_on_another_is_ordered():
    """owgs_update_health_device is asynchronous on its stream; a span replay issued next on ANOTHER stream must still
    see the new health (calls on one context are ordered as issued, include/owgs.h).  The health stream is held back
    by a spin kernel, so an unordered replay would read the old usable bitmap."""
    import torch
    from openwhisk_amd import cluster

    w = W.config("headline", n_activations=60_000, n_invokers=2000, conc_frac=0.2)
    s = w.stream
    sched = cluster.health_schedule(w.inv_status, s.n_batches, churn=0.05)
    b = gpu_for(w)
    st = O.state_for(w, zombies=True)
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    d_act, d_aid = t(s.act, np.int32), t(s.rel_aid, np.int64)
    d_out = torch.full((len(s.act),), -9, dtype=torch.int32, device=dev)
    d_fl = torch.zeros(len(s.act), dtype=torch.uint8, device=dev)
    d_rf = torch.zeros(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)
    d_h = [t(sched[k], np.uint8) for k in range(s.n_batches)]
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    n = len(s.act)
    o_inv, o_fl = np.full(n, -9, np.int32), np.zeros(n, np.uint8)
    o_rf = np.zeros(max(len(s.rel_aid), 1), np.uint8)
    P = O._ptr
    acq, rel = np.ascontiguousarray(s.acq_off, np.int64), np.ascontiguousarray(s.rel_off, np.int64)
    act, aid = np.ascontiguousarray(s.act, np.int32), np.ascontiguousarray(s.rel_aid, np.int64)
    for k in range(s.n_batches):
        with torch.cuda.stream(sa):
            torch.cuda._sleep(2_000_000)  # ~1 ms of spinning ahead of the health update on stream A
        b.update_health_device(len(w.inv_status), d_h[k].data_ptr(), stream=sa.cuda_stream)
        b.replay_device_span(s.acq_off[k], s.acq_off[k + 1], s.rel_off[k], s.rel_off[k + 1], d_act.data_ptr(),
                             d_aid.data_ptr(), s.seq_base, d_out.data_ptr(), d_fl.data_ptr(), d_rf.data_ptr(),
                             stream=sb.cuda_stream)
        st.update_invokers(w.inv_ids, w.inv_mem, sched[k])
        O.lib().owo_replay(st.h, 1, P(acq[k:]), P(act), P(rel[k:]), P(aid), int(s.seq_base), P(o_inv), P(o_fl), P(o_rf))
    torch.cuda.synchronize()
    g_inv = d_out.cpu().numpy()
    bad = np.nonzero(g_inv != o_inv)[0]
    assert len(bad) == 0, f"first mismatch at {bad[:5]}"
    assert np.array_equal(d_fl.cpu().numpy(), o_fl)
    assert np.array_equal(b.permits(), st.permits())


@pytest.mark.parametrize("cfg,kw,group,cluster_at", [
    ("headline", dict(n_activations=250_000, n_invokers=3000, conc_frac=0.3), 4, None),
    ("headline", dict(n_activations=250_000, n_invokers=3000, conc_frac=0.3), 1, None),
    ("c4", dict(n_activations=200_000), 5, None),
    ("c2", dict(n_activations=200_000), 64, None),
    ("headline", dict(n_activations=150_000, n_invokers=2000, conc_frac=0.3), 3, 2),
    # beyond the on-chip image: the large-state engine, per-batch health and a cluster change through the same call
    ("headline", dict(n_activations=300_000, n_invokers=25_000, conc_frac=0.3), 4, None),
    ("headline", dict(n_activations=300_000, n_invokers=25_000, conc_frac=0.3), 2, 1),
])
def test_group_replay_with_per_batch_health_matches_oracle(cfg, kw, group, cluster_at):
    """configs[4] cadence with several batches per engine launch (owgs_replay_device_group): the engine applies batch
    b's health vector itself before the batch's releases (updateInvokers, SCPB:512-551: usable bitmap, the usable flag
    of each changed invoker's permits, the pools' healthy counts), and the group's releases name activations decided
    by earlier launches (records written from those decisions) or by earlier batches of the group.  Bit-exact with the
    oracle applying the same vector before every batch; one variant changes the cluster size between groups (watched
    pairs: the call takes its batch-by-batch fallback)."""
    import torch
    from openwhisk_amd import cluster

    w = W.config(cfg, **kw)
    s = w.stream
    sched = cluster.health_schedule(w.inv_status, s.n_batches, churn=0.03)
    b = gpu_for(w)
    st = O.state_for(w, zombies=True)
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    d_act, d_aid = t(s.act, np.int32), t(s.rel_aid, np.int64)
    d_out = torch.full((len(s.act),), -9, dtype=torch.int32, device=dev)
    d_fl = torch.zeros(len(s.act), dtype=torch.uint8, device=dev)
    d_rf = torch.zeros(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)
    nid = len(w.inv_status)
    d_h = t(np.stack(sched), np.uint8)  # [n_batches][n_invokers]
    n = len(s.act)
    o_inv = np.full(n, -9, np.int32)
    o_fl = np.zeros(n, np.uint8)
    o_rf = np.zeros(max(len(s.rel_aid), 1), np.uint8)
    P = O._ptr
    acq = np.ascontiguousarray(s.acq_off, np.int64)
    rel = np.ascontiguousarray(s.rel_off, np.int64)
    act = np.ascontiguousarray(s.act, np.int32)
    aid = np.ascontiguousarray(s.rel_aid, np.int64)
    for g0 in range(0, s.n_batches, group):
        g1 = min(g0 + group, s.n_batches)
        if cluster_at is not None and g0 >= cluster_at and g0 - group < cluster_at:
            b.update_cluster(2)
            st.update_cluster(2)
        b.replay_device_group(acq[g0:g1 + 1], rel[g0:g1 + 1], d_act.data_ptr(), d_aid.data_ptr(), s.seq_base,
                              d_out.data_ptr(), d_fl.data_ptr(), d_rf.data_ptr(), d_h[g0].data_ptr(), nid, nid)
        for k in range(g0, g1):
            st.update_invokers(w.inv_ids, w.inv_mem, sched[k])
            O.lib().owo_replay(st.h, 1, P(acq[k:]), P(act), P(rel[k:]), P(aid), int(s.seq_base), P(o_inv), P(o_fl),
                               P(o_rf))
    torch.cuda.synchronize()
    g_inv = d_out.cpu().numpy()
    bad = np.nonzero(g_inv != o_inv)[0]
    assert len(bad) == 0, f"first mismatch at {bad[:5]} gpu {g_inv[bad[:5]]} oracle {o_inv[bad[:5]]}"
    assert np.array_equal(d_fl.cpu().numpy(), o_fl)
    assert np.array_equal(d_rf.cpu().numpy()[:len(s.rel_aid)], o_rf[:len(s.rel_aid)])
    assert np.array_equal(b.permits(), st.permits())
    assert b.resident_stats()["alive"] == 0
    # the context's health after the call is the last batch's row (the oracle's last update_invokers): publishes after
    # it walk past that row's unusable invokers and draw the fallback from its healthy count (SCPB:417-424)
    rng = np.random.default_rng(11)
    probe = rng.integers(0, len(w.actions), 4000).astype(np.int32)
    seq0 = int(s.seq_base) + n + 1
    g_p, g_pf = b.publish(probe, seq=np.arange(seq0, seq0 + len(probe), dtype=np.uint64))
    o_p = np.array([st.publish(int(a), seq0 + i) for i, a in enumerate(probe)], dtype=np.int64)
    assert np.array_equal(g_p, o_p[:, 0]) and np.array_equal(g_pf, o_p[:, 1])
    assert np.array_equal(b.permits(), st.permits())
    last_unusable = np.nonzero(sched[-1] != 0)[0]
    assert not np.isin(g_p[g_p >= 0], w.inv_ids[last_unusable]).any()  # (forced ones too: healthyInvokers)


# ----------------------------------------------------------------------------------------------- large-state engine
def test_large_pool_40k_invokers_stream_matches_oracle():
    """A 40,000-invoker pool (beyond every on-chip geometry, owgs_limits ~20.6k; 36,000 managed positions beyond the
    15-bit key and walk fields) runs on the large-state engine (owgs_seq.hip: permits in HBM, one HBM map keyed by
    the full (invoker, fqn@version) pair): the whole stream with concurrent actions and releases bit-exact with the
    oracle -- decisions, overload flags, release flags, final permits."""
    import ctypes as C
    from openwhisk_amd import _lib
    mx, ms = C.c_int32(), C.c_int32()
    _lib.lib().owgs_limits(C.byref(mx), C.byref(ms))
    w = W.config("headline", n_invokers=40_000, n_activations=80_000, n_actions=4000, n_namespaces=400,
                 conc_frac=0.3, user_memory_mb=1024)
    assert len(w.inv_ids) > mx.value and w.stream.n_batches > 3 and len(w.stream.rel_aid) > 10_000
    b, g_inv, g_fl = check_stream(w)
    assert (g_fl & 1).sum() >= 0 and (g_inv >= 0).all()


def test_large_pool_100k_invokers_beyond_the_old_step_kernel_range():
    """100,000 invokers: a managed pool of 90,000 positions, past the 65,535 the step-size kernel held until round 5
    (pairwiseCoprimeNumbersUntil now sieves one LDS bit per number) -- the stream bit-exact on the large-state engine."""
    w = W.config("headline", n_invokers=100_000, n_activations=150_000, n_actions=4000, n_namespaces=400,
                 conc_frac=0.3)
    b, g_inv, g_fl = check_stream(w)
    assert b.managed_size == 90_000 and (g_inv >= 0).all()


def test_large_pool_shim_sequence_with_membership_change():
    """The shim's call sequence (owgs_process_batch per drained batch) on a 25,000-invoker pool, with updateCluster
    mid-stream (SCPB:561-584: the entries of in-flight concurrent activations are discarded; their releases meet the
    new state and the empty entries failed tries leave, NS:61-62 -- the large-state engine keeps those literally),
    call by call against the literal oracle."""
    import test_gpu_resident as R
    w = W.config("headline", n_invokers=25_000, n_activations=70_000, n_actions=3000, n_namespaces=300,
                 conc_frac=0.4, load=1.1, user_memory_mb=1024)
    assert len(w.stream.rel_aid) > 10_000
    sh = R.Shim(w, shadow=True)
    rng = np.random.default_rng(9)
    half = len(sh.jobs) // 2
    changed = False
    while not sh.done():
        if not changed and sh.pos >= half:
            for x in (sh.g, sh.o, sh.z):
                x.update_cluster(2)
            changed = True
        sh.call(int(rng.integers(1, 3000)))
    assert np.array_equal(sh.g.permits(), sh.o.permits())
    assert sh.g.resident_stats()["served"] == 0  # (no resident engine for a large state)
    assert sh.z_rf != sh.o_rf  # releases only the reference's empty entries explain were reached


def test_maxconcurrent_beyond_4095_and_growth_into_the_large_engine():
    """maxConcurrent is bounded only by configuration in the reference (ConcurrencyLimit.scala:52,71); beyond the
    on-chip map's 12-bit field the context moves to the large-state engine, carrying the on-chip map's entries (and the
    empty entries watched pairs stand for) over -- here mid-stream, with activations in flight -- and so does a pool
    that grows past owgs_limits.  Call by call against the literal oracle."""
    from openwhisk_amd import Action
    MB = 1024 * 1024
    rng = np.random.default_rng(3)
    g = gpu(managed_fraction=1.0, blackbox_fraction=0.0, rng_seed=4)
    o = O.BalancerState(1.0, 0.0, rng_seed=4, zombies=True)
    n0 = 300
    ids, mem = np.arange(n0, dtype=np.int32), np.full(n0, 4096 * MB, np.int64)
    g.update_invokers_arrays(ids, mem, np.zeros(n0, np.uint8))
    o.update_invokers(ids, mem, np.zeros(n0, np.uint8))
    acts = [Action(f"ns{a % 5}", f"ns{a % 5}/p/a{a}", "0.0.1", int(rng.choice([128, 256, 512])),
                   int(rng.integers(2, 9)) if a % 3 else 1) for a in range(200)]
    gh, _ = g.register_actions(acts)
    oh = [o.register_action(a.namespace, a.path, k, a.mem_mb, a.max_concurrent) for k, a in enumerate(acts)]
    live, seq = [], 0

    def call(n_pub, n_rel):
        nonlocal live, seq
        pick = rng.choice(len(live), size=min(n_rel, len(live)), replace=False) if live else np.zeros(0, int)
        rel = [live[j] for j in sorted(pick)]
        keep = set(pick.tolist())
        live = [x for j, x in enumerate(live) if j not in keep]
        pubs = rng.integers(0, len(gh), size=n_pub)
        orf = [O._rel_bits(o.release(x, oh[a])) for x, a in rel]
        oi = [o.publish(oh[a], seq + k) for k, a in enumerate(pubs)]
        gi, gf, grf = g.process_batch([0, len(rel)], [x for x, _ in rel], [gh[a] for _, a in rel], [0, len(pubs)],
                                      [gh[a] for a in pubs], seq_base=seq)
        seq += len(pubs)
        assert grf.tolist() == orf
        assert [(int(x), int(f)) for x, f in zip(gi, gf)] == oi
        live += [(int(x), int(a)) for x, a in zip(gi, pubs) if x >= 0]

    for _ in range(20):
        call(400, 150)
    g.update_cluster(2)  # watched pairs on the on-chip engine ...
    o.update_cluster(2)
    for _ in range(5):
        call(300, 150)
    big = [Action("nsx", "nsx/p/big", "0.0.1", 256, 10_000), Action("nsx", "nsx/p/big2", "0.0.1", 128, 70_000)]
    gh2, _ = g.register_actions(big)  # ... carried into the large engine here
    oh += [o.register_action(a.namespace, a.path, len(oh) + k, a.mem_mb, a.max_concurrent) for k, a in enumerate(big)]
    gh = np.concatenate([gh, gh2])
    for _ in range(10):
        call(400, 200)
    n1 = 30_000  # the pool grows past owgs_limits (the large engine already holds the state)
    ids, mem = np.arange(n1, dtype=np.int32), np.full(n1, 2048 * MB, np.int64)
    g.update_invokers_arrays(ids, mem, np.zeros(n1, np.uint8))
    o.update_invokers(ids, mem, np.zeros(n1, np.uint8))
    for _ in range(10):
        call(400, 200)
    assert np.array_equal(g.permits(), o.permits())
