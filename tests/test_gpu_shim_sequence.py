"""The exact call sequence of the Scala shim (integration/GpuShardingContainerPoolBalancer.scala) through the C ABI,
against the oracle balancer driven one reference call at a time.

The shim's batching thread drains its queue in batches of up to 4096 jobs and, inside a batch, issues: one
owgs_update_invokers per CurrentInvokerPoolState (monitor actor, SCPB:226-227), one owgs_update_cluster per
membership change (SCPB:230-248), and for every maximal run of releases followed by publishes ONE owgs_release_batch
(releaseInvoker, SCPB:327-331) then ONE owgs_publish_batch (SCPB:257-290).  Actions are registered lazily, one
owgs_register_actions call per new (invoking namespace, fqn@version), and a release names a handle of its fqn@version
(the shim's byKey map).  Publishes that return no invoker create no ActivationEntry, so they are never released
(CLB:278-279).  The oracle replays the same jobs one reference call at a time; decisions, overload flags, release
flags and final permits must be bit-exact.  Variants change the cluster size mid-stream (updateCluster throws the
slot state away, SCPB:561-584), so the releases of earlier activations meet the new slots -- and, for concurrent
actions, the empty entries the reference's failed tries created (NestedSemaphore.scala:61-62): the comparison is
with the literal oracle, and with the non-materialising one to show those cases occur.
"""
import numpy as np
import pytest

import oracle as O
from openwhisk_amd import GpuShardingContainerPoolBalancer
from openwhisk_amd import workload as W
from openwhisk_amd.balancer import HEALTHY, UNHEALTHY

pytestmark = pytest.mark.gpu


def _jobs(w, rng, health_at, cluster_at):
    cluster_at = cluster_at or {}
    """Queue contents in arrival order: ('inv', status) / ('clu', n) / ('rel', activation) / ('pub', activation)."""
    s = w.stream
    jobs = [("inv", w.inv_status.copy())]
    for b in range(s.n_batches):
        if b == health_at:
            st = w.inv_status.copy()
            st[rng.choice(len(st), size=len(st) // 20, replace=False)] = UNHEALTHY
            st[rng.choice(len(st), size=len(st) // 50, replace=False)] = HEALTHY
            jobs.append(("inv", st))
        if b in cluster_at:
            jobs.append(("clu", cluster_at[b]))
        jobs += [("rel", int(a)) for a in s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]]]
        jobs += [("pub", i) for i in range(int(s.acq_off[b]), int(s.acq_off[b + 1]))]
    return jobs


@pytest.mark.parametrize("mode", ["calls", "fused"])
@pytest.mark.parametrize("seed,cluster_at,kw", [
    (1, None, {}),
    (2, {5: 2}, {}),
    # several membership changes while concurrent activations are in flight, small nearly full pools (failed tries)
    (3, {3: 2, 7: 3, 11: 1}, dict(conc_frac=0.5, conc_range=(2, 6), load=1.1)),
    (4, {4: 4, 9: 2}, dict(conc_frac=0.3, shared_frac=0.4, load=1.2, n_invokers=300)),
    (5, {2: 2, 6: 1, 10: 2}, dict(conc_frac=0.8, conc_range=(2, 3), n_invokers=200, load=1.3)),
])
def test_shim_call_sequence_matches_oracle(seed, cluster_at, kw, mode):
    """mode "calls": one owgs_release_batch per release run and one owgs_publish_batch per publish run; "fused": one
    owgs_process_batch per drained batch (all its runs between state updates), as the shim now does."""
    rng = np.random.default_rng(seed)
    base = dict(n_activations=40_000, n_invokers=600, n_actions=1500, n_namespaces=150)
    base.update(kw)
    w = W.config("headline", **base)
    acts = w.actions
    g = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    # the literal oracle: entries created on failed concurrent tries (NS:61-62); z = the oracle without them, to show
    # which variants reach the releases that tell the two apart
    o = O.BalancerState(w.managed_fraction, w.blackbox_fraction, rng_seed=w.rng_seed, zombies=True)
    z = O.BalancerState(w.managed_fraction, w.blackbox_fraction, rng_seed=w.rng_seed, zombies=False)
    z_rf = []
    z_h = {}
    g_h, o_h, by_key, o_key = {}, {}, {}, {}
    n = len(w.stream.act)
    g_inv = np.full(n, -9, np.int32)
    o_inv = np.full(n, -9, np.int32)
    g_fl = np.zeros(n, np.uint8)
    o_fl = np.zeros(n, np.uint8)
    g_rf, o_rf = [], []
    seq_of = {}

    def handle(a):  # handleOf: lazy registration per (namespace, fqn@version)
        x = acts[a]
        k = (x.namespace, x.key)
        if k not in g_h:
            (h,), _ = g.register_actions([x])
            g_h[k] = h
            by_key.setdefault(x.key, h)
            o_h[k] = o.register_action(x.namespace, x.path, o_key.setdefault(x.key, len(o_key)), x.mem_mb,
                                       x.max_concurrent, x.blackbox)
            z_h[k] = z.register_action(x.namespace, x.path, o_key[x.key], x.mem_mb, x.max_concurrent, x.blackbox)
        return g_h[k], o_h[k]

    jobs = _jobs(w, rng, health_at=3, cluster_at=cluster_at)
    seq = 0
    pos = 0
    fused = []  # (releases, publishes) runs collected for one owgs_process_batch call

    def flush():
        if not fused:
            return
        ro, po, ri, ra, pa, sq, pubs_all = [0], [0], [], [], [], [], []
        for rels, pubs, seqs in fused:
            ri += [int(o_inv[a]) for a in rels]
            ra += [by_key[acts[w.stream.act[a]].key] for a in rels]
            pa += [handle(int(w.stream.act[a]))[0] for a in pubs]
            sq += seqs
            pubs_all += pubs
            ro.append(len(ri))
            po.append(len(pa))
        r, f, rf = g.process_batch(ro, ri, ra, po, pa, seq=np.array(sq, np.uint64))
        g_inv[pubs_all], g_fl[pubs_all] = r, f
        if len(rf):
            g_rf.append(rf)
        fused.clear()

    while pos < len(jobs):
        batch = jobs[pos:pos + int(rng.integers(1, 4097))]  # queue.poll + drainTo(jobs, 4095)
        pos += len(batch)
        i = 0
        while i < len(batch):
            kind, x = batch[i]
            if kind in ("inv", "clu"):
                flush()
            if kind == "inv":
                g.update_invokers_arrays(w.inv_ids, w.inv_mem, x)
                o.update_invokers(w.inv_ids, w.inv_mem, x)
                z.update_invokers(w.inv_ids, w.inv_mem, x)
                i += 1
                continue
            if kind == "clu":
                g.update_cluster(x)
                o.update_cluster(x)
                z.update_cluster(x)
                i += 1
                continue
            rels = []
            while i < len(batch) and batch[i][0] == "rel":
                rels.append(batch[i][1])
                i += 1
            pubs = []
            while i < len(batch) and batch[i][0] == "pub":
                pubs.append(batch[i][1])
                i += 1
            # a fused call returns its decisions at its end: releases inside one drained batch name the invoker the
            # oracle chose (equal to the GPU's, which the final comparison checks)
            dec = o_inv if mode == "fused" else g_inv
            rels = [a for a in rels if dec[a] >= 0]  # no ActivationEntry for a failed publish
            if rels:
                inv = dec[rels]
                hk = [by_key[acts[w.stream.act[a]].key] for a in rels]
                if mode == "calls":
                    g_rf.append(g.release_invoker(inv, hk))
                ok = [(acts[w.stream.act[a]].namespace, acts[w.stream.act[a]].key) for a in rels]
                o_rf.append(np.array([{0: 0, O.THROW_NOSUCHELEMENT: 1, O.THROW_OVERFLOW: 2}.get(
                    o.release(int(iv), o_h[k]), 8) for iv, k in zip(inv, ok)], np.uint8))
                z_rf.append(np.array([O._rel_bits(z.release(int(iv), z_h[k])) for iv, k in zip(inv, ok)], np.uint8))
            if mode == "fused":
                fused.append((rels, pubs, list(range(seq, seq + len(pubs)))))
            if pubs:
                hs = [handle(int(w.stream.act[a])) for a in pubs]
                sq = np.arange(seq, seq + len(pubs), dtype=np.uint64)
                seq += len(pubs)
                if mode == "calls":
                    r, f = g.publish([h for h, _ in hs], seq=sq)
                    g_inv[pubs], g_fl[pubs] = r, f
                for k, (a, (_, oh)) in enumerate(zip(pubs, hs)):
                    o_inv[a], o_fl[a] = o.publish(oh, int(sq[k]))
                    z.publish(z_h[(acts[w.stream.act[a]].namespace, acts[w.stream.act[a]].key)], int(sq[k]))
                    seq_of[a] = int(sq[k])
        flush()  # one owgs_process_batch per drained batch (fused mode)
    flush()
    assert np.array_equal(g_inv, o_inv), np.nonzero(g_inv != o_inv)[0][:5]
    assert np.array_equal(g_fl, o_fl)
    assert np.array_equal(np.concatenate(g_rf), np.concatenate(o_rf))
    assert np.array_equal(g.permits(), o.permits())
    if cluster_at:  # these variants reach releases that only the reference's empty entries explain
        assert not np.array_equal(np.concatenate(z_rf), np.concatenate(o_rf))


def test_fused_batch_release_flags_follow_stream_order():
    """Releases the reference rejects, inside one owgs_process_batch call: a completion released twice in one run (the
    second finds the entry removed: NoSuchElementException, NS:103), a concurrent fqn never scheduled on that invoker,
    an invoker outside invokerSlots (lift: no-op, SCPB:329) and a release without ActivationEntry (CLB:278-279)."""
    from openwhisk_amd import Action, InvokerHealth
    MB = 1024 * 1024
    g = GpuShardingContainerPoolBalancer(managed_fraction=1.0, blackbox_fraction=0.0)
    o = O.BalancerState(1.0, 0.0, zombies=True)
    n = 6
    g.update_invokers([InvokerHealth(i, 8192 * MB) for i in range(n)])
    o.update_invokers(np.arange(n, dtype=np.int32), np.full(n, 8192 * MB, np.int64), np.zeros(n, np.uint8))
    acts = [Action("ns", "ns/c", "0.0.1", 256, 4), Action("ns", "ns/a", "0.0.1", 512, 1),
            Action("ns", "ns/d", "0.0.1", 128, 3)]
    hs, _ = g.register_actions(acts)
    oh = [o.register_action(a.namespace, a.path, k, a.mem_mb, a.max_concurrent, a.blackbox) for k, a in enumerate(acts)]
    pubs = [0, 0, 1, 2, 0, 2]
    gi, gf, _ = g.process_batch([0, 0], [], [], [0, len(pubs)], [hs[p] for p in pubs])
    oi = [o.publish(oh[p], k) for k, p in enumerate(pubs)]
    assert [(int(a), int(b)) for a, b in zip(gi, gf)] == oi
    x0, x2 = int(gi[0]), int(gi[3])
    other = (x0 + 1) % n
    # run 1: ns/c released once more than scheduled, ns/d on an invoker it never used, out of range, no entry;
    # run 2: publishes; run 3: the second ns/c activation (same entry) and the maxConcurrent == 1 one
    rel = [(x0, 0), (x0, 0), (other, 2), (x0, 0), (99, 1), (x0, 0), (-1, 1), (x2, 2)]  # ns/c: 3 scheduled, 4 released
    rel3 = [(x0, 0), (int(gi[2]), 1)]
    ri = [r for r, _ in rel] + [r for r, _ in rel3]
    ra = [hs[a] for _, a in rel] + [hs[a] for _, a in rel3]
    pubs2 = [2, 0, 1]
    gi2, gf2, grf = g.process_batch([0, len(rel), len(rel), len(ri)], ri, ra, [0, 0, len(pubs2), len(pubs2)],
                                    [hs[p] for p in pubs2], seq=np.arange(10, 13, dtype=np.uint64))
    orf = [O._rel_bits(o.release(r, oh[a])) for r, a in rel]
    oi2 = [o.publish(oh[p], 10 + k) for k, p in enumerate(pubs2)]
    orf += [O._rel_bits(o.release(r, oh[a])) for r, a in rel3]
    orf = [f if r >= 0 else 4 for f, r in zip(orf, ri)]
    assert [(int(a), int(b)) for a, b in zip(gi2, gf2)] == oi2
    assert grf.tolist() == orf
    assert 1 in orf  # NoSuchElement reached
    assert np.array_equal(g.permits(), o.permits())


def test_key_and_handle_recycling_over_a_controller_lifetime():
    """A long-running controller sees an unbounded number of fqn@version keys (every action update bumps the version).
    The reference's NestedSemaphore map holds an entry only while activations of its key are in flight
    (NestedSemaphore.scala:109-111); the shim drops cold handles with owgs_release_actions and the context recycles their
    ids, and the ids of keys nothing holds any more.  Over 140,000 distinct keys (more than the 131,070 key ids), with
    concurrent actions, releases one round later and a cluster change mid-stream (in-flight concurrent activations
    become watched pairs and keep their keys), every decision, overload flag, release flag and the final permits equal
    the literal oracle's, which never reuses a key."""
    from openwhisk_amd import Action
    MB = 1024 * 1024
    rng = np.random.default_rng(11)
    n_inv, total_keys, per_round = 200, 140_000, 4000
    g = GpuShardingContainerPoolBalancer(managed_fraction=1.0, blackbox_fraction=0.0, rng_seed=5)
    o = O.BalancerState(1.0, 0.0, rng_seed=5, zombies=True)
    ids, mem = np.arange(n_inv, dtype=np.int32), np.full(n_inv, 8192 * MB, np.int64)
    g.update_invokers_arrays(ids, mem, np.zeros(n_inv, np.uint8))
    o.update_invokers(ids, mem, np.zeros(n_inv, np.uint8))
    seq = 0
    inflight = []       # (gpu handle, oracle handle, invoker) of the previous round's scheduled activations
    live_prev = []      # gpu handles registered in the previous round (all of their activations complete next round)
    max_key = 0
    for r0 in range(0, total_keys, per_round):
        if r0 == 60_000:
            g.update_cluster(2)
            o.update_cluster(2)
        if r0 == 100_000:
            g.update_cluster(1)
            o.update_cluster(1)
        k = np.arange(r0, min(r0 + per_round, total_keys))
        conc = rng.random(len(k)) < 0.5
        acts = [Action(f"ns{x % 97}", f"ns{x % 97}/pkg/a{x}", "0.0.1", int(rng.choice([128, 256, 512])),
                       int(rng.integers(2, 5)) if c else 1) for x, c in zip(k, conc)]
        gh, _ = g.register_actions(acts)
        oh = [o.register_action(a.namespace, a.path, int(x), a.mem_mb, a.max_concurrent) for x, a in zip(k, acts)]
        max_key = max(max_key, max(g.key_id(int(h)) for h in gh))
        # one drained batch: the previous round's completions, then 1-2 publishes of every new action
        pubs = np.repeat(np.arange(len(k)), rng.integers(1, 3, len(k)))
        rng.shuffle(pubs)
        ri = [x for _, _, x in inflight]
        ra = [h for h, _, _ in inflight]
        gi, gf, grf = g.process_batch([0, len(ri)], ri, ra, [0, len(pubs)], [int(gh[p]) for p in pubs],
                                      seq_base=seq)
        orf = [O._rel_bits(o.release(x, oo)) for _, oo, x in inflight]
        oi = [o.publish(oh[p], seq + j) for j, p in enumerate(pubs)]
        seq += len(pubs)
        assert grf.tolist() == orf, r0
        assert [(int(a), int(b)) for a, b in zip(gi, gf)] == oi, r0
        # the previous round's actions have no activation in flight any more: drop their handles
        if live_prev:
            g.release_actions(live_prev)
        live_prev = [int(h) for h in gh]
        inflight = [(int(gh[p]), oh[p], int(x)) for p, x in zip(pubs, gi) if x >= 0]
    assert max_key <= 131_070
    assert np.array_equal(g.permits(), o.permits())
