"""The JNI binding (integration/owgs_jni.c) executed, not just compiled: tests/jni_stub/jni_harness.c supplies a JNIEnv
whose function table implements the JNI calls the binding makes over stand-in Java objects (arrays, Strings, direct
ByteBuffers), so these tests drive the exact native methods the Scala shim declares (OwgsNative in
integration/GpuShardingContainerPoolBalancer.scala) -- registerAction's String path, processBatch's direct-buffer layout
written the way BatchBuffers.ensure / processSegment write it, releaseActions, lastError -- and compare with the oracle.
The CPU tests check the binding's argument handling (nothing reaches the engine); the GPU test is a shim call sequence
against the literal oracle."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O
from openwhisk_amd import _lib
from openwhisk_amd import workload as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "integration", "build", "libowgs_jni_harness.so")
K_INTS, K_LONGS, K_BYTES, K_STRING, K_DIRECT = 1, 2, 3, 4, 5


class Jvm:
    """Stand-in Java objects over numpy buffers (kept alive here) and the binding's native methods."""

    def __init__(self):
        _lib.lib()  # the engine (and torch's HIP runtime) first: the harness links against the same libowgs.so
        if not os.path.exists(HARNESS):
            pytest.skip("integration/build/libowgs_jni_harness.so not built (make -C integration)")
        L = C.CDLL(HARNESS)
        P, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
        for name, res, args in [("h_obj", P, [C.c_int, P, i64]), ("h_free", None, [P]), ("h_oob", C.c_long, []),
                                ("h_strings_held", C.c_long, []),
                                ("h_create", i64, [C.c_double, C.c_double, i64, i32, i32, i64]),
                                ("h_destroy", None, [i64]), ("h_update_invokers", i32, [i64, P, P, P]),
                                ("h_update_cluster", i32, [i64, i32]),
                                ("h_register_action", i32, [i64, P, P, P, i32, i32, i32]),
                                ("h_process_batch", i32, [i64, P, P, i32, i32, i32, i64]),
                                ("h_release_actions", i32, [i64, P, i32]),
                                ("h_publish_batch", i32, [i64, P, P, i32, P, P]),
                                ("h_release_batch", i32, [i64, P, P, i32, P]), ("h_last_error", C.c_char_p, [i64])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L, self.keep, self.objs = L, [], []

    def obj(self, kind, arr, n=None):
        self.keep.append(arr)
        o = self.L.h_obj(kind, arr.ctypes.data_as(C.c_void_p), len(arr) if n is None else n)
        self.objs.append(o)
        return o

    def ints(self, a):
        return self.obj(K_INTS, np.ascontiguousarray(a, np.int32))

    def longs(self, a):
        return self.obj(K_LONGS, np.ascontiguousarray(a, np.int64))

    def bytes_(self, a):
        return self.obj(K_BYTES, np.ascontiguousarray(a, np.int8))

    def string(self, s):
        b = np.frombuffer(s.encode("utf-8") + b"\0", np.uint8).copy()
        return self.obj(K_STRING, b, len(b) - 1)

    def direct(self, buf):
        return self.obj(K_DIRECT, buf, buf.nbytes)

    def close(self):
        for o in self.objs:
            self.L.h_free(o)
        self.objs.clear()


class BatchBuffers:
    """Python mirror of the shim's BatchBuffers + processSegment's fill order: in = relOff[nRuns + 1], pubOff[nRuns + 1],
    relInvoker[nRel], relAction[nRel], pubAction[nPub] (native-order ints); out = outInvoker[nPub] (ints),
    outFlags[nPub], relFlags[nRel] (bytes)."""

    def __init__(self):
        self.inb = np.zeros(1 << 16, np.uint8)
        self.outb = np.zeros(1 << 15, np.uint8)

    def ensure(self, n_runs, n_rel, n_pub):
        in_bytes = 4 * (2 * (n_runs + 1) + 2 * n_rel + n_pub)
        out_bytes = 4 * n_pub + n_pub + n_rel
        if in_bytes > len(self.inb):
            self.inb = np.zeros(2 * in_bytes, np.uint8)
        if out_bytes > len(self.outb):
            self.outb = np.zeros(2 * out_bytes, np.uint8)

    def fill(self, runs):  # runs: [(rel invokers, rel handles, pub handles)]
        ints = [0]
        for r, _, _ in runs:
            ints.append(ints[-1] + len(r))
        po = [0]
        for _, _, p in runs:
            po.append(po[-1] + len(p))
        ints += po
        for r, _, _ in runs:
            ints += list(r)
        for _, h, _ in runs:
            ints += list(h)
        for _, _, p in runs:
            ints += list(p)
        a = np.array(ints, np.int32)
        self.inb[:4 * len(a)] = a.view(np.uint8)
        return len(runs), int(ints[len(runs)]), int(po[-1])


@pytest.fixture
def jvm():
    j = Jvm()
    yield j
    j.close()


def test_binding_rejects_bad_arguments_without_a_device(jvm):
    # no JVM object reaches the engine unless its shape is right; none of these needs a GPU
    L = jvm.L
    bufs = BatchBuffers()
    n_runs, n_rel, n_pub = bufs.fill([([0, 1], [0, 0], [0, 0, 0])])
    not_direct = jvm.ints(np.zeros(64, np.int32))
    out = jvm.direct(bufs.outb)
    assert L.h_process_batch(0, not_direct, out, n_runs, n_rel, n_pub, 0) == _lib.EINVAL  # not a direct buffer
    small = jvm.direct(np.zeros(8, np.uint8))
    assert L.h_process_batch(0, small, out, n_runs, n_rel, n_pub, 0) == _lib.EINVAL  # capacity below the layout
    bad_totals = jvm.direct(bufs.inb)
    assert L.h_process_batch(0, bad_totals, out, n_runs, n_rel + 1, n_pub, 0) == _lib.EINVAL  # offsets != counts
    assert L.h_release_actions(0, jvm.ints([1, 2]), 3) == _lib.EINVAL  # n beyond the array
    assert L.h_update_invokers(0, jvm.ints([0, 1]), jvm.longs([1]), jvm.bytes_([0, 0])) == _lib.EINVAL
    assert L.h_register_action(0, None, jvm.string("a"), jvm.string("b"), 256, 1, 0) == _lib.EINVAL
    assert L.h_oob() == 0 and L.h_strings_held() == 0


@pytest.mark.gpu
def test_shim_sequence_through_the_jni_binding_matches_oracle(jvm):
    """create -> updateInvokers -> (registerAction per new (namespace, fqn@version), processBatch per drained batch of
    (completions, publishes) runs through BatchBuffers) -> updateCluster mid-stream -> releaseActions of every handle,
    re-registration reusing the ids -> publishBatch / releaseBatch: decisions, overload flags, release flags and permits
    equal to the literal oracle driven one reference call at a time."""
    L = jvm.L
    w = W.config("headline", n_activations=30_000, n_invokers=600, n_actions=1200, n_namespaces=120, conc_frac=0.4)
    acts, s = w.actions, w.stream
    h = L.h_create(w.managed_fraction, w.blackbox_fraction, 128 * 1024 * 1024, 1, 0, w.rng_seed)
    assert h != 0
    o = O.BalancerState(w.managed_fraction, w.blackbox_fraction, rng_seed=w.rng_seed, zombies=True)
    try:
        rc = L.h_update_invokers(h, jvm.ints(w.inv_ids), jvm.longs(w.inv_mem), jvm.bytes_(w.inv_status))
        assert rc == 0, L.h_last_error(h)
        o.update_invokers(w.inv_ids, w.inv_mem, w.inv_status)
        g_h, o_h, by_key, o_key = {}, {}, {}, {}

        def handle(a):  # handleOf: registerAction through JNI Strings, once per (namespace, fqn@version)
            x = acts[a]
            k = (x.namespace, x.key)
            if k not in g_h:
                gh = L.h_register_action(h, jvm.string(x.namespace), jvm.string(x.path), jvm.string(x.key), x.mem_mb,
                                         x.max_concurrent, int(x.blackbox))
                assert gh >= 0, L.h_last_error(h)
                g_h[k] = gh
                by_key.setdefault(x.key, gh)
                o_h[k] = o.register_action(x.namespace, x.path, o_key.setdefault(x.key, len(o_key)), x.mem_mb,
                                           x.max_concurrent, x.blackbox)
            return g_h[k], o_h[k]

        bufs = BatchBuffers()
        n = len(s.act)
        o_inv = np.full(n, -9, np.int32)
        seq, drain = 0, 700
        jobs = []
        for b in range(s.n_batches):
            jobs += [("rel", int(a)) for a in s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]]]
            jobs += [("pub", i) for i in range(int(s.acq_off[b]), int(s.acq_off[b + 1]))]
        for j0 in range(0, len(jobs), drain):
            if j0 == (len(jobs) // drain // 2) * drain:  # membership change mid-stream (SCPB:561-584)
                assert L.h_update_cluster(h, 2) == 0
                o.update_cluster(2)
            batch, runs, o_runs, i = jobs[j0:j0 + drain], [], [], 0
            while i < len(batch):
                rels, pubs = [], []
                while i < len(batch) and batch[i][0] == "rel":
                    rels.append(batch[i][1])
                    i += 1
                while i < len(batch) and batch[i][0] == "pub":
                    pubs.append(batch[i][1])
                    i += 1
                rels = [a for a in rels if o_inv[a] >= 0]  # no ActivationEntry for a failed publish (CLB:278-279)
                runs.append(([int(o_inv[a]) for a in rels], [by_key[acts[s.act[a]].key] for a in rels],
                             [handle(int(s.act[a]))[0] for a in pubs]))
                o_runs.append((rels, pubs))
            bufs.ensure(len(runs), sum(len(r) for r, _, _ in runs), sum(len(p) for _, _, p in runs))
            n_runs, n_rel, n_pub = bufs.fill(runs)
            rc = L.h_process_batch(h, jvm.direct(bufs.inb), jvm.direct(bufs.outb), n_runs, n_rel, n_pub, seq)
            assert rc == 0, L.h_last_error(h)
            out_inv = bufs.outb[:4 * n_pub].view(np.int32)
            out_fl = bufs.outb[4 * n_pub:5 * n_pub]
            rel_fl = bufs.outb[5 * n_pub:5 * n_pub + n_rel]
            k_pub = k_rel = 0
            for rels, pubs in o_runs:
                for a in rels:
                    x = acts[s.act[a]]
                    assert int(rel_fl[k_rel]) == O._rel_bits(o.release(int(o_inv[a]), o_h[(x.namespace, x.key)]))
                    k_rel += 1
                for a in pubs:
                    oi, of = o.publish(handle(int(s.act[a]))[1], seq)
                    o_inv[a] = oi
                    assert (int(out_inv[k_pub]), int(out_fl[k_pub])) == (oi, of), (a, k_pub)
                    seq += 1
                    k_pub += 1
        # the completions still outstanding (a drained batch of releases only), then every handle back -- nothing of
        # them is in flight -- and a new registration reuses an id; the per-call array methods on the recycled handle
        done = set(int(a) for a in s.rel_aid)
        rest = [a for a in range(n) if o_inv[a] >= 0 and a not in done]
        runs = [([int(o_inv[a]) for a in rest], [by_key[acts[s.act[a]].key] for a in rest], [])]
        bufs.ensure(1, len(rest), 0)
        n_runs, n_rel, n_pub = bufs.fill(runs)
        assert L.h_process_batch(h, jvm.direct(bufs.inb), jvm.direct(bufs.outb), n_runs, n_rel, n_pub, seq) == 0
        for k, a in enumerate(rest):
            x = acts[s.act[a]]
            assert int(bufs.outb[k]) == O._rel_bits(o.release(int(o_inv[a]), o_h[(x.namespace, x.key)]))
        assert L.h_release_actions(h, jvm.ints(list(g_h.values())), len(g_h)) == 0
        x0 = acts[int(s.act[0])]
        gh = L.h_register_action(h, jvm.string(x0.namespace), jvm.string(x0.path), jvm.string(x0.key + "-v2"),
                                 x0.mem_mb, x0.max_concurrent, int(x0.blackbox))
        assert 0 <= gh < len(g_h), gh  # a recycled id
        oh = o.register_action(x0.namespace, x0.path, len(o_key) + 1, x0.mem_mb, x0.max_concurrent, x0.blackbox)
        pa, sq = np.full(5, gh, np.int32), np.arange(seq, seq + 5, dtype=np.int64)
        out, fl = np.zeros(5, np.int32), np.zeros(5, np.int8)
        assert L.h_publish_batch(h, jvm.ints(pa), jvm.longs(sq), 5, jvm.obj(K_INTS, out), jvm.obj(K_BYTES, fl)) == 0
        exp = [o.publish(oh, int(q)) for q in sq]
        assert [(int(a), int(b)) for a, b in zip(out, fl)] == exp
        rf = np.zeros(5, np.int8)
        assert L.h_release_batch(h, jvm.ints(out), jvm.ints(pa), 5, jvm.obj(K_BYTES, rf)) == 0
        assert [int(v) for v in rf] == [O._rel_bits(o.release(int(v), oh)) for v in out]
        assert L.h_oob() == 0 and L.h_strings_held() == 0
        perm = np.zeros(len(w.inv_ids), np.int32)
        assert _lib.lib().owgs_read_permits(C.c_void_p(h), perm.ctypes.data_as(C.c_void_p), len(perm), None) == 0
        assert np.array_equal(perm, o.permits())
    finally:
        L.h_destroy(h)
