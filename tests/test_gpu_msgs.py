"""ActivationMessage serialisation + per-invoker topic fan-out on the GPU (owgs_msgs.hip)
against the CPU oracle (oracle/owmsg_oracle.c) and the hand-written golden messages."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from openwhisk_amd import GpuShardingContainerPoolBalancer, OwgsError
from openwhisk_amd._lib import ERANGE, owgs_msg_batch
from test_msgs_cpu import GOLD, batch_of, check

pytestmark = pytest.mark.gpu


def gpu_balancer(templates=GOLD["templates"], rci=GOLD["rci"]):
    b = GpuShardingContainerPoolBalancer()
    assert b.register_templates(templates["a"], templates["b"]) == 0
    b.set_root_controller(rci)
    return b


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_gpu_msg_golden(case):
    out, off, order, topic = gpu_balancer().serialize_activations(**batch_of(case))
    check(case, out, off, order, topic)


def random_tid(rng):
    kind = rng.integers(0, 4)
    if kind == 0:
        return "sid_" + "".join(rng.choice(list("abcdefghijklmnopqrstuvwxyz0123456789"), size=int(rng.integers(1, 40))))
    if kind == 1:  # every escape class
        pool = ['"', "\\", "\b", "\f", "\n", "\r", "\t", "\x00", "\x1f", "\x7f", "a", "/", " "]
        return "".join(rng.choice(pool, size=int(rng.integers(0, 90))))
    if kind == 2:  # non-ASCII incl. supplementary planes, longer than one 64-byte window
        cps = rng.choice([0xE9, 0x3B1, 0x20AC, 0xFFFF, 0x1F600, 0x10FFFF, 0x41, 0x7E], size=int(rng.integers(1, 70)))
        return "".join(chr(int(c)) for c in cps)
    return ""


def random_batch(rng, n, n_topics, n_templates):
    inv = rng.integers(-1, n_topics, size=n).astype(np.int32)
    tmpl = rng.integers(0, n_templates, size=n).astype(np.int32)
    aid = rng.integers(0, 2 ** 63, size=(n, 2), dtype=np.int64).astype(np.uint64) * 2 + 1
    tids = [random_tid(rng) for _ in range(n)]
    start = rng.integers(-10 ** 15, 10 ** 15, size=n)
    start[: n // 2] = rng.integers(1_600_000_000_000, 1_800_000_000_000, size=n // 2)
    flags = rng.integers(0, 32, size=n).astype(np.uint8)
    # most messages fit the writer's 4 KB LDS staging buffer; some do not (direct path)
    contents = ['{"p":"' + "x" * int(rng.integers(0, 3000) if rng.random() > 0.05 else rng.integers(4000, 9000))
                + '"}' for _ in range(n)]
    causes = rng.integers(0, 2 ** 63, size=(n, 2), dtype=np.int64).astype(np.uint64)
    traces = ['{"t":"%d"}' % k for k in range(n)]
    return dict(invoker=inv, tmpl=tmpl, aid_words=aid, tids=tids, tid_start=start, flags=flags, contents=contents,
                causes=causes, traces=traces, n_topics=n_topics)


@pytest.mark.parametrize("seed,n,n_topics", [(1, 1, 1), (2, 300, 7), (3, 20000, 1000)])
def test_gpu_msg_random_vs_oracle(seed, n, n_topics):
    rng = np.random.default_rng(seed)
    ta = ['"action":{"path":"ns%d","name":"a%d"},"revision":null,"user":{"subject":"s%d"}' % (k, k, k)
          for k in range(50)]
    tb = ["[]" if k % 3 else '["x%d"]' % k for k in range(50)]
    T = {"a": ta, "b": tb}
    b = gpu_balancer(T, '{"asString":"7"}')
    B = random_batch(rng, n, n_topics, 50)
    g = b.serialize_activations(**B)
    o = O.serialize_activations(ta, tb, '{"asString":"7"}', **B)
    assert g[0] == o[0]
    for x, y in zip(g[1:], o[1:]):
        assert np.array_equal(x, y)


def test_gpu_msg_errors_and_capacity():
    b = gpu_balancer()
    B = batch_of(GOLD["cases"][4])
    with pytest.raises(OwgsError):
        b.serialize_activations(**{**B, "tmpl": [0, 0, 9, 0, 0]})
    with pytest.raises(OwgsError):
        b.serialize_activations(**{**B, "n_topics": 2})  # invoker 2 outside the topics
    with pytest.raises(OwgsError):
        b.serialize_activations(**{**B, "tids": ["a", b"\xe2\x82", "c", "d", "e"]})  # truncated UTF-8
    with pytest.raises(OwgsError) as e:
        b.serialize_activations(**B, cap=100)
    assert e.value.code == ERANGE
    out, off, order, topic = b.serialize_activations(**B)  # the context is still usable
    check(GOLD["cases"][4], out, off, order, topic)


def test_gpu_msg_device_pipeline_after_replay():
    """The engine's device-resident decisions feed the serialiser directly (no host round trip)."""
    import torch

    from openwhisk_amd import workload as W

    w = W.config("headline", n_activations=20_000, n_invokers=500)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed, device=0)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    inv, _, _ = b.replay(w.stream)
    na = len(w.actions)
    ta = ['"action":{"path":"%s","name":"a"},"revision":null,"user":{"subject":"u%d"}' % (a.path, k)
          for k, a in enumerate(w.actions)]
    tb = ["[]"] * na
    b.register_templates(ta, tb)
    rng = np.random.default_rng(4)
    n = len(inv)
    acts = np.asarray(w.stream.act, dtype=np.int32)
    B = dict(invoker=inv, tmpl=acts, aid_words=rng.integers(0, 2 ** 62, size=(n, 2)).astype(np.uint64),
             tids=["sid_%d" % k for k in range(n)], tid_start=np.arange(n) + 1_700_000_000_000,
             flags=np.zeros(n, np.uint8), n_topics=len(w.inv_ids))
    host = b.serialize_activations(**B)
    o = O.serialize_activations(ta, tb, '{"asString":"0"}', **B)
    assert host[0] == o[0]
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    tid_b = b"".join(s.encode() for s in B["tids"])
    tid_off = np.zeros(n + 1, np.int64)
    tid_off[1:] = np.cumsum([len(s) for s in B["tids"]])
    d = dict(inv=t(inv, np.int32), tmpl=t(acts, np.int32), aid=t(B["aid_words"].view(np.int64), np.int64),
             tid=t(np.frombuffer(tid_b, np.uint8), np.uint8), tid_off=t(tid_off, np.int64),
             start=t(B["tid_start"], np.int64), flags=t(B["flags"], np.uint8), zoff=t(np.zeros(n + 1), np.int64))
    cap = len(host[0])
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    topic = torch.empty(B["n_topics"] + 1, dtype=torch.int32, device=dev)
    P = lambda x: C.c_void_p(x.data_ptr())  # noqa: E731
    mb = owgs_msg_batch(n, P(d["inv"]), P(d["tmpl"]), P(d["aid"]), P(d["tid"]), P(d["tid_off"]), P(d["start"]),
                        P(d["flags"]), None, P(d["zoff"]), None, None, P(d["zoff"]))
    total, m = C.c_int64(0), C.c_int32(0)
    s = torch.cuda.current_stream().cuda_stream
    rc = b._L.owgs_serialize_activations_device(b._h, C.byref(mb), B["n_topics"], P(out), cap, P(off), P(order),
                                                P(topic), C.byref(total), C.byref(m), C.c_void_p(s))
    assert rc == 0
    assert total.value == cap and m.value == len(host[2])
    assert bytes(out.cpu().numpy()) == host[0]
    assert np.array_equal(topic.cpu().numpy(), host[3])
