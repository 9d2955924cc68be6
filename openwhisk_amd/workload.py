"""Synthetic activation streams (bench + parity tests).

A stream is a sequence of batches.  Batch b first releases activations of earlier batches (completion acks,
CLB:260-346 -> releaseInvoker SCPB:327-331), then publishes its own activations in order (SCPB:257-290).  Every
activation completes a geometric number (>= 1, mean D) of batches after it was published, so the shard runs in a
steady state whose in-flight memory is `load` x its usable capacity.  Action popularity is Zipf(s) over invocation
keys (invoking namespace, action), memory limits are drawn per action, a fraction of actions are concurrent
(maxConcurrent 2..500, NestedSemaphore slots) and a fraction are blackbox (action.exec.pull -> blackbox pool).

Configs (BASELINE.json "configs"):
  c1        10 managed invokers x 2000 MB, one 256 MB action, 10k activations (ShardingContainerPoolBalancerTests
            harness shape, T-SCPB:414-497)
  c2        1k invokers x 16 GiB, 10k actions / 1k namespaces, Zipf 1.0, 128..2048 MB, 1M activations in
            capacity-calibrated batches (~5.3k: each batch's releases and publishes keep the pool near its capacity)
  c2_64k    c2 in batches of 64k activations, as SURVEY 8(d) words configs[1]: releases come only between batches, so
            each batch fills the pool within its first few thousand activations and the rest fall back (SCPB:417-424)
  c3        10k invokers, 10 % unhealthy/offline, 10 % blackbox actions, load 1.2 x capacity (overload fallback)
  c4        c2 + 30 % concurrent actions (maxConcurrent 2..500) with completion releases
  headline  10k invokers x 16 GiB, 1M activations per shard, Zipf 1.0, 128..2048 MB, 10 % blackbox, 20 % concurrent,
            2 % unhealthy, clusterSize = number of shards (one shard per GPU, SCPB:485-499 / 561-584); all shards
            share invokers, health and actions, each has its own activation stream
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .balancer import HEALTHY, OFFLINE, UNHEALTHY, UNRESPONSIVE, Action

MB = 1024 * 1024
MEM_CHOICES = (128, 256, 512, 1024, 2048)


@dataclass
class Stream:
    act: np.ndarray       # int32 [n]   action handle (index into Workload.actions) of activation i
    acq_off: np.ndarray   # int64 [B+1] batch b publishes activations [acq_off[b], acq_off[b+1])
    rel_off: np.ndarray   # int64 [B+1] batch b first releases rel_aid[rel_off[b]:rel_off[b+1]]
    rel_aid: np.ndarray   # int64 [R]   activation ids (earlier batches)
    seq_base: int = 0     # activation i has seq = seq_base + i (overload RNG counter)

    @property
    def n_batches(self) -> int:
        return len(self.acq_off) - 1


@dataclass
class Workload:
    name: str
    inv_ids: np.ndarray
    inv_mem: np.ndarray    # bytes
    inv_status: np.ndarray
    managed_fraction: float
    blackbox_fraction: float
    actions: list
    stream: Stream
    cluster_size: int = 1
    rng_seed: int = 0
    info: dict = field(default_factory=dict)

    @property
    def n_activations(self) -> int:
        return len(self.stream.act)


def _zipf_sample(rng, n_keys, s, n):
    w = 1.0 / np.power(np.arange(1, n_keys + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n), side="right"), n_keys - 1).astype(np.int64)


def make_stream(rng, n_act, batch, delay_mean, n_keys_weights=None, keys=None):
    """Batches of `batch` activations; activation completes after 1 + Geometric batches (mean delay_mean)."""
    n_batches = max(1, -(-n_act // batch))
    acq_off = np.minimum(np.arange(n_batches + 1, dtype=np.int64) * batch, n_act)
    bidx = np.arange(n_act, dtype=np.int64) // batch
    p = 1.0 / max(delay_mean, 1.0)
    d = rng.geometric(p, size=n_act).astype(np.int64)  # >= 1
    rb = bidx + d
    keep = rb < n_batches
    aid = np.nonzero(keep)[0].astype(np.int64)
    rbk = rb[keep]
    order = np.lexsort((aid, rbk))
    rel_aid = aid[order]
    rel_off = np.zeros(n_batches + 1, dtype=np.int64)
    np.add.at(rel_off, rbk + 1, 1)
    rel_off = np.cumsum(rel_off)
    return Stream(act=keys.astype(np.int32), acq_off=acq_off, rel_off=rel_off, rel_aid=rel_aid)


def generate(name: str = "headline", n_invokers: int = 10_000, user_memory_mb: int = 16_384, n_actions: int = 10_000,
             n_namespaces: int = 1_000, zipf_s: float = 1.0, mem_choices=MEM_CHOICES, conc_frac: float = 0.2,
             conc_range=(2, 500), blackbox_frac: float = 0.1, unhealthy_frac: float = 0.02,
             shared_frac: float = 0.1, n_activations: int = 1_000_000, load: float = 0.9, delay_mean: float = 4.0,
             batch: int | None = None, managed_fraction: float = 0.9, blackbox_fraction: float = 0.1,
             cluster_size: int = 1, min_memory_mb: int = 128, seed: int = 0x0F15C005, rng_seed: int | None = None,
             fixed_actions: list | None = None, shard: int | None = None) -> Workload:
    """`seed` fixes the cluster (invokers, their health, the action universe and its popularity order), which every
    controller shard shares; `shard` (when given) seeds that controller's own activation stream."""
    rng = np.random.Generator(np.random.PCG64(seed))
    # ---- invokers (dense ids, as InvokerPool.registerInvoker pads them: InvokerSupervision.scala:191-207)
    inv_ids = np.arange(n_invokers, dtype=np.int32)
    inv_mem = np.full(n_invokers, user_memory_mb * MB, dtype=np.int64)
    inv_status = np.full(n_invokers, HEALTHY, dtype=np.uint8)
    n_bad = int(round(unhealthy_frac * n_invokers))
    if n_bad:
        bad = rng.choice(n_invokers, size=n_bad, replace=False)
        inv_status[bad] = rng.choice(np.array([UNHEALTHY, UNRESPONSIVE, OFFLINE], dtype=np.uint8), size=n_bad)
    # ---- actions / invocation keys
    if fixed_actions is not None:
        actions = list(fixed_actions)
    else:
        actions = []
        mem_a = rng.choice(np.array(mem_choices), size=n_actions)
        conc_a = np.where(rng.random(n_actions) < conc_frac,
                          rng.integers(conc_range[0], conc_range[1] + 1, size=n_actions), 1)
        bb_a = rng.random(n_actions) < blackbox_frac
        home_ns = rng.integers(0, n_namespaces, size=n_actions)
        for a in range(n_actions):
            ns = f"ns{home_ns[a]:05d}"
            path = f"{ns}/pkg{a % 7}/action{a:06d}"
            invokers_ns = [ns]
            if rng.random() < shared_frac:
                invokers_ns += [f"ns{x:05d}" for x in rng.integers(0, n_namespaces, size=rng.integers(1, 4))]
            for ins in invokers_ns:
                actions.append(Action(ins, path, "0.0.1", int(mem_a[a]), int(conc_a[a]), bool(bb_a[a])))
    n_keys = len(actions)
    perm = rng.permutation(n_keys)  # popularity rank -> key
    # ---- capacity-calibrated batch size
    slot_mb = max(min_memory_mb * MB, (user_memory_mb * MB) // max(cluster_size, 1)) // MB
    usable = int((inv_status == HEALTHY).sum())
    w = 1.0 / np.power(np.arange(1, n_keys + 1, dtype=np.float64), zipf_s)
    w /= w.sum()
    eff = np.array([a.mem_mb / a.max_concurrent for a in actions])[perm]
    mem_per_act = float((w * eff).sum())
    capacity = usable * slot_mb / max(mem_per_act, 1e-9)
    if batch is None:
        batch = max(1, int(load * capacity / delay_mean))
    srng = rng if shard is None else np.random.Generator(np.random.PCG64([seed, shard]))
    keys = perm[_zipf_sample(srng, n_keys, zipf_s, n_activations)]
    stream = make_stream(srng, n_activations, batch, delay_mean, keys=keys)
    info = dict(batch=batch, n_batches=stream.n_batches, capacity_activations=capacity, mem_per_activation=mem_per_act,
                slot_mb=int(slot_mb), usable=usable, n_keys=n_keys, load=load, delay_mean=delay_mean)
    return Workload(name, inv_ids, inv_mem, inv_status, managed_fraction, blackbox_fraction, actions, stream,
                    cluster_size, seed if rng_seed is None else rng_seed, info)


def config(name: str, n_activations: int | None = None, shard: int = 0, n_shards: int = 1, **kw) -> Workload:
    """Named BASELINE.json configs.  `n_activations` shrinks a config for fast parity tests.

    `n_shards` > 1 makes the workload controller shard `shard` of an `n_shards`-controller cluster for every config:
    clusterSize = n_shards (each slot holds 1/n_shards of every invoker, SCPB:485-499), the cluster (invokers, health,
    actions) shared, the activation stream and the overload RNG seed the shard's own."""
    if name == "c1":
        act = Action("invocationSpace", "testspace/testname", "0.0.1", 256, 1, False)
        base = dict(n_invokers=10, user_memory_mb=2000, unhealthy_frac=0.0, managed_fraction=1.0,
                    blackbox_fraction=0.0, fixed_actions=[act], n_activations=10_000, delay_mean=3.0, load=0.9,
                    seed=0x0F15C001)
    elif name == "c2":
        base = dict(n_invokers=1000, conc_frac=0.0, blackbox_frac=0.0, unhealthy_frac=0.0, seed=0x0F15C002)
    elif name == "c2_64k":  # configs[1] in SURVEY 8(d)'s literal batching: 64k activations per batch (overloaded)
        base = dict(n_invokers=1000, conc_frac=0.0, blackbox_frac=0.0, unhealthy_frac=0.0, seed=0x0F15C002,
                    batch=65_536)
    elif name == "c3":
        base = dict(n_invokers=10_000, conc_frac=0.0, blackbox_frac=0.1, unhealthy_frac=0.1, load=1.2,
                    seed=0x0F15C003)
    elif name == "c4":
        base = dict(n_invokers=1000, conc_frac=0.3, blackbox_frac=0.0, unhealthy_frac=0.0, seed=0x0F15C004)
    elif name in ("headline", "c5"):
        base = dict(n_invokers=10_000, conc_frac=0.2, blackbox_frac=0.1, unhealthy_frac=0.02,
                    seed=0x0F15C005, shard=shard, rng_seed=0x0F15C005 + shard, cluster_size=n_shards)
    else:
        raise ValueError(name)
    if name not in ("headline", "c5") and (n_shards > 1 or shard):
        base.update(shard=shard, rng_seed=base["seed"] + shard, cluster_size=n_shards)
    base.update(kw)
    if n_activations is not None:
        base["n_activations"] = n_activations
    return generate(name=name, **base)


# ------------------------------------------------------------------------------------------- completion acks
# Ack messages as the invoker's serializer writes them: CompletionMessage(...).serialize = jsonFormat4 compactPrint
# with fields transid, activationId, isSystemError, invoker (Message.scala:85-100, 204-216); InvokerInstanceId with
# its None options omitted and userMemory as ByteSize.toString "<n> MB" (InstanceId.scala:31-49, Size.scala:107-114);
# transid as [id, start] (TransactionId.scala:236-241).
TESTING_TID = ("sid_testing", 1700000000456)


def activation_ids(rng, n: int) -> list[str]:
    """ActivationId.generate(): a random UUID without dashes (32 lowercase hex chars, ActivationId.scala:77)."""
    hi = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64) * np.uint64(2) + rng.integers(0, 2, n).astype(np.uint64)
    lo = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64) * np.uint64(2) + rng.integers(0, 2, n).astype(np.uint64)
    return [f"{int(h):016x}{int(l):016x}" for h, l in zip(hi, lo)]


def completion_message(aid: str, instance: int, system_error: bool = False, tid=TESTING_TID,
                       user_memory_mb: int = 16384, unique_name: str | None = None) -> bytes:
    inv = '{"instance":%d%s,"userMemory":"%d MB"}' % (
        instance, (',"uniqueName":"%s"' % unique_name) if unique_name else "", user_memory_mb)
    return ('{"transid":["%s",%d],"activationId":"%s","isSystemError":%s,"invoker":%s}' % (
        tid[0], tid[1], aid, "true" if system_error else "false", inv)).encode("ascii")


def combined_message(aid: str, instance: int, user_memory_mb: int = 16384) -> bytes:
    """CombinedCompletionAndResultMessage after shrink (response = Left(activationId))."""
    return ('{"transid":["%s",%d],"response":"%s","isSystemError":false,"invoker":{"instance":%d,'
            '"userMemory":"%d MB"}}' % (TESTING_TID[0], TESTING_TID[1], aid, instance, user_memory_mb)).encode("ascii")


def ack_batch(rng, aids: list[str], invokers, health_start_ms: int, dup=0.05, unknown=0.03, health=0.02,
              out_of_range=0.02, combined=0.02, garbage=0.01, syserr=0.1):
    """Ack messages completing each (aid, invoker) once in a random order, mixed with the cases processCompletion
    distinguishes: duplicates (the second sees no entry), unknown ids, health acks, invoker ids outside the slots,
    combined messages (left to the JVM) and unparsable ones."""
    order = rng.permutation(len(aids))
    msgs = []
    for i in order:
        r = rng.random()
        if r < garbage:
            msgs.append(completion_message(aids[i], int(invokers[i]))[:-3])
            continue
        if r < garbage + combined:
            msgs.append(combined_message(aids[i], int(invokers[i])))
            continue
        inst = int(invokers[i]) if rng.random() >= out_of_range else int(rng.choice([-1, 99999, 2**31 - 1]))
        m = completion_message(aids[i], inst, bool(rng.random() < syserr))
        msgs.append(m)
        if rng.random() < dup:
            msgs.append(m)
        if rng.random() < unknown:
            msgs.append(completion_message(activation_ids(rng, 1)[0], inst))
        if rng.random() < health:
            msgs.append(completion_message(activation_ids(rng, 1)[0], inst, tid=("sid_invokerHealth", health_start_ms)))
    return msgs


def mutate(rng, m: bytes, k: int = 2) -> bytes:
    """Random byte-level edits of a message (parser fuzzing)."""
    b = bytearray(m)
    alphabet = b'{}[]",:\\ 0123456789-+.eEtrufalsn\t\nabcdefu\x01\xc3\xa9'
    for _ in range(k):
        op = rng.integers(0, 3)
        p = int(rng.integers(0, len(b) + 1))
        if op == 0 and b:
            del b[min(p, len(b) - 1)]
        elif op == 1:
            b.insert(p, alphabet[int(rng.integers(0, len(alphabet)))])
        elif b:
            b[min(p, len(b) - 1)] = alphabet[int(rng.integers(0, len(alphabet)))]
    return bytes(b)
