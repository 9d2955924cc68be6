"""Host-side mirror of the reference's balancer interface over the HIP engine (libowgs.so).

`GpuShardingContainerPoolBalancer` keeps the names, argument meaning and error behaviour of
ShardingContainerPoolBalancer / ShardingContainerPoolBalancerState
(core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/ShardingContainerPoolBalancer.scala, "SCPB")
for the scheduling hot path, batched: one call schedules or releases many activations with the sequential
semantics of calling the reference once per activation in array order.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import (ERANGE, FLAG_OVERLOAD, HEALTHY, NONE, OFFLINE, THROW_INDEX, UNHEALTHY, UNRESPONSIVE, OwgsError,
                   owgs_config)

__all__ = ["GpuShardingContainerPoolBalancer", "InvokerHealth", "Action", "NONE", "THROW_INDEX", "FLAG_OVERLOAD",
           "HEALTHY", "UNHEALTHY", "UNRESPONSIVE", "OFFLINE", "OwgsError"]

MB = 1024 * 1024


@dataclass(frozen=True)
class InvokerHealth:
    """InvokerHealth(InvokerInstanceId(id, userMemory), status) (LoadBalancer.scala:37-44)."""

    id: int
    user_memory_bytes: int
    status: int = HEALTHY


@dataclass(frozen=True)
class Action:
    """What publish() reads from an ExecutableWhiskActionMetaData + ActivationMessage (SCPB:260-276)."""

    namespace: str        # msg.user.namespace.name (invoking namespace, hashed)
    path: str             # action.fullyQualifiedName(false).asString ("ns/pkg/name", hashed)
    version: str = "0.0.1"
    mem_mb: int = 256     # action.limits.memory.megabytes
    max_concurrent: int = 1
    blackbox: bool = False  # action.exec.pull

    @property
    def key(self) -> str:  # fullyQualifiedName(true).asString: NestedSemaphore map key
        return f"{self.path}@{self.version}"


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _pack(strings: list[str]) -> tuple[bytes, np.ndarray]:
    enc = [s.encode("ascii") for s in strings]
    off = np.zeros(len(enc) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(b) for b in enc])
    return b"".join(enc), off


def _blob(items) -> tuple[np.ndarray, np.ndarray]:
    """str (UTF-8) or bytes items -> (byte buffer, int64 offsets[n + 1])."""
    enc = [x.encode("utf-8") if isinstance(x, str) else bytes(x) for x in items]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(b) for b in enc])
    return np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8), off


_RES_PROF = ("walk_rounds", "decisions", "stage_cycles", "release_cycles", "publish_cycles", "overflow_lookups",
             "cursor_walks", "bound_skips", "grouped_decisions", "validation_passes", "decided_alone",
             "alone_cycles", "speculation_cycles", "validation_cycles", "match_cycles", "plain_walk_cycles",
             "conc_walk_cycles", "insert_cycles", "conc_release_cycles", "prespec_chunks", "helper_cycles")
_NRP = len(_RES_PROF)


class GpuShardingContainerPoolBalancer:
    """One controller shard (SCPB:147-332) backed by the MI355X engine."""

    def __init__(self, managed_fraction: float = 0.9, blackbox_fraction: float = 0.1, min_memory_mb: int = 128,
                 cluster_size: int = 1, device: int = 0, rng_seed: int = 0):
        L = _lib.lib()
        cfg = owgs_config(managed_fraction, blackbox_fraction, min_memory_mb * MB, cluster_size, device, rng_seed)
        h = C.c_void_p()
        rc = L.owgs_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise OwgsError(rc, "owgs_create failed (is an MI355X visible?)")
        self._h = h
        self._L = L
        self.rng_seed = rng_seed

    def close(self):
        if getattr(self, "_h", None):
            self._L.owgs_destroy(self._h)
            self._h = None

    __del__ = close

    def _chk(self, rc: int) -> int:
        if rc < 0:
            raise OwgsError(rc, (self._L.owgs_last_error(self._h) or b"").decode())
        return rc

    # ------------------------------------------------------------------ state (SCPB:449-585)
    def update_invokers(self, invokers: list[InvokerHealth]):
        ids = np.array([i.id for i in invokers] or [0], dtype=np.int32)
        mem = np.array([i.user_memory_bytes for i in invokers] or [0], dtype=np.int64)
        st = np.array([i.status for i in invokers] or [0], dtype=np.uint8)
        self._chk(self._L.owgs_update_invokers(self._h, len(invokers), _p(ids), _p(mem), _p(st)))

    def update_invokers_arrays(self, ids, user_memory_bytes, status):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        mem = np.ascontiguousarray(user_memory_bytes, dtype=np.int64)
        st = np.ascontiguousarray(status, dtype=np.uint8)
        self._chk(self._L.owgs_update_invokers(self._h, len(ids), _p(ids), _p(mem), _p(st)))

    def update_cluster(self, new_size: int):
        self._chk(self._L.owgs_update_cluster(self._h, new_size))

    def _info(self):
        v = [C.c_int32() for _ in range(4)]
        self._chk(self._L.owgs_state_info(self._h, *[C.byref(x) for x in v]))
        return [x.value for x in v]

    @property
    def cluster_size(self) -> int:
        return self._info()[3]

    @property
    def managed_size(self) -> int:
        return self._info()[1]

    @property
    def blackbox_size(self) -> int:
        return self._info()[2]

    def _steps(self, pool):
        n = C.c_int32()
        self._chk(self._L.owgs_step_sizes(self._h, pool, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.int32)
        self._chk(self._L.owgs_step_sizes(self._h, pool, _p(out), n.value, None))
        return out[: n.value].tolist()

    # ------------------------------------------------------------------ completion path (CLB:148-166, 205-346)
    def health_events(self, invoker, kind, t_ms, user_memory, now_ms: int, apply: bool = False) -> None:
        """InvokerPool + InvokerActor FSMs (InvokerSupervision.scala:95-440) for a batch of supervision events in
        mailbox order; apply=True hands the status vector to updateInvokers (SCPB:226-227)."""
        inv = np.ascontiguousarray(invoker, dtype=np.int32)
        k = np.ascontiguousarray(kind, dtype=np.uint8)
        t = np.ascontiguousarray(t_ms, dtype=np.int64)
        m = np.ascontiguousarray(user_memory, dtype=np.int64)
        n = len(inv)
        if not (len(k) == len(t) == len(m) == n):
            raise ValueError("health_events: arrays of different lengths")
        self._chk(self._L.owgs_health_events(self._h, n, _p(inv) if n else None, _p(k) if n else None,
                                             _p(t) if n else None, _p(m) if n else None, int(now_ms), int(apply)))

    def health_read(self):
        """GetStatus (InvokerSupervision.scala:132): (status, userMemory, test actions of the last batch, ring, tick)."""
        n = C.c_int32(0)
        self._chk(self._L.owgs_health_read(self._h, 0, C.byref(n), None, None, None, None, None))
        m = n.value
        st = np.zeros(max(m, 1), np.uint8)
        mem = np.zeros(max(m, 1), np.int64)
        te = np.zeros(max(m, 1), np.int32)
        ring = np.zeros(max(m, 1), np.uint32)
        tick = np.zeros(max(m, 1), np.int64)
        self._chk(self._L.owgs_health_read(self._h, m, None, _p(st), _p(mem), _p(te), _p(ring), _p(tick)))
        return st[:m], mem[:m], te[:m], ring[:m], tick[:m]

    def register_templates(self, part_a: list[str], part_b: list[str]) -> int:
        """ActivationMessage invariant members per (action, identity): part A = '"action":..,"revision":..,"user":..',
        part B = the initArgs array.  Returns the first new template id."""
        ab, ao = _blob(part_a)
        bb, bo = _blob(part_b)
        first = C.c_int32(0)
        self._chk(self._L.owgs_register_templates(self._h, len(part_a), _p(ab), _p(ao), _p(bb), _p(bo),
                                                  C.byref(first)))
        return first.value

    def set_root_controller(self, json_value: str):
        b = json_value.encode()
        self._chk(self._L.owgs_set_root_controller(self._h, b, len(b)))

    def serialize_activations(self, invoker, tmpl, aid_words, tids: list[str], tid_start, flags, contents=None,
                              causes=None, traces=None, n_topics: int | None = None, cap: int | None = None):
        """ActivationMessage.serialize + the per-invoker fan-out of sendActivationToInvoker (Message.scala:51-70,
        CLB:175-198): (bytes, out_off, out_order, topic_start)."""
        from ._lib import owgs_msg_batch
        n = len(invoker)
        inv = np.ascontiguousarray(invoker, dtype=np.int32)
        tm = np.ascontiguousarray(tmpl, dtype=np.int32)
        aid = np.ascontiguousarray(aid_words, dtype=np.uint64).reshape(-1)
        tb, to = _blob(tids)
        ts = np.ascontiguousarray(tid_start, dtype=np.int64)
        fl = np.ascontiguousarray(flags, dtype=np.uint8)
        keep = [inv, tm, aid, tb, to, ts, fl]
        B = owgs_msg_batch(n, _p(inv), _p(tm), _p(aid), _p(tb), _p(to), _p(ts), _p(fl))
        if contents is not None:
            cb, co = _blob(contents)
            keep += [cb, co]
            B.content, B.content_off = _p(cb), _p(co)
        if causes is not None:
            cz = np.ascontiguousarray(causes, dtype=np.uint64).reshape(-1)
            keep.append(cz)
            B.cause = _p(cz)
        if traces is not None:
            rb, ro = _blob(traces)
            keep += [rb, ro]
            B.trace, B.trace_off = _p(rb), _p(ro)
        nt = int(n_topics if n_topics is not None else (inv.max() + 1 if n and inv.max() >= 0 else 0))
        off = np.zeros(n + 1, np.int64)
        order = np.zeros(max(n, 1), np.int32)
        topic = np.zeros(nt + 1, np.int32)
        total, m = C.c_int64(0), C.c_int32(0)
        if cap is None:  # size query first
            rc = self._L.owgs_serialize_activations(self._h, C.byref(B), nt, None, 0, _p(off), _p(order), _p(topic),
                                                    C.byref(total), C.byref(m))
            if rc not in (0, ERANGE):
                self._chk(rc)
            cap = total.value
        out = C.create_string_buffer(max(cap, 1))
        self._chk(self._L.owgs_serialize_activations(self._h, C.byref(B), nt, out, cap, _p(off), _p(order),
                                                     _p(topic), C.byref(total), C.byref(m)))
        mm = m.value
        return out.raw[:total.value], off[:mm + 1], order[:mm], topic

    def engine_ms(self) -> float:
        """Duration of the last engine kernel launch (HIP events on its stream)."""
        v = C.c_float(0)
        self._chk(self._L.owgs_engine_ms(self._h, C.byref(v)))
        return float(v.value)

    def resident_stats(self) -> dict:
        """owgs_process_batch's paths: calls the resident engine served, its launches, calls it refused untouched,
        calls the launch chain took, and whether a resident engine is live."""
        out = np.zeros(13 + 2 * _NRP, np.int64)
        n = self._L.owgs_resident_stats(self._h, _p(out), 13 + 2 * _NRP)
        if n < 0:
            self._chk(n)
        d = dict(zip(("served", "launches", "refused", "chained", "alive") + _RES_PROF + ("last_call_ns",),
                     (int(x) for x in out[:6 + _NRP])))
        d["life_exits"] = int(out[11 + 2 * _NRP])  # launches ended by the lifetime bound (OWGS_RES_LIFE_US)
        d["watch_calls"] = int(out[12 + 2 * _NRP])  # served calls while watched pairs existed
        return d

    def map_fill(self) -> dict:
        """The NestedSemaphore map's fill: live / deleted primary (LDS-image) entries, overflow entries and capacity."""
        v = [C.c_int32(0) for _ in range(4)]
        self._chk(self._L.owgs_map_fill(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("primary_live", "primary_deleted", "overflow_entries", "overflow_cap"), (x.value for x in v)))

    def resident_table_fill(self) -> tuple:
        """The largest primary-table fill (live + deleted entries) and deleted entries after a served resident call,
        and the host nanoseconds over served calls spent building them and waiting from bell to answer."""
        out = np.zeros(11 + 2 * _NRP, np.int64)
        self._chk(min(0, self._L.owgs_resident_stats(self._h, _p(out), 11 + 2 * _NRP)))
        return tuple(int(x) for x in out[7 + 2 * _NRP:11 + 2 * _NRP])

    def stream_mode_stats(self) -> dict | None:
        """The last replay's resident-engine counters when it ran in stream mode (OWGS_SPEC_REPLAY), else None."""
        out = np.zeros(7 + 2 * _NRP, np.int64)
        self._chk(min(0, self._L.owgs_resident_stats(self._h, _p(out), 7 + 2 * _NRP)))
        return dict(zip(_RES_PROF, (int(x) for x in out[7 + _NRP:]))) if out[6 + _NRP] else None

    def last_call_ns(self) -> int:
        """Duration of the last publish / release / process_batch call, timed inside the library (no ctypes cost)."""
        out = np.zeros(6 + _NRP, np.int64)
        self._L.owgs_resident_stats(self._h, _p(out), 6 + _NRP)
        return int(out[5 + _NRP])

    def set_health_tid(self, start_ms: int):
        """TransactionId.invokerHealth's start time (TransactionId.scala:225): health acks echo it."""
        self._chk(self._L.owgs_set_health_tid(self._h, start_ms))

    def track_activations(self, aids, actions, tickets):
        """setupActivation's activationSlots.getOrElseUpdate (CLB:148-166) for a batch: (ticket, existed)."""
        n = len(aids)
        buf = np.frombuffer(b"".join(a.encode("ascii") for a in aids) or b"\0", dtype=np.uint8)
        act = np.ascontiguousarray(actions, dtype=np.int32)
        tk = np.ascontiguousarray(tickets, dtype=np.int32)
        out = np.zeros(max(n, 1), dtype=np.int32)
        ex = np.zeros(max(n, 1), dtype=np.uint8)
        self._chk(self._L.owgs_track_activations(self._h, n, _p(buf), _p(act), _p(tk), _p(out), _p(ex)))
        return out[:n], ex[:n]

    def process_acks(self, msgs):
        """processAcknowledgement (CLB:205-232) for raw ack messages (bytes): (kind, invoker, ticket, flags)."""
        n = len(msgs)
        off = np.zeros(n + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(m) for m in msgs])
        buf = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
        kind = np.zeros(max(n, 1), dtype=np.uint8)
        inv = np.zeros(max(n, 1), dtype=np.int32)
        tk = np.zeros(max(n, 1), dtype=np.int32)
        fl = np.zeros(max(n, 1), dtype=np.uint8)
        self._chk(self._L.owgs_process_acks(self._h, n, _p(buf), _p(off), _p(kind), _p(inv), _p(tk), _p(fl)))
        return kind[:n], inv[:n], tk[:n], fl[:n]

    def complete_activations(self, aids, invokers, forced=None, system_error=None, health=None):
        """processCompletion (CLB:260-346) called directly (timeouts, JVM-parsed acks): (kind, ticket, flags)."""
        n = len(aids)
        buf = np.frombuffer(b"".join(a.encode("ascii") for a in aids) or b"\0", dtype=np.uint8)
        inv = np.ascontiguousarray(invokers, dtype=np.int32)
        z = np.zeros(n, dtype=np.uint8)
        f = ((np.asarray(forced if forced is not None else z, dtype=np.uint8) & 1)
             | (np.asarray(system_error if system_error is not None else z, dtype=np.uint8) & 1) << 1
             | (np.asarray(health if health is not None else z, dtype=np.uint8) & 1) << 2).astype(np.uint8)
        f = np.ascontiguousarray(f if n else np.zeros(1, np.uint8))
        kind = np.zeros(max(n, 1), dtype=np.uint8)
        tk = np.zeros(max(n, 1), dtype=np.int32)
        fl = np.zeros(max(n, 1), dtype=np.uint8)
        self._chk(self._L.owgs_complete_activations(self._h, n, _p(buf), _p(inv), _p(f), _p(kind), _p(tk), _p(fl)))
        return kind[:n], tk[:n], fl[:n]

    def activations_live(self) -> int:
        v = C.c_int64()
        self._chk(self._L.owgs_activations_live(self._h, C.byref(v)))
        return v.value

    def pairwise_coprime_numbers_until(self, x: int) -> list:
        """ShardingContainerPoolBalancer.pairwiseCoprimeNumbersUntil (SCPB:379-384), computed by owgs_coprime_kernel."""
        n = C.c_int32()
        self._chk(self._L.owgs_pairwise_coprime(self._h, x, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.int32)
        self._chk(self._L.owgs_pairwise_coprime(self._h, x, _p(out), n.value, None))
        return out[: n.value].tolist()

    @property
    def managed_step_sizes(self):
        return self._steps(0)

    @property
    def blackbox_step_sizes(self):
        return self._steps(1)

    def permits(self) -> np.ndarray:
        """availablePermits of every NestedSemaphore in invokerSlots."""
        n = C.c_int32()
        self._chk(self._L.owgs_read_permits(self._h, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.int32)
        self._chk(self._L.owgs_read_permits(self._h, _p(out), n.value, None))
        return out[: n.value]

    def concurrent_state(self, invoker: int, key: int):
        """NestedSemaphore(invoker).concurrentState(key) -> (availablePermits, counter) or None."""
        c, o = C.c_int32(), C.c_int32()
        r = self._chk(self._L.owgs_read_concurrent(self._h, invoker, key, C.byref(c), C.byref(o)))
        return (c.value, o.value) if r == 1 else None

    def set_slots(self, permits):
        p = np.ascontiguousarray(permits, dtype=np.int32)
        self._chk(self._L.owgs_set_slots(self._h, len(p), _p(p) if len(p) else None))

    def set_pool(self, pool: int, invokers: list[tuple[int, int]]):
        ids = np.array([i for i, _ in invokers] or [0], dtype=np.int32)
        st = np.array([s for _, s in invokers] or [0], dtype=np.uint8)
        self._chk(self._L.owgs_set_pool(self._h, pool, len(invokers), _p(ids), _p(st)))

    # ------------------------------------------------------------------ actions
    def register_actions(self, actions: list[Action]) -> tuple[np.ndarray, np.ndarray]:
        """Returns (action handles, generateHash values computed on the GPU)."""
        n = len(actions)
        nsb, nso = _pack([a.namespace for a in actions])
        pb, po = _pack([a.path for a in actions])
        kb, ko = _pack([a.key for a in actions])
        mem = np.array([a.mem_mb for a in actions], dtype=np.int32)
        mc = np.array([a.max_concurrent for a in actions], dtype=np.int32)
        bb = np.array([1 if a.blackbox else 0 for a in actions], dtype=np.uint8)
        out = np.zeros(max(n, 1), dtype=np.int32)
        hs = np.zeros(max(n, 1), dtype=np.int32)
        nsb_a = np.frombuffer(nsb or b"\0", dtype=np.uint8)
        pb_a = np.frombuffer(pb or b"\0", dtype=np.uint8)
        kb_a = np.frombuffer(kb or b"\0", dtype=np.uint8)
        self._chk(self._L.owgs_register_actions(self._h, n, _p(nsb_a), _p(nso), _p(pb_a), _p(po), _p(kb_a), _p(ko),
                                                _p(mem), _p(mc), _p(bb), _p(out), _p(hs)))
        return out[:n], hs[:n]

    def release_actions(self, handles) -> None:
        """Drop action handles no later call names (owgs_release_actions): their ids and unused fqn@version keys are
        reused by later registrations."""
        h = np.ascontiguousarray(handles, dtype=np.int32)
        self._chk(self._L.owgs_release_actions(self._h, len(h), _p(h if len(h) else np.zeros(1, np.int32))))

    def key_id(self, action: int) -> int:
        return self._chk(self._L.owgs_key_id(self._h, action))

    # ------------------------------------------------------------------ hot path
    def publish(self, actions, seq=None, seq_base: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """Scheduling half of publish (SCPB:257-290) for each activation, in order.
        Returns (invoker ids | NONE | THROW_INDEX, flags with bit0 = overload)."""
        a = np.ascontiguousarray(actions, dtype=np.int32)
        n = len(a)
        out = np.zeros(max(n, 1), dtype=np.int32)
        fl = np.zeros(max(n, 1), dtype=np.uint8)
        sq = None if seq is None else np.ascontiguousarray(seq, dtype=np.uint64)
        self._chk(self._L.owgs_publish_batch(self._h, n, _p(a), None if sq is None else _p(sq), seq_base, _p(out),
                                             _p(fl)))
        return out[:n], fl[:n]

    def release_invoker(self, invokers, actions) -> np.ndarray:
        """releaseInvoker (SCPB:327-331) per completion; returns release flags."""
        inv = np.ascontiguousarray(invokers, dtype=np.int32)
        a = np.ascontiguousarray(actions, dtype=np.int32)
        fl = np.zeros(max(len(a), 1), dtype=np.uint8)
        self._chk(self._L.owgs_release_batch(self._h, len(a), _p(inv), _p(a), _p(fl)))
        return fl[: len(a)]

    def process_batch(self, rel_off, rel_invokers, rel_actions, pub_off, pub_actions, seq=None, seq_base: int = 0):
        """One drained batch of the shim's batching thread (owgs_process_batch): for each run r, releaseInvoker for
        the completions [rel_off[r], rel_off[r+1]) then publish for [pub_off[r], pub_off[r+1]).  Returns
        (invoker ids, overload flags, release flags)."""
        ro = np.ascontiguousarray(rel_off, dtype=np.int32)
        po = np.ascontiguousarray(pub_off, dtype=np.int32)
        ri = np.ascontiguousarray(rel_invokers, dtype=np.int32)
        ra = np.ascontiguousarray(rel_actions, dtype=np.int32)
        pa = np.ascontiguousarray(pub_actions, dtype=np.int32)
        nr, npub = int(ro[-1]), int(po[-1])
        out = np.zeros(max(npub, 1), dtype=np.int32)
        fl = np.zeros(max(npub, 1), dtype=np.uint8)
        rf = np.zeros(max(nr, 1), dtype=np.uint8)
        sq = None if seq is None else np.ascontiguousarray(seq, dtype=np.uint64)
        z = np.zeros(1, np.int32)
        self._chk(self._L.owgs_process_batch(self._h, len(ro) - 1, _p(ro), _p(ri if nr else z), _p(ra if nr else z),
                                             _p(rf), _p(po), _p(pa if npub else z), None if sq is None else _p(sq),
                                             seq_base, _p(out), _p(fl)))
        return out[:npub], fl[:npub], rf[:nr]

    def schedule(self, max_concurrent, key, slots, index, step, pool=0, seq=None):
        """ShardingContainerPoolBalancer.schedule(maxConcurrent, fqn, invokers(pool), dispatched, slots, index, step)
        for arrays of calls (SCPB:398-436).  Scalars are broadcast.  Returns (ids, flags)."""
        n = max(np.size(x) for x in (max_concurrent, key, slots, index, step, pool, 1 if seq is None else seq))
        b = lambda x, dt: np.ascontiguousarray(np.broadcast_to(np.asarray(x, dtype=dt), (n,)))  # noqa: E731
        pl, ix, st = b(pool, np.uint8), b(index, np.int32), b(step, np.int32)
        mm, mc, ky = b(slots, np.int32), b(max_concurrent, np.int32), b(key, np.int32)
        sq = None if seq is None else b(seq, np.uint64)
        out = np.zeros(n, dtype=np.int32)
        fl = np.zeros(n, dtype=np.uint8)
        self._chk(self._L.owgs_schedule_walks(self._h, n, _p(pl), _p(ix), _p(st), _p(mm), _p(mc), _p(ky),
                                              None if sq is None else _p(sq), _p(out), _p(fl)))
        return out, fl

    def replay(self, stream) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Replay a workload.Stream with host buffers."""
        acq = np.ascontiguousarray(stream.acq_off, dtype=np.int64)
        rel = np.ascontiguousarray(stream.rel_off, dtype=np.int64)
        act = np.ascontiguousarray(stream.act, dtype=np.int32)
        aid = np.ascontiguousarray(stream.rel_aid, dtype=np.int64)
        n, nr = len(act), len(aid)
        out = np.zeros(max(n, 1), dtype=np.int32)
        fl = np.zeros(max(n, 1), dtype=np.uint8)
        rf = np.zeros(max(nr, 1), dtype=np.uint8)
        self._chk(self._L.owgs_replay(self._h, len(acq) - 1, _p(acq), _p(act), _p(rel), _p(aid if nr else
                                      np.zeros(1, np.int64)), int(stream.seq_base), _p(out), _p(fl), _p(rf)))
        return out[:n], fl[:n], rf[:nr]

    def replay_device(self, n_batches, acq_off, act, n_act, rel_off, rel_aid, n_rel, seq_base, out_inv, out_flags,
                      rel_flags, stream=None):
        """Replay with HBM-resident buffers given as device addresses (ints, e.g. torch tensor.data_ptr())."""
        vp = lambda x: C.c_void_p(int(x)) if x else None  # noqa: E731
        self._chk(self._L.owgs_replay_device(self._h, n_batches, vp(acq_off), vp(act), n_act, vp(rel_off),
                                             vp(rel_aid), n_rel, seq_base, vp(out_inv), vp(out_flags), vp(rel_flags),
                                             vp(stream)))

    def replay_device_span(self, a_beg, a_end, r_beg, r_end, act, rel_aid, seq_base, out_inv, out_flags, rel_flags,
                           stream=None):
        """One batch of a device-resident stream (owgs_replay_device_span): releases rel_aid[r_beg:r_end] of
        activations decided by earlier calls, then publishes act[a_beg:a_end]; whole-stream device addresses."""
        vp = lambda x: C.c_void_p(int(x)) if x else None  # noqa: E731
        self._chk(self._L.owgs_replay_device_span(self._h, int(a_beg), int(a_end), int(r_beg), int(r_end), vp(act),
                                                  vp(rel_aid), int(seq_base), vp(out_inv), vp(out_flags),
                                                  vp(rel_flags), vp(stream)))

    def replay_device_group(self, acq_off, rel_off, act, rel_aid, seq_base, out_inv, out_flags, rel_flags,
                            status=None, status_stride=0, n_status=0, stream=None):
        """Consecutive batches of a device-resident stream in one engine launch (owgs_replay_device_group):
        acq_off / rel_off are the group's host offsets (n_batches + 1 each, whole-stream indices); status (device
        address, optional): per batch a row of n_status InvokerState codes applied before the batch."""
        vp = lambda x: C.c_void_p(int(x)) if x else None  # noqa: E731
        ao = np.ascontiguousarray(acq_off, dtype=np.int64)
        ro = np.ascontiguousarray(rel_off, dtype=np.int64)
        self._chk(self._L.owgs_replay_device_group(self._h, len(ao) - 1, _p(ao), _p(ro), vp(act), vp(rel_aid),
                                                   int(seq_base), vp(out_inv), vp(out_flags), vp(rel_flags),
                                                   vp(status), int(status_stride), int(n_status), vp(stream)))

    @staticmethod
    def replay_device_multi(shards, stream=None):
        """Several controller shards in ONE engine launch (owgs_replay_device_multi, one workgroup per shard).
        `shards` = [(balancer, (n_batches, acq_off, act, n_act, rel_off, rel_aid, n_rel, seq_base, out_inv,
        out_flags, rel_flags)), ...] with device addresses as in replay_device."""
        from ._lib import owgs_replay_io

        k = len(shards)
        ios = (owgs_replay_io * k)()
        for j, (_, a) in enumerate(shards):
            ios[j] = owgs_replay_io(*[int(x) if x else 0 for x in a])
        hs = (C.c_void_p * k)(*[b._h for b, _ in shards])
        b0 = shards[0][0]
        b0._chk(b0._L.owgs_replay_device_multi(hs, k, ios, C.c_void_p(int(stream)) if stream else None))

    def snapshot(self):
        self._chk(self._L.owgs_snapshot(self._h))

    def restore(self, stream=None):
        self._chk(self._L.owgs_restore(self._h, C.c_void_p(int(stream)) if stream else None))

    def update_health_device(self, n: int, status_dev_ptr: int, stream=None):
        self._chk(self._L.owgs_update_health_device(self._h, n, C.c_void_p(int(status_dev_ptr)),
                                                    C.c_void_p(int(stream)) if stream else None))

    def selftest(self):
        self._chk(self._L.owgs_selftest(self._h))

    def stats(self) -> dict:
        out = (C.c_uint64 * 48)()
        self._chk(self._L.owgs_read_stats(self._h, out, 48))
        d = {"passes": out[0], "probes": out[1], "fallbacks": out[2], "long_walks": out[3], "chunks": out[4],
             "stops": out[5], "general_probes": out[6], "general_lanes": out[7], "redecided": out[31] & 0xFFFFFFFF}
        if out[31] >> 32:
            d["redecided_prewalk"] = out[31] >> 32
        if out[46] or out[47]:  # large-state engine: decisions kept from its group speculation / decided alone
            d["large_spec"], d["large_alone"] = out[46], out[47]
            d["large_cycles"] = {"releases": out[40], "speculation": out[41], "kept": out[42], "alone": out[43]}
        if any(out[28:31]) and not any(out[8:16]):  # -DOWGS_EXT_PROF build: in-pass re-decision costs
            d["redecide"] = {"cycles": out[28], "walk_rounds": out[29], "scans": out[30], "setup": out[20], "walk": out[21],
                             "apply": out[22], "scan": out[23]}
        if any(out[8:16]):
            names = ["batch", "chunk_start", "speculate", "tables_buckets", "validate", "commit", "worst_hot", "worst_lane"]
            d["cycles"] = {k: out[8 + i] for i, k in enumerate(names)}
            # profile build: slots 6/7 hold the cycles of the first and of the later passes of the chunks
            d["cycles"]["first_passes"] = d.pop("general_probes")
            d["cycles"]["later_passes"] = d.pop("general_lanes")
            walk = ["worst_long", "long_walks_worst_wave", "long_rounds", "conc_long", "conc_long_rounds",
                    "full_walks", "full_walk_rounds", "hot_rounds", "cyc_rounds_c1", "cyc_rounds_conc",
                    "worst_scan_push", "worst_barrier8", "worst_queue"]
            d["walks"] = {k: out[16 + i] for i, k in enumerate(walk[:10])}
            d["walks"].update({k: out[28 + i] for i, k in enumerate(walk[10:])})
            d["cycles"]["rel_sweep"] = out[26]
            d["cycles"]["ct_rebuild"] = out[27]
            d["kernel_cycles"] = {"state_load": out[40], "batches": out[41], "write_back": out[42]}
        return d
