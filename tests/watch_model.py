"""CPU model of the engine's NestedSemaphore handling after a slot-state reset (test infrastructure).

The HIP engine creates a concurrency entry only when an acquisition succeeds.  The reference also creates an empty
one on every failed concurrent try (`getOrElseUpdate`, NestedSemaphore.scala:61-62).  The two agree while every
release finds the entry of its own acquisition.  That stops holding once `updateCluster` (SCPB:561-584) throws the
slot state away with activations still in flight.  The engine then keeps a set W of *watched* pairs (invoker, fqn):

  d[p] = in-flight activations of p - operationCount of p's entry (0 when absent);  W = {p : d[p] > 0}

* reset (updateCluster / the slot test seam): d[p] = ops[p] + d_old[p] for every entry and every watched pair; the
  table is emptied;
* a publish run: decisions as always (no empty entries).  At its end, for every watched pair p that is absent from
  the table, Z[p] is set if a decision of p's fqn failed a try at p's invoker during the run: its walk passed that
  (usable) invoker before the step it took (every step for an overload fallback);
* a release of a watched pair: present -> RS.release(1, true) with a signed operationCount (removal clears Z);
  absent with Z -> the reference's empty entry takes it ({c = 1, ops = -1}); absent without Z -> NoSuchElement and
  d - 1 (the pair leaves W at 0).  Releases of other pairs are unchanged.

This module restates those rules in Python so tests/test_watch_model.py can check them against the literal oracle
(zombies=True) before (and independently of) the device kernels that implement them.
"""
from __future__ import annotations

import numpy as np

import oracle as O

HEALTHY = 0


def _rng_index(seed, seq, n):
    return O.rng_index(seed, seq, n)


class WatchModel:
    def __init__(self, ids, user_mem_bytes, status, mf, bf, rng_seed, min_mb=128):
        self.ids = np.asarray(ids)
        self.mem = np.asarray(user_mem_bytes, dtype=np.int64)
        self.status = np.asarray(status).copy()
        self.rng_seed = rng_seed
        self.min_mb = min_mb
        n = len(ids)
        mf = max(0.0, min(1.0, mf))
        bf = max(1.0 - mf, min(1.0, bf))
        import math
        self.nm = min(max(1, int(math.ceil(n * mf))), n)
        self.nb = min(max(1, int(math.floor(n * bf))), n)
        self.msteps = O.pairwise_coprime_numbers_until(max(1, int(math.ceil(n * mf))))
        self.bsteps = O.pairwise_coprime_numbers_until(max(1, int(math.floor(n * bf))))
        self.cluster = 1
        self.P = self._slots()
        self.T = {}        # (inv, key) -> [c, ops, R]
        self.W = {}        # (inv, key) -> [d, Z]
        self.D = {}        # action -> deepest walk step + 1 of this publish run
        self.actions = []  # (hash, key, mem, maxc, blackbox)
        self.stats = {"resurrected": 0, "nosuch_watched": 0, "z_set": 0}

    def _slots(self):
        return [max(self.min_mb * 1024 * 1024, int(m) // self.cluster) // (1024 * 1024) for m in self.mem]

    def register(self, h, key, mem, maxc, bb):
        self.actions.append((h, key, mem, maxc, bb))
        return len(self.actions) - 1

    def set_status(self, status):
        self.status = np.asarray(status).copy()

    # ------------------------------------------------------------------ walk
    def _pool(self, bb):
        n = self.nb if bb else self.nm
        base = len(self.ids) - n if bb else 0
        return n, base

    def _walk(self, a):
        h, key, mem, maxc, bb = self.actions[a]
        n, base = self._pool(bb)
        steps = self.bsteps if bb else self.msteps
        return n, base, h % n, steps[h % len(steps)]

    def publish(self, a, seq):
        h, key, mem, maxc, bb = self.actions[a]
        n, base = self._pool(bb)
        if n <= 0:
            return -1, 0
        if h < 0:  # Int.MinValue: home/step index negative -> throws before any try
            return -2, 0
        _, _, idx, step = self._walk(a)
        for s in range(n + 2):
            inv = int(self.ids[base + idx])
            if self.status[base + idx] == HEALTHY and self._try(inv, key, mem, maxc, False):
                if maxc > 1:
                    self.D[a] = max(self.D.get(a, 0), s + 1)
                return inv, 0
            idx = (idx + step) % n
        healthy = [int(self.ids[base + i]) for i in range(n) if self.status[base + i] == HEALTHY]
        if not healthy:
            return -1, 0
        r = healthy[_rng_index(self.rng_seed, seq, len(healthy))]
        self._try(r, key, mem, maxc, True)
        if maxc > 1:
            self.D[a] = n + 2
        return r, 1

    def _try(self, inv, key, mem, maxc, force):
        if maxc == 1:
            if force or self.P[inv] - mem >= 0:
                self.P[inv] -= mem
                return True
            return False
        e = self.T.get((inv, key))
        if e is not None and e[0] >= 1:
            e[0] -= 1
            e[1] += 1
            return True
        if force or self.P[inv] - mem >= 0:
            self.P[inv] -= mem
            if e is None:
                e = [0, 0, maxc]
                self.T[(inv, key)] = e
            self._rel(e, maxc - 1, False)
            return True
        return False

    @staticmethod
    def _rel(e, k, op_complete):
        e[1] += -1 if op_complete else 1
        nxt = e[0] + k
        if nxt % e[2] == 0:
            e[0] = nxt - e[2]
            return True
        e[0] = nxt
        return False

    def end_publish_run(self):
        """Z for watched pairs that are absent: did a decision of their fqn fail a try at their invoker?"""
        for p, w in self.W.items():
            if w[1] or p in self.T:
                continue
            inv, key = p
            for a, depth in self.D.items():
                if self.actions[a][1] != key:
                    continue
                n, base, home, step = self._walk(a)
                pos = inv - base
                if pos < 0 or pos >= n or self.status[base + pos] != HEALTHY:
                    continue
                idx = home
                for s in range(min(depth, n + 2)):
                    if idx == pos:
                        w[1] = True
                        self.stats["z_set"] += 1
                        break
                    idx = (idx + step) % n
                if w[1]:
                    break
        self.D = {}

    # ------------------------------------------------------------------ release
    def release(self, inv, a):
        """0 ok, 1 NoSuchElement, 2 overflow"""
        h, key, mem, maxc, bb = self.actions[a]
        if inv < 0 or inv >= len(self.P):
            return 0
        if maxc == 1:
            return self._mem_release(inv, mem)
        p = (inv, key)
        e = self.T.get(p)
        w = self.W.get(p)
        if e is None:
            if w is None or not w[1]:
                if w is not None:
                    self.stats["nosuch_watched"] += 1
                    w[0] -= 1
                    if w[0] == 0:
                        del self.W[p]
                return 1
            e = [0, 0, maxc]  # the reference's empty entry from a failed try
            self.T[p] = e
            self.stats["resurrected"] += 1
        if w is None:
            assert e[1] >= 1, "an unwatched entry always counts its own releases"
        memrel = self._rel(e, 1, True)
        f = self._mem_release(inv, mem) if memrel else 0
        if e[1] == 0 and f == 0:
            del self.T[p]
            if w is not None:
                w[1] = False
        return f

    def _mem_release(self, inv, mem):
        if self.P[inv] + mem > 0x7FFFFFFF:
            return 2
        self.P[inv] += mem
        return 0

    # ------------------------------------------------------------------ reset
    def update_cluster(self, size):
        size = max(1, size)
        if size == self.cluster:
            return
        keys = set(self.T) | set(self.W)
        nw = {}
        for p in keys:
            t = (self.T[p][1] if p in self.T else 0) + (self.W[p][0] if p in self.W else 0)
            if t > 0:
                nw[p] = [t, False]
        self.W = nw
        self.T = {}
        self.cluster = size
        self.P = self._slots()
