"""Diagnostic: the resident engine's per-call counters (owgs_resident_stats, balancer._RES_PROF) at given drain sizes:
where a served owgs_process_batch call's engine cycles go (speculation, validation, decisions made alone, ...).
Drives the headline shard's stream through owgs_process_batch as bench.shim_path does (fused mode), bit-exact check
against the oracle per call.  Prints one JSON line per drain size with per-call means."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402
from openwhisk_amd.balancer import _RES_PROF  # noqa: E402

drains = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,512").split(",")]
calls = int(os.environ.get("CALLS", "600"))
w = W.config(os.environ.get("CONFIG", "headline"))
o_inv, _, _ = O.state_for(w).replay(w.stream)
s = w.stream
kind = np.concatenate([np.concatenate([np.zeros(int(s.rel_off[b + 1] - s.rel_off[b]), np.int8),
                                       np.ones(int(s.acq_off[b + 1] - s.acq_off[b]), np.int8)]) for b in range(s.n_batches)])
ids = np.concatenate([np.concatenate([s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]], np.arange(s.acq_off[b], s.acq_off[b + 1])])
                      for b in range(s.n_batches)]).astype(np.int64)
act = np.ascontiguousarray(s.act, np.int32)
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.update_cluster(w.cluster_size)
b.register_actions(w.actions)
b.snapshot()
L, h = b._L, b._h
p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
for drain in drains:
    b.restore()
    inv = np.full(len(act), -9, np.int32)
    lat, n_pub, exact = [], 0, True
    st0 = b.resident_stats()
    served0 = st0["served"]
    for k0 in range(0, min(len(ids), calls * drain), drain):
        k, x = kind[k0:k0 + drain], ids[k0:k0 + drain]
        cut = np.nonzero((k[1:] == 0) & (k[:-1] == 1))[0] + 1
        bounds = np.concatenate([[0], cut, [len(k)]])
        ri, ra, pubs, ro, po = [], [], [], [0], [0]
        for r0, r1 in zip(bounds[:-1], bounds[1:]):
            kk, xx = k[r0:r1], x[r0:r1]
            rel = xx[kk == 0]
            rinv = np.where(inv[rel] == -9, o_inv[rel], inv[rel])
            keep = rinv >= 0
            ri.append(rinv[keep]), ra.append(act[rel[keep]]), pubs.append(xx[kk == 1])
            ro.append(ro[-1] + int(keep.sum())), po.append(po[-1] + int((kk == 1).sum()))
        ri = np.ascontiguousarray(np.concatenate(ri + [np.zeros(1, np.int32)]), np.int32)
        ra = np.ascontiguousarray(np.concatenate(ra + [np.zeros(1, np.int32)]), np.int32)
        pubs = np.concatenate(pubs).astype(np.int64)
        pa = np.ascontiguousarray(np.concatenate([act[pubs], np.zeros(1, np.int32)]), np.int32)
        sq = np.ascontiguousarray(np.concatenate([pubs, [0]]).astype(np.uint64))
        ro, po = np.array(ro, np.int32), np.array(po, np.int32)
        o = np.zeros(len(pubs) + 1, np.int32)
        f = np.zeros(len(pubs) + 1, np.uint8)
        rf = np.zeros(len(ri), np.uint8)
        args = (h, len(ro) - 1, p(ro), p(ri), p(ra), p(rf), p(po), p(pa), p(sq), 0, p(o), p(f))
        t0 = time.perf_counter()
        rc = L.owgs_process_batch(*args)
        lat.append(time.perf_counter() - t0)
        assert rc == 0, L.owgs_last_error(h)
        inv[pubs] = o[:len(pubs)]
        exact &= bool(np.array_equal(o[:len(pubs)], o_inv[pubs]))
        n_pub += len(pubs)
    st1 = b.resident_stats()
    served = max(st1["served"] - served0, 1)
    n = len(lat)
    out = {"drain": drain, "calls": n, "served": st1["served"] - served0, "publishes_per_call": n_pub / n,
           "p50_us": round(float(np.median(lat) * 1e6), 1), "p99_us": round(float(np.percentile(lat, 99) * 1e6), 1),
           "decisions_per_s": n_pub / float(np.sum(lat)), "exact": exact,
           "per_served_call": {k2: round((st1[k2] - st0[k2]) / served, 1) for k2 in _RES_PROF}}
    print(json.dumps(out), flush=True)
