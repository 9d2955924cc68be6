"""Why the shim path's tail latency is what it is: the headline stream through owgs_process_batch in
512-job drains (the bench's fused leg), with the resident engine's counters read after EVERY call, so each call's
latency can be set against its own work -- releases, publishes, decisions decided alone, walk rounds, staging,
cleanups and relaunches.  Prints the median call and the slowest 1 % side by side, as JSON."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import bench  # noqa: E402
import oracle as O  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="headline")
ap.add_argument("--drain", type=int, default=512)
ap.add_argument("--jobs", type=int, default=480_000)
a = ap.parse_args()
w = W.config(a.config)
o_inv, _, _ = O.state_for(w).replay(w.stream)
s = w.stream
kinds, ids = [], []
for b in range(s.n_batches):
    r = s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]]
    kinds.append(np.concatenate([np.zeros(len(r), np.int8), np.ones(int(s.acq_off[b + 1] - s.acq_off[b]), np.int8)]))
    ids.append(np.concatenate([r, np.arange(s.acq_off[b], s.acq_off[b + 1])]))
kind, ids = np.concatenate(kinds), np.concatenate(ids).astype(np.int64)
act = np.ascontiguousarray(s.act, np.int32)
g = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
g.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
g.update_cluster(w.cluster_size)
g.register_actions(w.actions)
inv = np.full(len(act), -9, np.int32)
rows = []
prev = g.resident_stats()
fill_prev = g.resident_table_fill()
n = min(a.jobs, len(ids))
for c0 in range(0, n, a.drain):
    c1 = min(c0 + a.drain, n)
    ns, npub = bench._fused_drain(g, kind, ids, act, inv, o_inv, c0, c1)
    st = g.resident_stats()
    fill = g.resident_table_fill()
    d = {k: st[k] - prev[k] for k in st if k not in ("alive", "last_call_ns")}
    d["us"] = ns * 1e-3
    d["releases"] = int((kind[c0:c1] == 0).sum())
    d["publishes"] = npub
    d["host_build_us"] = (fill[2] - fill_prev[2]) * 1e-3
    d["host_wait_us"] = (fill[3] - fill_prev[3]) * 1e-3
    rows.append(d)
    prev, fill_prev = st, fill
done = inv != -9
exact = bool(np.array_equal(inv[done], o_inv[done]))
lat = np.array([r["us"] for r in rows])
order = np.argsort(lat)
k = max(1, len(rows) // 100)
slow = [rows[i] for i in order[-k:]]
mid = [rows[i] for i in order[len(order) // 2 - k // 2: len(order) // 2 - k // 2 + k]]
keys = [x for x in rows[0] if isinstance(rows[0][x], (int, float))]


def mean(rs):
    return {x: round(float(np.mean([r[x] for r in rs])), 2) for x in keys}


lo, hi = np.percentile(lat, 97), np.percentile(lat, 99.5)
band = [r for r in rows if lo <= r["us"] <= hi and r["launches"] == 0 and r["chained"] == 0]
print(json.dumps({"config": a.config, "drain": a.drain, "calls": len(rows), "bit_exact": exact,
                  "p97_p995_band_no_relaunch": mean(band) if band else None, "band_calls": len(band),
                  "p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
                  "median_calls": mean(mid), "slowest_1pct": mean(slow),
                  "slowest_calls_index": [int(i) for i in order[-k:]],
                  "rows": [[round(r["us"], 1), r["decided_alone"], r["validation_passes"], r["launches"], r["chained"],
                            r["releases"], r["publishes"]] for r in rows],
                  "corr_us_vs": {x: round(float(np.corrcoef(lat, [r[x] for r in rows])[0, 1]), 3)
                                 for x in keys if x != "us" and np.std([r[x] for r in rows]) > 0}}))
