"""Diagnostic: per-phase engine cycles (OWGS_LIB=openwhisk_amd/libowgs_prof.so) for several workloads."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

configs = sys.argv[1:] or ["headline", "c2", "c3", "c4"]
for spec in configs:  # "name" or "name:shard/n_shards" (one controller shard of a clusterSize-n cluster)
    name, _, sh = spec.partition(":")
    shard, n_shards = (int(x) for x in sh.split("/")) if sh else (0, 1)
    n = int(os.environ["NACT"]) if os.environ.get("NACT") else None
    w = W.config(name, n_activations=n, shard=shard, n_shards=n_shards)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    b.snapshot()
    b.replay(w.stream)
    reps = int(os.environ.get("REPS", "5"))
    ts = []
    for _ in range(reps):  # min over repeats: single replays vary by a few percent
        b.restore()
        t = time.perf_counter()
        b.replay(w.stream)
        ts.append(time.perf_counter() - t)
    dt = min(ts)
    st = b.stats()
    cyc = st.pop("cycles", {})
    tot = sum(cyc.values()) or 1
    print(f"{spec}: n={w.n_activations} batches={w.stream.n_batches} {dt*1e3:.1f} ms (min of {reps}; median "
          f"{sorted(ts)[len(ts) // 2]*1e3:.1f})  {w.n_activations/dt:.3g}/s  {st}")
    print("   cycles/activation:", {k: round(v / w.n_activations, 1) for k, v in cyc.items()},
          "share:", {k: round(v / tot, 3) for k, v in cyc.items()})
