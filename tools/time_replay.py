"""Median engine replay time (device-resident replay via the host API, excluding host transfers) per workload."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

reps = int(os.environ.get("REPS", "5"))
tag = os.environ.get("OWGS_LIB", "default").split("/")[-1]
for name in (sys.argv[1:] or ["headline", "c2", "c4"]):
    w = W.config(name, n_activations=None if name != "c3" else 300_000)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    b.snapshot()
    ts = []
    for _ in range(reps):
        b.restore()
        t = time.perf_counter()
        out, fl, rf = b.replay(w.stream)
        ts.append(time.perf_counter() - t)
    ms = float(np.median(ts)) * 1e3
    print(f"{tag:>18} {name:>9}: {ms:8.1f} ms  {w.n_activations / ms * 1e3:.3g} dec/s  {b.stats()}", flush=True)
