"""Diagnostic: replay a (small) workload on the GPU and print the first mismatches against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else None
w = W.config(name, n_activations=n)
st = O.state_for(w, zombies=False)
o_inv, o_fl, o_rf = st.replay(w.stream)
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.update_cluster(w.cluster_size)
b.register_actions(w.actions)
try:
    g_inv, g_fl, g_rf = b.replay(w.stream)
except Exception as e:  # noqa: BLE001
    print("replay error:", e)
    g_inv = np.zeros_like(o_inv)
bad = np.nonzero(o_inv != g_inv)[0]
print(name, "n", len(o_inv), "mismatches", len(bad), "stats", b.stats())
acq = w.stream.acq_off
for i in bad[:12]:
    bt = int(np.searchsorted(acq, i, side="right") - 1)
    print(f"  i={i} batch={bt} chunk_lane={(i - acq[bt]) % 256} act={w.stream.act[i]} oracle={o_inv[i]} gpu={g_inv[i]}")
