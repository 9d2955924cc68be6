"""Diagnostic: first assignment mismatch of a build (OWGS_LIB) against the oracle on a named workload."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

name, n = sys.argv[1], int(sys.argv[2])
w = W.config(name, n_activations=n)
st = O.state_for(w)
o_inv, o_fl, o_rf = st.replay(w.stream)
for lib in sys.argv[3:]:
    os.environ["OWGS_LIB"] = lib
    import importlib
    import openwhisk_amd._lib as L
    importlib.reload(L)
    import openwhisk_amd.balancer as B
    importlib.reload(B)
    b = B.GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                           rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    g_inv, g_fl, g_rf = b.replay(w.stream)
    bad = np.nonzero(o_inv != g_inv)[0]
    print(lib, "mismatches", len(bad), "first", bad[:8].tolist(), b.stats(), flush=True)
    fb = np.nonzero(o_fl != g_fl)[0]
    if len(fb):
        print("  flag mismatches", len(fb), [(int(j), int(o_inv[j]), int(o_fl[j]), int(g_fl[j]), int(w.stream.act[j])) for j in fb[:10]], flush=True)
    if len(bad):
        i0 = int(bad[0])
        bs = np.searchsorted(w.stream.acq_off, i0, side="right") - 1
        print("  batch", bs, "batch start", int(w.stream.acq_off[bs]), "act", int(w.stream.act[i0]),
              "same-action lanes near:", [(int(j), int(o_inv[j]), int(g_inv[j])) for j in range(max(0, i0 - 300), min(n, i0 + 300))
                                          if w.stream.act[j] == w.stream.act[i0]][:12], flush=True)
