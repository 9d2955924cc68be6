"""Diagnostic: per-call pre-pass / engine kernel durations of small publish batches (the shim's drains), for a
rocprofv3 --kernel-trace run:  rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3
tools/prepass_probe.py [n_per_call] [calls]   (OWGS_DEAL / OWGS_CW select the pre-pass variants)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
w = W.config("headline", n_activations=n * calls)
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.update_cluster(w.cluster_size)
b.register_actions(w.actions)
act = w.stream.act
for k in range(calls):
    b.publish(act[k * n:(k + 1) * n], seq_base=k * n)
print("done", n, calls)
if os.environ.get("PROBE_STATS"):
    print(b.stats())
