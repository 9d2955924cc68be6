"""Run one engine replay of a workload (after one warm-up replay) -- target for rocprofv3 --pmc passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "headline"
w = W.config(name)
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.update_cluster(w.cluster_size)
b.register_actions(w.actions)
b.snapshot()
b.replay(w.stream)
b.restore()
b.replay(w.stream)
print(b.stats())
