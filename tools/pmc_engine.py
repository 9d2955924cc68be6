"""Target for rocprofv3 --pmc passes: one warm-up replay and one measured replay of the bench's workload (same
arguments as bench.py: --config, --n-activations, --cluster-size, --shard, --slots) on one GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402

args = bench.parse(sys.argv[1:])
n_ctl, shards = bench.cluster_geometry(args, 0, 1)
w = bench.shard_workload(args, shards[0], n_ctl)
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.update_cluster(w.cluster_size)
b.register_actions(w.actions)
b.snapshot()
b.replay(w.stream)
b.restore()
b.replay(w.stream)
print(b.stats(), flush=True)
