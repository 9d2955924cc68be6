"""Diagnostic: why passes stop (OWGS_LIB=openwhisk_amd/variants/libowgs_why.so, a -DOWGS_STOP_REASONS build).

stats[6] counts the reason of each stopping lane in 12-bit fields (keep streams short enough: < 4096 per reason):
1 maxConcurrent == 1 lane does not fit, 2 concurrent fallback not first in its bucket, 3 concurrent lane does not fit,
4 concurrent lane after an earlier concurrent forced acquire of the pass, 5 shared fqn@version under another action.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

n = int(os.environ.get("NACT", "150000"))
for spec in sys.argv[1:] or ["headline", "c2", "c4", "headline:0/8"]:
    name, _, sh = spec.partition(":")
    shard, n_shards = (int(x) for x in sh.split("/")) if sh else (0, 1)
    w = W.config(name, n_activations=n, shard=shard, n_shards=n_shards)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    b.replay(w.stream)
    st = b.stats()
    v = int(st["general_probes"])
    why = {k + 1: (v >> (12 * k)) & 0xFFF for k in range(5)}
    print(f"{spec}: n={n} passes {st['passes']} chunks {st['chunks']} stops {st['stops']} reasons {why}", flush=True)
