"""Diagnostic: the NestedSemaphore map's fill after a full replay of each workload (chunked engine): live and deleted
entries of the on-chip primary table (4,096 entries, new keys go to the HBM overflow past 3,840), entries in the HBM
overflow -- where map accesses cost HBM traffic (DESIGN.md 6, c4's write traffic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

for spec in (sys.argv[1:] or ["headline", "c2", "c4", "headline:0/8"]):
    cfg, _, sh = spec.partition(":")
    w = W.config(cfg, shard=int(sh.split("/")[0]), n_shards=int(sh.split("/")[1])) if sh else W.config(cfg)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    s = w.stream
    fills = []
    # batch by batch (host spans), the map's fill after each batch
    step = max(1, s.n_batches // 12)
    for b0 in range(0, s.n_batches, step):
        b1 = min(s.n_batches, b0 + step)
        sub = W.Stream(act=s.act[: s.acq_off[b1]], acq_off=s.acq_off[: b1 + 1], rel_off=s.rel_off[: b1 + 1],
                       rel_aid=s.rel_aid[: s.rel_off[b1]], seq_base=s.seq_base)
        if b0 == 0:
            b.snapshot()
        b.restore()
        b.replay(sub)
        fills.append((b1, b.map_fill()))
    peak = max(f["primary_live"] + f["overflow_entries"] for _, f in fills)
    print(json.dumps({"workload": spec, "batches": s.n_batches, "peak_entries": peak,
                      "fill_by_batch": [(k, f) for k, f in fills]}), flush=True)
