"""Host side of the configs[4] cadence (bench.py --health-churn): how long each library call of a batch takes on the
host (owgs_update_health_device, owgs_replay_device_span), to find calls that wait for the GPU -- the engine stream
then idles while the host prepares the next batch.  Prints per-call host microseconds (median, max, count > 200 us)
and the step's wall time against the GPU's kernel time."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

from openwhisk_amd import GpuShardingContainerPoolBalancer, cluster  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

n_shards = int(sys.argv[1]) if len(sys.argv) > 1 else 1
w = W.config("headline", n_shards=n_shards) if n_shards > 1 else W.config("headline")
dev = torch.device("cuda", 0)
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.update_cluster(w.cluster_size)
b.register_actions(w.actions)
b.snapshot()
s = w.stream
t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
d_act, d_aid = t(s.act, np.int32), t(s.rel_aid, np.int64)
d_out = torch.empty(len(s.act), dtype=torch.int32, device=dev)
d_fl = torch.empty(len(s.act), dtype=torch.uint8, device=dev)
d_rf = torch.empty(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)
health = [t(h, np.uint8) for h in cluster.health_schedule(w.inv_status, s.n_batches)]
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sp = stream.cuda_stream
res = {"restore": [], "health": [], "span": []}
walls = []
for step in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = time.perf_counter()
    b.restore(sp)
    res["restore"].append(time.perf_counter() - a)
    for k in range(s.n_batches):
        a = time.perf_counter()
        b.update_health_device(len(w.inv_status), health[k].data_ptr(), sp)
        res["health"].append(time.perf_counter() - a)
        a = time.perf_counter()
        b.replay_device_span(s.acq_off[k], s.acq_off[k + 1], s.rel_off[k], s.rel_off[k + 1], d_act.data_ptr(),
                             d_aid.data_ptr(), s.seq_base, d_out.data_ptr(), d_fl.data_ptr(), d_rf.data_ptr(), sp)
        res["span"].append(time.perf_counter() - a)
    torch.cuda.synchronize()
    walls.append(time.perf_counter() - t0)
out = {k: {"median_us": float(np.median(v) * 1e6), "max_us": float(np.max(v) * 1e6),
           "n_over_200us": int(np.sum(np.array(v) > 200e-6)), "n": len(v)} for k, v in res.items()}
slow = [i % s.n_batches for i, x in enumerate(res["span"]) if x > 200e-6]
print(json.dumps({"shards": n_shards, "batches": int(s.n_batches), "wall_ms": [round(x * 1e3, 2) for x in walls],
                  "calls": out, "slow_span_batches": slow[:40]}))
