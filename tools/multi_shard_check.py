"""Controller shards of one cluster on one GPU: each shard replayed alone (sequential), then all shards concurrently
(one HIP stream each); prints per-shard engine time and bit-exactness against the oracle for both."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer, cluster  # noqa: E402

N_ACT = int(os.environ.get("N_ACT", "1000000"))
dev = torch.device("cuda", 0)
t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731


def shard(idx, n):
    w = cluster.shard_workload("headline", idx, n, n_activations=N_ACT)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed, device=0)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    b.snapshot()
    s = w.stream
    d = dict(acq=t(s.acq_off, np.int64), rel=t(s.rel_off, np.int64), act=t(s.act, np.int32),
             aid=t(s.rel_aid if len(s.rel_aid) else np.zeros(1), np.int64),
             out=torch.empty(len(s.act), dtype=torch.int32, device=dev),
             fl=torch.empty(len(s.act), dtype=torch.uint8, device=dev),
             rf=torch.empty(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev))
    st = torch.cuda.Stream()
    o = O.state_for(w)
    ref = o.replay(s)
    return dict(w=w, b=b, d=d, st=st, ref=ref, ref_perm=o.permits())


def launch(x):
    s, d, sp = x["w"].stream, x["d"], x["st"].cuda_stream
    x["b"].restore(sp)
    x["b"].replay_device(s.n_batches, d["acq"].data_ptr(), d["act"].data_ptr(), len(s.act), d["rel"].data_ptr(),
                         d["aid"].data_ptr(), len(s.rel_aid), s.seq_base, d["out"].data_ptr(), d["fl"].data_ptr(),
                         d["rf"].data_ptr(), sp)


def exact(x):
    o_inv, o_fl, o_rf = x["ref"]
    d = x["d"]
    return (np.array_equal(o_inv, d["out"].cpu().numpy()) and np.array_equal(o_fl, d["fl"].cpu().numpy())
            and np.array_equal(o_rf, d["rf"].cpu().numpy()[: len(o_rf)])
            and np.array_equal(x["ref_perm"], x["b"].permits()))


for n in [int(v) for v in (sys.argv[1:] or ["2", "4", "8"])]:
    xs = [shard(i, n) for i in range(n)]
    for i, x in enumerate(xs):
        launch(x)
        torch.cuda.synchronize()
        print(f"cluster {n} shard {i} alone: engine {x['b'].engine_ms():.2f} ms exact {exact(x)} "
              f"batches {x['w'].stream.n_batches} stats {x['b'].stats()}", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for x in xs:
        launch(x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"cluster {n} concurrent: wall {dt * 1e3:.1f} ms, engines "
          f"{[round(x['b'].engine_ms(), 1) for x in xs]}, exact {[exact(x) for x in xs]}, "
          f"{n * N_ACT / dt / 1e6:.1f} M decisions/s", flush=True)
