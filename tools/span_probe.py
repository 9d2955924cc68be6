"""Per-batch engine time of the headline stream replayed batch by batch (owgs_replay_device_span) under three health
regimes: static (no update), static re-applied before every batch, and the per-batch churn schedule."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from openwhisk_amd import GpuShardingContainerPoolBalancer, cluster  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

w = W.config("headline")
s = w.stream
dev = torch.device("cuda", 0)
t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                     rng_seed=w.rng_seed)
b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
b.register_actions(w.actions)
b.snapshot()
d_act, d_aid = t(s.act, np.int32), t(s.rel_aid, np.int64)
d_acq, d_rel = t(s.acq_off, np.int64), t(s.rel_off, np.int64)
d_out = torch.empty(len(s.act), dtype=torch.int32, device=dev)
d_fl = torch.empty(len(s.act), dtype=torch.uint8, device=dev)
d_rf = torch.empty(len(s.rel_aid), dtype=torch.uint8, device=dev)
churn = cluster.health_schedule(w.inv_status, s.n_batches)
d_static = t(w.inv_status, np.uint8)
d_churn = [t(churn[k], np.uint8) for k in range(s.n_batches)]
for mode in ("one_launch", "static", "static_reapplied", "churn", "churn_again"):
    b.restore()
    torch.cuda.synchronize()
    if mode == "one_launch":
        t0 = time.perf_counter()
        b.replay_device(s.n_batches, d_acq.data_ptr(), d_act.data_ptr(), len(s.act), d_rel.data_ptr(),
                        d_aid.data_ptr(), len(s.rel_aid), s.seq_base, d_out.data_ptr(), d_fl.data_ptr(),
                        d_rf.data_ptr())
        ms = [b.engine_ms()]
        print(mode, f"wall {1e3 * (time.perf_counter() - t0):.1f} ms engine {ms[0]:.2f} ms", b.stats(), flush=True)
        if os.environ.get("PROBE_CYCLES"):
            print(" one launch", b.stats().get("cycles"), flush=True)
        continue
    ms, st = [], []
    t0 = time.perf_counter()
    for k in range(s.n_batches):
        if mode == "static_reapplied":
            b.update_health_device(len(w.inv_status), d_static.data_ptr())
        elif mode.startswith("churn"):
            b.update_health_device(len(w.inv_status), d_churn[k].data_ptr())
        b.replay_device_span(s.acq_off[k], s.acq_off[k + 1], s.rel_off[k], s.rel_off[k + 1], d_act.data_ptr(),
                             d_aid.data_ptr(), s.seq_base, d_out.data_ptr(), d_fl.data_ptr(), d_rf.data_ptr())
        ms.append(b.engine_ms())
        st.append(b.stats()["passes"])
        if os.environ.get("PROBE_CYCLES") and mode == "static" and k in (1, 8, 16):
            print(" batch", k, b.stats().get("cycles"), flush=True)
    print(mode, f"wall {1e3 * (time.perf_counter() - t0):.1f} ms engine {sum(ms):.2f} ms", "per batch",
          [round(x, 2) for x in ms], "passes", st, flush=True)
