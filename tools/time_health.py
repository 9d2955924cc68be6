"""Time owgs_health_events on the GPU: 10k invokers, batches of supervision events (pings every second from every
invoker + completion results), as a controller's health and ack feeds deliver them.  Prints one JSON line.
The ABI takes host buffers, so the time includes the H2D copy of the events and the host-side argument check."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402


def main(n_inv=10000, per_batch=1_000_000, batches=10):
    rng = np.random.default_rng(5)
    b = GpuShardingContainerPoolBalancer()
    t = 0
    evs = []
    for k in range(batches + 2):
        inv = rng.integers(0, n_inv, size=per_batch).astype(np.int32)
        inv[:n_inv] = np.arange(n_inv)
        kind = rng.choice(4, size=per_batch, p=[0.1, 0.8, 0.05, 0.05]).astype(np.uint8)
        kind[:n_inv] = 0
        ts = t + np.sort(rng.integers(0, 1000, size=per_batch)).astype(np.int64)
        mem = np.full(per_batch, 16 << 30, np.int64)
        t += 1000
        evs.append((inv, kind, ts, mem, t))
    for e in evs[:2]:
        b.health_events(*e)
    t0 = time.perf_counter()
    for e in evs[2:]:
        b.health_events(*e)
    dt = (time.perf_counter() - t0) / batches
    st = b.health_read()[0]
    print(json.dumps({"what": "owgs_health_events", "invokers": n_inv, "events_per_batch": per_batch,
                      "ms_per_batch": dt * 1e3, "events_per_s": per_batch / dt,
                      "status_counts": np.bincount(st, minlength=4).tolist()}), flush=True)


if __name__ == "__main__":
    main()
