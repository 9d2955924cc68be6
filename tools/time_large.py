"""Rate of the large-state engine (owgs_seq.hip): contexts beyond the on-chip image -- pools of more invoker ids than
owgs_limits reports, or maxConcurrent beyond 4095 -- against the one-core oracle on the same stream.  Each repeat builds
a fresh context (outside the clock) and replays the stream through the host ABI (owgs_replay: copies in and out
included, so this is the PCIe-inclusive rate).  Prints one JSON line per workload, with bit-exactness.
  python tools/time_large.py [n_invokers ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [40_000]
n_act = int(os.environ.get("NACT", "200000"))
for n_inv in sizes:
    mem = int(os.environ.get("INV_MB", "16384"))  # 16 GiB invokers as the headline (1024: the overloaded test pools)
    extra = {"conc_frac": float(os.environ["CONC"])} if os.environ.get("CONC") else {}
    w = W.config("headline", n_invokers=n_inv, n_activations=n_act, user_memory_mb=mem, **extra)
    t = time.perf_counter()
    o_inv, o_fl, _ = O.state_for(w).replay(w.stream)
    cpu_s = time.perf_counter() - t
    ts, exact = [], True
    for rep in range(3):
        b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction,
                                             blackbox_fraction=w.blackbox_fraction, rng_seed=w.rng_seed)
        b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
        b.update_cluster(w.cluster_size)
        b.register_actions(w.actions)
        t = time.perf_counter()
        g_inv, g_fl, _ = b.replay(w.stream)
        ts.append(time.perf_counter() - t)
        exact &= bool(np.array_equal(g_inv, o_inv) and np.array_equal(g_fl, o_fl))
        st = b.stats()
        b.close()
    dt = min(ts)
    print(json.dumps({"workload": f"headline-shaped, {n_inv} invokers x {mem} MB" + (f", conc {extra['conc_frac']}" if extra else ""),
                      "n_invokers": n_inv, "activations": n_act, "releases": int(len(w.stream.rel_aid)),
                      "batches": int(w.stream.n_batches), "gpu_ms": round(dt * 1e3, 2),
                      "gpu_decisions_per_s": n_act / dt, "oracle_1core_ms": round(cpu_s * 1e3, 1),
                      "oracle_decisions_per_s": n_act / cpu_s, "bit_exact": exact,
                      "speculated": st.get("large_spec"), "decided_alone": st.get("large_alone"),
                      "cycles": st.get("large_cycles"),
                      "note": "host ABI (owgs_replay), copies in and out inside the clock"}), flush=True)
