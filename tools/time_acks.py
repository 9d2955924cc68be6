"""Time the completion path on the GPU (owgs_process_acks_device): 1M tracked activations of the headline workload,
then one feed batch of 1M raw CompletionMessage records (~150 bytes each, inputs resident in HBM) parsed, looked up,
removed and released.  Prints one JSON line; per-kernel times come from rocprofv3 (tools/gpu_acks_prof.sh)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402


def main(n=1_000_000):
    rng = np.random.default_rng(3)
    w = W.config("headline", n_activations=100_000)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    b.set_health_tid(1_700_000_000_000)
    aids = W.activation_ids(rng, n)
    acts = rng.integers(0, len(w.actions), size=n).astype(np.int32)
    invs = rng.integers(0, len(w.inv_ids), size=n).astype(np.int32)
    msgs = [W.completion_message(a, int(i)) for a, i in zip(aids, invs)]
    blob = b"".join(msgs)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(np.frombuffer(blob + b"\0" * 16, np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    kind = torch.empty(n, dtype=torch.uint8, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    tk = torch.empty(n, dtype=torch.int32, device=dev)
    fl = torch.empty(n, dtype=torch.uint8, device=dev)
    P = lambda x: C.c_void_p(x.data_ptr())  # noqa: E731
    stream = torch.cuda.Stream()
    times = []
    for rep in range(4):
        b.track_activations(aids, acts, np.arange(n, dtype=np.int32))  # (re)insert the entries, outside the timing
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rc = b._L.owgs_process_acks_device(b._h, n, P(d_bytes), P(d_off), P(kind), P(inv), P(tk), P(fl),
                                           C.c_void_p(stream.cuda_stream))
        e1.record(stream)
        torch.cuda.synchronize()
        assert rc == 0, rc
        times.append(e0.elapsed_time(e1))
    k = kind.cpu().numpy()
    ms = float(np.median(times[1:]))
    print(json.dumps({"what": "owgs_process_acks_device", "messages": n, "bytes": int(off[-1]), "ms": ms,
                      "messages_per_s": n / (ms * 1e-3), "parse_GBps": off[-1] / (ms * 1e-3) / 1e9,
                      "released": int((k == 3).sum())}), flush=True)


if __name__ == "__main__":
    main()
