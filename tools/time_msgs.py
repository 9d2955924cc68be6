"""Time ActivationMessage serialisation + topic fan-out on the GPU (owgs_serialize_activations_device): 1M
publishes over 10k invoker topics, templates of ~330 bytes (action + revision + identity), content of 0-400 bytes,
inputs resident in HBM.  Prints one JSON line with the achieved output and algorithmic (read + write) bandwidth."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from openwhisk_amd import GpuShardingContainerPoolBalancer  # noqa: E402
from openwhisk_amd._lib import owgs_msg_batch  # noqa: E402


def main(n=1_000_000, n_topics=10_000, reps=10):
    rng = np.random.default_rng(9)
    b = GpuShardingContainerPoolBalancer()
    user = ('{"subject":"u%d","namespace":{"name":"ns%d","uuid":"23bc46b1-71f6-4ed5-8c54-816aa4f8c502"},"authkey":'
            '{"api_key":"23bc46b1-71f6-4ed5-8c54-816aa4f8c502:123zO3xZCLrMN6v2BKK1dXYFpXlPkccOFqm12CdAsMgRU4VrNZ9l'
            'yGVCGuMDGIwP"},"rights":["READ","PUT","DELETE","ACTIVATE"],"limits":{}}')
    ta = ['"action":{"path":"ns%d","name":"action%d","version":"0.0.1"},"revision":"1-%032x","user":%s'
          % (k % 1000, k, k, user % (k, k % 1000)) for k in range(10_000)]
    b.register_templates(ta, ["[]"] * len(ta))
    inv = rng.integers(0, n_topics, size=n).astype(np.int32)
    inv[rng.random(n) < 0.01] = -1
    tmpl = rng.integers(0, len(ta), size=n).astype(np.int32)
    aid = rng.integers(0, 2 ** 62, size=(n, 2)).astype(np.int64)
    tids = [b"sid_%028x" % k for k in range(n)]
    tid_off = np.zeros(n + 1, np.int64)
    tid_off[1:] = np.cumsum([len(t) for t in tids])
    clen = rng.integers(0, 400, size=n)
    content = np.frombuffer(b"".join(b'{"p":"' + b"x" * int(c) + b'"}' for c in clen), np.uint8)
    coff = np.zeros(n + 1, np.int64)
    coff[1:] = np.cumsum(clen + 8)
    flags = np.full(n, 4, np.uint8)
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    d = [t(inv, np.int32), t(tmpl, np.int32), t(aid, np.int64), t(np.frombuffer(b"".join(tids), np.uint8), np.uint8),
         t(tid_off, np.int64), t(1_700_000_000_000 + np.arange(n), np.int64), t(flags, np.uint8), t(content, np.uint8),
         t(coff, np.int64), t(np.zeros(n + 1), np.int64)]
    P = lambda x: C.c_void_p(x.data_ptr())  # noqa: E731
    mb = owgs_msg_batch(n, P(d[0]), P(d[1]), P(d[2]), P(d[3]), P(d[4]), P(d[5]), P(d[6]), P(d[7]), P(d[8]), None,
                        None, P(d[9]))
    total, m = C.c_int64(0), C.c_int32(0)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    topic = torch.empty(n_topics + 1, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream()
    s = C.c_void_p(stream.cuda_stream)
    rc = b._L.owgs_serialize_activations_device(b._h, C.byref(mb), n_topics, None, 0, P(off), P(order), P(topic),
                                                C.byref(total), C.byref(m), s)
    cap = total.value
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    call = lambda: b._L.owgs_serialize_activations_device(  # noqa: E731
        b._h, C.byref(mb), n_topics, P(out), cap, P(off), P(order), P(topic), C.byref(total), C.byref(m), s)
    assert call() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):
        assert call() == 0
    e1.record(stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ms = e0.elapsed_time(e1) / reps
    mm = m.value
    tmpl_bytes = sum(len(ta[k]) for k in tmpl[inv >= 0])
    read = int(tmpl_bytes + (tid_off[-1] + content.size) + n * (4 + 4 + 16 + 8 + 8 + 1 + 8))
    print(json.dumps({"what": "owgs_serialize_activations_device", "activations": n, "messages": mm,
                      "topics": n_topics, "bytes_out": cap, "ms_per_batch": ms, "wall_ms_per_batch": dt * 1e3,
                      "messages_per_s": mm / (ms * 1e-3), "out_GBps": cap / (ms * 1e-3) / 1e9,
                      "algorithmic_GBps": (cap + read) / (ms * 1e-3) / 1e9, "rc_size_query": rc}), flush=True)


if __name__ == "__main__":
    main()
