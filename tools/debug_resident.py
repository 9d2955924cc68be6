"""Diagnostic: drive test_gpu_resident's Shim call by call and compare permits after every call; prints the first
call after which the permits differ from the oracle (invokers, values, the call's jobs)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import test_gpu_resident as T  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "headline"
kw = dict(n_activations=30_000, n_invokers=1000, n_actions=2000, n_namespaces=200) if cfg == "headline" else \
    dict(n_activations=30_000)
w = T._hot_small_pool(11) if cfg == "hot" else W.config(cfg, **kw)
sh = T.Shim(w)
rng = np.random.default_rng(7)
k = 0
every = int(os.environ.get("EVERY", "1"))
while not sh.done():
    pos = sh.pos
    d = int(rng.integers(1, 601)) if cfg != "hot" else int(rng.integers(1, 300))
    sh.call(d)
    k += 1
    if k % every == 0 or sh.done():
        gp, op = sh.g.permits(), sh.o.permits()
        if not np.array_equal(gp, op):
            bad = np.nonzero(gp != op)[0]
            print(f"{cfg}: permits differ after call {k} (jobs {pos}..{sh.pos}): invokers {bad[:10]} gpu {gp[bad[:10]]} "
                  f"oracle {op[bad[:10]]}", flush=True)
            acts = w.stream.act
            for kind, a in sh.jobs[pos:sh.pos]:
                if kind == 1:
                    ac = w.actions[acts[a]]
                    if sh.dec[a] in bad:
                        print("  publish", a, "->", sh.dec[a], "mem", ac.mem_mb, "maxc", ac.max_concurrent)
            print(sh.g.resident_stats())
            sys.exit(1)
print(f"{cfg}: {k} calls, permits equal after every call", flush=True)
