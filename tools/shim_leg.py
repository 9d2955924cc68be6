"""The bench's shim-path leg alone (bench.shim_path): per-call latency of the C ABI as the JNI shim drives it, at the
given drain sizes, for the headline shard (or a config).  For rocprofv3 --kernel-trace --stats runs."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import bench  # noqa: E402
import oracle as O  # noqa: E402
from openwhisk_amd import workload as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="headline")
ap.add_argument("--drains", default="64,512,4096")
ap.add_argument("--budget", type=int, default=0, help="jobs per leg (0: the bench's)")
ap.add_argument("--modes", default="calls,fused")
a = ap.parse_args()
cfg, _, sh = a.config.partition(":")  # "headline:0/8" = shard 0 of an 8-controller cluster
w = W.config(cfg, shard=int(sh.split("/")[0]), n_shards=int(sh.split("/")[1])) if sh else W.config(cfg)
o_inv, _, _ = O.state_for(w).replay(w.stream)
dr = tuple(int(x) for x in a.drains.split(","))
bud = tuple([a.budget or None] * len(dr)) if a.budget else tuple({64: 120_000, 512: 480_000}.get(d) for d in dr)
print(json.dumps(bench.shim_path(w, o_inv, 0, drains=dr, budget_jobs=bud, modes=tuple(a.modes.split(",")))))
