#!/usr/bin/env python3
"""Benchmark: bit-exact scheduling decisions/s of ShardingContainerPoolBalancer.schedule() semantics on MI355X.

One step = one replay of every controller shard's activation stream on its GPU (1M activations per shard in
capacity-calibrated batches; each batch = completion releases then publishes; workload.py).  Inputs are resident in
HBM before the timed region; the slot state is restored before every step (inside the timed region).

Multi-GPU (BASELINE configs[4]): N GPUs = N controllers of one cluster (clusterSize = N x shards-per-GPU), one
process per GPU, each shard its own stream.  Slots are split: every invoker keeps 16 GiB of user memory and each
controller's slot holds 1/clusterSize of it (getInvokerSlot, SCPB:485-499) -- "10k invokers' slots split 1/8 per GPU".
The controllers exchange no scheduling state (SCPB:126-133), so the data path has no collective ("scaling": "weak":
each shard's stream is fixed at 1M activations); the invoker health vector is all-gathered over RCCL once per step
(every controller consumes the same health topic, SCPB:355).

`python bench.py --gpus N` with no torch.distributed environment starts the N ranks itself (torch.distributed.run as
a child process, before this process touches any GPU); the driver may also launch it under torch.distributed.run.

Prints ONE JSON line on rank 0.  The value counts only when every rank's assignment vector, flags and final permits
are bit-exact with the CPU oracle (checked after timing).
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

MULTI_MAX = 64  # controller shards per owgs_replay_device_multi launch (OWGS_MULTI_DEV_MAX)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
# algorithmic HBM bytes of the path
B_DECISION = 28  # activation record 8 + hash 4 + step 4 + permit read 4 + permit write 4 + decision 4
B_RELEASE = 20   # release record 8 + invoker 4 + permit read-modify-write 8
PMC_FILE = os.path.join(ROOT, "pmc_traffic.json")  # tools/pmc_traffic.py (rocprofv3 --pmc), per libowgs.so build
LIB = os.path.join(ROOT, "openwhisk_amd", "libowgs.so")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="headline", help="headline (= c5 shards for N > 1) | c1 | c2 | c2_64k | c3 | c4")
    ap.add_argument("--n-activations", type=int, default=None, help="per shard (default: the config's, 1M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-shim-path", action="store_true", help="skip the shim-path leg (per-call latency)")
    ap.add_argument("--health-group", type=int, default=8,
                    help="per-batch health cadence: batches per engine launch (owgs_replay_device_group; 1 = one "
                         "owgs_update_health_device + owgs_replay_device_span per batch)")
    ap.add_argument("--health-churn", action="store_true",
                    help="N = 1: replay batch by batch with the per-batch health schedule of the N > 1 runs "
                         "(cluster.health_schedule) instead of one launch per step")
    ap.add_argument("--health-static", action="store_true",
                    help="with --health-churn: every batch's all-gathered row is the initial health (the cadence's "
                         "mechanism -- exchange, per-batch application, group launches -- without the workload change)")
    ap.add_argument("--slots", choices=("split", "weak"), default="split",
                    help="'split' (default): 16 GiB invokers, each controller's slot = 1/clusterSize of them "
                         "(configs[4]); 'weak': invoker memory 16 GiB x clusterSize so every slot stays 16 GiB")
    ap.add_argument("--shards-per-gpu", type=int, default=1,
                    help="controller shards hosted per GPU (clusterSize = gpus x this), replayed by engine launches "
                         "of up to 64 shards (one workgroup each; 8 argument blocks in the kernarg segment, more in HBM)")
    ap.add_argument("--cluster-size", type=int, default=0,
                    help="single-GPU measurement of one shard of a larger cluster: clusterSize (default gpus x "
                         "shards-per-gpu)")
    ap.add_argument("--shard", type=int, default=0, help="with --cluster-size: which controller shard this GPU runs")
    ap.add_argument("--rccl", action="store_true",
                    help="N = 1 with --health-churn: initialise a one-rank RCCL ('nccl') process group and run the "
                         "per-batch health all-gathers through it instead of a local copy (the multi-GPU cadence's "
                         "collective, streams and ordering on one GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/collective plumbing only (gloo, CPU): no replay, value null (tests)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def warm_collective(dist, dev):
    """One all-gather right after the process group starts, with this process's stdout pointed at stderr: RCCL prints
    its version banner to stdout when the first collective creates the communicator (the bench's stdout is its one
    JSON line), and the communicator's internal stream is created here, before the shards' streams, so that it does not
    share a hardware queue (GPU_MAX_HW_QUEUES, round-robin over streams in creation order) with an engine stream."""
    import torch

    sys.stdout.flush()
    keep = os.dup(1)
    try:
        os.dup2(2, 1)
        x = torch.zeros(1, dtype=torch.uint8, device=dev)
        out = torch.empty(dist.get_world_size(), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, x)
        torch.cuda.synchronize()
    finally:
        sys.stdout.flush()
        os.dup2(keep, 1)
        os.close(keep)


def launch_ranks(args) -> int:
    """`--gpus N` without a torch.distributed environment: run N ranks under torch.distributed.run as a CHILD
    process (this process has not touched a GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    return subprocess.call(cmd, env=env)


def cluster_geometry(args, rank: int, world: int):
    """(clusterSize, controller shard indices this rank replays)."""
    K = max(1, args.shards_per_gpu)
    n_ctl = args.cluster_size if args.cluster_size > 0 else world * K
    base = args.shard if (args.cluster_size > 0 and world == 1) else rank * K
    if base + K > n_ctl:
        raise SystemExit(f"shards {base}..{base + K - 1} outside a {n_ctl}-controller cluster")
    return n_ctl, [base + k for k in range(K)]


def shard_workload(args, idx: int, n_ctl: int):
    """The stream and cluster of controller shard `idx` of `n_ctl` (workload.py; configs[4] for N > 1)."""
    from openwhisk_amd import cluster

    kw = {}
    if args.slots == "weak" and n_ctl > 1:
        kw["user_memory_mb"] = 16_384 * n_ctl
    return cluster.shard_workload(args.config, idx, n_ctl, n_activations=args.n_activations, **kw)


def algorithmic_bytes(w) -> dict:
    """Algorithmic HBM bytes of one shard's replay: SURVEY 8(d) (28 B per decision + 20 B per release) and the
    narrower stream-only count (decision in/out, release in/out, action table and slot state once)."""
    s = w.stream
    n, r = len(s.act), len(s.rel_aid)
    n_slots = len(w.inv_ids)
    stream = (n * (4 + 4 + 1) + r * (8 + 4 + 4 + 1) + len(w.actions) * (16 + 4) + n_slots * 4 * 2
              + (w.inv_ids.size + 64) * 4 + (s.n_batches + 1) * 16)
    return {"survey": n * B_DECISION + r * B_RELEASE, "stream": stream}


def lib_sha() -> str:
    try:
        with open(LIB, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return "missing"


def pmc_traffic(key: str):
    """HBM bytes per engine launch from a rocprofv3 --pmc pass of THIS build (same libowgs.so sha) on this workload,
    or None.  Counters cannot be read inside the timed run; tools/pmc_traffic.py records them per build."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None
    e = d.get(key)
    return e if e and e.get("lib_sha") == lib_sha() else None


def _oracle_replay(ws, reps=1):
    """Replay the shards `ws` on len(ws) host threads (one shard each), `reps` times; returns (decisions, s)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes as C

    import oracle as O

    acts = [np.ascontiguousarray(w.stream.act, dtype=np.int32) for w in ws]
    acqs = [np.ascontiguousarray(w.stream.acq_off, dtype=np.int64) for w in ws]
    rels = [np.ascontiguousarray(w.stream.rel_off, dtype=np.int64) for w in ws]
    aids = [np.ascontiguousarray(w.stream.rel_aid, dtype=np.int64) for w in ws]
    P = C.c_void_p
    total, dt = 0, 0.0
    for _ in range(reps):
        sts = [O.state_for(w) for w in ws]  # fresh slot state each repeat (outside the timed region)
        outs = [np.zeros(len(a), dtype=np.int32) for a in acts]
        fls = [np.zeros(len(a), dtype=np.uint8) for a in acts]
        t0 = time.perf_counter()
        if len(ws) == 1:
            s = ws[0].stream
            O.lib().owo_replay(sts[0].h, s.n_batches, acqs[0].ctypes.data_as(P), acts[0].ctypes.data_as(P),
                               rels[0].ctypes.data_as(P), aids[0].ctypes.data_as(P), C.c_uint64(s.seq_base),
                               outs[0].ctypes.data_as(P), fls[0].ctypes.data_as(P), None)
        else:
            import threading

            def run(k):
                s = ws[k].stream
                O.lib().owo_replay(sts[k].h, s.n_batches, acqs[k].ctypes.data_as(P), acts[k].ctypes.data_as(P),
                                   rels[k].ctypes.data_as(P), aids[k].ctypes.data_as(P), C.c_uint64(s.seq_base),
                                   outs[k].ctypes.data_as(P), fls[k].ctypes.data_as(P), None)

            th = [threading.Thread(target=run, args=(k,)) for k in range(len(ws))]
            for t in th:
                t.start()
            for t in th:
                t.join()
        dt += time.perf_counter() - t0
        total += sum(len(a) for a in acts)
    return total, dt


def cpu_baseline(args, w0, n_ctl, shard0):
    """The oracle (a literal C port of the reference schedule()/release path) replaying the bench's own shard stream
    on ONE host core -- one controller's schedule() runs on one thread in the reference (the balancer actor) and the
    stream is sequential -- repeated to ~10 s.  `parallel` adds T cores replaying T independent shards of the same
    cluster (T controllers on one host)."""
    n1, t1 = _oracle_replay([w0], reps=1)
    reps = max(1, min(20, int(10.0 / max(t1, 1e-3))))
    n, dt = _oracle_replay([w0], reps=reps)
    one = {"value": n / dt, "unit": "decisions/s", "cores": 1,
           "sample": f"shard {shard0} of {n_ctl} of the bench's {args.config} workload ({len(w0.stream.act)} "
                     f"activations) replayed {reps}x on 1 core (oracle/owsched_oracle.c, -O3), {dt:.2f} s"}
    out = dict(one, kind="port", single_core=one)
    T = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    if T > 1:
        # the line leads with the whole host: T cores replaying T independent shard streams of
        # the same cluster (T controllers on one host, the reference's own scaling model); one core stays beside it
        ws = [shard_workload(args, t % max(n_ctl, 1), max(n_ctl, 1)) if n_ctl > 1 else
              shard_workload(args, 0, 1) for t in range(T)]
        nt, dtt = _oracle_replay(ws, reps=1)
        out.update(value=nt / dtt, cores=T,
                   sample=(f"{T} host threads replaying {T} independent shard streams of the bench's {args.config} "
                           f"workload ({len(w0.stream.act)} activations each), {dtt:.2f} s wall: "
                           f"{nt / dtt / 1e6:.1f} M decisions/s aggregate; one core: {n / dt / 1e6:.2f} M/s "
                           f"(single_core)"))
    return out


def shim_path(w, o_inv, dev_index, drains=(64, 512, 4096), budget_jobs=(120_000, 480_000, None),
              modes=("calls", "fused")):
    """The path the JVM shim drives (integration/GpuShardingContainerPoolBalancer.scala): the shard's stream as the
    batching thread's queue -- per batch its completions, then its publishes -- drained `drain` jobs at a time.  Each
    drained batch splits into runs of releases followed by publishes; "calls" issues one owgs_release_batch per release
    run and one owgs_publish_batch per publish run (host buffers, as the JNI stub hands them over), "fused" one
    owgs_process_batch per drained batch.  Per-call latency is the C call alone (arguments prepared before the clock).
    Decisions are compared with the oracle's replay of the same prefix."""
    import ctypes as C

    from openwhisk_amd import GpuShardingContainerPoolBalancer

    s = w.stream
    jobs_rel, jobs_pub = [], []  # per batch: release activation ids, publish ids
    kinds = []
    for b in range(s.n_batches):
        r = s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]]
        kinds.append(np.concatenate([np.zeros(len(r), np.int8), np.ones(int(s.acq_off[b + 1] - s.acq_off[b]), np.int8)]))
        jobs_rel.append(r)
        jobs_pub.append(np.arange(s.acq_off[b], s.acq_off[b + 1]))
    kind = np.concatenate(kinds)
    ids = np.concatenate([np.concatenate([jobs_rel[b], jobs_pub[b]]) for b in range(s.n_batches)]).astype(np.int64)
    b = GpuShardingContainerPoolBalancer(managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction,
                                         rng_seed=w.rng_seed, device=dev_index)
    b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
    b.update_cluster(w.cluster_size)
    b.register_actions(w.actions)
    b.snapshot()
    L, h = b._L, b._h
    p = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    act = np.ascontiguousarray(s.act, np.int32)
    legs = []
    for drain, budget in zip(drains, budget_jobs):
        n_jobs = len(ids) if budget is None else min(budget, len(ids))
        for mode in modes:
            b.restore()
            rs0 = b.resident_stats()
            hn0 = b.resident_table_fill()[2:]
            inv = np.full(len(act), -9, np.int32)
            fl = np.zeros(len(act), np.uint8)
            lat, clat, n_pub = [], [], 0
            for c0 in range(0, n_jobs, drain):
                k = kind[c0:min(c0 + drain, n_jobs)]
                x = ids[c0:c0 + len(k)]
                # runs: maximal (releases, publishes) pairs
                cut = np.nonzero((k[1:] == 0) & (k[:-1] == 1))[0] + 1
                bounds = np.concatenate([[0], cut, [len(k)]])
                runs = []
                for r0, r1 in zip(bounds[:-1], bounds[1:]):
                    kk, xx = k[r0:r1], x[r0:r1]
                    rel = xx[kk == 0]
                    # a completion follows its publish; one published earlier in the SAME drained batch (the
                    # stream's one-batch delay at a drain boundary) names the oracle's invoker (= the GPU's, checked)
                    ri = inv[rel]
                    if o_inv is not None:
                        ri = np.where(ri == -9, o_inv[rel], ri)
                    keep = ri >= 0  # no ActivationEntry for a failed publish (CLB:278-279)
                    runs.append((np.ascontiguousarray(ri[keep]), np.ascontiguousarray(act[rel[keep]]),
                                 np.ascontiguousarray(xx[kk == 1])))
                if mode == "calls":
                    for ri, ra, pubs in runs:
                        if len(ri):
                            rf = np.zeros(len(ri), np.uint8)
                            args = (h, len(ri), p(ri), p(ra), p(rf))
                            t0 = time.perf_counter()
                            rc = L.owgs_release_batch(*args)
                            lat.append(time.perf_counter() - t0)
                            clat.append(b.last_call_ns())
                            assert rc == 0
                        if len(pubs):
                            pa = np.ascontiguousarray(act[pubs])
                            sq = pubs.astype(np.uint64)
                            o = np.zeros(len(pubs), np.int32)
                            f = np.zeros(len(pubs), np.uint8)
                            args = (h, len(pubs), p(pa), p(sq), 0, p(o), p(f))
                            t0 = time.perf_counter()
                            rc = L.owgs_publish_batch(*args)
                            lat.append(time.perf_counter() - t0)
                            clat.append(b.last_call_ns())
                            assert rc == 0
                            inv[pubs], fl[pubs] = o, f
                            n_pub += len(pubs)
                else:
                    ro = np.cumsum([0] + [len(r[0]) for r in runs]).astype(np.int32)
                    po = np.cumsum([0] + [len(r[2]) for r in runs]).astype(np.int32)
                    ri = np.concatenate([r[0] for r in runs] + [np.zeros(1, np.int32)]).astype(np.int32)
                    ra = np.concatenate([r[1] for r in runs] + [np.zeros(1, np.int32)]).astype(np.int32)
                    pubs = np.concatenate([r[2] for r in runs]).astype(np.int64)
                    pa = np.ascontiguousarray(np.concatenate([act[pubs], np.zeros(1, np.int32)]))
                    sq = np.ascontiguousarray(np.concatenate([pubs, [0]]).astype(np.uint64))
                    o = np.zeros(len(pubs) + 1, np.int32)
                    f = np.zeros(len(pubs) + 1, np.uint8)
                    rf = np.zeros(len(ri), np.uint8)
                    # (the buffers' addresses before the clock: the JNI shim hands over direct-buffer addresses; numpy's
                    # ctypes conversion costs ~2.7 us per pointer on the host, more than the call itself at small drains)
                    args = (h, len(runs), p(ro), p(ri), p(ra), p(rf), p(po), p(pa), p(sq), 0, p(o), p(f))
                    t0 = time.perf_counter()
                    rc = L.owgs_process_batch(*args)
                    lat.append(time.perf_counter() - t0)
                    clat.append(b.last_call_ns())
                    assert rc == 0, (rc, L.owgs_last_error(h))
                    inv[pubs], fl[pubs] = o[:len(pubs)], f[:len(pubs)]
                    n_pub += len(pubs)
            done = inv != -9
            exact = bool(np.array_equal(inv[done], o_inv[done])) if o_inv is not None else None
            lat_us = np.array(clat) * 1e-3  # the C call, timed inside the library
            py_us = np.array(lat) * 1e6     # the same calls seen from Python (+ ctypes' argument conversion)
            rs1 = b.resident_stats()
            fill = b.resident_table_fill()
            served, chained = rs1["served"] - rs0["served"], rs1["chained"] - rs0["chained"]
            legs.append({"drain": drain, "mode": mode, "jobs": n_jobs, "calls": len(lat), "publishes": int(n_pub),
                         "p50_us": float(np.percentile(lat_us, 50)), "p99_us": float(np.percentile(lat_us, 99)),
                         "decisions_per_s": n_pub / max(float(np.sum(lat_us)) * 1e-6, 1e-9),
                         "py_p50_us": float(np.percentile(py_us, 50)), "py_p99_us": float(np.percentile(py_us, 99)),
                         "bit_exact": exact,
                         # which engine served the leg's calls (a fused leg of drains over 1,024 jobs is all launch chain)
                         "engine": ("per-run launches" if mode == "calls" else "resident" if chained == 0 else
                                    "launch chain" if served == 0 else "resident + launch chain"),
                         # owgs_process_batch's paths in this leg: resident engine calls / launches, launch-chain calls
                         "resident": {k: rs1[k] - rs0[k] for k in rs1 if k not in ("alive", "last_call_ns")},
                         "map_fill_max": fill[0], "map_deleted_max": fill[1],
                         "host_build_us_mean": (fill[2] - hn0[0]) * 1e-3 / max(rs1["served"] - rs0["served"], 1),
                         "host_wait_us_mean": (fill[3] - hn0[1]) * 1e-3 / max(rs1["served"] - rs0["served"], 1)})
    legs += shim_extra_legs(w, b, kind, ids, act, o_inv)
    b.close()
    return {"path": "host buffers through the C ABI as the JNI shim calls it (queue order: each batch's completions, "
                    "then its publishes); calls = owgs_release_batch + owgs_publish_batch per run, fused = "
                    "owgs_process_batch per drained batch (small calls: the resident engine, owgs_resident.hip); "
                    "latency = the C call, timed inside the library (py_* = the same calls timed from Python, "
                    "ctypes' call overhead included)", "legs": legs}


def _fused_drain(b, kind, ids, act, inv, o_ref, c0, c1):
    """One drained batch jobs [c0, c1) through owgs_process_batch as the shim calls it; returns (C-call ns, publishes)."""
    import ctypes as C
    p = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    k, x = kind[c0:c1], ids[c0:c1]
    cut = np.nonzero((k[1:] == 0) & (k[:-1] == 1))[0] + 1
    bounds = np.concatenate([[0], cut, [len(k)]])
    runs = []
    for r0, r1 in zip(bounds[:-1], bounds[1:]):
        kk, xx = k[r0:r1], x[r0:r1]
        rel = xx[kk == 0]
        ri = inv[rel]
        ri = np.where(ri == -9, o_ref[rel], ri)  # (published earlier in this drained batch: the oracle's = the GPU's)
        keep = ri >= 0  # no ActivationEntry for a failed publish (CLB:278-279)
        runs.append((ri[keep], act[rel[keep]], xx[kk == 1]))
    ro = np.cumsum([0] + [len(r[0]) for r in runs]).astype(np.int32)
    po = np.cumsum([0] + [len(r[2]) for r in runs]).astype(np.int32)
    ri = np.concatenate([r[0] for r in runs] + [np.zeros(1, np.int32)]).astype(np.int32)
    ra = np.concatenate([r[1] for r in runs] + [np.zeros(1, np.int32)]).astype(np.int32)
    pubs = np.concatenate([r[2] for r in runs]).astype(np.int64)
    pa = np.ascontiguousarray(np.concatenate([act[pubs], np.zeros(1, np.int32)]))
    sq = np.ascontiguousarray(np.concatenate([pubs, [0]]).astype(np.uint64))
    o = np.zeros(len(pubs) + 1, np.int32)
    f = np.zeros(len(pubs) + 1, np.uint8)
    rf = np.zeros(len(ri), np.uint8)
    args = (b._h, len(runs), p(ro), p(ri), p(ra), p(rf), p(po), p(pa), p(sq), 0, p(o), p(f))
    rc = b._L.owgs_process_batch(*args)
    assert rc == 0, (rc, b._L.owgs_last_error(b._h))
    inv[pubs] = o[:len(pubs)]
    return b.last_call_ns(), len(pubs)


def shim_extra_legs(w, b, kind, ids, act, o_inv, budget=480_000, seed=0x5EED):
    """Two more fused legs of the shim path:
    "mixed": drain sizes as a loaded batching thread produces them -- log-uniform over 1..4096 jobs, so the calls flip
    between the resident engine (<= OWGS_RES_MAX jobs) and the launch chain; p50 / p99 per drain class and overall.
    "reset": 512-job drains with updateCluster(2) (SCPB:561-584) at a batch boundary a third into the leg: the
    activations in flight become watched pairs (their releases meet the new state, NS:61-62 / NS:98-113); what share
    of the calls after the change the resident engine serves, and their latency.  Both are checked against the oracle
    (the reset leg against an oracle replay with the same membership change)."""
    import oracle as O
    s = w.stream
    out = []
    n_jobs = min(budget, len(ids))
    # -- mixed drain sizes
    rng = np.random.default_rng(seed)
    b.restore()
    rs0 = b.resident_stats()
    inv = np.full(len(act), -9, np.int32)
    lat, sizes, n_pub, c0 = [], [], 0, 0
    while c0 < n_jobs:
        d = int(np.exp(rng.uniform(0.0, np.log(4096.0)))) or 1
        c1 = min(c0 + d, n_jobs)
        ns, npub = _fused_drain(b, kind, ids, act, inv, o_inv, c0, c1)
        lat.append(ns * 1e-3)
        sizes.append(c1 - c0)
        n_pub += npub
        c0 = c1
    rs1 = b.resident_stats()
    lat, sizes = np.array(lat), np.array(sizes)
    done = inv != -9
    small = sizes <= 1024
    flip = small & np.concatenate([[False], sizes[:-1] > 1024])  # a small call right after a chained one: relaunch
    out.append({"mode": "fused-mixed", "drain": "log-uniform 1..4096", "jobs": n_jobs, "calls": len(lat),
                "publishes": int(n_pub), "p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
                "p50_us_le1024": float(np.percentile(lat[small], 50)), "p99_us_le1024": float(np.percentile(lat[small], 99)),
                "p50_us_le1024_after_chain": float(np.percentile(lat[flip], 50)) if flip.any() else None,
                "p50_us_le1024_steady": float(np.percentile(lat[small & ~flip], 50)),
                "p99_us_le1024_steady": float(np.percentile(lat[small & ~flip], 99)),
                "p50_us_gt1024": float(np.percentile(lat[~small], 50)) if (~small).any() else None,
                "p99_us_gt1024": float(np.percentile(lat[~small], 99)) if (~small).any() else None,
                "decisions_per_s": n_pub / max(float(lat.sum()) * 1e-6, 1e-9),
                "bit_exact": bool(np.array_equal(inv[done], o_inv[done])),
                "resident": {k: rs1[k] - rs0[k] for k in rs1 if k not in ("alive", "last_call_ns")}})
    # -- membership change mid-leg
    job_batch = np.repeat(np.arange(s.n_batches), np.diff(s.rel_off) + np.diff(s.acq_off))
    first_job = np.concatenate([[0], np.cumsum(np.diff(s.rel_off) + np.diff(s.acq_off))])
    b0 = max(1, int(job_batch[min(n_jobs // 3, len(job_batch) - 1)]))
    end_b = int(job_batch[n_jobs - 1]) + 1  # (the leg stops at a batch end: the oracle replays whole batches)
    n_jobs_r = int(first_job[end_b])
    st = O.state_for(w)
    o_r = np.full(len(act), -9, np.int32)
    fl_r = np.zeros(len(act), np.uint8)
    rf_r = np.zeros(max(len(s.rel_aid), 1), np.uint8)
    acq = np.ascontiguousarray(s.acq_off, np.int64)
    rel = np.ascontiguousarray(s.rel_off, np.int64)
    aid = np.ascontiguousarray(s.rel_aid, np.int64)
    for bb in range(end_b):
        if bb == b0:
            st.update_cluster(2)
        O.lib().owo_replay(st.h, 1, O._ptr(acq[bb:]), O._ptr(np.ascontiguousarray(s.act, np.int32)),
                           O._ptr(rel[bb:]), O._ptr(aid), int(s.seq_base), O._ptr(o_r), O._ptr(fl_r), O._ptr(rf_r))
    b.restore()
    inv = np.full(len(act), -9, np.int32)
    lat_a, lat_b, n_pub, c0 = [], [], 0, 0
    cut = int(first_job[b0])
    st_mid = None
    while c0 < n_jobs_r:
        if c0 == cut:
            b.update_cluster(2)
            st_mid = b.resident_stats()
        c1 = min(c0 + 512, cut if c0 < cut else n_jobs_r)
        ns, npub = _fused_drain(b, kind, ids, act, inv, o_r, c0, c1)
        if c0 >= cut:
            lat_a.append(ns * 1e-3)
            n_pub += npub
        else:
            lat_b.append(ns * 1e-3)
        c0 = c1
    rs2 = b.resident_stats()
    b.update_cluster(w.cluster_size)  # (the context is restored by the next leg / closed)
    done = inv != -9
    lat_a = np.array(lat_a)
    served = rs2["served"] - st_mid["served"]
    out.append({"mode": "fused-reset", "drain": 512, "jobs": n_jobs_r, "reset_at_batch": b0, "cluster_size_after": 2,
                "calls_after": len(lat_a), "resident_served_after": int(served),
                "resident_fraction_after": served / max(len(lat_a), 1),
                "watch_calls": rs2["watch_calls"] - st_mid["watch_calls"],
                "p50_us_before": float(np.percentile(lat_b, 50)), "p99_us_before": float(np.percentile(lat_b, 99)),
                "p50_us_after": float(np.percentile(lat_a, 50)), "p99_us_after": float(np.percentile(lat_a, 99)),
                "decisions_per_s_after": n_pub / max(float(lat_a.sum()) * 1e-6, 1e-9),
                "bit_exact": bool(np.array_equal(inv[done], o_r[done])) and int(done.sum()) == int(s.acq_off[end_b])})
    return out


def dry_run(args):
    """Launcher + collective plumbing on the CPU (gloo): every rank builds its shard, the ranks all-gather health and
    reduce step times exactly as the GPU path does; no replay, value null."""
    import torch
    import torch.distributed as dist

    from openwhisk_amd import cluster

    rank, world, _ = cluster.env_rank()
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    else:
        dist = None
    n_ctl, shards = cluster_geometry(args, rank, world)
    ws = [shard_workload(args, g, n_ctl) for g in shards]
    hx = cluster.HealthExchange(dist, torch.from_numpy(ws[0].inv_status.copy()), world)
    health = [torch.from_numpy(h) for h in cluster.health_schedule(ws[0].inv_status, ws[0].stream.n_batches)]
    t0 = time.perf_counter()
    n_gather = 0
    flat = [torch.empty(world * len(health[0]), dtype=torch.uint8) for _ in health]  # one buffer per batch (GPU path)
    for _ in range(args.steps):
        for k, h in enumerate(health):  # the configs[4] cadence: one all-gather between batches
            agreed = hx.exchange_into(h, flat[k])
            assert torch.equal(agreed, h)
            n_gather += 1
    t_step = (time.perf_counter() - t0) / max(args.steps, 1)
    t_step, = cluster.max_over_ranks(dist, [t_step], torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"metric": "dry run", "value": None, "n_gpus": world, "dry_run": True,
                          "health_allgathers_per_step": n_gather / max(args.steps, 1),
                          "config": {"workload": args.config, "cluster_size": n_ctl, "slots": args.slots,
                                     "slot_mb": int(ws[0].info["slot_mb"]), "shards": shards,
                                     "health_disagree": hx.disagreeing_ranks(), "ms_per_step": t_step * 1e3}}),
              flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))  # before anything touches a GPU
    if args.dry_run:
        return dry_run(args)
    import torch

    from openwhisk_amd import cluster

    rank, world, local = cluster.env_rank()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
        warm_collective(dist, torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
        if args.rccl:  # one rank over RCCL: the collective the N > 1 cadence issues, on this lease's one GPU
            import torch.distributed as dist

            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
            warm_collective(dist, torch.device("cuda", 0))
    dev = torch.device("cuda", torch.cuda.current_device())

    from openwhisk_amd import GpuShardingContainerPoolBalancer

    n_ctl, shard_ids = cluster_geometry(args, rank, world)
    K = len(shard_ids)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731

    class Shard:
        """One controller shard: its own balancer context, stream buffers in HBM and HIP stream."""

        def __init__(self, idx, own_stream):
            self.idx = idx
            self.w = w = shard_workload(args, idx, n_ctl)
            self.b = b = GpuShardingContainerPoolBalancer(
                managed_fraction=w.managed_fraction, blackbox_fraction=w.blackbox_fraction, rng_seed=w.rng_seed,
                device=torch.cuda.current_device())
            b.update_invokers_arrays(w.inv_ids, w.inv_mem, w.inv_status)
            b.update_cluster(w.cluster_size)
            b.register_actions(w.actions)
            b.snapshot()
            s = self.s = w.stream
            self.d_acq, self.d_rel = t(s.acq_off, np.int64), t(s.rel_off, np.int64)
            self.d_act = t(s.act, np.int32)
            self.d_aid = t(s.rel_aid if len(s.rel_aid) else np.zeros(1), np.int64)
            self.d_out = torch.empty(len(s.act), dtype=torch.int32, device=dev)
            self.d_fl = torch.empty(len(s.act), dtype=torch.uint8, device=dev)
            self.d_rf = torch.empty(max(len(s.rel_aid), 1), dtype=torch.uint8, device=dev)
            # a real (non-null) HIP stream: engine and timing events share it.  Only the first shard of each
            # launch group gets one (HIP maps streams round-robin onto few hardware queues)
            self.stream = torch.cuda.Stream() if own_stream else None
            self.sp = self.stream.cuda_stream if own_stream else None

        def io(self):
            s = self.s
            return (s.n_batches, self.d_acq.data_ptr(), self.d_act.data_ptr(), len(s.act), self.d_rel.data_ptr(),
                    self.d_aid.data_ptr(), len(s.rel_aid), s.seq_base, self.d_out.data_ptr(), self.d_fl.data_ptr(),
                    self.d_rf.data_ptr())

        def replay(self):
            s = self.s
            self.b.restore(self.sp)
            self.b.replay_device(s.n_batches, self.d_acq.data_ptr(), self.d_act.data_ptr(), len(s.act),
                                 self.d_rel.data_ptr(), self.d_aid.data_ptr(), len(s.rel_aid), s.seq_base,
                                 self.d_out.data_ptr(), self.d_fl.data_ptr(), self.d_rf.data_ptr(), self.sp)

        def replay_batches(self, hx, timing=None):
            """configs[4] cadence: before each batch the shards all-gather their health view (the health topic,
            SCPB:355) and apply the agreed vector (owgs_update_health_device -> updateInvokers, SCPB:512-551); the
            batch is one engine launch (owgs_replay_device_span).  The health of batch k + 1 is an input known before
            the batch, so its all-gather runs on a side stream while batch k's engine runs (one batch ahead, its own
            buffer); the engine stream waits only for the exchange of the batch it is about to apply."""
            s, b = self.s, self.b
            # the stream the library runs this shard on (self.sp; torch's current one when the shard has none): every
            # wait for an exchange is that stream's, and the side stream waits for it before overwriting its buffers
            eng = self.stream if self.stream is not None else torch.cuda.current_stream()
            if getattr(self, "hside", None) is None:
                self.hside = torch.cuda.Stream()
                self.hflat = [torch.empty(hx.world * len(self.w.inv_status), dtype=torch.uint8, device=dev)
                              for _ in range(s.n_batches)]
                self.hev = [torch.cuda.Event() for _ in range(s.n_batches)]
            self.hside.wait_stream(eng)  # (the previous step has read every buffer it overwrites)
            agreed = [None] * s.n_batches

            def gather(k):
                with torch.cuda.stream(self.hside):
                    agreed[k] = hx.exchange_into(self.d_health[k], self.hflat[k])
                    self.hev[k].record(self.hside)

            b.restore(self.sp)
            G = max(1, args.health_group)
            if G == 1:
                gather(0)
                for k in range(s.n_batches):
                    if k + 1 < s.n_batches:
                        gather(k + 1)  # in flight while batch k's engine runs
                    eng.wait_event(self.hev[k])
                    h = agreed[k]
                    b.update_health_device(len(self.w.inv_status), h.data_ptr(), self.sp)
                    b.replay_device_span(s.acq_off[k], s.acq_off[k + 1], s.rel_off[k], s.rel_off[k + 1],
                                         self.d_act.data_ptr(), self.d_aid.data_ptr(), s.seq_base, self.d_out.data_ptr(),
                                         self.d_fl.data_ptr(), self.d_rf.data_ptr(), self.sp)
                    if timing is not None:
                        timing.append(b.engine_ms())
                return
            # G batches per engine launch (owgs_replay_device_group): the engine applies each batch's agreed health
            # itself; the exchanges of group g + 1 run on the side stream while group g's engine runs
            nid = len(self.w.inv_status)
            stride = hx.world * nid  # row k of the per-batch buffers (rank 0's row first: the agreed vector)
            if getattr(self, "hall", None) is None:
                self.hall = torch.empty((s.n_batches, stride), dtype=torch.uint8, device=dev)
                self.hflat = [self.hall[k] for k in range(s.n_batches)]
            groups = [(g0, min(g0 + G, s.n_batches)) for g0 in range(0, s.n_batches, G)]
            for k in range(groups[0][0], groups[0][1]):
                gather(k)
            for j, (g0, g1) in enumerate(groups):
                if j + 1 < len(groups):
                    for k in range(*groups[j + 1]):
                        gather(k)  # in flight while this group's engine runs
                eng.wait_event(self.hev[g1 - 1])
                b.replay_device_group(s.acq_off[g0:g1 + 1], s.rel_off[g0:g1 + 1], self.d_act.data_ptr(),
                                      self.d_aid.data_ptr(), s.seq_base, self.d_out.data_ptr(), self.d_fl.data_ptr(),
                                      self.d_rf.data_ptr(), self.hall[g0].data_ptr(), stride, nid, self.sp)
                if timing is not None:
                    timing.append(b.engine_ms())

    shards = [Shard(g, k % MULTI_MAX == 0) for k, g in enumerate(shard_ids)]
    w, s, b = shards[0].w, shards[0].s, shards[0].b
    hx = cluster.HealthExchange(dist, torch.from_numpy(w.inv_status.copy()).to(dev), world,
                                collective=world > 1 or (dist is not None and args.rccl))
    # health between batches (configs[4]) for one shard per GPU; several shards per GPU keep one exchange per step
    per_batch = K == 1 and (world > 1 or args.health_churn)
    if per_batch and dist is not None and world > 1:
        # every rank issues one all-gather per batch: the shards' batch counts must agree, or the collectives would
        # pair up wrongly and hang -- fail loudly instead
        nb = torch.tensor([s.n_batches], dtype=torch.int64, device=dev)
        nbs = [torch.zeros_like(nb) for _ in range(world)]
        dist.all_gather(nbs, nb)
        counts = [int(x.item()) for x in nbs]
        if len(set(counts)) != 1:
            raise SystemExit(f"shards disagree on the number of batches per step: {counts}")
    if per_batch:
        health = cluster.health_schedule(w.inv_status, s.n_batches)
        if args.health_static:
            health = np.repeat(np.asarray(w.inv_status, dtype=np.uint8)[None, :], max(s.n_batches, 1), axis=0)
        shards[0].health = health
        shards[0].d_health = [t(health[k], np.uint8) for k in range(s.n_batches)]
    torch.cuda.synchronize()
    stream = shards[0].stream
    torch.cuda.set_stream(stream)
    n_gathers = [0]

    def launch_all(timing=None):
        if per_batch:
            shards[0].replay_batches(hx, timing)
            n_gathers[0] += s.n_batches if hx.collective else 0
            return
        h = None
        if world > 1:  # the health topic every controller consumes (SCPB:355): one all-gather per step
            h = hx.exchange()
            n_gathers[0] += 1
        if K > 1:  # groups of up to 64 shards, each group ONE engine launch (one workgroup per shard) on its stream
            groups = [shards[j:j + MULTI_MAX] for j in range(0, K, MULTI_MAX)]
            for grp in groups:
                gs = grp[0].stream
                if gs is not stream:
                    gs.wait_stream(stream)
                for sh in grp:
                    if h is not None:
                        sh.b.update_health_device(len(w.inv_status), h.data_ptr(), gs.cuda_stream)
                    sh.b.restore(gs.cuda_stream)
                GpuShardingContainerPoolBalancer.replay_device_multi([(sh.b, sh.io()) for sh in grp], gs.cuda_stream)
            for grp in groups[1:]:
                stream.wait_stream(grp[0].stream)
            return
        if h is not None:
            shards[0].b.update_health_device(len(w.inv_status), h.data_ptr(), shards[0].sp)
        shards[0].replay()

    for _ in range(args.warmup):
        launch_all()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    n_gathers[0] = 0
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        launch_all()
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gathers_per_step = n_gathers[0] / max(args.steps, 1)
    replay_ms = float(np.mean([a.elapsed_time(c) for a, c in evs]))
    smode = b.stream_mode_stats()  # the replay ran through the resident engine's stream mode (OWGS_SPEC_REPLAY)
    stats = smode if smode is not None else b.stats()
    # the dominant kernel alone: HIP events the library records around each engine launch on the replay stream,
    # read after instrumented replays outside the timed region (reading them inside would add a sync per step)
    eng = []
    for _ in range(max(3, min(args.steps, 5))):
        if per_batch:  # one engine launch per batch: their durations add up to the step's kernel time
            tm = []
            launch_all(tm)
            eng.append(float(np.sum(tm)))
            continue
        launch_all()
        eng.append(float(np.mean([sh.b.engine_ms() for sh in shards[::MULTI_MAX]])))
    kern_ms = float(np.mean(eng))

    exact = True
    o_ref = None
    if not args.no_check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        for sh in shards:
            st = O.state_for(sh.w)
            if per_batch:  # the same health vector before each batch (every rank agreed: checked below)
                o_inv, o_fl, o_rf = O.replay_with_health(st, sh.s, sh.w.inv_ids, sh.w.inv_mem, sh.health)
            else:
                o_inv, o_fl, o_rf = st.replay(sh.s)
            if o_ref is None:
                o_ref = o_inv
            exact = exact and (np.array_equal(o_inv, sh.d_out.cpu().numpy())
                               and np.array_equal(o_fl, sh.d_fl.cpu().numpy())
                               and np.array_equal(o_rf, sh.d_rf.cpu().numpy()[: len(o_rf)])
                               and np.array_equal(st.permits(), sh.b.permits()))

    # host buffers through the C ABI (owgs_replay: argument checks, H2D of the stream, replay, D2H of the decisions):
    # the rate a JVM caller handing over host arrays would see; never the bench value
    h2d_ms = 0.0
    if not args.no_h2d and not per_batch:
        reps = 3
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            for sh in shards:
                sh.b.restore()
                sh.b.replay(sh.s)
        h2d_ms = (time.perf_counter() - t1) / reps * 1e3

    shim = None
    if world == 1 and K == 1 and not args.no_shim_path:
        shim = shim_path(w, o_ref, torch.cuda.current_device())

    n_dec = sum(len(sh.s.act) for sh in shards)  # this rank's decisions per step
    t_step = wall / args.steps
    disagree = float(len(hx.disagreeing_ranks())) if per_batch else 0.0
    t_step, bad, kern_ms, replay_ms, h2d_ms, disagree = cluster.max_over_ranks(
        dist, [t_step, 0.0 if exact else 1.0, kern_ms, replay_ms, h2d_ms, disagree], dev)
    exact = bad == 0.0
    value = cluster.whole_job_rate(n_dec, world, t_step)
    algo = algorithmic_bytes(w)
    per_launch = min(K, MULTI_MAX)  # shards one engine launch replays
    achieved = algo["survey"] * per_launch / (kern_ms * 1e-3) / 1e9
    key = f"{args.config}|n{len(s.act)}|c{n_ctl}|s{args.slots}|k{per_launch}"
    pmc = pmc_traffic(key)
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, w, n_ctl, shard_ids[0])
        line = {
            "metric": "scheduling decisions/sec (whole node) at 10k invokers, 1M-activation batch",
            "value": value if exact else 0.0,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (workload.py, seeded Zipf stream)",
            "bit_exact": exact,
            "config": {"workload": args.config, "invokers": int(len(w.inv_ids)), "activations_per_shard": len(s.act),
                       "batches": s.n_batches, "batch": w.info["batch"], "releases": int(len(s.rel_aid)),
                       "cluster_size": n_ctl, "slots": args.slots, "shards": shard_ids if world == 1 else None,
                       "invoker_memory_mb": int(w.inv_mem[0] // (1 << 20)), "slot_mb": int(w.info["slot_mb"]),
                       "health_allgathers_per_step": gathers_per_step,
                       "health": (("per batch: all-gathered one group ahead on a side stream, applied by the "
                                   f"engine before each batch, {args.health_group} batches per engine launch "
                                   f"(owgs_replay_device_group: {-(-s.n_batches // args.health_group)} launches per "
                                   "step; 1 % of invokers unresponsive, changing every batch)")
                                  if args.health_group > 1 else
                                  ("per batch: all-gathered one batch ahead, applied with owgs_update_health_device, "
                                   f"{s.n_batches} engine launches per step (1 % of invokers unresponsive, changing "
                                   "every batch)")) if per_batch else "static, one exchange per step",
                       "health_disagreeing_ranks": int(disagree),
                       "health_exchange": ("RCCL all_gather_into_tensor" if hx.collective else
                                           "local copy (one rank, no process group)"),
                       "parallelism": f"{n_ctl} controller shard(s), {K} per GPU, {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc["bytes"] if pmc else None,
                         "traffic_source": pmc["source"] if pmc else f"no --pmc pass recorded for this build ({key})",
                         # what limits this kernel instead: one CU's instruction issue along the decision chain
                         "issue": pmc.get("issue") if pmc else None,
                         "kernel": ("owgs_resident_kernel" if smode is not None else
                                    "owgs_engine_kernel" if K == 1 else "owgs_engine_multi_kernel"),
                         "kernel_ms": kern_ms, "replay_ms": replay_ms, "shards_per_launch": per_launch,
                         "algorithmic_bytes": algo["survey"] * per_launch,
                         "algorithmic_def": f"SURVEY 8(d): {B_DECISION} B/decision + {B_RELEASE} B/release",
                         "achieved_stream_bytes": algo["stream"] * per_launch / (kern_ms * 1e-3) / 1e9},
            "h2d_inclusive": None if (args.no_h2d or per_batch) else {
                "value": world * n_dec / (h2d_ms * 1e-3), "unit": "decisions/s", "ms_per_step": h2d_ms,
                "path": "owgs_replay host ABI: host checks + H2D stream + replay + D2H decisions"},
            "shim_path": shim,
            "engine_stats": stats,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
