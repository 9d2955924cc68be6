#!/usr/bin/env python3
"""Benchmark: bit-exact scheduling decisions/s of ShardingContainerPoolBalancer.schedule() semantics on MI355X.

One step = one replay of a controller shard's activation stream (1M activations in capacity-calibrated batches,
each batch = completion releases then publishes; workload.py "headline": 10k invokers, Zipf actions, 128..2048 MB,
concurrent + blackbox actions, 2 % unhealthy).  Inputs are resident in HBM before the timed region; the slot state is
restored before every step (included in the timed region).  N GPUs = N controller shards (clusterSize = N, one stream
each, weak scaling, no data-path collective; by default invoker memory is 16 GiB x N so each shard's 1/N slot stays
16 GiB -- `--slots split` keeps 16 GiB invokers split N ways); for N > 1 the invoker health vector is all-gathered over RCCL once per
step (the reference's controllers all consume the same health topic, SCPB:355).

Prints ONE JSON line on rank 0.  The value counts only when every rank's assignment vector is bit-exact with the
CPU oracle (checked after timing).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

MULTI_MAX = 64  # controller shards per owgs_replay_device_multi launch (OWGS_MULTI_DEV_MAX)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# HBM bytes of one owgs_engine_kernel launch on the headline config (1M activations), from separate rocprofv3 --pmc
# passes over `bench.py --steps 5` (tools/pmc_run.sh; summary committed as profiles/r01_v8_pmc.txt): FETCH_SIZE
# 12,920 KiB doubled for gfx950's half-counted 16 B/lane streaming reads (the engine reads by LDS-DMA dwordx4) +
# WRITE_SIZE 26,210 KiB.  Counters cannot be read live inside the timed run, so this is the profiled value of the
# same engine build; other configs report null.
ENGINE_PMC_TRAFFIC = {"bytes": (2 * 12920 + 26210) * 1024, "source": "profiles/r01_v8_pmc.txt (FETCH_SIZE x2 + WRITE_SIZE)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="headline")
    ap.add_argument("--n-activations", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--slots", choices=("weak", "split"), default="weak",
                    help="headline invoker memory: 'weak' = 16 GiB x clusterSize, so every controller shard's 1/N slot "
                         "(SCPB:485-499) is 16 GiB at every N; 'split' = 16 GiB invokers split N ways")
    ap.add_argument("--shards-per-gpu", type=int, default=1,
                    help="controller shards hosted per GPU (clusterSize = gpus x this), replayed by engine launches of "
                         "up to 8 shards (one workgroup each), one HIP stream per launch")
    return ap.parse_args()


def algorithmic_bytes(w) -> int:
    """Minimum HBM bytes one replay must move: stream in/out once, action table and slot state once."""
    s = w.stream
    n, r = len(s.act), len(s.rel_aid)
    n_slots = len(w.inv_ids)
    per_act = 4 + 4 + 1             # action id in, invoker out, flags out
    per_rel = 8 + 4 + 4 + 1         # release id in, its invoker and action (gathered), release flag out
    table = len(w.actions) * (16 + 4)  # {home, step, mem, meta} + slot key
    state = n_slots * 4 * 2 + (w.inv_ids.size + 64) * 4  # permits load + store, pool words
    offs = (s.n_batches + 1) * 16
    return n * per_act + r * per_rel + table + state + offs


def _oracle_replay(args, world, shards, reps=1):
    """Replay `shards` independent shard streams of the bench config on len(shards) host threads, `reps` times;
    returns (decisions, seconds)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes as C

    import oracle as O
    from openwhisk_amd import workload as W

    ws = [W.config(args.config, n_activations=args.n_activations, shard=t, n_shards=world) for t in shards]
    s0 = ws[0].stream  # owo_replay_parallel needs one batch structure: shard 0's offsets for every thread
    acts = [np.ascontiguousarray(w.stream.act, dtype=np.int32) for w in ws]
    acq = np.ascontiguousarray(s0.acq_off, dtype=np.int64)
    rel = np.ascontiguousarray(s0.rel_off, dtype=np.int64)
    aid = np.ascontiguousarray(s0.rel_aid, dtype=np.int64)
    P = C.c_void_p
    arr = lambda xs: (P * len(xs))(*[x.ctypes.data_as(P) for x in xs])  # noqa: E731
    total, dt = 0, 0.0
    for _ in range(reps):
        sts = [O.state_for(w) for w in ws]  # fresh slot state each repeat (outside the timed region)
        outs = [np.zeros(len(a), dtype=np.int32) for a in acts]
        fls = [np.zeros(len(a), dtype=np.uint8) for a in acts]
        sarr = (P * len(sts))(*[st.h for st in sts])
        t0 = time.perf_counter()
        O.lib().owo_replay_parallel(sarr, len(sts), len(acq) - 1, acq.ctypes.data_as(P), arr(acts),
                                    rel.ctypes.data_as(P), aid.ctypes.data_as(P), 0, arr(outs), arr(fls), None)
        dt += time.perf_counter() - t0
        total += sum(len(a) for a in acts)
    return total, dt


def cpu_baseline(args, world):
    """The oracle (a literal C port of the reference schedule()/release path) replaying the bench's own shard stream
    on ONE host core -- one controller's schedule() is single-threaded in the reference (SCPB:257-317 runs on the
    balancer's actor) and the stream is sequential, so this is the same workload on the CPU.  Repeated to ~5 s.
    `parallel` adds the aggregate of T cores replaying T independent shard streams (T controllers on one host)."""
    n1, t1 = _oracle_replay(args, world, [0], reps=1)
    reps = max(1, min(12, int(5.0 / max(t1, 1e-3))))
    n, dt = _oracle_replay(args, world, [0], reps=reps)
    out = {"value": n / dt, "unit": "decisions/s", "cores": 1, "kind": "port",
           "sample": f"the bench's {args.config} shard stream ({args.n_activations} activations) replayed "
                     f"{reps}x on 1 core (oracle/owsched_oracle.c, -O3), {dt:.2f} s"}
    T = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    if T > 1:
        nt, dtt = _oracle_replay(args, world, list(range(T)), reps=1)
        out["parallel"] = {"value": nt / dtt, "unit": "decisions/s", "cores": T,
                           "sample": f"{T} threads x an independent {args.config} shard stream each, {dtt:.2f} s wall"}
    return out


def main():
    args = parse()
    import torch

    from openwhisk_amd import cluster

    rank, world, local = cluster.env_rank()

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from openwhisk_amd import GpuShardingContainerPoolBalancer

    K = max(1, args.shards_per_gpu)
    n_ctl = world * K  # controllers in the cluster: rank r hosts shards r*K .. r*K+K-1
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731

    class Shard:
        """One controller shard: its own balancer context, stream buffers in HBM and HIP stream."""

        def __init__(self, idx, own_stream):
            kw = {}
            if args.slots == "weak" and args.config == "headline" and n_ctl > 1:
                kw["user_memory_mb"] = 16_384 * n_ctl
            self.w = w = cluster.shard_workload(args.config, idx, n_ctl, n_activations=args.n_activations, **kw)
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
            # launch group gets one: HIP maps streams round-robin onto few hardware queues, and two group streams
            # on one queue would serialise their launches
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

    shards = [Shard(rank * K + k, k % MULTI_MAX == 0) for k in range(K)]
    w, s, b = shards[0].w, shards[0].s, shards[0].b
    hx = cluster.HealthExchange(dist, torch.from_numpy(w.inv_status.copy()).to(dev), world)
    torch.cuda.synchronize()
    stream = shards[0].stream
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream

    def launch_all():
        if K > 1:  # groups of up to 8 shards, each group ONE engine launch (one workgroup per shard) on its stream
            h = hx.exchange() if world > 1 else None
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
        if world > 1:
            h = hx.exchange()  # on shards[0]'s stream; the other shards' streams wait for it
            for sh in shards:
                if sh is not shards[0]:
                    sh.stream.wait_stream(stream)
                sh.b.update_health_device(len(w.inv_status), h.data_ptr(), sh.sp)
        for sh in shards:
            sh.replay()
        for sh in shards[1:]:
            stream.wait_stream(sh.stream)  # the step ends when every shard's replay has ended

    for _ in range(args.warmup):
        launch_all()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
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
    replay_ms = float(np.mean([a.elapsed_time(c) for a, c in evs]))
    stats = b.stats()
    # the dominant kernel alone: HIP events the library records around each engine launch on the replay stream,
    # read after instrumented replays outside the timed region (reading them inside would add a sync per step)
    eng = []
    for _ in range(max(3, min(args.steps, 5))):
        launch_all()
        eng.append(float(np.mean([sh.b.engine_ms() for sh in shards])))
    kern_ms = float(np.mean(eng))

    exact = True
    if not args.no_check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        for sh in shards:
            st = O.state_for(sh.w)
            o_inv, o_fl, o_rf = st.replay(sh.s)
            exact = exact and (np.array_equal(o_inv, sh.d_out.cpu().numpy())
                               and np.array_equal(o_fl, sh.d_fl.cpu().numpy())
                               and np.array_equal(o_rf, sh.d_rf.cpu().numpy()[: len(o_rf)])
                               and np.array_equal(st.permits(), sh.b.permits()))

    n_dec = sum(len(sh.s.act) for sh in shards)  # this rank's decisions per step
    t_step = wall / args.steps
    t_step, bad, kern_ms, replay_ms = cluster.max_over_ranks(dist, [t_step, 0.0 if exact else 1.0, kern_ms, replay_ms],
                                                             dev)
    exact = bad == 0.0
    value = cluster.whole_job_rate(n_dec, world, t_step)
    algo = algorithmic_bytes(w)
    achieved = algo / (kern_ms * 1e-3) / 1e9
    headline = args.config == "headline" and args.n_activations == 1_000_000
    traffic = ENGINE_PMC_TRAFFIC["bytes"] if headline else None
    traffic_src = ENGINE_PMC_TRAFFIC["source"] if headline else None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, world)
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
                       "cluster_size": w.cluster_size,
                       "invoker_memory_mb": int(w.inv_mem[0] // (1 << 20)), "slot_mb": int(w.info["slot_mb"]), "parallelism": f"{n_ctl} controller shard(s), {K} per GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "owgs_engine_kernel", "kernel_ms": kern_ms, "replay_ms": replay_ms,
                         "algorithmic_bytes": algo},
            "engine_stats": stats,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
