"""Multi-controller path on the CPU: world_size 2 over gloo (the GPU run uses RCCL with the same code).

Each rank is one controller shard (clusterSize = 2, SCPB:485-507): it builds its shard workload, agrees on invoker
health with the other rank (HealthExchange), replays its own stream through the oracle, and the ranks combine step
times by max (bench.py's aggregation).  Checks: shards share cluster + health but not streams, each shard's slots hold
half of every invoker (getInvokerSlot), shard replays are independent of each other (replaying rank r's stream alone
gives the same answer as inside the 2-rank job), and the whole-job rate uses the slowest rank.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_ACT = 20_000
KW = dict(n_invokers=400, n_actions=800, n_namespaces=80)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    for p in (ROOT, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    import oracle as O
    from openwhisk_amd import cluster

    w = cluster.shard_workload("headline", rank, world, n_activations=N_ACT, **KW)
    health = torch.from_numpy(w.inv_status.copy())
    hx = cluster.HealthExchange(dist, health, world)
    agreed = hx.exchange().numpy().copy()
    st = O.state_for(w)
    inv, fl, rf = st.replay(w.stream)
    # configs[4] cadence: each rank all-gathers its health view between batches and applies the agreed vector
    # (updateInvokers, SCPB:512-551) before the batch; the schedule changes the unresponsive set every batch
    sched = cluster.health_schedule(w.inv_status, w.stream.n_batches)
    agreed_b = np.stack([hx.exchange(torch.from_numpy(sched[b])).numpy().copy() for b in range(len(sched))])
    st2 = O.state_for(w)
    inv2, fl2, rf2 = O.replay_with_health(st2, w.stream, w.inv_ids, w.inv_mem, agreed_b)
    t_step = 0.010 * (rank + 1)  # synthetic per-rank step times: the max must win
    t_max, = cluster.max_over_ranks(dist, [t_step], torch.device("cpu"))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), agreed=agreed, disagree=np.array(hx.disagreeing_ranks()),
             inv=inv, fl=fl, rf=rf, permits=st.permits(), act=w.stream.act, t_max=t_max,
             agreed_b=agreed_b, inv2=inv2, fl2=fl2, rf2=rf2, permits2=st2.permits(),
             rate=cluster.whole_job_rate(len(w.stream.act), world, t_max))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_ranks(tmp_path_factory):
    out = tmp_path_factory.mktemp("dist")
    mp.start_processes(_rank_main, args=(2, _free_port(), str(out)), nprocs=2, join=True, start_method="spawn")
    return [dict(np.load(out / f"rank{r}.npz")) for r in range(2)]


def test_shards_share_cluster_not_streams(two_ranks):
    r0, r1 = two_ranks
    assert np.array_equal(r0["agreed"], r1["agreed"])
    assert len(r0["disagree"]) == 0 and len(r1["disagree"]) == 0
    assert not np.array_equal(r0["act"], r1["act"])


def test_shard_slots_hold_half_of_each_invoker(two_ranks):
    from openwhisk_amd import cluster
    import oracle as O

    w = cluster.shard_workload("headline", 0, 2, n_activations=10, **KW)
    st = O.state_for(w)
    assert st.permits().tolist() == [16_384 // 2] * KW["n_invokers"]  # getInvokerSlot: 16 GiB / clusterSize 2


def test_shard_replay_is_independent_of_the_job(two_ranks):
    from openwhisk_amd import cluster
    import oracle as O

    for r in (0, 1):
        w = cluster.shard_workload("headline", r, 2, n_activations=N_ACT, **KW)
        st = O.state_for(w)
        inv, fl, rf = st.replay(w.stream)
        assert np.array_equal(inv, two_ranks[r]["inv"]) and np.array_equal(fl, two_ranks[r]["fl"])
        assert np.array_equal(rf, two_ranks[r]["rf"])
        assert np.array_equal(st.permits(), two_ranks[r]["permits"])


def test_assignments_respect_health(two_ranks):
    health = two_ranks[0]["agreed"]
    for r in two_ranks:
        inv = r["inv"]
        placed = inv[inv >= 0]
        assert len(placed) > 0.9 * len(inv)
        # normal placements (no overload flag) only go to healthy invokers
        normal = inv[(inv >= 0) & ((r["fl"] & 1) == 0)]
        assert np.all(health[normal] == 0)


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` without a torch.distributed environment starts 2 ranks itself (torch.distributed.run as a
    child), each rank takes its controller shard of a 2-controller cluster with split slots (configs[4]), the ranks
    all-gather health once per step and rank 0 prints one line.  --dry-run swaps RCCL for gloo and skips the replay."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                          "--n-activations", "200000"], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] and d["value"] is None
    assert d["config"]["cluster_size"] == 2 and d["config"]["slots"] == "split"
    assert d["config"]["slot_mb"] == 16_384 // 2  # getInvokerSlot: 16 GiB / clusterSize 2
    assert d["config"]["health_disagree"] == []
    assert d["health_allgathers_per_step"] > 1  # one all-gather between batches, not one per step


def test_max_over_ranks_and_rate(two_ranks):
    for r in two_ranks:
        assert float(r["t_max"]) == pytest.approx(0.020)
        assert float(r["rate"]) == pytest.approx(2 * N_ACT / 0.020)


def test_health_change_between_batches_keeps_every_shard_exact(two_ranks):
    """The per-batch health all-gather: both ranks agree on every batch's vector (the shared health topic), and each
    rank's replay with that vector applied before every batch equals its shard replayed alone with the schedule --
    the exchange adds nothing but agreement.  The changing unresponsive sets do change decisions, and normal
    placements of batch b only go to invokers usable in batch b."""
    from openwhisk_amd import cluster
    import oracle as O

    for r in (0, 1):
        w = cluster.shard_workload("headline", r, 2, n_activations=N_ACT, **KW)
        sched = cluster.health_schedule(w.inv_status, w.stream.n_batches)
        assert np.array_equal(two_ranks[r]["agreed_b"], sched)
        st = O.state_for(w)
        inv, fl, rf = O.replay_with_health(st, w.stream, w.inv_ids, w.inv_mem, sched)
        assert np.array_equal(inv, two_ranks[r]["inv2"]) and np.array_equal(fl, two_ranks[r]["fl2"])
        assert np.array_equal(rf, two_ranks[r]["rf2"]) and np.array_equal(st.permits(), two_ranks[r]["permits2"])
        assert not np.array_equal(inv, two_ranks[r]["inv"])  # the schedule matters
        s = w.stream
        for b in range(s.n_batches):
            sl = slice(int(s.acq_off[b]), int(s.acq_off[b + 1]))
            ib, fb = inv[sl], fl[sl]
            normal = ib[(ib >= 0) & ((fb & 1) == 0)]
            assert np.all(sched[b][normal] == 0)
