"""Pins the CPU oracle to the reference's own unit-test vectors (tests/golden/reference_unit_vectors.json).

Each case cites the reference test it re-expresses.  CPU only.
"""
import numpy as np
import pytest

import oracle as O

ST = {"healthy": O.HEALTHY, "unhealthy": O.UNHEALTHY, "unresponsive": O.UNRESPONSIVE, "offline": O.OFFLINE}
MB = 1024 * 1024


def test_coprime(golden):
    for x, exp in golden["pairwise_coprime_numbers_until"]["expect"].items():
        assert O.pairwise_coprime_numbers_until(int(x)) == exp


def test_coprime_sizes_at_bench_pools():
    # |f(900)|, |f(1000)|, |f(9000)|, |f(10000)|
    assert [len(O.pairwise_coprime_numbers_until(x)) for x in (900, 1000, 9000, 10000)] == [152, 167, 1115, 1228]
    f9000 = O.pairwise_coprime_numbers_until(9000)
    assert f9000[:4] == [1, 7, 11, 13] and f9000[-1] == 8999


def test_walk_doc_example(golden):
    c = golden["walk_doc_example"]
    assert O.pairwise_coprime_numbers_until(c["n"]) == c["step_sizes"]
    home = c["hash"] % c["n"]
    step = c["step_sizes"][c["hash"] % len(c["step_sizes"])]
    assert (home, step) == (c["home"], c["step"])
    assert [(home + s * step) % c["n"] for s in range(c["n"])] == c["order"]


def test_java_hash(golden):
    for s, h in golden["java_string_hashcode"]["expect"].items():
        assert O.java_hash(s) == h
    assert O.generate_hash("x", "polygenelubricants") != -2**31  # xor with a nonzero hash
    # Int.MinValue.abs stays negative (SCPB:371)
    assert O.generate_hash("", "polygenelubricants") == -2**31


def _run_schedule_case(c, zombies):
    inv = [(i, ST[s]) for i, s in c["invokers"]]
    slots = O.Slots(c["slots"]["count"], c["slots"]["permits"], zombies=zombies)
    key = 7
    for call in c["calls"]:
        r = O.schedule(c["max_concurrent"], key, inv, slots, call["mem"], call["index"], call["step"])
        exp = call["expect"]
        assert (r is None and exp is None) or (r is not None and list(r) == exp)
        if "concurrent_permits_after" in call:
            cp = call["concurrent_permits_after"]
            st = slots[cp["invoker"]].concurrent_state(key)
            assert st is not None and st[0] == cp["permits"]
    if "then_overload" in c:
        t = c["then_overload"]
        res = [O.schedule(c["max_concurrent"], key, inv, slots, t["mem"], t["index"], t["step"], seq=s, rng_seed=99)
               for s in range(t["calls"])]
        ids = {r[0] for r in res}
        assert set(t["ids_contain_all"]) <= ids <= set(t["ids_subset_of"])
        assert all(r[1] for r in res)
    if "final_permits" in c:
        assert [slots[i].available_permits for i in range(len(slots))] == c["final_permits"]


@pytest.mark.parametrize("zombies", [True, False])
@pytest.mark.parametrize("name", ["schedule_empty_invokers", "schedule_no_healthy", "schedule_step_then_overload",
                                  "schedule_ignore_unhealthy_offline", "schedule_enough_free_slots",
                                  "schedule_concurrent_actions"])
def test_schedule(golden, name, zombies):
    _run_schedule_case(golden[name], zombies)


def _run_state_steps(c):
    s = O.BalancerState(c["managed_fraction"], c["blackbox_fraction"])
    for step in c["steps"]:
        if "update_invokers" in step:
            u = step["update_invokers"]
            s.update_invokers([x[0] for x in u], [x[1] for x in u], [ST[x[2]] for x in u])
            ids = [x[0] for x in u]
        if "try_acquire" in step:
            i, m = step["try_acquire"]
            assert s.invoker_slots[i].try_acquire(m)
        if "update_cluster" in step:
            s.update_cluster(step["update_cluster"])
        e = step.get("expect", {})
        if "permits" in e:
            assert s.permits().tolist() == e["permits"]
        if "n_slots" in e:
            assert len(s.invoker_slots) == e["n_slots"]
        if "managed" in e:
            assert ids[: s.managed_size] == e["managed"]
        if "blackbox" in e:
            assert ids[len(ids) - s.blackbox_size:] == e["blackbox"]
        if "managed_steps" in e:
            assert s.managed_step_sizes == e["managed_steps"]
            assert s.blackbox_step_sizes == e["blackbox_steps"]


@pytest.mark.parametrize("name", ["state_grow_keep_old", "state_update_cluster", "state_cluster_below_one",
                                  "state_cluster_min_memory"])
def test_state(golden, name):
    _run_state_steps(golden[name])


def test_state_overlap(golden):
    c = golden["state_overlap_small_n"]
    states = {}
    for row in c["rows"]:
        bf = row["bf"]
        if bf not in states:
            states[bf] = O.BalancerState(1.0 - bf, bf)
        s = states[bf]
        i = row["i"]
        s.update_invokers([1] * i, [c["user_memory_mb"] * MB] * i, [O.HEALTHY] * i)
        assert s.managed_size <= i
        assert s.blackbox_size == row["blackbox_size"]
        assert s.managed_size + s.blackbox_size == row["managed_plus_blackbox"]


def test_state_full_overlap(golden):
    c = golden["state_full_overlap"]
    s = O.BalancerState(c["managed_fraction"], c["blackbox_fraction"])
    for i in range(1, c["n"] + 1):
        s.update_invokers([1] * i, [256 * MB] * i, [O.HEALTHY] * i)
    assert s.managed_size == c["managed_size"] and s.blackbox_size == c["blackbox_size"]


@pytest.mark.parametrize("zombies", [True, False])
def test_balancer_activation_batch(golden, zombies):
    c = golden["balancer_activation_batch"]
    n_inv = c["n_invokers"]
    for row in c["rows"]:
        s = O.BalancerState(c["managed_fraction"], c["blackbox_fraction"], zombies=zombies)
        s.update_invokers(list(range(n_inv)), [c["invoker_memory_mb"] * MB] * n_inv, [O.HEALTHY] * n_inv)
        a = s.register_action(c["namespace"], c["action_path"], 1, c["action_memory_mb"], c["max_concurrent"])
        h = s.action_hash(a)
        assert h == O.generate_hash(c["namespace"], c["action_path"])
        steps = O.pairwise_coprime_numbers_until(n_inv)
        home, step = h % n_inv, steps[h % len(steps)]
        got = [s.publish(a, i) for i in range(row["activations"])]
        assert all(f == 0 for _, f in got)
        nxt = home
        for g in row["groups_in_walk_order"]:
            st = s.invoker_slots[nxt].concurrent_state(1)
            assert st == (g["remaining"], g["count"])
            nxt = (nxt + step) % n_inv
        for inv, _ in got:
            assert s.release(inv, a) == 0
        assert s.permits().tolist() == c["after_release"]["permits"]
        assert all(s.invoker_slots[i].concurrent_state(1) is None for i in range(n_inv))


def test_nested_semaphore(golden):
    c = golden["nested_semaphore_concurrency_first"]
    s = O.NestedSemaphore(c["permits"])
    assert s.available_permits == c["permits"]
    for st in c["steps"]:
        res = [s.try_acquire_concurrent(c["key"], c["max_concurrent"], c["mem"]) for _ in range(st["acquire_n"])]
        assert all(r == st["expect_all"] for r in res)
        if "expect_permits" in st:
            assert s.available_permits == st["expect_permits"]
            assert s.concurrent_state(c["key"])[0] == st["expect_concurrent"]


def test_forcible_semaphore(golden):
    c = golden["forcible_semaphore"]
    for op, arg in c["invalid"]:
        with pytest.raises(ValueError):
            getattr(O.NestedSemaphore(2), op)(arg)
    for seq in c["sequences"]:
        s = O.NestedSemaphore(seq["permits"])
        for op, arg, exp in seq["ops"]:
            r = getattr(s, op)(arg)
            if exp is not None:
                assert r == exp


def test_resizable_semaphore(golden):
    c = golden["resizable_semaphore_trace"]
    for op, arg in c["invalid"]:
        s = O.ResizableSemaphore(2, 5)
        with pytest.raises(ValueError):
            s.try_acquire(arg) if op == "try_acquire" else s.release(arg, True)
    s = O.ResizableSemaphore(c["max_allowed"], c["reduction_size"])
    for op, arg, exp, counter, avail in c["ops"]:
        if op == "try_acquire":
            r = s.try_acquire(arg)
        else:
            r = list(s.release(arg, op == "release_complete"))
        assert r == exp, (op, arg)
        assert s.counter == counter
        if avail is not None:
            assert s.available_permits == avail


def test_rng_is_uniform_enough():
    n = 7
    counts = np.bincount([O.rng_index(1234, s, n) for s in range(70000)], minlength=n)
    assert counts.min() > 9000 and counts.max() < 11000
