"""Writes tests/golden/reference_unit_vectors.json: the golden vectors held by the reference's own unit tests
for the invoker-assignment path, re-expressed as data (inputs + expected outputs).

Every case cites the reference test it transcribes (paths relative to the reference repository root).  This script
only writes literals and the closed-form expectations the reference tests themselves state (e.g. T-SCPB:158-171
asserts `blackboxInvokers.size == max(1, (bf * i).toInt)`); it does not execute any reference code.

Run:  python tests/golden/make_golden.py
"""
import json
import os

T_SCPB = "tests/src/test/scala/org/apache/openwhisk/core/loadBalancer/test/ShardingContainerPoolBalancerTests.scala"
T_NS = "tests/src/test/scala/org/apache/openwhisk/common/NestedSemaphoreTests.scala"
T_FS = "tests/src/test/scala/org/apache/openwhisk/common/ForcibleSemaphoreTests.scala"
T_RS = "tests/src/test/scala/org/apache/openwhisk/common/ResizableSemaphoreTests.scala"

MB = 1024 * 1024
MIN_MEMORY_MB = 128  # common/scala/src/main/resources/application.conf:377 (memory.min = 128 m)
STD_MEMORY_MB = 256  # application.conf:379

cases = []

# --------------------------------------------------------------------------------------------- coprime lists
cases.append({
    "name": "pairwise_coprime_numbers_until",
    "source": f"{T_SCPB}:371-384",
    "expect": {"0": [], "-1": [], "1": [1], "2": [1], "3": [1, 2], "4": [1, 3], "5": [1, 2, 3], "9": [1, 2, 5, 7],
               "10": [1, 3, 7]},
})
cases.append({
    "name": "walk_doc_example",
    "source": "core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/"
              "ShardingContainerPoolBalancer.scala:70-77",
    "n": 10, "hash": 13, "home": 3, "step_sizes": [1, 3, 7], "step": 3,
    "order": [3, 6, 9, 2, 5, 8, 1, 4, 7, 0],
})

# --------------------------------------------------------------------------------------------- java hashCode
# JLS String.hashCode; widely published values (collision "Aa"/"BB", MIN_VALUE for "polygenelubricants").
cases.append({
    "name": "java_string_hashcode",
    "source": "JLS java.lang.String.hashCode (JDK 11, un-vendored; call site SCPB:371)",
    "expect": {"": 0, "a": 97, "Aa": 2112, "BB": 2112, "hello": 99162322, "polygenelubricants": -2147483648},
})

# --------------------------------------------------------------------------------------------- schedule
cases.append({
    "name": "schedule_empty_invokers",
    "source": f"{T_SCPB}:248-258",
    "invokers": [], "slots": {"count": 0, "permits": 0}, "max_concurrent": 1,
    "calls": [{"mem": MIN_MEMORY_MB, "index": 0, "step": 2, "expect": None}],
})
cases.append({
    "name": "schedule_no_healthy",
    "source": f"{T_SCPB}:260-272",
    "invokers": [[0, "unhealthy"], [1, "unhealthy"], [2, "unhealthy"]], "slots": {"count": 3, "permits": 3},
    "max_concurrent": 1,
    "calls": [{"mem": MIN_MEMORY_MB, "index": 0, "step": 2, "expect": None}],
})
cases.append({
    "name": "schedule_step_then_overload",
    "source": f"{T_SCPB}:274-299",
    "invokers": [[3, "healthy"], [4, "healthy"], [5, "healthy"]], "slots": {"count": 6, "permits": 3},
    "max_concurrent": 1,
    "calls": [{"mem": 1, "index": 0, "step": 2, "expect": [i, False]} for i in [3, 3, 3, 5, 5, 5, 4, 4, 4]],
    "then_overload": {"calls": 101, "mem": 1, "index": 0, "step": 2, "ids_contain_all": [3, 4, 5],
                      "ids_subset_of": [3, 4, 5]},
})
cases.append({
    "name": "schedule_ignore_unhealthy_offline",
    "source": f"{T_SCPB}:301-327",
    "invokers": [[0, "healthy"], [1, "unhealthy"], [2, "offline"], [3, "healthy"]],
    "slots": {"count": 4, "permits": 3}, "max_concurrent": 1,
    "calls": [{"mem": 1, "index": 0, "step": 1, "expect": [i, False]} for i in [0, 0, 0, 3, 3, 3]],
    "then_overload": {"calls": 101, "mem": 1, "index": 0, "step": 1, "ids_contain_all": [0, 3],
                      "ids_subset_of": [0, 3]},
})
cases.append({
    "name": "schedule_enough_free_slots",
    "source": f"{T_SCPB}:329-367",
    "invokers": [[0, "healthy"], [1, "healthy"], [2, "healthy"]], "slots": {"count": 3, "permits": 4},
    "max_concurrent": 1,
    "calls": [{"mem": m, "index": 0, "step": 1, "expect": [i, False]}
              for m, i in [(3, 0), (2, 1), (1, 0), (4, 2), (2, 1)]],
    "final_permits": [0, 0, 0],
})
calls = []
for i in range(3):
    for _s in range(2):
        for c in range(1, 4):
            calls.append({"mem": 1, "index": 0, "step": 1, "expect": [i, False],
                          "concurrent_permits_after": {"invoker": i, "permits": 3 - c}})
cases.append({
    "name": "schedule_concurrent_actions",
    "source": f"{T_SCPB}:386-412",
    "invokers": [[0, "healthy"], [1, "healthy"], [2, "healthy"]], "slots": {"count": 3, "permits": 2},
    "max_concurrent": 3, "calls": calls,
})

# --------------------------------------------------------------------------------------------- state
cases.append({
    "name": "state_grow_keep_old",
    "source": f"{T_SCPB}:105-148",
    "blackbox_fraction": 0.5, "managed_fraction": 0.5,
    "steps": [
        {"update_invokers": [[0, 1280 * MB, "healthy"]],
         "expect": {"managed": [0], "blackbox": [0], "n_slots": 1, "permits": [1280], "managed_steps": [1],
                    "blackbox_steps": [1]}},
        {"try_acquire": [0, 128], "expect": {"permits": [1152]}},
        {"update_invokers": [[0, 1280 * MB, "healthy"], [1, 2560 * MB, "healthy"]],
         "expect": {"managed": [0], "blackbox": [1], "n_slots": 2, "permits": [1152, 2560], "managed_steps": [1],
                    "blackbox_steps": [1]}},
        {"try_acquire": [1, 128], "expect": {"permits": [1152, 2432]}},
    ],
})
overlap = []
small = {0.1: 10, 0.2: 5, 0.3: 4, 0.4: 3, 0.5: 2}  # T-SCPB:163-169: m + b == i + 1 for i < bound
for bf in [0.1, 0.2, 0.3, 0.4, 0.5]:
    for i in range(1, 101):
        b = max(1, int(bf * i))  # T-SCPB:159 `Math.max(1, (bf * i).toInt)`
        overlap.append({"bf": bf, "i": i, "blackbox_size": b, "managed_plus_blackbox": i + 1 if i < small[bf] else i})
cases.append({"name": "state_overlap_small_n", "source": f"{T_SCPB}:150-175", "user_memory_mb": STD_MEMORY_MB,
              "rows": overlap})
cases.append({"name": "state_full_overlap", "source": f"{T_SCPB}:177-188", "blackbox_fraction": 1.0,
              "managed_fraction": 1.0, "n": 100, "managed_size": 100, "blackbox_size": 100})
cases.append({
    "name": "state_update_cluster",
    "source": f"{T_SCPB}:190-206",
    "blackbox_fraction": 0.5, "managed_fraction": 0.5,
    "steps": [
        {"update_invokers": [[0, 1280 * MB, "healthy"], [1, 2560 * MB, "healthy"]]},
        {"try_acquire": [0, 128], "expect": {"permits": [1152, 2560]}},
        {"try_acquire": [1, 128], "expect": {"permits": [1152, 2432]}},
        {"update_cluster": 2, "expect": {"permits": [640, 1280]}},
    ],
})
cases.append({
    "name": "state_cluster_below_one",
    "source": f"{T_SCPB}:208-225",
    "blackbox_fraction": 0.5, "managed_fraction": 0.5,
    "steps": [
        {"update_invokers": [[0, 1280 * MB, "healthy"]], "expect": {"permits": [1280]}},
        {"update_cluster": 2, "expect": {"permits": [640]}},
        {"update_cluster": 0, "expect": {"permits": [1280]}},
        {"update_cluster": -1, "expect": {"permits": [1280]}},
    ],
})
cases.append({
    "name": "state_cluster_min_memory",
    "source": f"{T_SCPB}:227-239",
    "blackbox_fraction": 0.5, "managed_fraction": 0.5,
    "steps": [
        {"update_invokers": [[0, 1280 * MB, "healthy"]], "expect": {"permits": [1280]}},
        {"update_cluster": 20, "expect": {"permits": [MIN_MEMORY_MB]}},
    ],
})

# --------------------------------------------------------------------------------------------- batch (component)
# T-SCPB:414-569 with whisk.action.concurrency=true (CI local env, ansible/environments/local/group_vars/all:49):
# 3 invokers x 2000 MB, action testspace/testname 256 MB, concurrency 5, namespace invocationSpace, i in [75,105).
conc, inv_mem, act_mem, n_inv = 5, 2000, 256, 3
max_containers = inv_mem // act_mem
per_inv = conc * max_containers
rows = []
for n in range(75, max_containers * n_inv * conc):
    groups, left = [], n
    while left > 0:
        g = min(per_inv, left)
        groups.append({"count": g, "remaining": (conc - g % conc) if g % conc > 0 else 0})
        left -= g
    rows.append({"activations": n, "groups_in_walk_order": groups})
cases.append({
    "name": "balancer_activation_batch",
    "source": f"{T_SCPB}:414-569",
    "namespace": "invocationSpace", "action_path": "testspace/testname", "invoker_memory_mb": inv_mem,
    "action_memory_mb": act_mem, "max_concurrent": conc, "n_invokers": n_inv,
    "managed_fraction": 0.9, "blackbox_fraction": 0.1,  # core/controller/src/main/resources/reference.conf:22-32
    "rows": rows, "after_release": {"permits": [inv_mem] * n_inv, "entries": None},
})

# --------------------------------------------------------------------------------------------- semaphores
cases.append({
    "name": "nested_semaphore_concurrency_first",
    "source": f"{T_NS}:29-51",
    "permits": 20, "key": 1, "max_concurrent": 5, "mem": 3,
    "steps": [
        {"acquire_n": 5, "expect_all": True, "expect_permits": 17, "expect_concurrent": 0},
        {"acquire_n": 25, "expect_all": True, "expect_permits": 2, "expect_concurrent": 0},
        {"acquire_n": 1, "expect_all": False},
    ],
})
cases.append({
    "name": "forcible_semaphore",
    "source": f"{T_FS}:28-75",
    "invalid": [["try_acquire", 0], ["try_acquire", -1], ["force_acquire", 0], ["force_acquire", -1],
                ["release", 0], ["release", -1]],
    "sequences": [
        {"permits": 2, "ops": [["try_acquire", 1, True], ["try_acquire", 1, True], ["try_acquire", 1, False]]},
        {"permits": 4, "ops": [["try_acquire", 5, False], ["try_acquire", 3, True], ["try_acquire", 2, False],
                               ["try_acquire", 1, True]]},
        {"permits": 2, "ops": [["try_acquire", 1, True], ["try_acquire", 1, True], ["try_acquire", 1, False],
                               ["release", 1, None], ["try_acquire", 1, True], ["release", 2, None],
                               ["try_acquire", 2, True]]},
        {"permits": 2, "ops": [["try_acquire", 2, True], ["force_acquire", 5, None], ["try_acquire", 1, False],
                               ["release", 4, None], ["try_acquire", 1, False], ["release", 1, None],
                               ["try_acquire", 1, False], ["release", 1, None], ["try_acquire", 1, True]]},
    ],
})
# T-RS:62-159 verbatim: [op, arg, expected result, expected counter, expected availablePermits or None]
rs_ops = [
    ["try_acquire", 1, True, 1, None], ["try_acquire", 1, True, 2, None], ["try_acquire", 1, False, 2, None],
    ["release_open", 4, [False, False], 3, None], ["try_acquire", 4, True, 4, None],
    ["try_acquire", 1, False, 4, None], ["release_open", 5, [True, False], 5, None],
    ["try_acquire", 1, False, 5, None], ["release_open", 6, [False, False], 6, None],
    ["try_acquire", 1, True, 7, None], ["try_acquire", 1, True, 8, None], ["try_acquire", 1, True, 9, None],
    ["try_acquire", 1, True, 10, None], ["try_acquire", 1, True, 11, None], ["try_acquire", 1, True, 12, None],
    ["try_acquire", 1, False, 12, None], ["release_open", 10, [True, False], 13, None],
    ["try_acquire", 1, True, 14, 4],
]
for res, cnt, av in [([True, False], 13, 0), ([False, False], 12, 1), ([False, False], 11, 2), ([False, False], 10, 3),
                     ([False, False], 9, 4), ([True, False], 8, 0), ([False, False], 7, 1), ([False, False], 6, 2),
                     ([False, False], 5, 3), ([False, False], 4, 4), ([True, False], 3, 0), ([False, False], 2, 1),
                     ([False, False], 1, 2), ([False, True], 0, 3)]:
    rs_ops.append(["release_complete", 1, res, cnt, av])
cases.append({
    "name": "resizable_semaphore_trace",
    "source": f"{T_RS}:29-159",
    "invalid": [["try_acquire", 0], ["try_acquire", -1], ["release_complete", 0], ["release_complete", -1]],
    "max_allowed": 2, "reduction_size": 5, "ops": rs_ops,
})

out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_unit_vectors.json")
with open(out, "w") as f:
    json.dump({"generated_by": "tests/golden/make_golden.py", "cases": cases}, f, indent=1)
print(out, len(cases))
