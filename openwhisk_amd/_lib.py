"""ctypes binding of libowgs.so (the C ABI in include/owgs.h).

The product path has no CPU fallback: if the HIP library is missing or no MI355X is visible, every constructor
raises.  build() compiles the library in-tree (hipcc --offload-arch=gfx950).
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_PATH = os.environ.get("OWGS_LIB") or os.path.join(PKG, "libowgs.so")
HEADER = os.path.join(ROOT, "include", "owgs.h")

OK = 0
EINVAL, ENOMEM, EDEVICE, ERANGE, ENOENT = -22, -12, -5, -34, -2
NONE, THROW_INDEX = -1, -2
FLAG_OVERLOAD = 1
REL_NOSUCHELEMENT, REL_OVERFLOW, REL_NOENTRY = 1, 2, 4
ACK_FAIL, ACK_JVM, ACK_UNSUPPORTED, ACK_RELEASED, ACK_HEALTH, ACK_NOENTRY, ACK_FORCED_NOENTRY = range(7)
HEALTHY, UNHEALTHY, UNRESPONSIVE, OFFLINE = 0, 1, 2, 3


class OwgsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"owgs error {code}: {msg}")
        self.code = code


class owgs_config(C.Structure):
    _fields_ = [
        ("managed_fraction", C.c_double),
        ("blackbox_fraction", C.c_double),
        ("min_memory_bytes", C.c_int64),
        ("cluster_size", C.c_int32),
        ("device", C.c_int32),
        ("rng_seed", C.c_uint64),
    ]


class owgs_replay_io(C.Structure):
    """include/owgs.h: owgs_replay_io (one controller shard of owgs_replay_device_multi)."""
    _fields_ = [("n_batches", C.c_int32), ("acq_off", C.c_void_p), ("act", C.c_void_p),
                ("n_activations", C.c_int64), ("rel_off", C.c_void_p), ("rel_aid", C.c_void_p),
                ("n_releases", C.c_int64), ("seq_base", C.c_uint64), ("out_invoker", C.c_void_p),
                ("out_flags", C.c_void_p), ("rel_flags", C.c_void_p)]


class owgs_msg_batch(C.Structure):
    _fields_ = [("n", C.c_int32)] + [(k, C.c_void_p) for k in (
        "invoker", "tmpl", "aid", "tid", "tid_off", "tid_start", "flags", "content", "content_off", "cause", "trace",
        "trace_off")]


def build(verbose: bool = False) -> str:
    """Compile libowgs.so for gfx950 in-tree."""
    out = subprocess.run(["make", "-s", "-C", PKG], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"libowgs build failed:\n{out.stdout}\n{out.stderr}")
    return LIB_PATH


def header_functions() -> list[str]:
    """Names of every function declared in include/owgs.h."""
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(owgs_\w+)\s*\(", src, flags=re.M)))


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OwgsError(EDEVICE, f"{LIB_PATH} is missing: run openwhisk_amd._lib.build() (hipcc, gfx950)")
    # PyTorch-ROCm ships its own HIP runtime: when both are used in one process, torch's must be the one loaded
    # (libowgs.so then binds to it by soname); loading libowgs first leaves torch without a visible device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    i32, u64, P = C.c_int32, C.c_uint64, C.c_void_p
    sig = {
        "owgs_abi_version": (C.c_int, []),
        "owgs_limits": (C.c_int, [P, P]),
        "owgs_create": (C.c_int, [P, P]),
        "owgs_destroy": (None, [P]),
        "owgs_last_error": (C.c_char_p, [P]),
        "owgs_update_invokers": (C.c_int, [P, i32, P, P, P]),
        "owgs_update_cluster": (C.c_int, [P, i32]),
        "owgs_health_events": (C.c_int, [P, i32, P, P, P, P, C.c_int64, i32]),
        "owgs_register_templates": (C.c_int, [P, i32, P, P, P, P, P]),
        "owgs_engine_ms": (C.c_int, [P, P]),
        "owgs_resident_stats": (C.c_int, [P, P, i32]),
        "owgs_set_root_controller": (C.c_int, [P, C.c_char_p, i32]),
        "owgs_serialize_activations": (C.c_int, [P, P, i32, P, C.c_int64, P, P, P, P, P]),
        "owgs_serialize_activations_device": (C.c_int, [P, P, i32, P, C.c_int64, P, P, P, P, P, P]),
        "owgs_health_read": (C.c_int, [P, i32, P, P, P, P, P, P]),
        "owgs_register_actions": (C.c_int, [P, i32, P, P, P, P, P, P, P, P, P, P, P]),
        "owgs_publish_batch": (C.c_int, [P, i32, P, P, u64, P, P]),
        "owgs_release_batch": (C.c_int, [P, i32, P, P, P]),
        "owgs_process_batch": (C.c_int, [P, i32, P, P, P, P, P, P, P, u64, P, P]),
        "owgs_schedule_walks": (C.c_int, [P, i32, P, P, P, P, P, P, P, P, P]),
        "owgs_set_slots": (C.c_int, [P, i32, P]),
        "owgs_set_pool": (C.c_int, [P, i32, i32, P, P]),
        "owgs_read_permits": (C.c_int, [P, P, i32, P]),
        "owgs_read_concurrent": (C.c_int, [P, i32, i32, P, P]),
        "owgs_key_id": (C.c_int, [P, i32]),
        "owgs_map_fill": (C.c_int, [P, P, P, P, P]),
        "owgs_release_actions": (C.c_int, [P, i32, P]),
        "owgs_geometry_selfcheck": (C.c_int, []),
        "owgs_state_info": (C.c_int, [P, P, P, P, P]),
        "owgs_step_sizes": (C.c_int, [P, i32, P, i32, P]),
        "owgs_pairwise_coprime": (C.c_int, [P, i32, P, i32, P]),
        "owgs_set_health_tid": (C.c_int, [P, C.c_int64]),
        "owgs_track_activations": (C.c_int, [P, i32, P, P, P, P, P]),
        "owgs_process_acks": (C.c_int, [P, i32, P, P, P, P, P, P]),
        "owgs_process_acks_device": (C.c_int, [P, i32, P, P, P, P, P, P, P]),
        "owgs_complete_activations": (C.c_int, [P, i32, P, P, P, P, P, P]),
        "owgs_activations_live": (C.c_int, [P, P]),
        "owgs_replay_device": (C.c_int, [P, i32, P, P, C.c_int64, P, P, C.c_int64, u64, P, P, P, P]),
        "owgs_replay_device_multi": (C.c_int, [P, i32, P, P]),
        "owgs_replay_device_span": (C.c_int, [P, C.c_int64, C.c_int64, C.c_int64, C.c_int64, P, P, u64, P, P, P, P]),
        "owgs_replay_device_group": (C.c_int, [P, C.c_int32, P, P, P, P, u64, P, P, P, P, C.c_int64, C.c_int32, P]),
        "owgs_replay": (C.c_int, [P, i32, P, P, P, P, u64, P, P, P]),
        "owgs_snapshot": (C.c_int, [P]),
        "owgs_restore": (C.c_int, [P, P]),
        "owgs_update_health_device": (C.c_int, [P, i32, P, P]),
        "owgs_read_stats": (C.c_int, [P, P, i32]),
        "owgs_selftest": (C.c_int, [P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L
