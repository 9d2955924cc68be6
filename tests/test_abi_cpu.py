"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every symbol include/owgs.h declares,
and refuses to run without a GPU (no silent CPU fallback).  No compute calls."""
import ctypes as C
import os

import numpy as np
import pytest

import openwhisk_amd as ow
from openwhisk_amd import _lib
from openwhisk_amd import workload as W


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def test_header_declares_the_boundary():
    fns = ow.header_functions()
    for required in ["owgs_create", "owgs_destroy", "owgs_update_invokers", "owgs_update_cluster",
                     "owgs_register_actions", "owgs_publish_batch", "owgs_release_batch", "owgs_schedule_walks",
                     "owgs_replay_device", "owgs_last_error"]:
        assert required in fns


def test_library_exports_every_header_symbol(L):
    missing = [f for f in ow.header_functions() if not hasattr(L, f)]
    assert not missing, missing


def test_abi_version_and_limits(L):
    assert L.owgs_abi_version() == 1
    mi, ms = C.c_int32(), C.c_int32()
    assert L.owgs_limits(C.byref(mi), C.byref(ms)) == 0
    assert mi.value >= 20_000 and ms.value >= 20_000  # BASELINE: 10k invokers; the narrow engine geometry holds 20k


def test_engine_objects_refuse_another_geometry(L):
    # a host sized for one engine geometry must never drive the other geometry's object (round 3: a host built for
    # narrower chunks against the regular narrow engine wrote chunk tables out of bounds and the engine spun); both
    # objects' launch wrappers refuse the other's tag before touching the device -- this runs without a GPU
    assert L.owgs_geometry_selfcheck() == 0


def test_no_cpu_fallback_without_gpu(L):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(ow.OwgsError):
        ow.GpuShardingContainerPoolBalancer()


def test_null_arguments_are_rejected_not_crashing(L):
    assert L.owgs_create(None, None) == _lib.EINVAL
    assert L.owgs_update_cluster(None, 2) == _lib.EINVAL
    assert L.owgs_publish_batch(None, 0, None, None, 0, None, None) == _lib.EINVAL
    assert L.owgs_last_error(None) == b"null context"


def test_workload_streams_are_well_formed():
    for name in ["c1", "c2", "c3", "c4", "headline"]:
        w = W.config(name, n_activations=20_000)
        s = w.stream
        n = len(s.act)
        assert s.acq_off[0] == 0 and s.acq_off[-1] == n and np.all(np.diff(s.acq_off) >= 0)
        assert s.rel_off[0] == 0 and s.rel_off[-1] == len(s.rel_aid) and np.all(np.diff(s.rel_off) >= 0)
        assert s.act.min() >= 0 and s.act.max() < len(w.actions)
        # releases only reference activations of strictly earlier batches
        for b in range(s.n_batches):
            r = s.rel_aid[s.rel_off[b]:s.rel_off[b + 1]]
            assert np.all(r < s.acq_off[b])
        assert len(np.unique(s.rel_aid)) == len(s.rel_aid)


def test_workload_is_deterministic():
    a = W.config("headline", n_activations=5000)
    b = W.config("headline", n_activations=5000)
    assert np.array_equal(a.stream.act, b.stream.act) and np.array_equal(a.stream.rel_aid, b.stream.rel_aid)
    assert a.actions == b.actions


def _engine_static_lds(obj: str) -> dict:
    """group_segment_fixed_size (static LDS bytes) of every engine kernel in a built object's gfx950 code object."""
    import re
    import subprocess
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    with tempfile.TemporaryDirectory() as d:
        co, fat = os.path.join(d, "k.co"), os.path.join(d, "fat.bin")
        subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "h.o")],
                       check=True)
        subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, size = {}, None
    for line in notes.splitlines():
        m = re.search(r"\.group_segment_fixed_size:\s+(\d+)", line)
        if m:
            size = int(m.group(1))
        m = re.search(r"\.name:\s+(\S+)", line)
        if m and size is not None:
            out[m.group(1)] = size
            size = None
    return {k: v for k, v in out.items() if "engine" in k and "kernel" in k}


@pytest.mark.parametrize("obj", ["owgs_kernels.o", "owgs_engine_narrow.o"])
def test_engine_kernels_use_no_static_lds(L, obj):
    # the engine's LDS image is dynamic and fills up to 159.5 of 160 KB at the headline: any static __shared__ (a
    # __syncthreads_or, a helper's scratch) would make every launch fail with "invalid argument"
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "build", obj)
    if not os.path.exists(path) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"):
        pytest.skip("build objects or ROCm llvm tools missing")
    sizes = _engine_static_lds(path)
    assert sizes, "no engine kernels found"
    assert all(v == 0 for v in sizes.values()), {k: v for k, v in sizes.items() if v}
