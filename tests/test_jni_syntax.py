"""The JNI binding (integration/owgs_jni.c) compiles cleanly (-Wall -Wextra -Werror) against a minimal jni.h
stand-in (this image has no JDK) and the shim's native methods all have a C implementation with the JNI name."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_jni_binding_compiles(tmp_path):
    out = tmp_path / "owgs_jni.o"
    r = subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-fPIC",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"), "-c",
                        os.path.join(ROOT, "integration", "owgs_jni.c"), "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_native_method_is_bound():
    scala = open(os.path.join(ROOT, "integration", "GpuShardingContainerPoolBalancer.scala")).read()
    natives = set(re.findall(r"@native def (\w+)", scala))
    c = open(os.path.join(ROOT, "integration", "owgs_jni.c")).read()
    bound = set(re.findall(r"Java_org_apache_openwhisk_core_loadBalancer_OwgsNative_00024_(\w+)\(", c))
    assert natives and natives <= bound, natives - bound
