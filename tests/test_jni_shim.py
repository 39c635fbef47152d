"""CPU: the JNI shim (jni/stcjni.c) compiled and exercised without a JDK or a GPU.

No JDK exists in this container, so tests/jni_stub/jni.h stands in for <jni.h> (the JNI types and the
JNIEnv function-table entries the shim uses, with the specification's signatures).  gcc type-checks the
shim against it with every warning an error, and tests/jni_stub/mock_env.c runs the wrappers against a
mock JNIEnv and the real libstc.so: a Java array shorter than what the C ABI would read or write must
throw IllegalArgumentException before anything is pinned (advisor round 2), and a correctly sized
call must reach the library.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "jni_stub")
LIBDIR = os.path.join(ROOT, "spark-text-clustering_amd", "stc")
GCC = shutil.which("gcc")


@pytest.mark.skipif(GCC is None, reason="gcc not found")
def test_shim_type_checks_against_the_jni_signatures():
    r = subprocess.run([GCC, "-fsyntax-only", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-I", STUB, "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "jni", "stcjni.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(GCC is None or not os.path.exists(os.path.join(LIBDIR, "libstc.so")),
                    reason="gcc or libstc.so missing (run __graft_entry__.build())")
def test_short_java_arrays_throw_before_the_library_is_called(tmp_path):
    exe = str(tmp_path / "mock_env")
    r = subprocess.run([GCC, "-std=c99", "-Wall", "-Wno-unused-parameter", "-I", STUB, "-I", os.path.join(ROOT, "include"),
                        os.path.join(STUB, "mock_env.c"), "-L", LIBDIR, "-lstc", "-Wl,-rpath," + LIBDIR, "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rows = {}
    for line in out.stdout.strip().splitlines():
        name, cls, msg = line.split("\t")
        rows[name] = (cls, msg)
    iae = "java/lang/IllegalArgumentException"
    short = {"hashingTf_short_indices": ("hashingTf indicesOut", 2, 3), "hashingTf_short_indptr": ("hashingTf indptrOut", 2, 3),
             "hashTokens_short": ("hashTokens idxOut", 2, 3), "tokenize_short_tokoff": ("tokenize tokOffOut", 6, 7),
             "tokenize_short_utf8": ("tokenize utf8Out", 6, 7), "dcsrUpload_short_indices": ("dcsrUpload indices", 4, 5),
             "dcsrUpload_short_indptr": ("dcsrUpload indptr", 3, 4), "ldaCounters_short": ("ldaCounters out", 3, 4),
             "ldaPhaseTimes_short": ("ldaPhaseTimes msOut", 4, 5)}
    for name, (what, have, need) in short.items():
        assert rows[name] == (iae, f"{what}: the Java array has {have} elements, the call needs {need}"), (name, rows[name])
    # a correctly sized call reaches the library (which rejects the null context itself)
    assert rows["hashingTf_sized"][0] == iae and rows["hashingTf_sized"][1].startswith("requirement failed: ctx")
    # the handle's shape is looked up (and fails on a null handle) before any array is touched
    assert rows["ldaGetTopics_null_handle"] == (iae, "requirement failed: lda")
    # idfGet sizes its checks from the model (stc_didf_shape), not from the caller's cols
    assert rows["idfGet_null_model"] == (iae, "requirement failed: model")
    # the ml transform's batched call (HipLDAModel → groupTopicDistribution) reaches stc_group_topic_distribution
    assert rows["groupTopicDistribution_null_group"] == (iae, "requirement failed: group/member index")
