"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the host code.

* oracle/sgm_oracle.c with the seeded fuzz driver oracle/asan_fuzz.c: every entry point over
  random geometries, parameters and OpenCV build-variant switches (the oracle pins every GPU
  parity claim, and once read past a row: commit 96b0ed7);
* the plugin core (hip_sgm_core.cpp) with its C++ driver, `plugin_core_test setters`.

Host code only (GPU sanitizers are not available on the pool). CPU tests.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.fixture(scope="module")
def outdir(tmp_path_factory):
    return tmp_path_factory.mktemp("san")


def _env():
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "abort_on_error=0:halt_on_error=1:detect_leaks=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    return env


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
@pytest.mark.parametrize("first,count", [(1, 400), (5000, 400)])
def test_oracle_asan_ubsan_fuzz(outdir, first, count):
    exe = os.path.join(outdir, "asan_fuzz")
    if not os.path.exists(exe):
        subprocess.check_call(["gcc", "-std=gnu11", "-Wall"] + SAN + ["-I" + os.path.join(ROOT, "include"),
                               os.path.join(ROOT, "oracle", "sgm_oracle.c"),
                               os.path.join(ROOT, "oracle", "asan_fuzz.c"), "-o", exe])
    r = subprocess.run([exe, str(first), str(count)], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip() == f"ok {count}"


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_plugin_core_setters_asan_ubsan(outdir):
    plug = os.path.join(ROOT, "i3dr_stereo_camera-ros_amd", "plugin")
    lib = os.path.join(ROOT, "i3dr_stereo_camera-ros_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libsgm_hip.so")):
        pytest.fail("libsgm_hip.so missing: run build() first")
    exe = os.path.join(outdir, "plugin_core_test_asan")
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Wextra"] + SAN +
                          ["-I" + plug, "-I" + os.path.join(ROOT, "include"),
                           os.path.join(plug, "plugin_core_test.cpp"), os.path.join(plug, "hip_sgm_core.cpp"),
                           "-o", exe, "-L" + lib, "-lsgm_hip", "-Wl,-rpath," + lib])
    env = _env()
    # the HIP runtime (not our code) keeps process-lifetime allocations: no leak report
    env["ASAN_OPTIONS"] = "halt_on_error=1:detect_leaks=0"
    r = subprocess.run([exe, "setters"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "setters ok" in r.stdout
