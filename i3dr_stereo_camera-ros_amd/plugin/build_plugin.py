"""Build the OpenCV-free plugin core (hip_sgm_core.cpp) into lib/libsgm_plugin_core.so and
its C++ test driver lib/plugin_core_test, both linked against lib/libsgm_hip.so with g++.
(matcherHIPSGM.cpp needs OpenCV + the reference headers and is built inside the ROS tree.)"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
LIBDIR = os.path.join(PKG, "lib")


def _stale(out, deps):
    return not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps)


def build():
    os.makedirs(LIBDIR, exist_ok=True)
    inc = ["-I" + HERE, "-I" + os.path.join(ROOT, "include")]
    core_src = os.path.join(HERE, "hip_sgm_core.cpp")
    deps = [core_src, os.path.join(HERE, "hip_sgm_core.h"), os.path.join(ROOT, "include", "sgm_hip.h")]
    so = os.path.join(LIBDIR, "libsgm_plugin_core.so")
    link = ["-L" + LIBDIR, "-lsgm_hip", "-Wl,-rpath,$ORIGIN"]
    if _stale(so, deps):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra"] + inc +
                              [core_src, "-o", so] + link)
    drv_src = os.path.join(HERE, "plugin_core_test.cpp")
    drv = os.path.join(LIBDIR, "plugin_core_test")
    if _stale(drv, deps + [drv_src]):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra"] + inc +
                              [drv_src, core_src, "-o", drv] + link)
    return so


if __name__ == "__main__":
    build()
