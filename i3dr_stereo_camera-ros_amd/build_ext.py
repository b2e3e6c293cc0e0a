"""In-tree build of libsgm_hip.so (hand-written HIP for gfx950) and the host plugin core.

`python build_ext.py` or `build()` — hipcc cross-compiles for gfx950 without a GPU.
The .so lands in lib/ next to this file (git-ignored, but it travels to the GPU box).
"""
import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
BUILDDIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIBDIR, "libsgm_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["census_sgm.hip", "ocv_sgm.hip", "post.hip", "depth.hip", "rectify.hip", "sgm_api.cpp"]
HEADERS = ["sgm_device.h"]


def _flags():
    return ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I" + CSRC,
            "-I" + os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function"]


def _compile(src):
    obj = os.path.join(BUILDDIR, os.path.basename(src) + ".o")
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(ROOT, "include", "sgm_hip.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    lang = ["-x", "hip"]
    cmd = [HIPCC] + _flags() + lang + ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return obj


def build(verbose=True):
    os.makedirs(BUILDDIR, exist_ok=True)
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(o) for o in objs):
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build()
