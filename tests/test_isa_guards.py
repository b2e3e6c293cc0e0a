"""Code-generation guards on the built libsgm_hip.so (CPU only: the gfx950 code objects are read
out of the library's .hip_fatbin section and disassembled with the ROCm LLVM tools).

Round 5 found a silent regression that no parity test could see: after the round-robin deal of
the path directions, hipcc no longer proved the block's volume slot uniform and wrapped every
buffer load and store of the small-D `k_ocv_paths` instantiations in a readfirstlane waterfall
loop (135 `v_readfirstlane_b32` per kernel; C1 paths 0.080 -> 0.101 ms). The kernel now states
the values uniform; this test keeps it that way for every path-kernel instantiation and for the
census path / fused kernels and the packed OCV WTA.

Round 6 found another: `k_ocv_vwta_pk` kept 8 steps of operands in flight whatever the values per
lane, so at 16 per lane (D > 512, the processing launch's D = 752) it spilled 904 B per lane to
scratch (MODE_HH fused vertical WTA 21.3 ms, 7.85 ms without). `test_no_scratch_spills` reads every
kernel's private segment size from the code objects' metadata.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "i3dr_stereo_camera-ros_amd", "lib", "libsgm_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(tmp_path):
    """The gfx950 code objects of the library (paths of unbundled .co files)."""
    if not os.path.exists(LIB):
        pytest.skip("libsgm_hip.so not built")
    for tool in ("clang-offload-bundler", "llvm-objdump"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            pytest.skip(f"{tool} not available")
    objcopy = shutil.which("objcopy")
    if not objcopy:
        pytest.skip("objcopy not available")
    # objcopy rewrites its input when no output file is given: work on a copy, never on the
    # library a test process may have mapped
    lib = tmp_path / "lib.so"
    shutil.copyfile(LIB, lib)
    fat = tmp_path / "fatbin"
    subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", str(lib), str(tmp_path / "lib_out.so")],
                   check=True, capture_output=True)
    data = fat.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in .hip_fatbin"
    cos = []
    for i, s in enumerate(starts):
        part = tmp_path / f"b{i}"
        part.write_bytes(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = tmp_path / f"b{i}.co"
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode != 0 or not co.exists() or co.stat().st_size == 0:
            continue
        cos.append(co)
    return cos


def _disassembly(tmp_path):
    text = []
    for co in _code_objects(tmp_path):
        d = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                           capture_output=True, text=True)
        text.append(d.stdout)
    return "\n".join(text)


def _scratch_sizes(tmp_path):
    """{kernel symbol: private segment bytes per lane} from the code objects' AMDGPU metadata."""
    out = {}
    for co in _code_objects(tmp_path):
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], capture_output=True,
                               text=True).stdout
        for blk in notes.split("  - .")[1:]:
            nm = re.search(r"\.name:\s+(\S+)", blk)
            ps = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
            if nm and ps:
                out[nm.group(1)] = int(ps.group(1))
    return out


def _kernels(asm, prefix):
    out = {}
    for m in re.finditer(r"^[0-9a-f]+ <(" + re.escape(prefix) + r"\S*)>:\n", asm, re.M):
        end = asm.find("\n\n", m.end())
        out[m.group(1)] = asm[m.end():end if end > 0 else len(asm)]
    return out


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    return _disassembly(tmp_path_factory.mktemp("isa"))


def test_path_kernels_have_no_waterfall_loops(asm):
    ks = _kernels(asm, "_ZN3sgm11k_ocv_paths")
    assert len(ks) >= 30, f"expected every k_ocv_paths instantiation, found {len(ks)}"
    for name, body in ks.items():
        n = body.count("v_readfirstlane_b32")
        assert n <= 16, f"{name}: {n} v_readfirstlane (a waterfall loop around non-uniform buffer descriptors?)"


def test_census_and_wta_kernels_have_no_waterfall_loops(asm):
    for prefix in ("_ZN3sgm16k_census_fused16", "_ZN3sgm16k_census_paths16", "_ZN3sgm14k_ocv_wta16_pk"):
        ks = _kernels(asm, prefix)
        assert ks, f"no {prefix} in the library"
        for name, body in ks.items():
            n = body.count("v_readfirstlane_b32")
            assert n <= 16, f"{name}: {n} v_readfirstlane"


# Instantiations allowed to use scratch, with the reason: 32 values per path lane are D > 1024, which
# no configuration of the reference reaches (its widest search is D = 752). (The shipped block-21 cost
# kernel had kept ring slot 0 in 12 B of scratch until round 6; that slot now lives in LDS.)
SCRATCH_ALLOWED = ("_ZN3sgm10k_ocv_vwtaILi32E", "_ZN3sgm13k_ocv_vwta_pkILi32E")


def test_no_scratch_spills(tmp_path):
    sizes = _scratch_sizes(tmp_path)
    assert len(sizes) > 200, f"expected the library's kernels, found {len(sizes)}"
    bad = {k: v for k, v in sizes.items() if v > 0 and not k.startswith(SCRATCH_ALLOWED)}
    assert not bad, f"kernels spilling to scratch: {bad}"
