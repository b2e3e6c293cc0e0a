"""The MatcherHIPSGM adapter (plugin/matcherHIPSGM.{h,cpp}) against the reference's own plugin
header: a `-fsyntax-only` compile of the adapter with the reference's
include/stereoMatcher/abstractStereoMatcher.h:12-92 and a declaration-only opencv2 stub
(tests/stub/opencv2/opencv.hpp). It checks that every pure virtual is overridden with the right
signature and that the adapter only uses what the base class provides; nothing is linked or
run. Skipped where the reference tree is absent (the GPU box)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_INC = "/root/reference/include"
PLUG = os.path.join(ROOT, "i3dr_stereo_camera-ros_amd", "plugin")


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_INC, "stereoMatcher", "abstractStereoMatcher.h")),
                    reason="reference tree not present")
def test_adapter_compiles_against_reference_header(tmp_path):
    # the adapter includes "stereoMatcher/matcherHIPSGM.h" like the other matchers: lay the
    # two adapter files out as they would sit in the reference tree
    inc = tmp_path / "include" / "stereoMatcher"
    inc.mkdir(parents=True)
    shutil.copy(os.path.join(PLUG, "matcherHIPSGM.h"), inc / "matcherHIPSGM.h")
    # the reference's base header stays where it is: only its directory goes on the path
    cmd = ["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Werror",
           "-I", str(tmp_path / "include"), "-I", REF_INC, "-I", os.path.join(ROOT, "tests", "stub"),
           "-I", PLUG, "-I", os.path.join(ROOT, "include"), os.path.join(PLUG, "matcherHIPSGM.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # and it is a concrete class: instantiating it needs every pure virtual overridden
    probe = tmp_path / "probe.cpp"
    probe.write_text('#include "stereoMatcher/matcherHIPSGM.h"\n'
                     'AbstractStereoMatcher* make(std::string& f) { return new MatcherHIPSGM(f, cv::Size(640, 480)); }\n')
    r = subprocess.run(cmd[:-1] + [str(probe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
