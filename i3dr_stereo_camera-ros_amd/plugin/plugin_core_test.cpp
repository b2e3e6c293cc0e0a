// plugin_core_test — C++ driver of the plugin core, the C++ analogue of the reference's
// only executable check, init_stereo_matchers (src/init_stereo_matchers.cpp:39-66): build
// a matcher, match a 10x10 zero pair, fail on a non-zero exit code or an empty result.
// Modes:  plugin_core_test init              (the warm-up; needs a GPU)
//         plugin_core_test setters           (setter semantics; no GPU)
//         plugin_core_test match <L.raw> <R.raw> <W> <H> <out.f32> [algo params...]
//         plugin_core_test time <L.raw> <R.raw> <W> <H> <algo> <D> <minD> <block> <reps>
//                          (ms per forwardMatch: the node's host-buffer call, float output)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <vector>

#include "hip_sgm_core.h"

static int fail(const char* m) { std::fprintf(stderr, "FAIL: %s\n", m); return 1; }

int main(int argc, char** argv)
{
    const char* mode = argc > 1 ? argv[1] : "setters";
    if (!std::strcmp(mode, "setters")) {
        sgm_hip::MatcherCore m(0, SGM_MODE_OCV_SGBM5);
        if (m.params().min_disparity != 64 || m.params().num_disparities != 9 || m.params().block_size != 5)
            return fail("create(64, 9, 5) defaults");
        m.setDisparityRange(0, 640);
        if (m.disparityRange() != ((640 / 8 + 15) & -16)) return fail("setDisparityRange(<=0)");
        m.setDisparityRange(96, 640);
        if (m.disparityRange() != 96) return fail("setDisparityRange");
        m.setP1(200.9f);
        m.setP2(-3.5f);
        if (m.params().p1 != 200 || m.params().p2 != -3) return fail("float -> int truncation");
        m.setMinDisparity(9);
        sgm_params r = sgm_hip::MatcherCore::rightMatcherParams(m.params());
        if (r.min_disparity != -(9 + 96) + 1 || r.uniqueness_ratio != 0 || r.disp12_max_diff != 1000000 ||
            r.speckle_window_size != 0)
            return fail("right matcher params");
        std::printf("setters ok\n");
        return 0;
    }
    if (!std::strcmp(mode, "compat")) {          // SGM_HIP_OCV_COMPAT as the adapter core reads it
        std::printf("%d\n", sgm_hip::ocv_compat_from_env(SGM_OCV_COMPAT_MELODIC));
        return 0;
    }
    if (!std::strcmp(mode, "init")) {
        sgm_hip::MatcherCore m(0, SGM_MODE_OCV_SGBM5);
        m.setDisparityRange(16, 10);
        m.setMinDisparity(0);
        m.setWindowSize(3);
        std::vector<uint8_t> z(100, 0);
        std::vector<float> d(100, -1.f);
        int rc = m.forwardMatch(z.data(), z.data(), 10, 10, 10, d.data(), 10);
        if (rc != 0) return fail("Failed to compute stereo match");
        std::printf("Stereo matchers init complete. d[0]=%g\n", d[0]);
        return 0;
    }
    if (!std::strcmp(mode, "match") && argc >= 7) {
        const int W = std::atoi(argv[4]), H = std::atoi(argv[5]);
        std::vector<uint8_t> L((size_t)W * H), R((size_t)W * H);
        std::ifstream(argv[2], std::ios::binary).read((char*)L.data(), L.size());
        std::ifstream(argv[3], std::ios::binary).read((char*)R.data(), R.size());
        sgm_hip::MatcherCore m(0, argc > 7 ? std::atoi(argv[7]) : SGM_MODE_OCV_SGBM5);
        // updateMatcher() with the node defaults (generate_disparity.cpp:100-112, :241-261)
        m.setDisparityRange(argc > 8 ? std::atoi(argv[8]) : 64, W);
        m.setWindowSize(15);
        m.setMinDisparity(argc > 9 ? std::atoi(argv[9]) : 9);
        m.setUniquenessRatio(15);
        m.setSpeckleFilterRange(4);
        m.setSpeckleFilterWindow(100);
        m.setPreFilterCap(31);
        m.setP1(200);
        m.setP2(400);
        m.setInterpolation(argc > 10 && std::atoi(argv[10]) != 0);
        std::vector<float> d((size_t)W * H);
        if (m.forwardMatch(L.data(), R.data(), W, H, W, d.data(), W) != 0) return fail("match");
        std::ofstream(argv[6], std::ios::binary).write((const char*)d.data(), d.size() * sizeof(float));
        return 0;
    }
    if (!std::strcmp(mode, "time") && argc >= 11) {
        const int W = std::atoi(argv[4]), H = std::atoi(argv[5]), reps = std::max(std::atoi(argv[10]), 1);
        std::vector<uint8_t> L((size_t)W * H), R((size_t)W * H);
        std::ifstream(argv[2], std::ios::binary).read((char*)L.data(), L.size());
        std::ifstream(argv[3], std::ios::binary).read((char*)R.data(), R.size());
        sgm_hip::MatcherCore m(0, std::atoi(argv[6]));
        m.setDisparityRange(std::atoi(argv[7]), W);
        m.setMinDisparity(std::atoi(argv[8]));
        m.setWindowSize(std::atoi(argv[9]));
        m.setUniquenessRatio(15);
        m.setSpeckleFilterRange(4);
        m.setSpeckleFilterWindow(100);
        m.setPreFilterCap(31);
        m.setP1(200);
        m.setP2(400);
        if (argc > 11) m.setSpeckleFilterWindow(std::atoi(argv[11]));
        // the adapter keeps its persistent disparity_lr page-locked (matcherHIPSGM.cpp init)
        m.keepOutputRegistered(argc > 12 ? std::atoi(argv[12]) != 0 : true);
        std::vector<float> d((size_t)W * H);
        if (m.forwardMatch(L.data(), R.data(), W, H, W, d.data(), W) != 0) return fail("match");   // warm-up
        std::vector<double> t;
        for (int i = 0; i < reps; i++) {
            const auto a = std::chrono::steady_clock::now();
            if (m.forwardMatch(L.data(), R.data(), W, H, W, d.data(), W) != 0) return fail("match");
            t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
        }
        std::sort(t.begin(), t.end());
        std::printf("{\"ms_median\": %.4f, \"ms_min\": %.4f, \"reps\": %d}\n", t[t.size() / 2], t[0], reps);
        return 0;
    }
    return fail("usage");
}
