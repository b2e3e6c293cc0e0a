// hip_sgm_core.cpp — see hip_sgm_core.h.
#include "hip_sgm_core.h"

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

namespace sgm_hip {

// SGM_HIP_OCV_COMPAT = melodic | noetic | scalar | <bits>: the OpenCV build the OCV modes
// reproduce (include/sgm_hip.h SGM_OCV_*); unset: sgm_default_params' melodic default.
// Case and surrounding blanks are ignored; an unparseable value warns on stderr and keeps
// the fallback (the Python mirror's ocv_compat_from_env does the same).
int ocv_compat_from_env(int fallback)
{
    const char* e = std::getenv("SGM_HIP_OCV_COMPAT");
    if (!e) return fallback;
    std::string v(e);
    while (!v.empty() && std::isspace((unsigned char)v.back())) v.pop_back();
    size_t b = 0;
    while (b < v.size() && std::isspace((unsigned char)v[b])) b++;
    v = v.substr(b);
    if (v.empty()) return fallback;
    for (char& c : v) c = (char)std::tolower((unsigned char)c);
    if (v == "melodic") return SGM_OCV_COMPAT_MELODIC;
    if (v == "noetic") return SGM_OCV_COMPAT_NOETIC;
    if (v == "scalar") return SGM_OCV_COMPAT_SCALAR;
    char* end = nullptr;
    const long bits = std::strtol(v.c_str(), &end, 0);
    if (end == v.c_str() || *end) {
        std::cerr << "SGM_HIP_OCV_COMPAT=\"" << e << "\" is not melodic | noetic | scalar | <bits>: using "
                  << fallback << std::endl;
        return fallback;
    }
    return (int)bits & (SGM_OCV_COL0_LEGACY | SGM_OCV_SIMD_SAT | SGM_OCV_LANE_TIE);
}

MatcherCore::MatcherCore(int device, int mode) : device_(device)
{
    if (mode < 0) {
        const char* env = std::getenv("SGM_HIP_MODE");
        mode = env ? std::atoi(env) : SGM_MODE_OCV_SGBM5;
    }
    sgm_default_params(&params_, mode);
    params_.ocv_compat = ocv_compat_from_env(params_.ocv_compat);
    // cv::StereoSGBM::create(64, 9, 5) (matcherOpenCVSGBM.cpp:14): overwritten by the setters
    params_.min_disparity = 64;
    params_.num_disparities = 9;
    params_.block_size = 5;
    params_.p1 = params_.p2 = params_.uniqueness_ratio = params_.disp12_max_diff = 0;
    params_.prefilter_cap = params_.speckle_window_size = params_.speckle_range = 0;
}

MatcherCore::~MatcherCore()
{
    releaseOutput();
    sgm_destroy(handle_);
}

void MatcherCore::keepOutputRegistered(bool enable)
{
    keep_reg_ = enable;
    if (!enable) releaseOutput();
}

void MatcherCore::releaseOutput()
{
    if (reg_ptr_ && handle_) (void)sgm_host_unregister(handle_, reg_ptr_);
    reg_ptr_ = nullptr;
    reg_bytes_ = 0;
}

void MatcherCore::setDisparityRange(int r, int image_width)
{
    r = r > 0 ? r : ((image_width / 8) + 15) & -16;
    params_.num_disparities = r;
}
void MatcherCore::setWindowSize(int w) { params_.block_size = w; }
void MatcherCore::setMinDisparity(int d) { params_.min_disparity = d; }
void MatcherCore::setUniquenessRatio(int r) { params_.uniqueness_ratio = r; }
void MatcherCore::setSpeckleFilterWindow(int w) { params_.speckle_window_size = w; }
void MatcherCore::setSpeckleFilterRange(int r) { params_.speckle_range = r; }
void MatcherCore::setDisp12MaxDiff(int d) { params_.disp12_max_diff = d; }
void MatcherCore::setPreFilterCap(int c) { params_.prefilter_cap = c; }
void MatcherCore::setP1(float p1) { params_.p1 = (int)p1; }
void MatcherCore::setP2(float p2) { params_.p2 = (int)p2; }
void MatcherCore::setInterpolation(bool e) { interpolate_ = e; }
void MatcherCore::setMode(int m) { params_.mode = m; }
void MatcherCore::setOcvCompat(int bits) { params_.ocv_compat = bits; }

sgm_params MatcherCore::rightMatcherParams(const sgm_params& p)
{
    sgm_params r = p;
    r.min_disparity = -(p.min_disparity + p.num_disparities) + 1;
    r.uniqueness_ratio = 0;
    r.disp12_max_diff = 1000000;
    r.speckle_window_size = 0;
    return r;
}

// One host-buffer match: float32 output (the CV_32FC1 of matcherOpenCVSGBM.cpp:34, converted
// on the device by sgm_match_f32) or int16 (CV_16S, the right matcher's disparity_rl).
int MatcherCore::run(const sgm_params& p, const uint8_t* a, const uint8_t* b, int w, int h, size_t stride, float* outf,
                     int16_t* out16, size_t out_stride)
{
    int rc = SGM_OK;
    if (!handle_) rc = sgm_create(&handle_, device_);
    if (rc == SGM_OK) rc = sgm_set_params(handle_, &p);
    if (rc == SGM_OK && keep_reg_ && outf) {
        const size_t bytes = out_stride * sizeof(float) * (size_t)(h - 1) + (size_t)w * sizeof(float);
        if (reg_ptr_ != (void*)outf || reg_bytes_ != bytes) {
            releaseOutput();
            // not fatal: an unregistered output takes one synchronous copy
            if (sgm_host_register(handle_, outf, bytes) == SGM_OK) { reg_ptr_ = outf; reg_bytes_ = bytes; }
        }
    }
    if (rc == SGM_OK)
        rc = outf ? sgm_match_f32(handle_, a, b, w, h, stride, outf, out_stride)
                  : sgm_match(handle_, a, b, w, h, stride, out16, out_stride);
    if (rc != SGM_OK) {
        err_ = handle_ ? sgm_last_error(handle_) : "no HIP device";
        std::cerr << "Error in HIP SGM parameters" << std::endl << err_ << " (status " << rc << ")" << std::endl;
        return -1;
    }
    return 0;
}

int MatcherCore::forwardMatch(const uint8_t* left, const uint8_t* right, int w, int h, size_t stride, float* out,
                              size_t out_stride)
{
    if (interpolate_)  // Q3: WLS output discarded, right-view disparity returned
        return backwardMatch(left, right, w, h, stride, out, out_stride);
    return run(params_, left, right, w, h, stride, out, nullptr, out_stride);
}

int MatcherCore::backwardMatch(const uint8_t* left, const uint8_t* right, int w, int h, size_t stride, float* out,
                               size_t out_stride)
{
    return run(rightMatcherParams(params_), right, left, w, h, stride, out, nullptr, out_stride);
}

int MatcherCore::backwardMatch16(const uint8_t* left, const uint8_t* right, int w, int h, size_t stride, int16_t* out,
                                 size_t out_stride)
{
    return run(rightMatcherParams(params_), right, left, w, h, stride, nullptr, out, out_stride);
}

}  // namespace sgm_hip
