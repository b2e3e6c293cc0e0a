// hip_sgm_core.h — OpenCV-free core of the MatcherHIPSGM plugin.
//
// Holds the matcher parameters with the reference's setter semantics
// (src/stereoMatcher/matcherOpenCVSGBM.cpp:53-110) and runs the match through the C-ABI
// (include/sgm_hip.h). MatcherHIPSGM (matcherHIPSGM.{h,cpp}) is a thin cv::Mat shell
// around it, so everything with behaviour is compiled and tested without OpenCV/ROS.
#ifndef HIP_SGM_CORE_H
#define HIP_SGM_CORE_H

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "sgm_hip.h"

namespace sgm_hip {

// SGM_HIP_OCV_COMPAT (melodic | noetic | scalar | <bits>), else `fallback`
int ocv_compat_from_env(int fallback);

class MatcherCore {
public:
    // mode < 0: SGM_HIP_MODE env var, default SGM_MODE_OCV_SGBM5 (the reference's SGBM
    // path never sets a mode, generate_disparity.cpp:241-261 -> cv::StereoSGBM::MODE_SGBM).
    explicit MatcherCore(int device = 0, int mode = -1);
    ~MatcherCore();
    MatcherCore(const MatcherCore&) = delete;
    MatcherCore& operator=(const MatcherCore&) = delete;

    // --- setters, reference semantics ------------------------------------------------
    void setDisparityRange(int disparity_range, int image_width);  // <=0 -> ((W/8)+15)&-16
    void setWindowSize(int window_size);
    void setMinDisparity(int min_disparity);
    void setUniquenessRatio(int ratio);
    void setSpeckleFilterWindow(int window);
    void setSpeckleFilterRange(int range);
    void setDisp12MaxDiff(int diff);
    void setPreFilterCap(int cap);
    void setP1(float p1);   // OpenCV's setP1(int) truncates the reference's float
    void setP2(float p2);
    void setInterpolation(bool enable);
    void setMode(int mode);
    void setOcvCompat(int bits);   // SGM_OCV_* (default: SGM_HIP_OCV_COMPAT env, else melodic)

    // --- matching -------------------------------------------------------------------
    // u8 mono rectified pair -> CV_32FC1-layout disparity in 1/16 px (x16 fixed point,
    // invalid = (minD-1)*16). Returns 0, or -1 after printing to stderr (the reference's
    // catch(cv::Exception&) behaviour, matcherOpenCVSGBM.cpp:37-43).
    int forwardMatch(const uint8_t* left, const uint8_t* right, int width, int height, size_t stride,
                     float* out, size_t out_stride);
    // right-view match (cv::ximgproc::createRightMatcher semantics) into `out`: float32, or
    // int16 (backwardMatch16: the CV_16S disparity_rl of matcherOpenCVSGBM.cpp:46-51).
    int backwardMatch(const uint8_t* left, const uint8_t* right, int width, int height, size_t stride,
                      float* out, size_t out_stride);
    int backwardMatch16(const uint8_t* left, const uint8_t* right, int width, int height, size_t stride,
                        int16_t* out, size_t out_stride);

    // Keep the forwardMatch output buffer page-locked between frames (sgm_host_register) so the
    // copy-out overlaps the match; the caller must call releaseOutput() before that buffer is
    // freed or reallocated (MatcherHIPSGM: before disparity_lr.create() changes its size/type).
    void keepOutputRegistered(bool enable);
    void releaseOutput();

    const sgm_params& params() const { return params_; }
    bool interpolation() const { return interpolate_; }
    int disparityRange() const { return params_.num_disparities; }
    const std::string& lastError() const { return err_; }
    static sgm_params rightMatcherParams(const sgm_params& p);

private:
    int run(const sgm_params& p, const uint8_t* a, const uint8_t* b, int w, int h, size_t stride, float* outf,
            int16_t* out16, size_t out_stride);
    int device_;
    sgm_handle* handle_ = nullptr;   // opened lazily at the first match
    sgm_params params_{};
    bool interpolate_ = false;
    bool keep_reg_ = false;
    void* reg_ptr_ = nullptr;        // the registered output range
    size_t reg_bytes_ = 0;
    std::string err_;
};

}  // namespace sgm_hip
#endif
