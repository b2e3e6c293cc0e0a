// matcherHIPSGM.cpp — cv::Mat shell over sgm_hip::MatcherCore (compute: libsgm_hip.so).
// Behaviour mirrors src/stereoMatcher/matcherOpenCVSGBM.cpp:1-110 of the reference.
#include "stereoMatcher/matcherHIPSGM.h"

void MatcherHIPSGM::init(void)
{
  // Setup for 16-bit disparity, like MatcherOpenCVSGBM::init (device opened lazily)
  cv::Mat(image_size, CV_16S).copyTo(disparity_lr);
  cv::Mat(image_size, CV_16S).copyTo(disparity_rl);
  // disparity_lr persists across frames: keep it page-locked (released before it is reallocated)
  core_.keepOutputRegistered(true);
}

int MatcherHIPSGM::forwardMatch()
{
  if (left->type() != CV_8UC1 || right->type() != CV_8UC1 || left->size() != right->size())
  {
    std::cerr << "Error in HIP SGM parameters" << std::endl << "expects equal-size CV_8UC1 images" << std::endl;
    return -1;
  }
  if (interpolate)
  {
    // Q3 (matcherOpenCVSGBM.cpp:22-33): the WLS output is discarded and the right-view
    // disparity (CV_16S in disparity_rl) replaces disparity_lr
    int rc = backwardMatch();
    if (rc == 0)
    {
      if (disparity_lr.size() != disparity_rl.size() || disparity_lr.type() != CV_32FC1)
        core_.releaseOutput();  // convertTo reallocates disparity_lr
      disparity_rl.convertTo(disparity_lr, CV_32FC1);
    }
    return rc;
  }
  // CV_32FC1 straight from the device (matcherOpenCVSGBM.cpp:34's convertTo runs there)
  if (disparity_lr.size() != left->size() || disparity_lr.type() != CV_32FC1)
    core_.releaseOutput();  // create() reallocates: unregister the old buffer before it is freed
  disparity_lr.create(left->size(), CV_32FC1);
  return core_.forwardMatch(left->data, right->data, left->cols, left->rows, left->step,
                            (float *)disparity_lr.data, disparity_lr.step / sizeof(float));
}

int MatcherHIPSGM::backwardMatch()
{
  // CV_16S like createRightMatcher(matcher)->compute(*right, *left, disparity_rl) (:46-51)
  disparity_rl.create(left->size(), CV_16S);
  return core_.backwardMatch16(left->data, right->data, left->cols, left->rows, left->step,
                               (int16_t *)disparity_rl.data, disparity_rl.step / sizeof(int16_t));
}

void MatcherHIPSGM::setMinDisparity(int min_disparity)
{
  core_.setMinDisparity(min_disparity);
  this->min_disparity = min_disparity;
}

void MatcherHIPSGM::setDisparityRange(int disparity_range)
{
  core_.setDisparityRange(disparity_range, image_size.width);
  this->disparity_range = core_.disparityRange();
}

void MatcherHIPSGM::setWindowSize(int window_size)
{
  this->window_size = window_size;
  core_.setWindowSize(window_size);
}

void MatcherHIPSGM::setUniquenessRatio(int ratio) { core_.setUniquenessRatio(ratio); }
void MatcherHIPSGM::setSpeckleFilterWindow(int window) { core_.setSpeckleFilterWindow(window); }
void MatcherHIPSGM::setSpeckleFilterRange(int range) { core_.setSpeckleFilterRange(range); }
void MatcherHIPSGM::setDisp12MaxDiff(int diff) { core_.setDisp12MaxDiff(diff); }
void MatcherHIPSGM::setP1(float p1) { core_.setP1(p1); }
void MatcherHIPSGM::setP2(float p2) { core_.setP2(p2); }
void MatcherHIPSGM::setPreFilterCap(int cap) { core_.setPreFilterCap(cap); }

void MatcherHIPSGM::setInterpolation(bool enable)
{
  this->interpolate = enable;
  core_.setInterpolation(enable);
}
