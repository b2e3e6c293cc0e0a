// matcherHIPSGM.cpp — cv::Mat shell over sgm_hip::MatcherCore (compute: libsgm_hip.so).
// Behaviour mirrors src/stereoMatcher/matcherOpenCVSGBM.cpp:1-110 of the reference.
#include "stereoMatcher/matcherHIPSGM.h"

void MatcherHIPSGM::init(void)
{
  // Setup for 16-bit disparity, like MatcherOpenCVSGBM::init (device opened lazily)
  cv::Mat(image_size, CV_16S).copyTo(disparity_lr);
  cv::Mat(image_size, CV_16S).copyTo(disparity_rl);
}

int MatcherHIPSGM::forwardMatch()
{
  if (left->type() != CV_8UC1 || right->type() != CV_8UC1 || left->size() != right->size())
  {
    std::cerr << "Error in HIP SGM parameters" << std::endl << "expects equal-size CV_8UC1 images" << std::endl;
    return -1;
  }
  disparity_lr.create(left->size(), CV_32FC1);
  int rc = core_.forwardMatch(left->data, right->data, left->cols, left->rows, left->step,
                              (float *)disparity_lr.data, disparity_lr.step / sizeof(float));
  if (rc == 0 && interpolate)
    disparity_lr.copyTo(disparity_rl);   // Q3: the interp result IS the right-view disparity
  return rc;
}

int MatcherHIPSGM::backwardMatch()
{
  disparity_rl.create(left->size(), CV_32FC1);
  return core_.backwardMatch(left->data, right->data, left->cols, left->rows, left->step,
                             (float *)disparity_rl.data, disparity_rl.step / sizeof(float));
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
