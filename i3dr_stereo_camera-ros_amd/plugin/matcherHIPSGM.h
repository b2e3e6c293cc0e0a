// matcherHIPSGM.h — drop-in AbstractStereoMatcher subclass for the reference ROS package.
// Copy into include/stereoMatcher/ of i3dr_stereo_camera-ros; it
// mirrors matcherOpenCVSGBM.h:6-39 and delegates compute to libsgm_hip.so.
#ifndef MATCHERHIPSGM_H
#define MATCHERHIPSGM_H

#include "stereoMatcher/abstractStereoMatcher.h"
#include "hip_sgm_core.h"

class MatcherHIPSGM : public AbstractStereoMatcher
{
public:
  explicit MatcherHIPSGM(std::string &param_file, cv::Size _image_size)
      : AbstractStereoMatcher(param_file, _image_size), core_(0, -1)
  {
    init();
  }

  int forwardMatch(void);
  int backwardMatch(void);

  void setMinDisparity(int min_disparity);
  void setDisparityRange(int disparity_range);
  void setWindowSize(int window_size);
  void setUniquenessRatio(int ratio);
  void setSpeckleFilterWindow(int window);
  void setSpeckleFilterRange(int range);
  void setP1(float p1);
  void setP2(float p2);
  void setDisp12MaxDiff(int diff);
  void setInterpolation(bool enable);
  void setPreFilterCap(int cap);

  // Not used by SGM (no-ops, as matcherOpenCVSGBM.h:31-34)
  void setTextureThreshold(int threshold){};
  void setPreFilterSize(int size){};
  void setOcclusionDetection(bool enable){};

private:
  sgm_hip::MatcherCore core_;
  void init(void);
};

#endif // MATCHERHIPSGM_H
