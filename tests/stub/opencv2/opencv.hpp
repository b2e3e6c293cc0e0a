// Declaration-only stand-in for <opencv2/opencv.hpp>, just enough of cv::Mat / cv::Size for a
// -fsyntax-only compile of the MatcherHIPSGM adapter against the reference's
// include/stereoMatcher/abstractStereoMatcher.h (tests/test_adapter_syntax.py). It is NOT an
// OpenCV implementation and is never linked or run.
#pragma once
#include <cstddef>
#include <iostream>
#include <string>

#define CV_8U 0
#define CV_16S 3
#define CV_32F 5
#define CV_8UC1 0
#define CV_16SC1 3
#define CV_32FC1 5

namespace cv {
struct Size {
    int width = 0, height = 0;
    Size() = default;
    Size(int w, int h) : width(w), height(h) {}
    bool operator==(const Size& o) const { return width == o.width && height == o.height; }
    bool operator!=(const Size& o) const { return !(*this == o); }
};
struct Scalar { explicit Scalar(double) {} };
class Mat {
public:
    Mat();
    Mat(Size size, int type);
    Mat(Size size, int type, const Scalar& s);
    Mat(int rows, int cols, int type);
    Mat(int rows, int cols, int type, void* data, size_t step = 0);
    void create(Size size, int type);
    void create(int rows, int cols, int type);
    void copyTo(Mat& dst) const;
    void convertTo(Mat& dst, int rtype, double alpha = 1, double beta = 0) const;
    int type() const;
    Size size() const;
    bool empty() const;
    int rows = 0, cols = 0;
    unsigned char* data = nullptr;
    size_t step = 0;
};
}  // namespace cv
