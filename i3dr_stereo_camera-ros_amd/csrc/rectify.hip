// rectify.hip — the node's rectify() on the device:
//   cv::initUndistortRectifyMap(K, D, R, P, size, CV_32FC1, map_x, map_y)
//   cv::remap(raw, rect, map_x, map_y, INTER_CUBIC, BORDER_CONSTANT)
// (generate_disparity.cpp:370-386, rectify.cpp:111-127). The reference recomputes the map on
// every frame on the CPU; here it is computed once per calibration (k_rectify_map, double
// precision, the scalar OpenCV loop) and every frame is one HBM-bound remap pass
// (k_remap_cubic: 8 B of map + 1 B out per pixel, the 4x4 source taps from L1/L2).
//
//  k_rectify_map   one thread per map row: the row start i*ir1 + ir2 (etc.) advanced by
//                  += ir0 per column exactly as the scalar loop does (the rounding of the
//                  running sums is part of the result), then the rational + tangential +
//                  thin-prism distortion model, identity tilt, stored as float.
//  k_remap_cubic   OpenCV's fixed-point bicubic remap for u8: X = cvRound(map_x * 32) ->
//                  integer part X >> 5 (saturated to short), fraction X & 31; 16 int16 weights
//                  of the 32 x 32 sub-pixel table (cubic_table, built on the host exactly as
//                  initInterTab2D builds it); taps outside the image read 0 (BORDER_CONSTANT);
//                  dst = sat_u8((sum + 2^14) >> 15).
//
// FMA contraction is off for this file: the double map and the float cubic coefficients
// are bit-identical to the scalar C++ evaluation (oracle/sgm_oracle.py rectify_map /
// cubic_table / remap_cubic).
#include "sgm_device.h"

#include <cmath>

#pragma clang fp contract(off)

namespace sgm {

constexpr int kInterBits = 5;
constexpr int kInterTab = 1 << kInterBits;       // 32 sub-pixel positions per axis
constexpr int kCoefBits = 15;
constexpr int kCoefScale = 1 << kCoefBits;

struct RectMap {
    double ir[9];                                // (P[:, :3] * R)^-1, row-major
    double fx, fy, u0, v0;
    double k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4;
};

__global__ __launch_bounds__(64) void k_rectify_map(RectMap m, int W, int H, float* __restrict__ mx,
                                                    float* __restrict__ my, size_t stride)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= H) return;
    const double* ir = m.ir;
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    float* rx = mx + (size_t)i * stride;
    float* ry = my + (size_t)i * stride;
    for (int j = 0; j < W; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
        const double w = 1. / _w, x = _x * w, y = _y * w;
        const double x2 = x * x, y2 = y * y;
        const double r2 = x2 + y2, _2xy = 2 * x * y;
        const double kr = (1 + ((m.k3 * r2 + m.k2) * r2 + m.k1) * r2) / (1 + ((m.k6 * r2 + m.k5) * r2 + m.k4) * r2);
        const double xd = (x * kr + m.p1 * _2xy + m.p2 * (r2 + 2 * x2) + m.s1 * r2 + m.s2 * r2 * r2);
        const double yd = (y * kr + m.p1 * (r2 + 2 * y2) + m.p2 * _2xy + m.s3 * r2 + m.s4 * r2 * r2);
        // identity tilt matrix times (xd, yd, 1), Matx order: s = 0; s += a(i,k) * b(k)
        double t0 = 0.0, t1 = 0.0, t2 = 0.0;
        t0 += 1.0 * xd; t0 += 0.0 * yd; t0 += 0.0 * 1.0;
        t1 += 0.0 * xd; t1 += 1.0 * yd; t1 += 0.0 * 1.0;
        t2 += 0.0 * xd; t2 += 0.0 * yd; t2 += 1.0 * 1.0;
        const double inv = t2 != 0.0 ? 1. / t2 : 1;
        const double u = m.fx * inv * t0 + m.u0;
        const double v = m.fy * inv * t1 + m.v0;
        rx[j] = (float)u;
        ry[j] = (float)v;
    }
}

// One output pixel per thread; a 64 x 4 block covers 64 consecutive columns of 4 rows.
__global__ __launch_bounds__(256) void k_remap_cubic(const uint8_t* __restrict__ src, size_t sstride, int sw, int sh,
                                                     const float* __restrict__ mx, const float* __restrict__ my,
                                                     size_t mstride, int W, int H, const int16_t* __restrict__ tab,
                                                     uint8_t* __restrict__ dst, size_t dstride)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    const size_t m = (size_t)y * mstride + x;
    dst[(size_t)y * dstride + x] = remap_cubic_px(src, sstride, sw, sh, mx[m], my[m], tab);
}

// ---- host -------------------------------------------------------------------------------

// imgwarp.cpp interpolateCubic (float, A = -0.75)
static void cubic_coeffs(float x, float* c)
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

// initInterTab2D(INTER_CUBIC, fixpt = true): [32 * 32][16] int16, entry fy * 32 + fx
void cubic_table(int16_t* tab)
{
    float t1[kInterTab][4];
    const float scale = 1.f / kInterTab;
    for (int i = 0; i < kInterTab; i++) cubic_coeffs(i * scale, t1[i]);
    for (int i = 0; i < kInterTab; i++)
        for (int j = 0; j < kInterTab; j++) {
            int16_t* it = tab + (size_t)(i * kInterTab + j) * 16;
            int isum = 0;
            for (int k1 = 0; k1 < 4; k1++) {
                const float vy = t1[i][k1];
                for (int k2 = 0; k2 < 4; k2++) {
                    const float v = vy * t1[j][k2];
                    const float sv = v * (float)kCoefScale;
                    const long r = std::lrint(sv);          // cvRound: half to even
                    it[k1 * 4 + k2] = (int16_t)std::min(std::max(r, -32768L), 32767L);
                    isum += it[k1 * 4 + k2];
                }
            }
            if (isum != kCoefScale) {    // the difference goes to one tap of rows/columns 2..3
                const int diff = isum - kCoefScale;
                int Mk1 = 2, Mk2 = 2, mk1 = 2, mk2 = 2;
                for (int k1 = 2; k1 < 4; k1++)
                    for (int k2 = 2; k2 < 4; k2++) {
                        if (it[k1 * 4 + k2] < it[mk1 * 4 + mk2]) mk1 = k1, mk2 = k2;
                        else if (it[k1 * 4 + k2] > it[Mk1 * 4 + Mk2]) Mk1 = k1, Mk2 = k2;
                    }
                if (diff < 0) it[Mk1 * 4 + Mk2] = (int16_t)(it[Mk1 * 4 + Mk2] - diff);
                else it[mk1 * 4 + mk2] = (int16_t)(it[mk1 * 4 + mk2] - diff);
            }
        }
}

// (P[:, :3] * R)^-1: the product summed k = 0..2 in order, cv::invert's 3x3 closed form.
// Returns false when singular.
bool rectify_inverse(const double* P, const double* R, double* ir)
{
    double m[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += P[i * 4 + k] * (R ? R[k * 3 + j] : (k == j ? 1.0 : 0.0));
            m[i * 3 + j] = s;
        }
    auto M = [&](int r, int c) { return m[r * 3 + c]; };
    const double det = M(0, 0) * (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) - M(0, 1) * (M(1, 0) * M(2, 2) - M(1, 2) * M(2, 0)) +
                       M(0, 2) * (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0));
    if (det == 0.0) return false;
    const double d = 1. / det;
    ir[0] = (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d;
    ir[1] = (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d;
    ir[2] = (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d;
    ir[3] = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d;
    ir[4] = (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d;
    ir[5] = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d;
    ir[6] = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d;
    ir[7] = (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d;
    ir[8] = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d;
    return true;
}

// K 3x3, dist[12] = k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4, ir from rectify_inverse
hipError_t launch_rectify_map(const double* K, const double* dist, const double* ir, int W, int H, float* mx,
                              float* my, size_t stride, hipStream_t st)
{
    RectMap m;
    for (int i = 0; i < 9; i++) m.ir[i] = ir[i];
    m.fx = K[0]; m.fy = K[4]; m.u0 = K[2]; m.v0 = K[5];
    m.k1 = dist[0]; m.k2 = dist[1]; m.p1 = dist[2]; m.p2 = dist[3]; m.k3 = dist[4];
    m.k4 = dist[5]; m.k5 = dist[6]; m.k6 = dist[7];
    m.s1 = dist[8]; m.s2 = dist[9]; m.s3 = dist[10]; m.s4 = dist[11];
    hipLaunchKernelGGL(k_rectify_map, dim3((H + 63) / 64), dim3(64), 0, st, m, W, H, mx, my, stride);
    return hipGetLastError();
}

hipError_t launch_remap_cubic(const uint8_t* src, size_t sstride, int sw, int sh, const float* mx, const float* my,
                              size_t mstride, int W, int H, const int16_t* tab, uint8_t* dst, size_t dstride,
                              hipStream_t st)
{
    hipLaunchKernelGGL(k_remap_cubic, dim3((W + 63) / 64, (H + 3) / 4), dim3(256), 0, st, src, sstride, sw, sh, mx, my,
                       mstride, W, H, tab, dst, dstride);
    return hipGetLastError();
}

}  // namespace sgm
