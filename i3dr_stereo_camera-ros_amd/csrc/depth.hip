// depth.hip — the two per-frame passes after the matcher.
//
//  k_disp_to_msg   int16 ×16 disparity -> the DisparityImage float image
//                  (generate_disparity.cpp:426-452: convertTo(..., 1/16), then
//                  setTo(MISSING_Z) below min_disparity and above max_disparity)
//  k_depth_count / k_depth_scan / k_depth_write
//                  DisparityImage float image -> depth image + XYZRGB point list in raster
//                  order (disparity_to_depth.cpp:127-205, Q from calc_q :62-84)
//
// Float arithmetic follows the reference's expression order, one IEEE rounding per
// operation: FMA contraction is off for this file (hipcc contracts a*b+c by default) and
// float division is the correctly rounded one, so results are bit-identical to a float32
// evaluation of the same C++ expressions.
#include "sgm_device.h"

#pragma clang fp contract(off)

namespace sgm {

constexpr float kMissingZ = 10000.0f;    // image_geometry::StereoCameraModel::MISSING_Z

__global__ __launch_bounds__(256) void k_disp_to_msg(const int16_t* __restrict__ disp, size_t disp_stride, int W, int H,
                                                     float min_disp, float max_disp, float* __restrict__ out,
                                                     size_t out_stride)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    float v = (float)disp[(size_t)y * disp_stride + x] * 0.0625f;   // exact: power of two
    if (v < min_disp) v = kMissingZ;
    if (v > max_disp) v = kMissingZ;      // second setTo sees the first one's MISSING_Z (reference order)
    out[(size_t)y * out_stride + x] = v;
}

struct DepthQ {
    float wz, q03, q13, q32, q33;    // Q(2,3), Q(0,3), Q(1,3), Q(3,2), Q(3,3) cast to float (:134-138)
    double zmin, zmax;               // _depth_min / _depth_max (double in the reference)
};

// One pixel: returns true when the reference emits a point (and writes depth).
__device__ __forceinline__ bool depth_pixel(float d, int i, int j, const DepthQ& q, float& x, float& y, float& z)
{
    if (!(d != 0.0f && d != kMissingZ)) return false;
    const float w = d * q.q32 + q.q33;
    x = ((float)j + q.q03) / w;
    y = ((float)i + q.q13) / w;
    z = q.wz / w;
    if (!(w > 0.0f && z > 0.0f)) return false;
    return (double)z <= q.zmax && (double)z >= q.zmin;
}

// pass 1: depth image (0 where no point) and the number of points of every row
__global__ __launch_bounds__(256) void k_depth_count(const float* __restrict__ disp, size_t disp_stride, int W, DepthQ q,
                                                     float* __restrict__ depth, size_t depth_stride,
                                                     int* __restrict__ row_count)
{
    __shared__ int cnt;
    const int i = blockIdx.x;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    int mine = 0;
    for (int j = threadIdx.x; j < W; j += 256) {
        float x, y, z;
        const bool ok = depth_pixel(disp[(size_t)i * disp_stride + j], i, j, q, x, y, z);
        if (depth) depth[(size_t)i * depth_stride + j] = ok ? z : 0.0f;
        mine += ok ? 1 : 0;
    }
    atomicAdd(&cnt, mine);
    __syncthreads();
    if (threadIdx.x == 0) row_count[i] = cnt;
}

// pass 2 (one workgroup): exclusive prefix over rows -> row_off[H], total in row_off[H]
__global__ __launch_bounds__(1024) void k_depth_scan(const int* __restrict__ row_count, int H, int* __restrict__ row_off)
{
    __shared__ int part[1024];
    const int t = threadIdx.x;
    const int per = (H + 1023) / 1024;
    const int b = t * per, e = min(b + per, H);
    int s = 0;
    for (int r = b; r < e; r++) s += row_count[r];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {      // Hillis-Steele inclusive scan of the partials
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = t ? part[t - 1] : 0;
    for (int r = b; r < e; r++) { row_off[r] = run; run += row_count[r]; }
    if (t == 1023) row_off[H] = part[1023];
}

// pass 3: points of row i in raster order at row_off[i] (a wave-ballot prefix per chunk)
__global__ __launch_bounds__(256) void k_depth_write(const float* __restrict__ disp, size_t disp_stride, int W, DepthQ q,
                                                     const uint8_t* __restrict__ color, size_t color_stride,
                                                     int channels, const int* __restrict__ row_off,
                                                     float4* __restrict__ points, int max_points)
{
    __shared__ int wave_n[4];
    const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    int base = row_off[i];
    for (int j0 = 0; j0 < W; j0 += 256) {
        const int j = j0 + t;
        float x = 0.f, y = 0.f, z = 0.f;
        const bool ok = j < W && depth_pixel(disp[(size_t)i * disp_stride + j], i, j, q, x, y, z);
        const uint64_t m = __ballot(ok);
        if (lane == 0) wave_n[w] = __popcll(m);
        __syncthreads();
        int before = __popcll(m & ((1ull << lane) - 1ull));
        for (int k = 0; k < w; k++) before += wave_n[k];
        if (ok && base + before < max_points) {
            uint32_t b, gch, r;
            if (channels == 1) {
                b = gch = r = color ? color[(size_t)i * color_stride + j] : 0u;
            } else if (channels == 3) {
                const uint8_t* px = color + (size_t)i * color_stride + 3 * (size_t)j;
                b = px[0]; gch = px[1]; r = px[2];
            } else {
                b = gch = r = 0u;
            }
            const uint32_t rgba = 0xFF000000u | (r << 16) | (gch << 8) | b;   // pcl rgba (a = 255)
            points[base + before] = make_float4(x, y, z, __uint_as_float(rgba));
        }
        base += wave_n[0] + wave_n[1] + wave_n[2] + wave_n[3];
        __syncthreads();
    }
}

hipError_t launch_disp_to_msg(const int16_t* disp, size_t disp_stride, int W, int H, float min_disp, float max_disp,
                              float* out, size_t out_stride, hipStream_t st)
{
    hipLaunchKernelGGL(k_disp_to_msg, dim3((W + 255) / 256, H), dim3(256), 0, st, disp, disp_stride, W, H, min_disp,
                       max_disp, out, out_stride);
    return hipGetLastError();
}

hipError_t launch_depth_points(const float* disp, size_t disp_stride, int W, int H, const float qf[5], double zmin,
                               double zmax, const uint8_t* color, size_t color_stride, int channels, float* depth,
                               size_t depth_stride, float4* points, int max_points, int* row_count, int* row_off,
                               hipStream_t st)
{
    DepthQ q{qf[0], qf[1], qf[2], qf[3], qf[4], zmin, zmax};
    hipLaunchKernelGGL(k_depth_count, dim3(H), dim3(256), 0, st, disp, disp_stride, W, q, depth, depth_stride, row_count);
    hipLaunchKernelGGL(k_depth_scan, dim3(1), dim3(1024), 0, st, row_count, H, row_off);
    if (points && max_points > 0)
        hipLaunchKernelGGL(k_depth_write, dim3(H), dim3(256), 0, st, disp, disp_stride, W, q, color, color_stride,
                           channels, row_off, points, max_points);
    return hipGetLastError();
}

}  // namespace sgm
