/*
 * sgm_hip.h — C-ABI of the MI355X-native Semi-Global Matching engine (libsgm_hip.so).
 *
 * This is the drop-in boundary for the reference's stereo-matcher plugin surface.
 * It replaces the work that `MatcherOpenCVSGBM::forwardMatch` delegates to
 * `cv::StereoSGBM::compute` (reference: src/stereoMatcher/matcherOpenCVSGBM.cpp:17-44,
 * call at :21) and is called from the plugin adapter `MatcherHIPSGM`
 * (i3dr_stereo_camera-ros_amd/plugin/matcherHIPSGM.{h,cpp}), a subclass of the
 * reference's `AbstractStereoMatcher` (include/stereoMatcher/abstractStereoMatcher.h:12-92).
 *
 * Plain C types only: pointers, sizes, ints. No torch / OpenCV / HIP types in signatures
 * (streams are passed as `void*` = hipStream_t).
 *
 * Output contract (identical to the reference's SGBM path, abstractStereoMatcher.cpp:44-53,
 * generate_disparity.cpp:403-436): int16 disparity in 1/16-pixel fixed point
 * (OpenCV DISP_SCALE = 16); invalid pixels = (min_disparity - 1) * 16; columns outside
 * [max(maxD,0), W + min(minD,0)) are invalid.
 *
 * Error convention (reference: matcherOpenCVSGBM.cpp:37-43 returns -1 on cv::Exception;
 * generate_disparity.cpp:355-365 logs and publishes nothing): every call returns an int
 * status, 0 = OK, < 0 = error class below; `sgm_last_error()` gives the text. The adapter
 * maps any non-zero status to -1, exactly like the OpenCV wrapper.
 */
#ifndef SGM_HIP_H
#define SGM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ABI version ------------------------------------------------------------------- */
/* Bumped whenever a struct or signature of this header changes. Round 3 grew sgm_params
 * from 14 to 15 ints (ocv_compat, version 3); round 4 added sgm_match_tiled_device
 * (version 4). A caller compiled against an older header must check sgm_abi_version()
 * == SGM_ABI_VERSION before passing an sgm_params (a 14-int struct would be read one int
 * past its end).                                                                         */
#define SGM_ABI_VERSION 4
int  sgm_abi_version(void);

/* ---- status codes ------------------------------------------------------------------ */
#define SGM_OK                0
#define SGM_ERR_ARG          -1   /* null pointer, bad size / stride                      */
#define SGM_ERR_PARAM        -2   /* invalid matcher parameters (e.g. D % 16 != 0)       */
#define SGM_ERR_DEVICE       -3   /* no HIP device / HIP runtime failure                  */
#define SGM_ERR_ALLOC        -4   /* device / host allocation failure                     */
#define SGM_ERR_UNSUPPORTED  -5   /* parameter combination this build does not implement */

/* ---- matching modes ---------------------------------------------------------------- */
/* OpenCV-compatible modes: Birchfield-Tomasi cost on the Sobel-prefiltered + raw image,
 * SAD block aggregation, int16 path costs. Bit-exact with the CPU oracle's restatement of
 * cv::StereoSGBM (oracle/sgm_oracle.c).                                                   */
#define SGM_MODE_OCV_SGBM5    0   /* cv::StereoSGBM::MODE_SGBM: 5 directions (reference default, Q1) */
#define SGM_MODE_OCV_HH8      1   /* cv::StereoSGBM::MODE_HH: 8 directions (cfg `fullDP`)             */
/* North-star mode: 9x7 census, Hamming cost, 8 directions, u8 path costs, u16 sums.       */
#define SGM_MODE_CENSUS8      2

/* OpenCV build variants of the OCV modes (`sgm_params.ocv_compat`, a bitfield). The reference
 * pins OpenCV only through its ROS distro — melodic (OpenCV 3.2.0, the reference's Dockerfile:1,
 * amd64) and noetic (OpenCV 4.2.0; CI matrix .github/workflows/ros-build.yml:14-21) — and
 * computeDisparitySGBM differs between those releases and between its scalar and SIMD (SSE2 /
 * universal-intrinsic, every x86-64 build) branches. Bits:
 *   COL0_LEGACY  3.x cost loop: C' column 0 is never updated for rows y > 0
 *   SIMD_SAT     saturating int16 box sums, path recurrence and S (SIMD branches)
 *   LANE_TIE     3.x SSE2 MODE_SGBM WTA: among equal minimal sums the lowest lane (d mod 8) wins
 * The three agree with the scalar restatement except on column 0 (COL0, every frame), on int16
 * overflow (SIMD_SAT) and on exact cross-lane ties (LANE_TIE). Census mode ignores the field. */
#define SGM_OCV_COL0_LEGACY   1
#define SGM_OCV_SIMD_SAT      2
#define SGM_OCV_LANE_TIE      4
#define SGM_OCV_COMPAT_SCALAR   0                      /* the scalar 4.x restatement            */
#define SGM_OCV_COMPAT_NOETIC   SGM_OCV_SIMD_SAT      /* noetic x86-64: OpenCV 4.2, SIMD        */
#define SGM_OCV_COMPAT_MELODIC  (SGM_OCV_COL0_LEGACY | SGM_OCV_SIMD_SAT | SGM_OCV_LANE_TIE)
                                                       /* melodic x86-64 (the Docker image): 3.2, SSE2;
                                                        * the default of sgm_default_params      */

/* Parameter block. Field names follow the reference's setters
 * (abstractStereoMatcher.h:27-48) and cfg/i3DR_Disparity.cfg:21-39.                      */
typedef struct sgm_params {
    int mode;                 /* SGM_MODE_*                                               */
    int min_disparity;        /* setMinDisparity                  (cfg min_disparity)     */
    int num_disparities;      /* setDisparityRange, multiple of 16 (cfg disparity_range)  */
    int block_size;           /* setWindowSize: OCV SAD window (cfg correlation_window_size); census: ignored */
    int p1;                   /* setP1 (float in the reference API, truncated like OpenCV's int setter) */
    int p2;                   /* setP2                                                    */
    int uniqueness_ratio;     /* setUniquenessRatio (percent)                             */
    int disp12_max_diff;      /* setDisp12MaxDiff (<=0 -> 1, as OpenCV SGBM)              */
    int prefilter_cap;        /* setPreFilterCap (OCV modes)                              */
    int speckle_window_size;  /* setSpeckleFilterWindow (0 = speckle filter off)          */
    int speckle_range;        /* setSpeckleFilterRange (max diff in pixels; x16 internally) */
    int subpixel;             /* census: parabolic 1/16 interpolation on/off (OCV: always on) */
    int lr_check;             /* census: left-right (disp2) check on/off (OCV: always on)     */
    int median;               /* census: 3x3 median post-filter on/off (OCV: always on)       */
    int ocv_compat;           /* OCV modes: SGM_OCV_* bits of the OpenCV build to reproduce   */
} sgm_params;

typedef struct sgm_handle sgm_handle;

/* ---- device / handle management ------------------------------------------------------ */
/* Number of visible HIP devices (0 if none / runtime unavailable). Never throws.           */
int  sgm_device_count(void);

/* Create a matcher handle bound to `device` (reference ctor: abstractStereoMatcher.h:15,
 * subclasses call init(), matcherOpenCVSGBM.h:10-14). Cheap: no device allocation happens
 * until the first match (the reference constructs every matcher lazily on the first frame,
 * generate_disparity.cpp:268-278). Returns SGM_ERR_DEVICE if `device` is not visible.     */
int  sgm_create(sgm_handle** out, int device);
void sgm_destroy(sgm_handle* h);

/* Page-lock and map a caller's host buffer (hipHostRegister, mapped) for as long as it stays
 * registered: a registered output of sgm_match / sgm_match_f32 is copied back by DMA without the
 * runtime's pageable staging, or — sgm_match_f32 in the census mode without median / speckles —
 * written by the WTA kernel itself as the rows finish. The caller must unregister a buffer
 * before freeing it (unregistering waits for the handle's last call; on failure the buffer stays
 * registered and mapped). sgm_destroy unregisters every buffer still registered through the
 * handle: HIP registrations are process-wide, so a caller that keeps using a buffer page-locked
 * after destroying the handle registers it again. The MatcherHIPSGM adapter registers its
 * persistent disparity_lr, matcherOpenCVSGBM.cpp:34's output Mat.                              */
int  sgm_host_register(sgm_handle* h, void* ptr, size_t bytes);
int  sgm_host_unregister(sgm_handle* h, void* ptr);

/* Defaults: census mode = north-star config (P1 10, P2 120, uniq 5, subpixel+LR on);
 * OCV modes = the generate_disparity node defaults (generate_disparity.cpp:100-112) and
 * ocv_compat = SGM_OCV_COMPAT_MELODIC (the OpenCV the reference's Dockerfile:1 ships).     */
void sgm_default_params(sgm_params* p, int mode);

/* Store parameters. Like the reference's setters this never fails on values; invalid
 * combinations surface at match time (matcherOpenCVSGBM.cpp:37-43 behaviour).            */
int  sgm_set_params(sgm_handle* h, const sgm_params* p);
int  sgm_get_params(const sgm_handle* h, sgm_params* p);

/* Validate parameters for a W-wide image without matching (0 = would run).                */
int  sgm_check_params(const sgm_params* p, int width, int height);

/* ---- matching -------------------------------------------------------------------------- */
/* Host buffers in, host buffer out; synchronous. L/R: W x H u8 mono (stride bytes);
 * disp: W x H int16 (out_stride in elements). Replaces cv::StereoSGBM::compute
 * (matcherOpenCVSGBM.cpp:21).                                                              */
int  sgm_match(sgm_handle* h, const uint8_t* left, const uint8_t* right,
               int width, int height, size_t stride,
               int16_t* disp, size_t out_stride);

/* sgm_match with the CV_32FC1 output of the reference's matcher contract
 * (matcherOpenCVSGBM.cpp:34 `disparity_lr.convertTo(disparity_lr, CV_32FC1)`, still x16 fixed
 * point): the int16 -> float conversion runs on the device, so the caller's buffer is filled by
 * the D2H itself (out_stride in floats). Host buffers; synchronous.                        */
int  sgm_match_f32(sgm_handle* h, const uint8_t* left, const uint8_t* right,
                   int width, int height, size_t stride, float* disp, size_t out_stride);

/* Device buffers in/out (already resident in HBM), asynchronous on `stream` (hipStream_t,
 * NULL = the handle's own stream). The handle's device must own the buffers. Calls on one
 * handle share its workspace, so each call is ordered after the previous one whatever the
 * streams (an event recorded at the end of every call is waited on at the start of the next);
 * use one handle per concurrent stream to overlap matches.                                  */
int  sgm_match_device(sgm_handle* h, const uint8_t* d_left, const uint8_t* d_right,
                      int width, int height, size_t stride,
                      int16_t* d_disp, size_t out_stride, void* stream);

/* Frame batch, sharded frame i -> devices[i % n_dev] (SURVEY §8e "frame batch"). Each
 * device gets a driver thread, a packer and an unpacker thread, a compute stream and two
 * high-priority copy streams: its frames stream through pinned host rings (user rows ->
 * pinned -> H2D -> pipelined census batch / per-frame OCV pipeline -> D2H -> user rows), so
 * host copies, PCIe and kernels overlap. Host buffers with one row stride per side (stride,
 * out_stride in elements); synchronous; no cross-device traffic. n_dev <= 0 or
 * devices == NULL: all visible devices; a device may be listed more than once (one handle
 * per entry). Results equal sgm_match per frame.                                            */
int  sgm_match_batch(sgm_handle* h, const uint8_t* const* lefts, const uint8_t* const* rights,
                     int n_frames, int width, int height, size_t stride,
                     int16_t* const* disps, size_t out_stride,
                     const int* devices, int n_dev);

/* One large frame split into n_bands row bands (band b -> devices[b % n_dev]), SURVEY §8(e)
 * "single huge frame" in overlap mode: each band is matched on its rows extended by `halo`
 * rows above and below, and only its own rows are kept. No path state crosses bands, so
 * pixels near band seams can differ from the full-frame result (the tests report the
 * disagreement); n_bands = 1 is exactly sgm_match. Host buffers; synchronous.          */
int  sgm_match_tiled(sgm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height,
                     size_t stride, int16_t* disp, size_t out_stride, int n_bands, int halo,
                     const int* devices, int n_dev);

/* Overlap mode on device buffers (C5 with the frame already in HBM of h's device): band b's
 * rows + halo are copied to devices[b % n_dev] (hipMemcpyPeerAsync over xGMI when the device
 * differs), matched there with sgm_match_device on that device's sub-handle, and the band's
 * own rows are copied back into d_disp. One host thread + stream per device. Work queued on
 * `stream` (may be NULL) before the call is complete before the band copies start;
 * synchronous: d_disp is complete on return. Same results as sgm_match_tiled.             */
int  sgm_match_tiled_device(sgm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                            size_t stride, int16_t* d_disp, size_t out_stride, int n_bands, int halo,
                            const int* devices, int n_dev, void* stream);

/* The same band split in exact mode (SURVEY §8(e) "exact mode", census mode only): band b
 * continues the path lines of its neighbours. Its downward sweeps start from the last
 * volume row of band b-1 and its upward sweeps from the first row of band b+1. Those
 * boundary rows (3 directions x width1 x D u8 per seam) move device to device with
 * hipMemcpyPeerAsync (xGMI). The top-down and bottom-up chains run concurrently; the WTA of a
 * band uses only its own rows, and median/speckle filters run on the assembled frame on h's
 * device. The result is bit-identical to sgm_match for any band count. Host buffers;
 * synchronous. Replaces nothing in the reference (no reference tile mode exists); the
 * per-frame contract is that of cv::StereoSGBM::compute (matcherOpenCVSGBM.cpp:21).       */
int  sgm_match_tiled_exact(sgm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height,
                           size_t stride, int16_t* disp, size_t out_stride, int n_bands,
                           const int* devices, int n_dev);

/* Frame batch on device buffers (host arrays of n_frames device pointers), asynchronous on
 * `stream`. Census mode pipelines the frames: the path aggregation of frame i+1 and the
 * WTA of frame i run in ONE launch (VALU-bound and HBM-bound work side by side), with two
 * workspace volume sets. Results are identical to n_frames sgm_match_device calls.     */
int  sgm_match_device_batch(sgm_handle* h, const uint8_t* const* d_lefts, const uint8_t* const* d_rights,
                            int n_frames, int width, int height, size_t stride,
                            int16_t* const* d_disps, size_t out_stride, void* stream);

/* Synchronise the handle's stream (after sgm_match_device with stream == NULL).          */
int  sgm_synchronize(sgm_handle* h);

const char* sgm_last_error(const sgm_handle* h);

/* ---- profiling: per-stage device time (hipEvents on the handle's stream) ---------------- */
#define SGM_MAX_STAGES 16
/* enable != 0: (re)start recording a hipEvent around every kernel launch ("stage") of
 * every match; records since the last enable are kept (no host sync per match).          */
int  sgm_set_profiling(sgm_handle* h, int enable);
/* Synchronises on the last record and fills up to `max` per-stage AVERAGE times (ms per
 * launch) — stages are identified by name, in first-launch order; returns their number. */
int  sgm_get_stage_times(sgm_handle* h, float* ms, int max);
/* Number of frames matched while profiling.                                               */
int  sgm_profiled_matches(const sgm_handle* h);
const char* sgm_stage_name(const sgm_handle* h, int i);
/* Algorithmic HBM bytes per launch of stage i.                         */
double sgm_stage_bytes(const sgm_handle* h, int i);
/* Number of launches of stage i recorded since profiling was enabled.                    */
int  sgm_stage_launches(const sgm_handle* h, int i);

/* ---- after the matcher: DisparityImage packing and disparity -> depth / point cloud ----- */
/* The node's processDisparity tail (generate_disparity.cpp:426-452) on device buffers:
 * out = disp * (1/16) as float, then MISSING_Z (10000) where out < min_disparity and where
 * out > max_disparity (min/max = T*f/depth_max and T*f/depth_min, as float, :447-450).
 * Asynchronous on `stream` (NULL = the handle's stream).                                   */
int  sgm_disparity_to_msg(sgm_handle* h, const int16_t* d_disp, size_t disp_stride, int width, int height,
                          float min_disparity, float max_disparity, float* d_out, size_t out_stride,
                          void* stream);

/* Q of disparity_to_depth.cpp calc_q (:62-84) from the left camera matrix K (3x3) and the
 * rectified projections P_right, P_left (3x4), all row-major doubles. Host-only.          */
void sgm_calc_q(const double K_left[9], const double P_right[12], const double P_left[12], double Q[16]);

/* One point of the cloud: pcl::PointXYZRGB's x, y, z and its packed rgba (b | g<<8 | r<<16 |
 * 255<<24).                                                                                 */
typedef struct sgm_point_xyzrgb { float x, y, z; uint32_t rgba; } sgm_point_xyzrgb;

/* disparity_to_depth.cpp:127-205 on device buffers, asynchronous on `stream`:
 *   d_disp     DisparityImage float image (pixels; 0 and MISSING_Z are skipped)
 *   d_color    MONO8 (channels 1) / BGR8 (channels 3) image, or NULL with channels 0 (black)
 *   q          {Q(2,3), Q(0,3), Q(1,3), Q(3,2), Q(3,3)} (cast to float, as the node does)
 *   depth_min/max  the node's depth window (z kept when depth_min <= z <= depth_max)
 *   d_depth    (may be NULL) W x H float depth, 0 where no point
 *   d_points   (may be NULL) the first max_points points in raster order (pcl push_back order)
 *   d_num_points (device int, may be NULL) receives the total number of points.           */
int  sgm_depth_points(sgm_handle* h, const float* d_disp, size_t disp_stride, int width, int height,
                      const uint8_t* d_color, size_t color_stride, int channels, const double q[5],
                      double depth_min, double depth_max, float* d_depth, size_t depth_stride,
                      sgm_point_xyzrgb* d_points, int max_points, int* d_num_points, void* stream);

/* ---- rectification: the node's rectify(), generate_disparity.cpp:370-386
 * and rectify.cpp:111-127 — cv::initUndistortRectifyMap(K, D, R, P, size, CV_32FC1) then
 * cv::remap(INTER_CUBIC, BORDER_CONSTANT 0) — with the map computed once per calibration. */

/* Float rectification maps (map_x, map_y: W x H, row stride map_stride floats) on the device
 * from the CameraInfo matrices (row-major doubles): K 3x3, D (n_dist = 0, 4, 5, 8 or 12:
 * k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4]]]; the node passes 5), R 3x3 (NULL = identity),
 * P 3x4 (its left 3x3 is the new camera matrix). Asynchronous on `stream`.
 * SGM_ERR_UNSUPPORTED for other n_dist (the tilted-sensor model); SGM_ERR_ARG if P*R is
 * singular.                                                                                */
int  sgm_rectify_map(sgm_handle* h, const double K[9], const double* D, int n_dist, const double R[9],
                     const double P[12], int width, int height, float* d_map_x, float* d_map_y,
                     size_t map_stride, void* stream);
/* One remapped u8 image: dst(x, y) = bicubic(src at (map_x, map_y)), OpenCV's fixed-point
 * INTER_CUBIC (1/32 px positions, 15-bit weights), source pixels outside src_w x src_h read
 * 0. dst is width x height like the maps. Asynchronous on `stream`.                        */
int  sgm_remap_cubic(sgm_handle* h, const uint8_t* d_src, size_t src_stride, int src_w, int src_h,
                     const float* d_map_x, const float* d_map_y, size_t map_stride, int width, int height,
                     uint8_t* d_dst, size_t dst_stride, void* stream);
/* Rectification fused into the census (census mode): after this call the device matches
 * (sgm_match_device, sgm_match_device_batch, sgm_match_device_batch_rect) take RAW images of
 * src_width x src_height (their stride argument = the raw stride) and rectify them inside
 * the census tiles through the maps (W x H = the match geometry, e.g. from sgm_rectify_map;
 * left x/y, right x/y). The maps must stay valid while set. All four maps NULL switches it
 * off. sgm_match (host buffers) returns SGM_ERR_UNSUPPORTED while it is on, as do the OCV
 * modes (rectify those with sgm_remap_cubic).                                               */
int  sgm_set_rectification(sgm_handle* h, const float* d_map_xl, const float* d_map_yl, const float* d_map_xr,
                           const float* d_map_yr, size_t map_stride, int src_width, int src_height);
/* sgm_match_device_batch that also returns the rectified images (d_rect_lefts /
 * d_rect_rights: arrays of n device pointers, W x H u8 with row stride rect_stride; either
 * array may be NULL). Needs sgm_set_rectification.                                          */
int  sgm_match_device_batch_rect(sgm_handle* h, const uint8_t* const* d_raw_lefts, const uint8_t* const* d_raw_rights,
                                 int n_frames, int width, int height, size_t raw_stride,
                                 uint8_t* const* d_rect_lefts, uint8_t* const* d_rect_rights, size_t rect_stride,
                                 int16_t* const* d_disps, size_t out_stride, void* stream);
/* The 32 x 32 x 16 int16 INTER_CUBIC weight table (entry fy*32 + fx, tap row*4 + col) the
 * remap uses. Host-only.                                                                   */
void sgm_cubic_table(int16_t tab[16384]);

/* ---- stage entry points (parity tests compare each stage with the CPU oracle) ----------- */
/* 9x7 census codes of one image (host buffers; out: W x H uint64, row-major).             */
int  sgm_debug_census(sgm_handle* h, const uint8_t* img, int width, int height,
                      size_t stride, uint64_t* out);
/* Census mode: u8 path-cost volume of direction `dir` (0..7; see DESIGN.md for the order),
 * layout [H][width1][D]. Runs census + that direction only.                               */
int  sgm_debug_census_path(sgm_handle* h, const uint8_t* left, const uint8_t* right,
                           int width, int height, size_t stride, int dir, uint8_t* vol);
/* OCV modes: int16 aggregated matching cost C' = SAD + P2 used by the path recurrence,
 * layout [H][width1][D].                                                                  */
int  sgm_debug_ocv_cost(sgm_handle* h, const uint8_t* left, const uint8_t* right,
                        int width, int height, size_t stride, int16_t* cost);
/* Census mode: the path work list one launch would dispatch (host-only, no device): every
 * 16-line block of the directions in dir_mask (bit d) of `group` frames, plus the up+WTA
 * blocks (code 8) of `up_group` frames, as dir << 24 | frame << 22 | block, longest first,
 * dealt in a snake over rounds of n_slots. Returns the entry count (out may be NULL), or
 * < 0 on an error (cap too small: SGM_ERR_ARG).                                           */
int  sgm_debug_path_items(const sgm_params* p, int width, int height, unsigned dir_mask, int n_slots,
                          int group, int up_group, uint32_t* out, int cap);
/* 3x3 median (replicate border) and speckle filter on a host int16 image, in place.       */
int  sgm_debug_median3(sgm_handle* h, int16_t* disp, int width, int height);
int  sgm_debug_speckle(sgm_handle* h, int16_t* disp, int width, int height,
                       int new_val, int max_size, int max_diff);

#ifdef __cplusplus
}
#endif
#endif /* SGM_HIP_H */
