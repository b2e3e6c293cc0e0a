/*
 * sgm_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement ("oracle") of the reference's
 * disparity hot path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library; the product path (libsgm_hip.so) never does.
 *
 * PARITY STATUS: **parity unpinned** against the reference's real arithmetic.
 *   The reference delegates its arithmetic to third-party OpenCV (`cv::StereoSGBM`,
 *   modules/calib3d/src/stereosgbm.cpp + imgproc medianBlur), pinned only by ROS distro
 *   (melodic -> OpenCV 3.2.0, noetic -> 4.2.0; reference .github/workflows/ros-build.yml:14-21,
 *   CMakeLists.txt:48-51). OpenCV is absent from this image and the reference holds no
 *   tests, fixtures or golden vectors, so this file restates OpenCV's
 *   published algorithm (OpenCV >= 3.4 / 4.x semantics) and is pinned
 *   by analytic known-answer tests (tests/test_oracle.py) and its own committed fixtures.
 *
 * Reference call sites the restatement follows:
 *   - cv::StereoSGBM::create(64, 9, 5) then 10 setters    matcherOpenCVSGBM.cpp:14, :53-110
 *   - matcher->compute(left, right, disparity_lr)          matcherOpenCVSGBM.cpp:21
 *   - node defaults minD 9, D 64, block 15, P1 200, P2 400 generate_disparity.cpp:100-112
 *   - mode never set -> MODE_SGBM (5 dirs); disp12MaxDiff never forwarded (Q1)
 *                                                          generate_disparity.cpp:241-261
 *
 * Census-SGM (SGM_MODE_CENSUS8) has NO reference implementation (the closest analogue is
 * the closed Phobos library, I3DRSGM.cpp:158-165); it follows the build-defined spec of
 * SURVEY.md Appendix B and this file is its definition.
 */
#include "sgm_hip.h"

#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define DISP_SHIFT 4
#define DISP_SCALE 16
#define MAX_COST 32767

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iclamp(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int16_t sat16(int v) { return (int16_t)iclamp(v, SHRT_MIN, SHRT_MAX); }

/* ======================================================================================
 * OpenCV build variants (oracle switches; DESIGN.md §3 "OpenCV semantics targets").
 * The reference pins OpenCV only by ROS distro (melodic -> 3.2.0, noetic -> 4.2.0;
 * .github/workflows/ros-build.yml:14-21, CMakeLists.txt:48-51), and computeDisparitySGBM
 * differs between versions and between its scalar and CV_SIMD branches. The bits come from
 * `sgm_params.ocv_compat` (include/sgm_hip.h SGM_OCV_*; the GPU engine reproduces every
 * combination), OR-ed with the process-wide switch below (the KATs' context manager).
 * 0 is the scalar branch with the column-0 update of the refactored 4.x loop. Bits:
 *   SGMREF_OCV_COL0_LEGACY  the 3.x loop `for (x = D; x < width1*D; x += D)`: for y > 0 the
 *                           vertical running sum never updates C' column 0 (x = minX1), so it
 *                           keeps its row-0 value (MODE_SGBM, one C row buffer) or the P2
 *                           initialisation (MODE_HH, one C row per image row).
 *   SGMREF_OCV_SIMD_SAT     the CV_SIMD (SSE2 / universal-intrinsic) branches, taken by every
 *                           x86-64 build: int16 saturating adds/subs in the y > 0 horizontal and
 *                           vertical running sums ((h - sub) + add, (C - hsub) + h), in the path
 *                           recurrence (L = sat(sat(min - delta) + C), Lp(d+-1) + P1 saturated,
 *                           delta = (short)(minLr + P2)), Lr and minLr kept as the saturated
 *                           int16 values, and S = sat(sat(S + sat(L0+L1)) + sat(L2+L3)) (+ the
 *                           fifth path saturated alone). Scalar: int arithmetic, int16 wrapping
 *                           stores, S += saturate_cast(L0+L1+L2+L3). They agree while no box
 *                           sum or path cost leaves int16.
 *   SGMREF_OCV_LANE_TIE     MODE_SGBM's SSE2 WTA (3.x: per-lane strict minima over 8 int16
 *                           lanes, then LSBTab of the lanes holding the minimum): among equal
 *                           minimal S the winner is the one in the lowest lane (d mod 8), then
 *                           the smallest d in that lane, instead of the smallest d.
 * ====================================================================================== */
#define SGMREF_OCV_COL0_LEGACY SGM_OCV_COL0_LEGACY
#define SGMREF_OCV_SIMD_SAT SGM_OCV_SIMD_SAT
#define SGMREF_OCV_LANE_TIE SGM_OCV_LANE_TIE
static int g_ocv_compat = 0;
void sgmref_set_ocv_compat(int flags) { g_ocv_compat = flags; }
int sgmref_get_ocv_compat(void) { return g_ocv_compat; }
static inline int16_t adds16(int a, int b) { return sat16(a + b); }   /* _mm_adds_epi16 */
static inline int16_t subs16(int a, int b) { return sat16(a - b); }   /* _mm_subs_epi16 */

/* Effective parameters: head of OpenCV computeDisparitySGBM. */
typedef struct {
    int minD, maxD, D;
    int SW2, SH2, ftzero, uniq, disp12, P1, P2;
    int minX1, maxX1, width1;
    int invalid_scaled;
    int subpix, lr, median, census;
    int npasses;
    int compat;          /* SGMREF_OCV_* bits (OCV modes only) */
} eff_t;

int sgmref_effective(const sgm_params* p, int width, int height, int* out /* 16 ints */);

static int effective(const sgm_params* p, int width, int height, eff_t* e)
{
    if (!p || width <= 0 || height <= 0) return SGM_ERR_ARG;
    if (p->mode < SGM_MODE_OCV_SGBM5 || p->mode > SGM_MODE_CENSUS8) return SGM_ERR_PARAM;
    if (p->num_disparities <= 0 || p->num_disparities % 16 != 0) return SGM_ERR_PARAM;
    e->census = p->mode == SGM_MODE_CENSUS8;
    e->minD = p->min_disparity;
    e->D = p->num_disparities;
    e->maxD = e->minD + e->D;
    if (e->census) {
        /* Appendix B: u8 path costs need C + P2 <= 255 with C <= 62 -> P2 <= 193. */
        e->SW2 = 4; e->SH2 = 3;
        e->P1 = p->p1 > 0 ? p->p1 : 10;
        e->P2 = imax(p->p2 > 0 ? p->p2 : 120, e->P1 + 1);
        if (e->P2 > 193) e->P2 = 193;
        if (e->P1 >= e->P2) e->P1 = e->P2 - 1;
        e->ftzero = 0;
        e->subpix = p->subpixel != 0;
        e->lr = p->lr_check != 0;
        e->median = p->median != 0;
        e->npasses = 1;
    } else {
        int sw = p->block_size > 0 ? p->block_size : 5;
        e->SW2 = sw / 2; e->SH2 = sw / 2;
        e->ftzero = imax(p->prefilter_cap, 15) | 1;
        e->P1 = p->p1 > 0 ? p->p1 : 2;
        e->P2 = imax(p->p2 > 0 ? p->p2 : 5, e->P1 + 1);
        e->subpix = 1; e->lr = 1; e->median = 1;
        e->npasses = p->mode == SGM_MODE_OCV_HH8 ? 2 : 1;
    }
    e->compat = e->census ? 0 : ((p->ocv_compat | g_ocv_compat) & 7);
    e->uniq = p->uniqueness_ratio >= 0 ? p->uniqueness_ratio : 10;
    e->disp12 = p->disp12_max_diff > 0 ? p->disp12_max_diff : 1;
    e->minX1 = imax(e->maxD, 0);
    e->maxX1 = width + imin(e->minD, 0);
    e->width1 = e->maxX1 - e->minX1;
    e->invalid_scaled = (e->minD - 1) * DISP_SCALE;
    /* the engine's limits: census 512 (u8 path engine), OpenCV modes 2048 (the node's cfg) */
    if (e->D > (e->census ? 512 : 2048)) return SGM_ERR_UNSUPPORTED;
    if (width > 32767 || height > 32767) return SGM_ERR_UNSUPPORTED;
    return SGM_OK;
}

int sgmref_effective(const sgm_params* p, int width, int height, int* out)
{
    eff_t e;
    int rc = effective(p, width, height, &e);
    if (rc) return rc;
    int v[16] = {e.minD, e.D, e.SW2, e.SH2, e.ftzero, e.uniq, e.disp12, e.P1, e.P2,
                 e.minX1, e.maxX1, e.width1, e.invalid_scaled, e.subpix, e.lr, e.median};
    memcpy(out, v, sizeof(v));
    return SGM_OK;
}

/* ======================================================================================
 * Post filters shared by all modes
 * ====================================================================================== */

/* medianBlur(disp, disp, 3) on CV_16S, BORDER_REPLICATE (imgproc median_blur.cpp). */
int sgmref_median3(int16_t* img, int w, int h, size_t stride)
{
    if (!img || w <= 0 || h <= 0) return SGM_ERR_ARG;
    int16_t* src = (int16_t*)malloc(sizeof(int16_t) * (size_t)w * h);
    if (!src) return SGM_ERR_ALLOC;
    for (int y = 0; y < h; y++) memcpy(src + (size_t)y * w, img + (size_t)y * stride, sizeof(int16_t) * w);
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            int v[9], n = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++)
                    v[n++] = src[(size_t)iclamp(y + dy, 0, h - 1) * w + iclamp(x + dx, 0, w - 1)];
            for (int i = 1; i < 9; i++) { /* insertion sort, 9 elements */
                int t = v[i], j = i - 1;
                while (j >= 0 && v[j] > t) { v[j + 1] = v[j]; j--; }
                v[j + 1] = t;
            }
            img[(size_t)y * stride + x] = (int16_t)v[4];
        }
    }
    free(src);
    return SGM_OK;
}

/* filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) — calib3d filterSpecklesImpl:
 * 4-connected flood fill over pixels != newVal, neighbours joined when |p - q| <= maxDiff;
 * every region with <= maxSpeckleSize pixels is set to newVal. Raster seed order,
 * LIFO wavefront, region membership decided on the unmodified values. */
int sgmref_filter_speckles(int16_t* img, int w, int h, size_t stride, int newVal, int maxSize, int maxDiff)
{
    if (!img || w <= 0 || h <= 0) return SGM_ERR_ARG;
    size_t n = (size_t)w * h;
    int* labels = (int*)calloc(n, sizeof(int));
    int* stack = (int*)malloc(sizeof(int) * n);
    unsigned char* rtype = (unsigned char*)calloc(n + 1, 1);
    if (!labels || !stack || !rtype) { free(labels); free(stack); free(rtype); return SGM_ERR_ALLOC; }
    int curlabel = 0;
    for (int i = 0; i < h; i++) {
        int16_t* ds = img + (size_t)i * stride;
        int* ls = labels + (size_t)w * i;
        for (int j = 0; j < w; j++) {
            if (ds[j] == newVal) continue;
            if (ls[j]) {
                if (rtype[ls[j]]) ds[j] = (int16_t)newVal;
                continue;
            }
            int top = 0, count = 0;
            curlabel++;
            ls[j] = curlabel;
            int px = j, py = i;
            for (;;) {
                count++;
                int16_t* dpp = img + (size_t)py * stride + px;
                int dp = *dpp;
                int* lpp = labels + (size_t)w * py + px;
                if (py < h - 1 && !lpp[w] && dpp[stride] != newVal && abs(dp - dpp[stride]) <= maxDiff) {
                    lpp[w] = curlabel; stack[top++] = (py + 1) * w + px;
                }
                if (py > 0 && !lpp[-w] && dpp[-(ptrdiff_t)stride] != newVal && abs(dp - dpp[-(ptrdiff_t)stride]) <= maxDiff) {
                    lpp[-w] = curlabel; stack[top++] = (py - 1) * w + px;
                }
                if (px < w - 1 && !lpp[1] && dpp[1] != newVal && abs(dp - dpp[1]) <= maxDiff) {
                    lpp[1] = curlabel; stack[top++] = py * w + px + 1;
                }
                if (px > 0 && !lpp[-1] && dpp[-1] != newVal && abs(dp - dpp[-1]) <= maxDiff) {
                    lpp[-1] = curlabel; stack[top++] = py * w + px - 1;
                }
                if (top == 0) break;
                int q = stack[--top];
                py = q / w; px = q % w;
            }
            if (count <= maxSize) { rtype[ls[j]] = 1; ds[j] = (int16_t)newVal; }
            else rtype[ls[j]] = 0;
        }
    }
    free(labels); free(stack); free(rtype);
    return SGM_OK;
}

/* ======================================================================================
 * Winner-take-all + uniqueness + subpixel + disp2 (right view) + LR check, one row.
 * OpenCV computeDisparitySGBM, `if( pass == npasses )` block.
 * `S` holds width1*D sums (non-negative, <= 32767). For the OCV 5-direction mode the
 * fifth path is folded into S by the caller before each pixel is visited (see below).
 * ====================================================================================== */
typedef struct {
    int16_t* disp2;     /* width */
    int* disp2cost;     /* width */
} wta_buf_t;

static void wta_row_begin(const eff_t* e, int width, int16_t* disp_row, wta_buf_t* b)
{
    for (int x = 0; x < width; x++) {
        disp_row[x] = (int16_t)e->invalid_scaled;
        b->disp2[x] = (int16_t)e->invalid_scaled;
        b->disp2cost[x] = MAX_COST;
    }
}

/* One pixel x (0-based inside [0,width1)), visited in descending x order. */
static void wta_pixel(const eff_t* e, int x, const int* Sp, int16_t* disp_row, wta_buf_t* b)
{
    const int D = e->D;
    int minS = MAX_COST, bestDisp = -1, d;
    if ((e->compat & SGMREF_OCV_LANE_TIE) && e->npasses == 1) {
        /* SSE2: lane l (d = l, l+8, ...) keeps its first strict minimum from MAX_COST; the
         * lowest lane holding the overall minimum wins (LSBTab) */
        int lmin[8], lbest[8];
        for (int l = 0; l < 8; l++) { lmin[l] = MAX_COST; lbest[l] = -1; }
        for (d = 0; d < D; d++)
            if (Sp[d] < lmin[d & 7]) { lmin[d & 7] = Sp[d]; lbest[d & 7] = d; }
        for (int l = 0; l < 8; l++) minS = imin(minS, lmin[l]);
        for (int l = 0; l < 8; l++)
            if (lmin[l] == minS) { bestDisp = lbest[l]; break; }
    } else {
        for (d = 0; d < D; d++)
            if (Sp[d] < minS) { minS = Sp[d]; bestDisp = d; }
    }
    for (d = 0; d < D; d++)
        if (Sp[d] * (100 - e->uniq) < minS * 100 && abs(bestDisp - d) > 1) break;
    if (d < D) return;                         /* uniqueness reject: no disp2 update either */
    d = bestDisp;
    /* bestDisp == -1 (every S saturated at MAX_COST) puts x2 one past the row; OpenCV reads
     * a CostType there, which can never exceed minS == MAX_COST: no update */
    int x2 = x + e->minX1 - d - e->minD;
    if (d >= 0 && b->disp2cost[x2] > minS) { b->disp2cost[x2] = minS; b->disp2[x2] = (int16_t)(d + e->minD); }
    if (e->subpix && 0 < d && d < D - 1) {
        int denom2 = imax(Sp[d - 1] + Sp[d + 1] - 2 * Sp[d], 1);
        d = d * DISP_SCALE + ((Sp[d - 1] - Sp[d + 1]) * DISP_SCALE + denom2) / (denom2 * 2);
    } else {
        d *= DISP_SCALE;
    }
    disp_row[x + e->minX1] = (int16_t)(d + e->minD * DISP_SCALE);
}

static void wta_row_lrcheck(const eff_t* e, int width, int16_t* disp_row, const wta_buf_t* b)
{
    if (!e->lr) return;
    for (int x = e->minX1; x < e->maxX1; x++) {
        int d1 = disp_row[x];
        if (d1 == e->invalid_scaled) continue;
        int _d = d1 >> DISP_SHIFT;
        int d_ = (d1 + DISP_SCALE - 1) >> DISP_SHIFT;
        int _x = x - _d, x_ = x - d_;
        if (0 <= _x && _x < width && b->disp2[_x] >= e->minD && abs(b->disp2[_x] - _d) > e->disp12 &&
            0 <= x_ && x_ < width && b->disp2[x_] >= e->minD && abs(b->disp2[x_] - d_) > e->disp12)
            disp_row[x] = (int16_t)e->invalid_scaled;
    }
}

/* Public helper for stage tests: WTA/LR over a full S volume [H][width1][D]. */
int sgmref_wta(const sgm_params* p, int width, int height, const uint16_t* S, int16_t* disp, size_t out_stride)
{
    eff_t e;
    int rc = effective(p, width, height, &e);
    if (rc) return rc;
    wta_buf_t b;
    b.disp2 = (int16_t*)malloc(sizeof(int16_t) * width);
    b.disp2cost = (int*)malloc(sizeof(int) * width);
    int* tmp = (int*)malloc(sizeof(int) * e.D);
    if (!b.disp2 || !b.disp2cost || !tmp) { free(b.disp2); free(b.disp2cost); free(tmp); return SGM_ERR_ALLOC; }
    for (int y = 0; y < height; y++) {
        int16_t* row = disp + (size_t)y * out_stride;
        wta_row_begin(&e, width, row, &b);
        if (e.width1 > 0)
            for (int x = e.width1 - 1; x >= 0; x--) {
                const uint16_t* Sp = S + ((size_t)y * e.width1 + x) * e.D;
                for (int d = 0; d < e.D; d++) tmp[d] = Sp[d];
                wta_pixel(&e, x, tmp, row, &b);
            }
        wta_row_lrcheck(&e, width, row, &b);
    }
    free(b.disp2); free(b.disp2cost); free(tmp);
    return SGM_OK;
}

/* ======================================================================================
 * OpenCV-compatible modes (SGM_MODE_OCV_SGBM5 / SGM_MODE_OCV_HH8)
 * ====================================================================================== */

/* calcPixelCostBT (mono): adds the Birchfield-Tomasi dissimilarity of the prefiltered
 * image (shift 0) and of the raw image (shift 2) for every x in [minX1,maxX1), d in
 * [minD,maxD). Prefilter: clip(2(r[x+1]-r[x-1]) + n[x+1]-n[x-1] + s[x+1]-s[x-1]) + ftzero
 * with n/s the rows above/below (replicated at the image edges); columns 0 and W-1 of
 * BOTH channels are forced to ftzero (= clipTab[TAB_OFS]). */
static void ocv_prefilter_row(const uint8_t* img, int w, int h, size_t stride, int y, int ftzero,
                              uint8_t* pf, uint8_t* raw)
{
    const uint8_t* r = img + (size_t)y * stride;
    const uint8_t* n = y > 0 ? r - stride : r;
    const uint8_t* s = y < h - 1 ? r + stride : r;
    pf[0] = pf[w - 1] = raw[0] = raw[w - 1] = (uint8_t)ftzero;
    for (int x = 1; x < w - 1; x++) {
        int v = (r[x + 1] - r[x - 1]) * 2 + n[x + 1] - n[x - 1] + s[x + 1] - s[x - 1];
        pf[x] = (uint8_t)(iclamp(v, -ftzero, ftzero) + ftzero);
        raw[x] = r[x];
    }
}

/* half-pixel min/max of a channel row: lo/hi of {(u+u_l)/2, u, (u+u_r)/2} */
static void bt_minmax(const uint8_t* a, int w, uint8_t* lo, uint8_t* hi)
{
    for (int x = 0; x < w; x++) {
        int u = a[x];
        int ul = x > 0 ? (u + a[x - 1]) / 2 : u;
        int ur = x < w - 1 ? (u + a[x + 1]) / 2 : u;
        lo[x] = (uint8_t)imin(imin(ul, ur), u);
        hi[x] = (uint8_t)imax(imax(ul, ur), u);
    }
}

static void ocv_pixel_cost_bt(const uint8_t* L, const uint8_t* R, int w, int h, size_t stride, int y,
                              const eff_t* e, int16_t* cost /* width1*D */, uint8_t* tmp /* 16*w */)
{
    uint8_t *pf1 = tmp, *raw1 = tmp + w, *pf2 = tmp + 2 * w, *raw2 = tmp + 3 * w;
    uint8_t *lo1 = tmp + 4 * w, *hi1 = tmp + 5 * w, *lo2 = tmp + 6 * w, *hi2 = tmp + 7 * w;
    ocv_prefilter_row(L, w, h, stride, y, e->ftzero, pf1, raw1);
    ocv_prefilter_row(R, w, h, stride, y, e->ftzero, pf2, raw2);
    memset(cost, 0, sizeof(int16_t) * (size_t)e->width1 * e->D);
    for (int c = 0; c < 2; c++) {
        const uint8_t* p1 = c == 0 ? pf1 : raw1;
        const uint8_t* p2 = c == 0 ? pf2 : raw2;
        int shift = c == 0 ? 0 : 2;
        bt_minmax(p1, w, lo1, hi1);
        bt_minmax(p2, w, lo2, hi2);
        for (int x = e->minX1; x < e->maxX1; x++) {
            int u = p1[x], u0 = lo1[x], u1 = hi1[x];
            int16_t* cx = cost + (size_t)(x - e->minX1) * e->D;
            for (int d = e->minD; d < e->maxD; d++) {
                int xr = x - d;
                int v = p2[xr], v0 = lo2[xr], v1 = hi2[xr];
                int c0 = imax(0, imax(u - v1, v0 - u));
                int c1 = imax(0, imax(v - u1, u0 - v));
                cx[d - e->minD] = (int16_t)(cx[d - e->minD] + (imin(c0, c1) >> shift));
            }
        }
    }
}

/* Computes, for every row y, the cost row C'(y) = P2 + SAD used by the recurrence,
 * following OpenCV's row loop: a ring of SH2*2+2 horizontal-sum rows, a vertical running
 * sum Cprev + hsum(y+SH2) - hsum(max(y-SH2-1,0)), and the quirk that rows with
 * y + SH2 >= H are never recomputed (MODE_SGBM keeps the last computed row; MODE_HH keeps
 * the P2 initialisation). `emit(y, Crow)` receives each row. */
typedef void (*cost_row_cb)(void* ctx, int y, const int16_t* Crow);

static int ocv_cost_rows(const uint8_t* L, const uint8_t* R, int w, int h, size_t stride,
                         const eff_t* e, cost_row_cb emit, void* ctx)
{
    const int D = e->D, width1 = e->width1, SW2 = e->SW2, SH2 = e->SH2;
    const size_t costBufSize = (size_t)width1 * D;
    const int hsumBufNRows = SH2 * 2 + 2;
    int16_t* hsumBuf = (int16_t*)malloc(sizeof(int16_t) * costBufSize * hsumBufNRows);
    int16_t* pixDiff = (int16_t*)malloc(sizeof(int16_t) * costBufSize);
    int16_t* C = (int16_t*)malloc(sizeof(int16_t) * costBufSize);      /* current row  */
    int16_t* Cprev = (int16_t*)malloc(sizeof(int16_t) * costBufSize);  /* row y-1 (HH) */
    uint8_t* tmp = (uint8_t*)malloc((size_t)16 * w);
    if (!hsumBuf || !pixDiff || !C || !Cprev || !tmp) {
        free(hsumBuf); free(pixDiff); free(C); free(Cprev); free(tmp);
        return SGM_ERR_ALLOC;
    }
    const int fullDP = e->npasses == 2;
    for (size_t k = 0; k < costBufSize; k++) C[k] = (int16_t)e->P2;
    for (int y = 0; y < h; y++) {
        if (fullDP) {                    /* HH: every row has its own C, initialised to P2 */
            memcpy(Cprev, C, sizeof(int16_t) * costBufSize);
            for (size_t k = 0; k < costBufSize; k++) C[k] = (int16_t)e->P2;
        } else {
            memcpy(Cprev, C, sizeof(int16_t) * costBufSize);   /* single buffer: Cprev == C */
        }
        int dy1 = y == 0 ? 0 : y + SH2, dy2 = y == 0 ? SH2 : dy1;
        for (int k = dy1; k <= dy2; k++) {
            int16_t* hsumAdd = hsumBuf + (size_t)(imin(k, h - 1) % hsumBufNRows) * costBufSize;
            if (k < h) {
                ocv_pixel_cost_bt(L, R, w, h, stride, k, e, pixDiff, tmp);
                for (int d = 0; d < D; d++) {
                    int s = pixDiff[d] * (SW2 + 1);
                    for (int x = 1; x <= SW2; x++) s += pixDiff[(size_t)imin(x, width1 - 1) * D + d];
                    hsumAdd[d] = (int16_t)s;
                }
                /* CV_SIMD saturates the running sums of rows y > 0 (the y == 0 rows run the
                 * scalar loop in every version) */
                const int sat = (e->compat & SGMREF_OCV_SIMD_SAT) && y > 0;
                for (int x = 1; x < width1; x++) {
                    const int16_t* pixAdd = pixDiff + (size_t)imin(x + SW2, width1 - 1) * D;
                    const int16_t* pixSub = pixDiff + (size_t)imax(x - SW2 - 1, 0) * D;
                    int16_t* hx = hsumAdd + (size_t)x * D;
                    const int16_t* hp = hsumAdd + (size_t)(x - 1) * D;
                    for (int d = 0; d < D; d++)
                        hx[d] = sat ? adds16(subs16(hp[d], pixSub[d]), pixAdd[d])
                                    : (int16_t)(hp[d] + pixAdd[d] - pixSub[d]);
                }
                if (y > 0) {
                    const int16_t* hsumSub = hsumBuf + (size_t)(imax(y - SH2 - 1, 0) % hsumBufNRows) * costBufSize;
                    /* 3.x: the vertical update starts at column 1 (x = D) */
                    const size_t i0 = (e->compat & SGMREF_OCV_COL0_LEGACY) ? (size_t)D : 0;
                    for (size_t i = i0; i < costBufSize; i++)
                        C[i] = sat ? adds16(subs16(Cprev[i], hsumSub[i]), hsumAdd[i])
                                   : (int16_t)(Cprev[i] + hsumAdd[i] - hsumSub[i]);
                }
            }
            if (y == 0) {
                int scale = k == 0 ? SH2 + 1 : 1;
                for (size_t i = 0; i < costBufSize; i++) C[i] = (int16_t)(C[i] + hsumAdd[i] * scale);
            }
        }
        emit(ctx, y, C);
    }
    free(hsumBuf); free(pixDiff); free(C); free(Cprev); free(tmp);
    return SGM_OK;
}

typedef struct { int16_t* vol; size_t row; } cost_vol_ctx;
static void emit_to_volume(void* ctx, int y, const int16_t* Crow)
{
    cost_vol_ctx* c = (cost_vol_ctx*)ctx;
    memcpy(c->vol + (size_t)y * c->row, Crow, sizeof(int16_t) * c->row);
}

/* Stage helper: the aggregated cost volume C' [H][width1][D] (int16, includes +P2). */
int sgmref_ocv_cost(const sgm_params* p, const uint8_t* L, const uint8_t* R, int w, int h, size_t stride,
                    int16_t* vol)
{
    eff_t e;
    int rc = effective(p, w, h, &e);
    if (rc) return rc;
    if (e.census) return SGM_ERR_PARAM;
    if (e.width1 <= 0) return SGM_OK;
    cost_vol_ctx c = {vol, (size_t)e.width1 * e.D};
    return ocv_cost_rows(L, R, w, h, stride, &e, emit_to_volume, &c);
}

/* The OpenCV raster SGM (computeDisparitySGBM): pass 1 top->bottom, ascending x, paths
 * r0=(x-1,y) r1=(x-1,y-1) r2=(x,y-1) r3=(x+1,y-1); MODE_HH pass 2 bottom->top, descending
 * x, r0=(x+1,y) r1=(x-1,y+1) r2=(x,y+1) r3=(x+1,y+1); MODE_SGBM adds r=(x+1,y) inside
 * the descending WTA loop. Lr rows keep one border column on each side and the d=-1/D
 * slots at MAX_COST; previous-row state outside the image is 0 (path start L = C). */
typedef struct {
    const eff_t* e;
    int16_t* Cvol;   /* MODE_HH: full cost volume; MODE_SGBM: NULL (rows streamed) */
} ocv_ctx;

static int ocv_match(const eff_t* e, const uint8_t* L, const uint8_t* R, int w, int h, size_t stride,
                     int16_t* disp, size_t out_stride)
{
    const int D = e->D, width1 = e->width1, P1 = e->P1, P2 = e->P2;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) disp[(size_t)y * out_stride + x] = (int16_t)e->invalid_scaled;
    if (e->minX1 >= e->maxX1) return SGM_OK;

    const size_t costBufSize = (size_t)width1 * D;
    const int fullDP = e->npasses == 2;
    int16_t* Cvol = (int16_t*)malloc(sizeof(int16_t) * costBufSize * h);
    uint16_t* Svol = (uint16_t*)malloc(sizeof(uint16_t) * costBufSize * (fullDP ? h : 1));
    /* Lr[k]: (width1+2) columns x 4 slots x (D+2) entries (d=-1..D) */
    const int D2 = D + 2;
    const size_t LrRow = (size_t)(width1 + 2) * 4 * D2;
    int* Lr[2] = {(int*)malloc(sizeof(int) * LrRow), (int*)malloc(sizeof(int) * LrRow)};
    int* minLr[2] = {(int*)malloc(sizeof(int) * (width1 + 2) * 4), (int*)malloc(sizeof(int) * (width1 + 2) * 4)};
    wta_buf_t b;
    b.disp2 = (int16_t*)malloc(sizeof(int16_t) * w);
    b.disp2cost = (int*)malloc(sizeof(int) * w);
    int* Stmp = (int*)malloc(sizeof(int) * D);
    int rc = SGM_OK;
    if (!Cvol || !Svol || !Lr[0] || !Lr[1] || !minLr[0] || !minLr[1] || !b.disp2 || !b.disp2cost || !Stmp) {
        rc = SGM_ERR_ALLOC;
        goto done;
    }
    {
        cost_vol_ctx cc = {Cvol, costBufSize};
        rc = ocv_cost_rows(L, R, w, h, stride, e, emit_to_volume, &cc);
        if (rc) goto done;
    }
#define LR(buf, x, k) ((buf) + ((size_t)((x) + 1) * 4 + (k)) * D2 + 1) /* d index 0..D-1, [-1],[D] valid */
#define MINLR(buf, x, k) ((buf)[((x) + 1) * 4 + (k)])
    for (int pass = 1; pass <= e->npasses; pass++) {
        int y1, y2, dy, x1, x2, dx;
        if (pass == 1) { y1 = 0; y2 = h; dy = 1; x1 = 0; x2 = width1; dx = 1; }
        else { y1 = h - 1; y2 = -1; dy = -1; x1 = width1 - 1; x2 = -1; dx = -1; }
        memset(Lr[0], 0, sizeof(int) * LrRow); memset(Lr[1], 0, sizeof(int) * LrRow);
        memset(minLr[0], 0, sizeof(int) * (width1 + 2) * 4); memset(minLr[1], 0, sizeof(int) * (width1 + 2) * 4);
        for (int y = y1; y != y2; y += dy) {
            const int16_t* C = Cvol + (size_t)y * costBufSize;
            uint16_t* S = Svol + (fullDP ? (size_t)y * costBufSize : 0);
            if (pass == 1) memset(S, 0, sizeof(uint16_t) * costBufSize);
            /* clear the left/right border columns of the current row */
            for (int k = 0; k < 4; k++) {
                int* l = LR(Lr[0], -1, k); int* r = LR(Lr[0], width1, k);
                for (int d = -1; d <= D; d++) { l[d] = 0; r[d] = 0; }
                MINLR(minLr[0], -1, k) = 0; MINLR(minLr[0], width1, k) = 0;
            }
            for (int x = x1; x != x2; x += dx) {
                int delta0 = MINLR(minLr[0], x - dx, 0) + P2, delta1 = MINLR(minLr[1], x - 1, 1) + P2;
                int delta2 = MINLR(minLr[1], x, 2) + P2, delta3 = MINLR(minLr[1], x + 1, 3) + P2;
                int* Lp0 = LR(Lr[0], x - dx, 0); int* Lp1 = LR(Lr[1], x - 1, 1);
                int* Lp2 = LR(Lr[1], x, 2);      int* Lp3 = LR(Lr[1], x + 1, 3);
                Lp0[-1] = Lp0[D] = Lp1[-1] = Lp1[D] = Lp2[-1] = Lp2[D] = Lp3[-1] = Lp3[D] = MAX_COST;
                const int16_t* Cp = C + (size_t)x * D;
                uint16_t* Sp = S + (size_t)x * D;
                int minL0 = MAX_COST, minL1 = MAX_COST, minL2 = MAX_COST, minL3 = MAX_COST;
                if (e->compat & SGMREF_OCV_SIMD_SAT) {
                    /* _delta = v_setall_s16((short)delta): the int sum wraps to int16 */
                    const int dl0 = (int16_t)delta0, dl1 = (int16_t)delta1, dl2 = (int16_t)delta2, dl3 = (int16_t)delta3;
                    for (int d = 0; d < D; d++) {
                        int Cpd = Cp[d];
                        int L0 = adds16(subs16(imin(imin(Lp0[d], adds16(Lp0[d - 1], P1)), imin(adds16(Lp0[d + 1], P1), dl0)), dl0), Cpd);
                        int L1 = adds16(subs16(imin(imin(Lp1[d], adds16(Lp1[d - 1], P1)), imin(adds16(Lp1[d + 1], P1), dl1)), dl1), Cpd);
                        int L2 = adds16(subs16(imin(imin(Lp2[d], adds16(Lp2[d - 1], P1)), imin(adds16(Lp2[d + 1], P1), dl2)), dl2), Cpd);
                        int L3 = adds16(subs16(imin(imin(Lp3[d], adds16(Lp3[d - 1], P1)), imin(adds16(Lp3[d + 1], P1), dl3)), dl3), Cpd);
                        LR(Lr[0], x, 0)[d] = L0; minL0 = imin(minL0, L0);
                        LR(Lr[0], x, 1)[d] = L1; minL1 = imin(minL1, L1);
                        LR(Lr[0], x, 2)[d] = L2; minL2 = imin(minL2, L2);
                        LR(Lr[0], x, 3)[d] = L3; minL3 = imin(minL3, L3);
                        Sp[d] = (uint16_t)adds16(adds16((int16_t)Sp[d], adds16(L0, L1)), adds16(L2, L3));
                    }
                } else {
                    for (int d = 0; d < D; d++) {
                        int Cpd = Cp[d];
                        int L0 = Cpd + imin(Lp0[d], imin(Lp0[d - 1] + P1, imin(Lp0[d + 1] + P1, delta0))) - delta0;
                        int L1 = Cpd + imin(Lp1[d], imin(Lp1[d - 1] + P1, imin(Lp1[d + 1] + P1, delta1))) - delta1;
                        int L2 = Cpd + imin(Lp2[d], imin(Lp2[d - 1] + P1, imin(Lp2[d + 1] + P1, delta2))) - delta2;
                        int L3 = Cpd + imin(Lp3[d], imin(Lp3[d - 1] + P1, imin(Lp3[d + 1] + P1, delta3))) - delta3;
                        /* Lr rows are CostType (int16) in OpenCV */
                        LR(Lr[0], x, 0)[d] = (int16_t)L0; minL0 = imin(minL0, L0);
                        LR(Lr[0], x, 1)[d] = (int16_t)L1; minL1 = imin(minL1, L1);
                        LR(Lr[0], x, 2)[d] = (int16_t)L2; minL2 = imin(minL2, L2);
                        LR(Lr[0], x, 3)[d] = (int16_t)L3; minL3 = imin(minL3, L3);
                        Sp[d] = (uint16_t)sat16((int)(int16_t)Sp[d] + L0 + L1 + L2 + L3);
                    }
                }
                MINLR(minLr[0], x, 0) = (int16_t)minL0; MINLR(minLr[0], x, 1) = (int16_t)minL1;
                MINLR(minLr[0], x, 2) = (int16_t)minL2; MINLR(minLr[0], x, 3) = (int16_t)minL3;
            }
            if (pass == e->npasses) {
                int16_t* drow = disp + (size_t)y * out_stride;
                wta_row_begin(e, w, drow, &b);
                for (int x = width1 - 1; x >= 0; x--) {
                    uint16_t* Sp = S + (size_t)x * D;
                    if (e->npasses == 1) {        /* fifth path r=(x+1,y), fused into WTA */
                        int minL0 = MAX_COST;
                        int delta0 = MINLR(minLr[0], x + 1, 0) + P2;
                        int* Lp0 = LR(Lr[0], x + 1, 0);
                        Lp0[-1] = Lp0[D] = MAX_COST;
                        const int16_t* Cp = C + (size_t)x * D;
                        const int simd = (e->compat & SGMREF_OCV_SIMD_SAT) != 0;
                        const int dl0 = (int16_t)delta0;
                        for (int d = 0; d < D; d++) {
                            if (simd) {
                                int L0 = adds16(subs16(imin(imin(Lp0[d], adds16(Lp0[d - 1], P1)), imin(adds16(Lp0[d + 1], P1), dl0)), dl0), Cp[d]);
                                LR(Lr[0], x, 0)[d] = L0;
                                minL0 = imin(minL0, L0);
                                Sp[d] = (uint16_t)adds16(L0, (int16_t)Sp[d]);
                                continue;
                            }
                            int L0 = Cp[d] + imin(Lp0[d], imin(Lp0[d - 1] + P1, imin(Lp0[d + 1] + P1, delta0))) - delta0;
                            LR(Lr[0], x, 0)[d] = (int16_t)L0;
                            minL0 = imin(minL0, L0);
                            Sp[d] = (uint16_t)sat16((int)(int16_t)Sp[d] + L0);
                        }
                        MINLR(minLr[0], x, 0) = (int16_t)minL0;
                    }
                    for (int d = 0; d < D; d++) Stmp[d] = (int16_t)Sp[d];   /* CostType */
                    wta_pixel(e, x, Stmp, drow, &b);
                }
                wta_row_lrcheck(e, w, drow, &b);
            }
            int* t = Lr[0]; Lr[0] = Lr[1]; Lr[1] = t;
            t = minLr[0]; minLr[0] = minLr[1]; minLr[1] = t;
        }
    }
#undef LR
#undef MINLR
done:
    free(Cvol); free(Svol); free(Lr[0]); free(Lr[1]); free(minLr[0]); free(minLr[1]);
    free(b.disp2); free(b.disp2cost); free(Stmp);
    return rc;
}

/* ======================================================================================
 * Census-SGM (SGM_MODE_CENSUS8) — build-defined spec, SURVEY Appendix B
 * ====================================================================================== */

/* 9x7 census: bit i (raster order over dy=-3..3, dx=-4..4, centre skipped, LSB first)
 * is 1 iff I(y+dy, x+dx) < I(y, x); coordinates clamped to the image (replicate). */
int sgmref_census9x7(const uint8_t* img, int w, int h, size_t stride, uint64_t* out)
{
    if (!img || !out || w <= 0 || h <= 0) return SGM_ERR_ARG;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            int c = img[(size_t)y * stride + x];
            uint64_t code = 0;
            int bit = 0;
            for (int dy = -3; dy <= 3; dy++) {
                const uint8_t* row = img + (size_t)iclamp(y + dy, 0, h - 1) * stride;
                for (int dx = -4; dx <= 4; dx++) {
                    if (dx == 0 && dy == 0) continue;
                    if (row[iclamp(x + dx, 0, w - 1)] < c) code |= (uint64_t)1 << bit;
                    bit++;
                }
            }
            out[(size_t)y * w + x] = code;
        }
    }
    return SGM_OK;
}

/* Direction table: L(p) depends on L(p - r). Index order is the engine's volume order
 * (DESIGN.md): 0 r=(0,1) 1 r=(0,-1) 2 r=(1,1) 3 r=(-1,1) 4 r=(1,-1) 5 r=(-1,-1)
 * 6 r=(1,0) 7 r=(-1,0). */
static const int kDirRX[8] = {0, 0, 1, -1, 1, -1, 1, -1};
static const int kDirRY[8] = {1, -1, 1, 1, -1, -1, 0, 0};

static inline int census_cost(uint64_t a, uint64_t b) { return __builtin_popcountll(a ^ b); }

/* One path recurrence step for one pixel: Lc[d] from previous state Lp (NULL = start). */
static inline void census_step(const eff_t* e, const uint64_t* cLrow, const uint64_t* cRrow, int x,
                               const uint8_t* Lp, int minLp, uint8_t* Lc, int* minOut)
{
    const int D = e->D, P1 = e->P1, P2 = e->P2;
    uint64_t cl = cLrow[x];
    int mn = 1 << 30;
    for (int d = 0; d < D; d++) {
        int c = census_cost(cl, cRrow[x - e->minD - d]);
        int L;
        if (!Lp) {
            L = c;
        } else {
            int best = Lp[d];
            if (d > 0) best = imin(best, Lp[d - 1] + P1);
            if (d < D - 1) best = imin(best, Lp[d + 1] + P1);
            best = imin(best, minLp + P2);
            L = c + best - minLp;
        }
        Lc[d] = (uint8_t)L;   /* L <= 62 + P2 <= 255 by construction */
        mn = imin(mn, L);
    }
    *minOut = mn;
}

/* Path volume of one direction, layout [H][width1][D] u8. Lines with ry != 0 are swept
 * row by row (all columns of a row in parallel); ry == 0 lines are rows. */
static int census_path(const eff_t* e, const uint64_t* cL, const uint64_t* cR, int w, int h, int dir,
                       uint8_t* vol /* may be NULL */, uint16_t* S /* may be NULL: += */)
{
    const int D = e->D, width1 = e->width1, rx = kDirRX[dir], ry = kDirRY[dir];
    if (width1 <= 0) return SGM_OK;
    const size_t rowCells = (size_t)width1 * D;
    if (ry == 0) {
#pragma omp parallel
        {
            uint8_t* buf = (uint8_t*)malloc((size_t)2 * D);
#pragma omp for schedule(dynamic, 4)
            for (int y = 0; y < h; y++) {
                uint8_t* Lp = NULL;
                int minLp = 0;
                int xs = rx > 0 ? 0 : width1 - 1;
                for (int i = 0, x1 = xs; i < width1; i++, x1 += rx) {
                    uint8_t* Lc = buf + (i & 1) * D;
                    int mn;
                    census_step(e, cL + (size_t)y * w, cR + (size_t)y * w, x1 + e->minX1, Lp, minLp, Lc, &mn);
                    size_t off = (size_t)y * rowCells + (size_t)x1 * D;
                    if (vol) memcpy(vol + off, Lc, D);
                    if (S) for (int d = 0; d < D; d++) S[off + d] = (uint16_t)(S[off + d] + Lc[d]);
                    Lp = Lc; minLp = mn;
                }
            }
            free(buf);
        }
        return SGM_OK;
    }
    uint8_t* prev = (uint8_t*)malloc(rowCells);
    uint8_t* cur = (uint8_t*)malloc(rowCells);
    int* minPrev = (int*)malloc(sizeof(int) * width1);
    int* minCur = (int*)malloc(sizeof(int) * width1);
    if (!prev || !cur || !minPrev || !minCur) { free(prev); free(cur); free(minPrev); free(minCur); return SGM_ERR_ALLOC; }
    for (int i = 0; i < h; i++) {
        int y = ry > 0 ? i : h - 1 - i;
#pragma omp parallel for schedule(static)
        for (int x1 = 0; x1 < width1; x1++) {
            int xp = x1 - rx;
            const uint8_t* Lp = (i > 0 && xp >= 0 && xp < width1) ? prev + (size_t)xp * D : NULL;
            int mn;
            census_step(e, cL + (size_t)y * w, cR + (size_t)y * w, x1 + e->minX1, Lp, Lp ? minPrev[xp] : 0,
                        cur + (size_t)x1 * D, &mn);
            minCur[x1] = mn;
            size_t off = (size_t)y * rowCells + (size_t)x1 * D;
            if (vol) memcpy(vol + off, cur + (size_t)x1 * D, D);
            if (S) for (int d = 0; d < D; d++) S[off + d] = (uint16_t)(S[off + d] + cur[(size_t)x1 * D + d]);
        }
        uint8_t* t = prev; prev = cur; cur = t;
        int* tm = minPrev; minPrev = minCur; minCur = tm;
    }
    free(prev); free(cur); free(minPrev); free(minCur);
    return SGM_OK;
}

/* Stage helper: one direction's u8 volume [H][width1][D]. */
int sgmref_census_path(const sgm_params* p, const uint8_t* L, const uint8_t* R, int w, int h, size_t stride,
                       int dir, uint8_t* vol)
{
    eff_t e;
    int rc = effective(p, w, h, &e);
    if (rc) return rc;
    if (!e.census || dir < 0 || dir > 7) return SGM_ERR_PARAM;
    uint64_t* cL = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)w * h);
    uint64_t* cR = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)w * h);
    if (!cL || !cR) { free(cL); free(cR); return SGM_ERR_ALLOC; }
    sgmref_census9x7(L, w, h, stride, cL);
    sgmref_census9x7(R, w, h, stride, cR);
    rc = census_path(&e, cL, cR, w, h, dir, vol, NULL);
    free(cL); free(cR);
    return rc;
}

/* Stage helper: S = sum of the 8 path volumes, u16 [H][width1][D]. */
int sgmref_census_sum(const sgm_params* p, const uint8_t* L, const uint8_t* R, int w, int h, size_t stride,
                      uint16_t* S)
{
    eff_t e;
    int rc = effective(p, w, h, &e);
    if (rc) return rc;
    if (!e.census) return SGM_ERR_PARAM;
    if (e.width1 <= 0) return SGM_OK;
    uint64_t* cL = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)w * h);
    uint64_t* cR = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)w * h);
    if (!cL || !cR) { free(cL); free(cR); return SGM_ERR_ALLOC; }
    sgmref_census9x7(L, w, h, stride, cL);
    sgmref_census9x7(R, w, h, stride, cR);
    memset(S, 0, sizeof(uint16_t) * (size_t)e.width1 * e.D * h);
    for (int dir = 0; dir < 8 && !rc; dir++) rc = census_path(&e, cL, cR, w, h, dir, NULL, S);
    free(cL); free(cR);
    return rc;
}

/* ======================================================================================
 * Full pipeline — what StereoSGBMImpl::compute does:
 * disparity -> medianBlur(3) -> filterSpeckles(newVal=(minD-1)*16, window, 16*range).
 * ====================================================================================== */
int sgmref_match(const sgm_params* p, const uint8_t* L, const uint8_t* R, int w, int h, size_t stride,
                 int16_t* disp, size_t out_stride)
{
    eff_t e;
    if (!L || !R || !disp) return SGM_ERR_ARG;
    int rc = effective(p, w, h, &e);
    if (rc) return rc;
    if (stride < (size_t)w || out_stride < (size_t)w) return SGM_ERR_ARG;
    if (!e.census) {
        rc = ocv_match(&e, L, R, w, h, stride, disp, out_stride);
    } else {
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) disp[(size_t)y * out_stride + x] = (int16_t)e.invalid_scaled;
        if (e.width1 > 0) {
            uint16_t* S = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)e.width1 * e.D * h);
            if (!S) return SGM_ERR_ALLOC;
            rc = sgmref_census_sum(p, L, R, w, h, stride, S);
            if (!rc) rc = sgmref_wta(p, w, h, S, disp, out_stride);
            free(S);
        }
    }
    if (rc) return rc;
    if (e.median) rc = sgmref_median3(disp, w, h, out_stride);
    if (!rc && p->speckle_window_size > 0)
        rc = sgmref_filter_speckles(disp, w, h, out_stride, e.invalid_scaled, p->speckle_window_size,
                                    DISP_SCALE * p->speckle_range);
    return rc;
}

int sgmref_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void sgmref_set_num_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
