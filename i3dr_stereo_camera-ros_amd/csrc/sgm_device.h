// sgm_device.h — shared types and wave-level primitives of the HIP SGM engine (gfx950).
//
// Wave = 64 lanes. A wave owns all D disparities of a pixel: lane l holds
// d = l*DPL .. l*DPL + DPL-1 (DPL = disparities per lane, D <= 64*DPL). Cross-lane
// traffic uses DPP (wave_shr/shl:1 for the d-1 / d+1 neighbours, quad_perm + row_ror
// + 4 readlanes for the min over D), never LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sgm_hip.h"

#include <type_traits>

namespace sgm {

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Readable codes kept before and after every census code image in the workspace: the row
// sweeps' segment loads run unclamped past the row ends (census_sgm.hip seg_load_u).
constexpr int kCodeMargin = 1024;
constexpr int kInf = 0x3FFF;  // > any u8 path cost and any census S (<= 8*255)

// Geometry + effective parameters of one match (computed on the host, passed by value).
struct Geom {
    int W, H;               // image size
    int minD, D;            // disparity search [minD, minD + D)
    int minX1, maxX1;       // processed columns [max(maxD,0), W + min(minD,0))
    int width1;             // maxX1 - minX1
    int P1, P2;             // smoothness penalties (effective)
    int uniq;               // uniqueness ratio (percent)
    int disp12;             // LR tolerance (>= 1)
    int subpix, lr;         // census: subpixel / LR-check flags (OCV: 1, 1)
    int invalid;            // (minD - 1) * 16
    int SW2, SH2, ftzero;   // OCV: SAD half window, prefilter cap
    int wide;               // OCV overflow regime: 0 the plain int16 kernels; 1 the "flagged"
                            // kernels (scalar branch: int32 path volumes, exact S; SIMD_SAT: the
                            // sequential saturating cost + saturating int16 paths and sums);
                            // 2 gated: the cost kernel sets *ovf when a frame needs the flagged
                            // kernels, and both kinds are launched, each running only on its case
    int* ovf;               // device flag of wide == 2 (null otherwise)
    int compat;             // OCV: SGM_OCV_* bits (sgm_params.ocv_compat); census: 0
    int ovf_thr;            // OCV: largest C' the plain kernels reproduce exactly (32767, or
                            // 32767 - P2 under SIMD_SAT: (short)(minLr + P2) must not wrap)
    int evol;               // OCV: the plain kernels' path volumes hold deficit planes (C' - L in
                            // 9 bits: ocv_evol_ok) instead of int16 L
};

// OCV workspace: the four u8 prefilter planes, then (256-B aligned) the four u32 planes of
// packed Birchfield-Tomasi intervals that the fused cost stages per row.
__host__ __device__ inline size_t ocv_planes_bytes(int W, int H) { return ((size_t)W * H * 4 + 255) / 256 * 256; }
__host__ __device__ inline size_t ocv_planes_total(int W, int H) { return ocv_planes_bytes(W, H) + (size_t)W * H * 16; }

// Elements of one OCV path volume of `cells` cells at es bytes per cell (256-B aligned
// slices; the host layout and the kernels' launchers agree on it).
__host__ __device__ inline size_t ocv_vol_elems(size_t cells, size_t es) { return (cells * es + 255) / 256 * 256 / es; }
#ifndef SGM_LRPRIO_SCALE
#define SGM_LRPRIO_SCALE 8
#endif
// Wave priority from the work a block still has (rem: remaining steps in row-sweep step
// units, uniform; span: the longest chain of the launch): level = SCALE * rem / span, capped
// at 3. A paths launch of one frame has
// fewer blocks than resident slots, so every block starts at once and each CU's set is fixed;
// the arbiter favours the oldest waves, which starved the youngest long diagonal blocks (a
// C2 trace: diagonal steps took 0.72 us against 0.41 for the oldest vertical blocks, and
// the launch ended on them). Longest-remaining-first lets the long chains issue first and
// the short blocks fill the gaps: single frame C2 1.15 -> 1.05 ms, C3 1.86 -> 1.70 ms. The
// batch's fused launches have more blocks than slots (the dispatcher balances) and measured
// 0-3 % slower with it, so they keep the default priority.
__device__ __forceinline__ void lr_prio(int rem, int span)
{
    const int lvl = min(3, SGM_LRPRIO_SCALE * rem / (span + 1));
    if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
    else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
    else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// Gate of the wide == 2 launches: true when this launch's kind (FLAGGED: the overflow-regime
// kernels) is not the one the frame needs (uniform: a kernel argument and one scalar load).
template <bool FLAGGED>
__device__ __forceinline__ bool ocv_gate_skip(const Geom& g)
{
    return g.wide == 2 && ((*g.ovf != 0) != FLAGGED);
}
// The frame takes the flagged kernels (wide == 1 always, wide == 2 when the cost kernel said so)
__device__ __forceinline__ bool ocv_flagged(const Geom& g)
{
    return g.wide == 1 || (g.wide == 2 && *g.ovf != 0);
}

// Direction r = (rx, ry): L_r(p) depends on L_r(p - r). Engine volume order.
__host__ __device__ constexpr int dir_rx(int i) { return i == 2 || i == 4 || i == 6 ? 1 : (i == 3 || i == 5 || i == 7 ? -1 : 0); }
__host__ __device__ constexpr int dir_ry(int i) { return i == 0 || i == 2 || i == 3 ? 1 : (i == 1 || i == 4 || i == 5 ? -1 : 0); }

// lane i <- lane i-1 (lane 0 <- old)
__device__ __forceinline__ int dpp_shr1(int v, int old) {
    return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false);
}
// lane i <- lane i+1 (lane 63 <- old)
__device__ __forceinline__ int dpp_shl1(int v, int old) {
    return __builtin_amdgcn_update_dpp(old, v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint64_t dpp_shr1_u64(uint64_t v, uint64_t old) {
    int lo = dpp_shr1((int)(uint32_t)v, (int)(uint32_t)old);
    int hi = dpp_shr1((int)(uint32_t)(v >> 32), (int)(uint32_t)(old >> 32));
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t dpp_shl1_u64(uint64_t v, uint64_t old) {
    int lo = dpp_shl1((int)(uint32_t)v, (int)(uint32_t)old);
    int hi = dpp_shl1((int)(uint32_t)(v >> 32), (int)(uint32_t)(old >> 32));
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Min over the 64 lanes, returned wave-uniform (SGPR). EXEC must be full. quad_perm and
// row_ror never read outside the wave, so no identity element is needed.
__device__ __forceinline__ int wave_min(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false));  // row_ror:4
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false));  // row_ror:8
    int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return min(min(a, b), min(c, d));
}

__device__ __forceinline__ int popc64(uint64_t a) { return __builtin_popcountll(a); }

// C-style truncating division for small ints (|num| < 2^24, den > 0): float estimate + fix.
__device__ __forceinline__ int tdiv(int num, int den) {
    int q = (int)__builtin_truncf((float)num / (float)den);
    int r = num - q * den;
    if (num >= 0) { if (r >= den) q++; else if (r < 0) q--; }
    else          { if (r <= -den) q--; else if (r > 0) q++; }
    return q;
}

template <int DPL>
__device__ __forceinline__ int pick(const int (&S)[DPL], int k) {
    int r = S[0];
#pragma unroll
    for (int i = 1; i < DPL; i++) r = (k == i) ? S[i] : r;
    return r;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Winner-take-all of U pixels at once (OpenCV computeDisparitySGBM semantics, SURVEY
// Appendix A.6), branch-free so the U independent reduction chains interleave:
//   best  = first d with the minimal S;
//   reject if some d with |d - best| > 1 has S[d]*(100-uniq) < minS*100;
//   subpixel d16 = 16*best + ((S[best-1]-S[best+1])*16 + den) / (2*den), C truncation,
//   den = max(S[best-1] + S[best+1] - 2*S[best], 1), only for 0 < best < D-1.
// S[u][k] holds d = lane*DPL + k; entries with d >= D must be larger than any real S.
// Results for pixel u (columns xs[u], u < nvalid) go to LDS from lane 0:
//   drow[x] = d16 + 16*minD (left untouched when rejected), bst[x] = best (-1 if rejected),
//   mins[x] = minS. disp2 is derived later from (bst, mins) by row_finish().
template <int DPL, int U>
__device__ __forceinline__ void wta_batch(const int (&S)[U][DPL], int lane, const int (&xs)[U], int nvalid,
                                          const Geom& g, int16_t* drow, int16_t* bst, uint16_t* mins)
{
    int lmin[U], lk[U], minS[U], best[U], d16[U];
    bool rej[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        lmin[u] = S[u][0]; lk[u] = 0;
#pragma unroll
        for (int k = 1; k < DPL; k++) {
            const bool lt = S[u][k] < lmin[u];
            lmin[u] = lt ? S[u][k] : lmin[u];
            lk[u] = lt ? k : lk[u];
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) minS[u] = wave_min(lmin[u]);
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int bl = __builtin_ctzll(__ballot(lmin[u] == minS[u]));
        best[u] = bl * DPL + __builtin_amdgcn_readlane(lk[u], bl);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        bool r = false;
#pragma unroll
        for (int k = 0; k < DPL; k++) {
            const int d = lane * DPL + k;
            r |= (d < g.D) && (S[u][k] * (100 - g.uniq) < minS[u] * 100) && (abs(d - best[u]) > 1);
        }
        rej[u] = __ballot(r) != 0ull;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        // S[best-1], S[best+1]: masked per-lane contribution + readlane (no dynamic
        // register indexing, which hipcc would lower to scratch)
        const int bm = max(best[u] - 1, 0), bp = min(best[u] + 1, g.D - 1);
        int vm = 0, vp = 0;
#pragma unroll
        for (int k = 0; k < DPL; k++) {
            const int d = lane * DPL + k;
            vm += d == bm ? S[u][k] : 0;
            vp += d == bp ? S[u][k] : 0;
        }
        const int sm = __builtin_amdgcn_readlane(vm, bm / DPL);
        const int sp = __builtin_amdgcn_readlane(vp, bp / DPL);
        const int den = max(sm + sp - 2 * minS[u], 1);
        const bool use = g.subpix && best[u] > 0 && best[u] < g.D - 1;
        d16[u] = best[u] * 16 + (use ? tdiv((sm - sp) * 16 + den, 2 * den) : 0);
    }
    // lane u stores pixel u; every other lane (and pixels u >= nvalid) hits its own dummy
    // slot at index W + lane, so the LDS stores need no exec-masked branch. (Dummy slots are
    // shared by the waves of a workgroup: their content is never read.)
    int x = g.W + lane, b = -1, m = 32767, dv = 0, keep = 1;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const bool me = lane == u && u < nvalid;
        x = me ? xs[u] : x;
        b = me ? (rej[u] ? -1 : best[u]) : b;
        m = me ? minS[u] : m;
        dv = me ? d16[u] + g.minD * 16 : dv;
        keep = me ? (rej[u] ? 1 : 0) : keep;
    }
    bst[x] = (int16_t)b;
    mins[x] = (uint16_t)m;
    drow[keep ? g.W + lane : x] = (int16_t)dv;   // rejected pixels keep the invalid value
}

// Row epilogue, after every pixel of the row went through wta_batch:
//  1. disp2 (right-view disparity, OpenCV's x-descending "strictly better" rule): for each
//     target column x2 the pixel with the smallest minS wins, ties -> the largest x. This
//     is an LDS atomicMin over key = minS << 16 | (0xFFFF - x). disp2 starts at the SCALED
//     invalid value (OpenCV quirk: it can look valid when minD > 0), and minS = 32767
//     never updates (disp2cost starts at MAX_COST).
//  2. LR check: invalid iff both rounded candidates are in range, have disp2 >= minD and
//     differ by more than disp12.
//  3. store of the full row (columns outside [minX1, maxX1) stay invalid).
// `key` needs W uint32; `d2` may alias `mins` (mins is dead after step 1). OutT = float: the
// row goes out as the node's CV_32FC1 (every int16 is exact in float).
template <typename OutT>
__device__ __forceinline__ void row_finish(const Geom& g, int tid, int nthr, const int16_t* drow, const int16_t* bst,
                                           const uint16_t* mins, uint32_t* key, int16_t* d2, OutT* orow)
{
    __syncthreads();
    for (int x = g.minX1 + tid; x < g.maxX1; x += nthr) {
        const int b = bst[x];
        const int m = (int16_t)mins[x];     // minS is a CostType: negative once OCV costs wrap
        if (b >= 0 && m < 32767) {
            const int x2 = x - b - g.minD;
            atomicMin(&key[x2], ((uint32_t)(m + 32768) << 16) | (uint32_t)(0xFFFF - x));
        }
    }
    __syncthreads();
    for (int x2 = tid; x2 < g.W; x2 += nthr) {
        const uint32_t k = key[x2];
        d2[x2] = (int16_t)(k == 0xFFFFFFFFu ? g.invalid : bst[0xFFFF - (int)(k & 0xFFFF)] + g.minD);
    }
    __syncthreads();
    for (int x = tid; x < g.W; x += nthr) {
        int d1 = drow[x];
        if (g.lr && d1 != g.invalid) {
            const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            const int _x = x - _d, x_ = x - d_;
            if (0 <= _x && _x < g.W && d2[_x] >= g.minD && abs(d2[_x] - _d) > g.disp12 &&
                0 <= x_ && x_ < g.W && d2[x_] >= g.minD && abs(d2[x_] - d_) > g.disp12)
                d1 = g.invalid;
        }
        orow[x] = (OutT)d1;
    }
}

// LDS carve-up of the per-row WTA state: key u32 [W] | drow i16 | bst i16 | mins u16, the
// last three with 64 extra dummy slots (index W + lane) for branch-free stores.
// A group of frames handled by one launch (frame pipelining): per frame its census codes
// and volume set (paths) or volume set and output (WTA). Frames >= n are skipped.
constexpr int kMaxGroup = 4;
struct PathFrames {
    const uint64_t* cL[kMaxGroup];
    const uint64_t* cR[kMaxGroup];
    uint8_t* vols[kMaxGroup];
    int n;
    unsigned skip_dirs;     // work-list directions this launch skips (bit d: direction d)
};
struct WtaFrames {
    const uint8_t* vols[kMaxGroup];
    int16_t* out[kMaxGroup];
    int n;
    // the standalone WTA launch only: when outf[0] is set, the rows go out as float (CV_32FC1)
    // to outf (a host buffer mapped into the device's address space, sgm_host_register) instead
    // of int16 to out, with this row stride in floats
    float* outf[kMaxGroup];
    size_t outf_stride;
    // up+WTA blocks (census_sgm.hip UpWta): the frames' codes and per-pixel result images
    const uint64_t* cL[kMaxGroup];
    const uint64_t* cR[kMaxGroup];
    uint64_t* res[kMaxGroup];
};
// Rectification fused into the census: the census tile reads
// remap(raw, map) instead of a rectified image. map[0..1] = left x/y, map[2..3] = right x/y,
// each W x H of the rectified geometry; the raw images are src_w x src_h.
struct RectifyIn {
    const float* map[4];
    size_t map_stride;
    int src_w, src_h;
    const int16_t* tab;          // INTER_CUBIC weights (rectify.hip cubic_table)
};
// census transforms of the next group, run in the tail of a fused launch. With rect.tab
// set, L/R are raw images (stride = raw stride) and the rectified pixels are also written
// to rectL/rectR (when not null).
struct CensusFrames {
    const uint8_t* L[kMaxGroup];
    const uint8_t* R[kMaxGroup];
    uint64_t* cL[kMaxGroup];
    uint64_t* cR[kMaxGroup];
    uint8_t* rectL[kMaxGroup];
    uint8_t* rectR[kMaxGroup];
    size_t stride, rect_stride;
    int n;
    RectifyIn rect;
};

// One pixel of cv::remap(src, map_x, map_y, INTER_CUBIC, BORDER_CONSTANT 0) for u8 (rectify.hip)
__device__ __forceinline__ int remap_round_sat(float v)
{
    return (v > -2147483648.0f && v < 2147483648.0f) ? (int)__builtin_rintf(v) : (int)0x80000000u;
}
__device__ __forceinline__ uint8_t remap_cubic_px(const uint8_t* __restrict__ src, size_t sstride, int sw, int sh,
                                                  float fx, float fy, const int16_t* __restrict__ tab)
{
    const int X = remap_round_sat(fx * 32.0f), Y = remap_round_sat(fy * 32.0f);
    const int sx = min(max(X >> 5, -32768), 32767) - 1, sy = min(max(Y >> 5, -32768), 32767) - 1;
    const int16_t* w = tab + (size_t)(((Y & 31) * 32 + (X & 31)) * 16);
    int sum = 0;
    if ((unsigned)sx < (unsigned)max(sw - 3, 0) && (unsigned)sy < (unsigned)max(sh - 3, 0)) {
        const uint8_t* s = src + (size_t)sy * sstride + sx;
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++, s += sstride)
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) sum += (int)s[k2] * (int)w[k1 * 4 + k2];
    } else {
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++) {
            const int yy = sy + k1;
            if (yy < 0 || yy >= sh) continue;
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) {
                const int xx = sx + k2;
                if (xx >= 0 && xx < sw) sum += (int)src[(size_t)yy * sstride + xx] * (int)w[k1 * 4 + k2];
            }
        }
    }
    return (uint8_t)min(max((sum + (1 << 14)) >> 15, 0), 255);
}

struct RowLds {
    uint32_t* key; int16_t* drow; int16_t* bst; uint16_t* mins;
    static size_t bytes(int W) { return (size_t)4 * W + (size_t)6 * (W + 64) + 16; }
    __device__ RowLds(void* base, int W) : RowLds(base, (uint32_t*)base + W, W) {}
    // key at key_base, the rest at rest (key may alias scratch the caller uses before
    // row_finish: then init(.., false) and init_key() afterwards)
    __device__ RowLds(void* key_base, void* rest, int W) {
        key = (uint32_t*)key_base;
        drow = (int16_t*)rest;
        bst = drow + W + 64;
        mins = (uint16_t*)(bst + W + 64);
    }
    static size_t rest_bytes(int W) { return (size_t)6 * (W + 64) + 16; }
    __device__ void init(const Geom& g, int tid, int nthr, bool with_key = true) {
        for (int x = tid; x < g.W; x += nthr) {
            if (with_key) key[x] = 0xFFFFFFFFu;
            drow[x] = (int16_t)g.invalid; bst[x] = -1; mins[x] = 32767;
        }
        __syncthreads();
    }
    __device__ void init_key(const Geom& g, int tid, int nthr) {
        __syncthreads();
        for (int x = tid; x < g.W; x += nthr) key[x] = 0xFFFFFFFFu;
    }
};

// ---- packed u16x2 arithmetic (v_pk_*_u16): two path costs per 32-bit register ----------
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2_t as_v2(uint32_t v) { return __builtin_bit_cast(u16x2_t, v); }
__device__ __forceinline__ uint32_t as_u(u16x2_t v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_min(as_v2(a), as_v2(b))); }
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return as_u(as_v2(a) + as_v2(b)); }
__device__ __forceinline__ uint32_t pk_adds(uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_add_sat(as_v2(a), as_v2(b))); }
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) { return as_u(as_v2(a) - as_v2(b)); }
// (hi:lo) >> 16 — e.g. alignbit16(x, y) = (x.lo, y.hi) as (hi, lo) halves
__device__ __forceinline__ uint32_t alignbit16(uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbit(hi, lo, 16); }

// DPP inside 16-lane rows (lanes outside the row read `old`)
__device__ __forceinline__ uint32_t row_shr1(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x111, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t row_shl1(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x101, 0xf, 0xf, false);
}
__device__ __forceinline__ uint64_t row_shr1_u64(uint64_t v, uint64_t old) {
    return ((uint64_t)row_shr1((uint32_t)(v >> 32), (uint32_t)(old >> 32)) << 32) | row_shr1((uint32_t)v, (uint32_t)old);
}
__device__ __forceinline__ uint64_t row_shl1_u64(uint64_t v, uint64_t old) {
    return ((uint64_t)row_shl1((uint32_t)(v >> 32), (uint32_t)(old >> 32)) << 32) | row_shl1((uint32_t)v, (uint32_t)old);
}
// shift by N lanes inside 16-lane rows (lanes whose source is outside the row read `old`)
template <int N>
__device__ __forceinline__ uint32_t row_shr_n(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x110 + N, 0xf, 0xf, false);
}
template <int N>
__device__ __forceinline__ uint32_t row_shl_n(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x100 + N, 0xf, 0xf, false);
}
// unsigned min over the lanes of one path line, result in every lane of the line:
// LPL = 16: the whole 16-lane row; LPL = 8: the lanes of one parity in the row (two
// interleaved lines per row, lane = 2 * p + line); LPL = 32: a row pair (rows 0-1, 2-3),
// the two row minima joined by v_permlane16_swap
template <int LPL>
__device__ __forceinline__ uint32_t line_min_u32(uint32_t v) {
    if constexpr (LPL >= 16)
        v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, true));       // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, true));      // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, true));      // row_ror:8
    if constexpr (LPL == 32) {
        const auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);         // rows (0,1), (2,3) exchanged
        v = min((uint32_t)sw[0], (uint32_t)sw[1]);
    }
    return v;
}
// neighbour lanes inside 32-lane lines (lane i <- i - 1 / i + 1 across the row boundary of
// the line; the line's first / last lane reads `old`): wave_shr/shl:1 + one select for the
// lane that would read the other line of the wave
__device__ __forceinline__ uint32_t line32_shr1(uint32_t v, uint32_t old) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
    return (threadIdx.x & 31) == 0 ? old : t;
}
__device__ __forceinline__ uint32_t line32_shl1(uint32_t v, uint32_t old) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
    return (threadIdx.x & 31) == 31 ? old : t;
}
__device__ __forceinline__ uint64_t line32_shr1_u64(uint64_t v, uint64_t old) {
    return ((uint64_t)line32_shr1((uint32_t)(v >> 32), (uint32_t)(old >> 32)) << 32) | line32_shr1((uint32_t)v, (uint32_t)old);
}
__device__ __forceinline__ uint64_t line32_shl1_u64(uint64_t v, uint64_t old) {
    return ((uint64_t)line32_shl1((uint32_t)(v >> 32), (uint32_t)(old >> 32)) << 32) | line32_shl1((uint32_t)v, (uint32_t)old);
}
// unsigned min over the 16 lanes of each row, result in every lane of the row
__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true));    // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, true));    // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, true));   // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, true));   // row_ror:8
    return v;
}
// sum over the 16 lanes of each row, result in every lane of the row
__device__ __forceinline__ uint32_t row_sum_u32(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true);    // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, true);    // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, true);   // row_ror:4
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, true);   // row_ror:8
    return v;
}
// C-style truncating num / den (|num| < 2^24, den > 0) from the hardware reciprocal: the
// estimate is within one of the quotient, then fixed like tdiv()
__device__ __forceinline__ int tdiv_rcp(int num, int den)
{
    int q = (int)__builtin_truncf((float)num * __builtin_amdgcn_rcpf((float)den));
    const int r = num - q * den;
    if (num >= 0) q += (r >= den) ? 1 : (r < 0 ? -1 : 0);
    else          q += (r <= -den) ? -1 : (r > 0 ? 1 : 0);
    return q;
}

// broadcast lane J of each 16-lane row (ds_swizzle bit-mask mode: and 0x10, or J)
template <int J>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x10 | (J << 5));
}
template <int J>
__device__ __forceinline__ uint64_t row_bcast_u64(uint64_t v) {
    return ((uint64_t)row_bcast<J>((uint32_t)(v >> 32)) << 32) | row_bcast<J>((uint32_t)v);
}

// Pack DPL u8 path costs of one lane into the per-lane store word.
template <int DPL> struct LaneVec;
template <> struct LaneVec<1> { using T = uint8_t; };
template <> struct LaneVec<2> { using T = uint16_t; };
template <> struct LaneVec<4> { using T = uint32_t; };
template <> struct LaneVec<8> { using T = uint64_t; };

template <int DPL>
__device__ __forceinline__ typename LaneVec<DPL>::T pack_u8(const int (&L)[DPL]) {
    typename LaneVec<DPL>::T v = 0;
#pragma unroll
    for (int k = 0; k < DPL; k++) v |= (typename LaneVec<DPL>::T)(L[k] & 0xFF) << (8 * k);
    return v;
}

}  // namespace sgm
