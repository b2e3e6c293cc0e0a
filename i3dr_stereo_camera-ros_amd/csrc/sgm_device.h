// sgm_device.h — shared types and wave-level primitives of the HIP SGM engine (gfx950).
//
// Wave = 64 lanes. A wave owns all D disparities of a pixel: lane l holds
// d = l*DPL .. l*DPL + DPL-1 (DPL = disparities per lane, D <= 64*DPL). Cross-lane
// traffic uses DPP (wave_shr/shl:1 for the d-1 / d+1 neighbours, quad_perm + row_ror
// + 4 readlanes for the min over D), never LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgm {

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
};

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

// Winner-take-all for the pixel at image column x (x descending over a row), OpenCV
// computeDisparitySGBM semantics: first minimal S, uniqueness
// reject (no disp2 update), disp2 "strictly better" update, parabolic subpixel with C
// truncating division. S[k] for d = lane*DPL + k; lanes/entries with d >= D hold a value
// larger than any real S. Writes drow[x] / d2 / d2c (LDS) from lane 0.
template <int DPL>
__device__ __forceinline__ void wta_pixel(const int (&S)[DPL], int lane, int x, const Geom& g,
                                          int16_t* drow, int16_t* d2, int* d2c)
{
    int lminS = S[0], lk = 0;
#pragma unroll
    for (int k = 1; k < DPL; k++)
        if (S[k] < lminS) { lminS = S[k]; lk = k; }
    const int minS = wave_min(lminS);
    const unsigned long long mm = __ballot(lminS == minS);
    const int bl = __builtin_ctzll(mm);
    const int best = bl * DPL + __builtin_amdgcn_readlane(lk, bl);
    bool rej = false;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
        const int d = lane * DPL + k;
        rej |= (d < g.D) && (S[k] * (100 - g.uniq) < minS * 100) && (abs(d - best) > 1);
    }
    if (__ballot(rej) != 0ull) return;
    int d16 = best * 16;
    if (g.subpix && best > 0 && best < g.D - 1) {
        const int sm = __builtin_amdgcn_readlane(pick<DPL>(S, (best - 1) % DPL), (best - 1) / DPL);
        const int sp = __builtin_amdgcn_readlane(pick<DPL>(S, (best + 1) % DPL), (best + 1) / DPL);
        const int den = max(sm + sp - 2 * minS, 1);
        d16 += tdiv((sm - sp) * 16 + den, 2 * den);
    }
    if (lane == 0) {
        const int x2 = x - best - g.minD;
        if (d2c[x2] > minS) { d2c[x2] = minS; d2[x2] = (int16_t)(best + g.minD); }
        drow[x] = (int16_t)(d16 + g.minD * 16);
    }
}

// Row epilogue: LR check (OpenCV: both rounded candidates inconsistent -> invalid) and
// store of the full row (columns outside [minX1, maxX1) stay invalid).
__device__ __forceinline__ void lr_check_store(const Geom& g, int lane, const int16_t* drow, const int16_t* d2,
                                               int16_t* orow)
{
    for (int x = lane; x < g.W; x += 64) {
        int d1 = drow[x];
        if (g.lr && d1 != g.invalid) {
            const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            const int _x = x - _d, x_ = x - d_;
            if (0 <= _x && _x < g.W && d2[_x] >= g.minD && abs(d2[_x] - _d) > g.disp12 &&
                0 <= x_ && x_ < g.W && d2[x_] >= g.minD && abs(d2[x_] - d_) > g.disp12)
                d1 = g.invalid;
        }
        orow[x] = (int16_t)d1;
    }
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
