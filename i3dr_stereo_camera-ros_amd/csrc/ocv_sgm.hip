// ocv_sgm.hip — OpenCV-StereoSGBM-compatible modes on gfx950 (SGM_MODE_OCV_SGBM5 / _HH8).
//
// Bit-exact with the CPU restatement oracle/sgm_oracle.c `ocv_match` (which follows
// OpenCV's sequential raster loop); here every stage is re-expressed in parallel form:
//   k_ocv_prefilter  Sobel-x prefilter + raw channel, columns 0 / W-1 forced to ftzero
//   k_ocv_pixhsum    Birchfield-Tomasi cost of both channels (raw >> 2) and the horizontal
//                    SAD box (replicate clamp to [0, width1)) in one pass through LDS;
//                    k_ocv_pixcost + k_ocv_hsum unfused when the LDS tile would not fit
//   k_ocv_vsum_seg   vertical box + P2 offset + OpenCV's bottom-row quirk:
//                    rows with y + SH2 >= H are never recomputed (MODE_SGBM keeps the
//                    last computed row, MODE_HH keeps the P2 initialisation)
//   k_ocv_paths      each direction independently (L depends only on its own path), four
//                    lines per wave (16 lanes each);
//                    int16 storage of L and minL as OpenCV's CostType
//   k_ocv_wta16      S = the sum of L in OpenCV's saturating order, 16 lanes per pixel, + the
//                    shared disp2 / LR row code (k_ocv_wta64 for D > 512); k_ocv_wta16_pk the
//                    same in packed u16 pairs where no cost leaves int16.
// Volumes: int16 while no path cost can leave int16; otherwise (Geom::wide, e.g. the shipped
// 2448x2048 D=480 block-21 config) int32 path volumes, gated per frame by the cost kernel's
// overflow flag ("OpenCV semantics targets").
#include "sgm_device.h"
#include <algorithm>
#include <atomic>
#include <cstdlib>

namespace sgm {

constexpr int kMaxCost = 32767;
#ifndef SGM_OCV_PF
#define SGM_OCV_PF 8       // cost rows in flight per path line (D <= 64)
#endif
#ifndef SGM_OCV_PRIO
#define SGM_OCV_PRIO 1     // longest-remaining-first wave priority (lr_prio) in k_ocv_paths: 1 on the packed
                           // lines of <= 4 dwords per lane, 2 on every line, 0 off
#endif
#ifndef SGM_OCV_VWTA_THR
#define SGM_OCV_VWTA_THR 0   // k_ocv_vwta: uniqueness as one threshold per pixel (A/B knob)
#endif
#ifndef SGM_OCV_VWTA_PF
#define SGM_OCV_VWTA_PF 3    // steps whose operands k_ocv_vwta keeps in flight (DPL <= 8)
#endif
#ifndef SGM_OCV_VWTA_RL
#define SGM_OCV_VWTA_RL 0    // k_ocv_vwta: S[best +- 1] by one readlane per element (0: select, then one readlane;
                             // the select is folded into an LDS-indexed load, 86 % bank-conflict cycles, but the
                             // kernel is memory-bound: 3.67 vs 3.66 ms, profiles/r04_ocv_vwta_rl_ab.jsonl)
#endif
#ifndef SGM_OCV_PF_WIDE32
#define SGM_OCV_PF_WIDE32 4  // 32-lane lines with more than 4 values per lane (D > 256: the shipped
                             // 2448x2048 D=480 config, 1 / 2 / 3 / 4 rows: MODE_SGBM 15.01 / 14.86 /
                             // 14.80 / 14.79 ms per frame, MODE_HH 22.3 / 21.9 / 21.55 / 21.5)
#endif
#ifndef SGM_OCV_PF_WIDE
#define SGM_OCV_PF_WIDE 2  // the same for more disparities per lane (1080p D=128 MODE_SGBM paths:
                           // 1 step 1.42 ms, 2 steps 0.95, 3 steps 1.57, 4 steps 1.25)
#endif

// bt (optional, the fused cost's input): the Birchfield-Tomasi intervals of both channels at x,
// packed u | lo << 8 | hi << 16, from the prefiltered / raw values at x - 1, x, x + 1 computed in
// the thread (what bt_lohi reads from the planes)
// Four adjacent pixels per thread (round 5; was one, with ~15 byte loads each): the 8 source bytes
// x0 - 2 .. x0 + 5 of the three rows feed the six prefiltered values x0 - 1 .. x0 + 4 (the BT
// intervals need both neighbours), and the four pixels of each plane go out as one dword / dwordx4
// store where the address is aligned (else byte / dword stores).
__global__ __launch_bounds__(256) void k_ocv_prefilter(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                       size_t stride, int W, int H, int ftzero,
                                                       uint8_t* __restrict__ planes /* 4 x W x H */,
                                                       uint32_t* __restrict__ bt /* 4 x W x H, or null */)
{
    const int x0 = 4 * (blockIdx.x * 256 + threadIdx.x), y = blockIdx.y;
    if (x0 >= W) return;
    const int img = blockIdx.z;
    const uint8_t* src = img ? R : L;
    uint8_t* pf = planes + (size_t)(2 * img) * W * H;
    uint8_t* raw = planes + (size_t)(2 * img + 1) * W * H;
    const size_t o = (size_t)y * W + x0;
    const uint8_t* r = src + (size_t)y * stride;
    const uint8_t* n = y > 0 ? r - stride : r;
    const uint8_t* s = y < H - 1 ? r + stride : r;
    // source bytes x0 - 2 + i (clamped reads: the columns they reach outside [1, W - 2] are forced
    // to ftzero below)
    int cr[8], cn[8], cs[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int xx = min(max(x0 - 2 + i, 0), W - 1);
        cr[i] = r[xx]; cn[i] = n[xx]; cs[i] = s[xx];
    }
    int p[6], q[6];                                      // columns x0 - 1 + j; 0 and W - 1 are ftzero
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int xx = x0 - 1 + j;
        const int v = (cr[j + 2] - cr[j]) * 2 + cn[j + 2] - cn[j] + cs[j + 2] - cs[j];
        const bool edge = xx <= 0 || xx >= W - 1;
        p[j] = edge ? ftzero : min(max(v, -ftzero), ftzero) + ftzero;
        q[j] = edge ? ftzero : cr[j + 1];
    }
    const bool full = x0 + 3 < W && (((uintptr_t)(pf + o) | (uintptr_t)(raw + o)) & 3) == 0;
    if (full) {
        *(uint32_t*)(pf + o) = (uint32_t)p[1] | (uint32_t)p[2] << 8 | (uint32_t)p[3] << 16 | (uint32_t)p[4] << 24;
        *(uint32_t*)(raw + o) = (uint32_t)q[1] | (uint32_t)q[2] << 8 | (uint32_t)q[3] << 16 | (uint32_t)q[4] << 24;
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (x0 + k < W) { pf[o + k] = (uint8_t)p[k + 1]; raw[o + k] = (uint8_t)q[k + 1]; }
    }
    if (!bt) return;
    // bt_lohi of pixel k with neighbours k - 1 and k + 1 (the frame's first / last column takes
    // itself as the missing neighbour)
    auto pack = [&](const int (&a)[6], int k) {
        const int u = a[k + 1];
        const int l = x0 + k > 0 ? a[k] : u, rr = x0 + k < W - 1 ? a[k + 2] : u;
        const int ul = (u + l) / 2, ur = (u + rr) / 2;
        return (uint32_t)u | (uint32_t)min(min(ul, ur), u) << 8 | (uint32_t)max(max(ul, ur), u) << 16;
    };
    const size_t plane = (size_t)W * H;
    uint32_t* bp = bt + (size_t)(2 * img) * plane + o;
    uint32_t* bq = bt + (size_t)(2 * img + 1) * plane + o;
    if (x0 + 3 < W && (((uintptr_t)bp | (uintptr_t)bq) & 15) == 0) {
        *(uint4*)bp = make_uint4(pack(p, 0), pack(p, 1), pack(p, 2), pack(p, 3));
        *(uint4*)bq = make_uint4(pack(q, 0), pack(q, 1), pack(q, 2), pack(q, 3));
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (x0 + k < W) { bp[k] = pack(p, k); bq[k] = pack(q, k); }
    }
}

__device__ __forceinline__ void bt_lohi(const uint8_t* a, int x, int W, int& u, int& lo, int& hi)
{
    u = a[x];
    const int ul = x > 0 ? (u + a[x - 1]) / 2 : u;
    const int ur = x < W - 1 ? (u + a[x + 1]) / 2 : u;
    lo = min(min(ul, ur), u);
    hi = max(max(ul, ur), u);
}

__device__ __forceinline__ int sat16(int v) { return min(max(v, -32768), 32767); }

__device__ __forceinline__ void pixcost_cell(const uint8_t* __restrict__ planes, const Geom& g, int x1, int y,
                                             int16_t* __restrict__ cost)
{
    const int x = x1 + g.minX1;
    const size_t plane = (size_t)g.W * g.H;
    int c_u[2], c_lo[2], c_hi[2];
#pragma unroll
    for (int c = 0; c < 2; c++) bt_lohi(planes + c * plane + (size_t)y * g.W, x, g.W, c_u[c], c_lo[c], c_hi[c]);
    int16_t* out = cost + ((size_t)y * g.width1 + x1) * g.D;
    for (int d = threadIdx.x; d < g.D; d += 256) {
        const int xr = x - g.minD - d;
        int acc = 0;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            int v, v0, v1;
            bt_lohi(planes + (2 + c) * plane + (size_t)y * g.W, xr, g.W, v, v0, v1);
            const int c0 = max(0, max(c_u[c] - v1, v0 - c_u[c]));
            const int c1 = max(0, max(v - c_hi[c], c_lo[c] - v));
            acc += min(c0, c1) >> (c == 0 ? 0 : 2);
        }
        out[d] = (int16_t)acc;
    }
}

// grid (width1, H), block 256 over d
__global__ __launch_bounds__(256) void k_ocv_pixcost(const uint8_t* __restrict__ planes, Geom g,
                                                     int16_t* __restrict__ cost)
{
    pixcost_cell(planes, g, blockIdx.x, blockIdx.y, cost);
}

// thread per (y, d): running horizontal box along x
__global__ __launch_bounds__(256) void k_ocv_hsum(const int16_t* __restrict__ pix, Geom g, int16_t* __restrict__ hs)
{
    const int d = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (d >= g.D) return;
    const size_t rb = (size_t)y * g.width1 * g.D + d;
    const int W1 = g.width1, SW2 = g.SW2;
    int s = pix[rb] * (SW2 + 1);
    for (int i = 1; i <= SW2; i++) s += pix[rb + (size_t)min(i, W1 - 1) * g.D];
    hs[rb] = (int16_t)s;
    for (int x = 1; x < W1; x++) {
        s += pix[rb + (size_t)min(x + SW2, W1 - 1) * g.D] - pix[rb + (size_t)max(x - SW2 - 1, 0) * g.D];
        hs[rb + (size_t)x * g.D] = (int16_t)s;
    }
}

// Pixel cost + horizontal SAD box fused: one block per XB output pixels x DC disparities of
// a row (blockIdx.z: the disparity chunk). Chunking the disparities lets a block take many
// output columns (few halo columns recomputed) at any D: with all D in one block it could
// take only 32 columns, and a 21-wide box recomputed 52 columns per 32 outputs (the shipped
// 2448x2048 D=480 block-21 config: 5.38 -> 3.38 ms).
// Every value is handled as a packed pair of ADJACENT DISPARITIES (d, d+1) in one u32, the
// layout of the output volume, so the box and its stores take one op per two cells:
//   stage:  the Birchfield-Tomasi intervals (u, lo, hi) of both channels of the NX = XB + 2*SW2
//           left columns, each duplicated into both halves of a u32, 6 words per column; the
//           right entries the cells reach (r = 0 .. NX + DC - 2), indexed j = M - 1 - r, as pair
//           words W[j] = (entry j, entry j + 1) per plane: the right entries of (d, d+1) at one
//           column are W[j] of d (low = d, high = d + 1). Records of 6 words (+ 1 pad) per j,
//           even and odd j apart: the lanes of a wave read j, j + 2, ... at a stride of 7 words
//           (conflict-free), the planes at immediate offsets;
//   cost:   P[k][dp] = the cells (k, 2dp) and (k, 2dp + 1): 12 u32 reads at immediate offsets
//           from two running addresses, packed u16 saturating subtracts (max(a - b, 0) in one
//           op): 16 packed ops for two cells;
//   edges:  staged columns outside [0, width1) take the edge column's P (the running sum's
//           replicate rule), in a short pass that only edge blocks run;
//   box:    thread (segment, dp) slides its window over the segment's outputs: two u32 LDS
//           reads, one packed subtract and add, one u32 store per two cells (u16 wrap-around
//           = OpenCV's int16 truncation of the int sum).
#ifndef SGM_PIX_XB
#define SGM_PIX_XB 96
#endif
#ifndef SGM_PIX_DC
#define SGM_PIX_DC 128
#endif
constexpr int kPixXB = SGM_PIX_XB;     // output columns per block (32-128 measured: 96 best at the shipped config)
constexpr int kPixDC = SGM_PIX_DC;     // disparities per block
__host__ __device__ inline int pix_xb(const Geom& g) { return g.D >= kPixDC ? kPixXB : kPixXB * 2; }
__host__ __device__ inline int pix_dc(const Geom& g) { return g.D < kPixDC ? g.D : kPixDC; }
struct PixGeo {
    int XB, DC, NX, M, PP;      // NX even >= XB + 2*SW2; M: right pair words (j < M);
                                // PP: P's row pitch in u32 (odd below 64 pairs: rows spread over banks)
    __host__ __device__ PixGeo(const Geom& g) {
        XB = pix_xb(g); DC = pix_dc(g);
        NX = (XB + 2 * g.SW2 + 1) & ~1;
        M = ((NX + DC) & ~1) + 2;                   // even, > NX + DC - 1; M / 2 records per parity
        PP = DC / 2 >= 64 ? DC / 2 : DC / 2 + 1;
    }
    __host__ __device__ size_t bytes() const { return (size_t)4 * ((size_t)NX * PP + 6 * NX + 7 * M); }
};
__host__ inline size_t pix_lds_bytes(const Geom& g) { return PixGeo(g).bytes(); }
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
template <bool GATED>      // GATED: only for the flagged frames (the fused cost made C' for the others)
__global__ __launch_bounds__(256) void k_ocv_pixhsum(const uint8_t* __restrict__ planes, Geom g,
                                                     int16_t* __restrict__ hs)
{
    if (GATED && !ocv_flagged(g)) return;
    extern __shared__ uint32_t lds_pix32[];
    const PixGeo pg(g);
    const int XB = pg.XB, DCmax = pg.DC, NX = pg.NX, M = pg.M, PP = pg.PP;
    const int y = blockIdx.y, x0 = blockIdx.x * XB, tid = threadIdx.x;
    const int d0 = blockIdx.z * DCmax, DC = min(DCmax, g.D - d0), DPC = DC / 2;   // D % 16 == 0: DC even
    const int SW2 = g.SW2;
    const size_t plane = (size_t)g.W * g.H;
    uint32_t* P = lds_pix32;                               // [NX][PP] packed (d, d+1)
    uint32_t* Lx = P + (size_t)NX * PP;                    // [NX][6]: (u, lo, hi) of channel 0, then 1
    uint32_t* Rw = Lx + 6 * NX;                            // [j & 1][j >> 1][7] pair words, same plane order
    const int MH = M / 2;
    // staged column k <-> x = minX1 + x0 - SW2 + k (not clamped: out-of-frame columns get
    // clamped BT entries and are replaced by the edge pass); right entry r <-> xr = x(0) - minD - (d0 + DC - 1) + r
    const int xs = g.minX1 + x0 - SW2;
    for (int i = tid; i < 2 * NX; i += 256) {
        const int c = i / NX, k = i - c * NX;
        int u, lo, hi;
        bt_lohi(planes + c * plane + (size_t)y * g.W, min(max(xs + k, 0), g.W - 1), g.W, u, lo, hi);
        uint32_t* o = Lx + 6 * k + 3 * c;
        o[0] = (uint32_t)u * 0x10001u; o[1] = (uint32_t)lo * 0x10001u; o[2] = (uint32_t)hi * 0x10001u;
    }
    const int xr0 = xs - g.minD - (d0 + DC - 1);
    const int NRr = NX + DC - 1;                           // right entries the cells reach
    uint16_t* Rh = (uint16_t*)Rw;
    for (int i = tid; i < 2 * NRr; i += 256) {
        const int c = i / NRr, r = i - c * NRr;
        int v, lo, hi;
        bt_lohi(planes + (2 + c) * plane + (size_t)y * g.W, min(max(xr0 + r, 0), g.W - 1), g.W, v, lo, hi);
        // entry j = M - 1 - r: low half of word j, high half of word j - 1 (j >= 2)
        const int j = M - 1 - r;
        uint16_t* lo16 = Rh + 2 * (7 * ((j & 1) * MH + (j >> 1)) + 3 * c);
        uint16_t* hi16 = Rh + 2 * (7 * (((j - 1) & 1) * MH + ((j - 1) >> 1)) + 3 * c) + 1;
        lo16[0] = (uint16_t)v; lo16[2] = (uint16_t)lo; lo16[4] = (uint16_t)hi;
        hi16[0] = (uint16_t)v; hi16[2] = (uint16_t)lo; hi16[4] = (uint16_t)hi;
    }
    __syncthreads();
    // thread -> disparity pair dp (fixed), columns k = kg, kg + tpd, ...
    // cell (k, d): r = k + DC - 1 - d, j = M - 1 - r = M - DC - k + d; the pair (2dp, 2dp + 1)
    // reads word j of d = 2dp (entries j and j + 1 = the right entries of d and d + 1). tpd is
    // even, so a thread's j keeps its parity (j = k mod 2) and steps tpd / 2 records down.
    const int tpd = (256 / DPC) & ~1, dp = tid % DPC, kg = tid / DPC;
    if (kg < tpd) {
        auto sat = [](u16x2_t a, u16x2_t b) { return __builtin_elementwise_sub_sat(a, b); };
        auto w = [](const uint32_t* p, int o) { return __builtin_bit_cast(u16x2_t, p[o]); };
        const uint32_t* Lk = Lx + 6 * kg;
        const int j0 = M - DC - kg + 2 * dp;
        const uint32_t* Rk = Rw + 7 * ((j0 & 1) * MH + (j0 >> 1));
        uint32_t* Pk = P + (size_t)kg * PP + dp;
        for (int k = kg; k < NX; k += tpd, Lk += 6 * tpd, Rk -= 7 * (tpd / 2), Pk += tpd * PP) {
            u16x2_t m[2];
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const u16x2_t u = w(Lk, 3 * c), ulo = w(Lk, 3 * c + 1), uhi = w(Lk, 3 * c + 2);
                const u16x2_t v = w(Rk, 3 * c), v0 = w(Rk, 3 * c + 1), v1 = w(Rk, 3 * c + 2);
                const u16x2_t c0 = __builtin_elementwise_max(sat(u, v1), sat(v0, u));
                const u16x2_t c1 = __builtin_elementwise_max(sat(v, uhi), sat(ulo, v));
                m[c] = __builtin_elementwise_min(c0, c1);
            }
            *Pk = __builtin_bit_cast(uint32_t, m[0] + (m[1] >> (u16x2_t){2, 2}));
        }
    }
    __syncthreads();
    const int nout = min(XB, g.width1 - x0);
    const int klo = SW2 - x0, khi = g.width1 - 1 - x0 + SW2;   // staged columns inside [0, width1)
    if (klo > 0 || khi < NX - 1) {                              // uniform: an edge block
        const int nlo = max(klo, 0), nhi = max(NX - 1 - khi, 0);
        for (int i = tid; i < (nlo + nhi) * DPC; i += 256) {
            const int e = i / DPC, p = i - e * DPC;
            const int k = e < nlo ? e : khi + 1 + (e - nlo);
            P[(size_t)k * PP + p] = P[(size_t)(e < nlo ? klo : khi) * PP + p];
        }
        __syncthreads();
    }
    // horizontal box: thread (segment, dp) slides its window over the segment's outputs
    int16_t* dst = hs + ((size_t)y * g.width1 + x0) * g.D + d0;
    const int nseg = max(256 / DPC, 1), seglen = (nout + nseg - 1) / nseg, BW = 2 * SW2;
    for (int t = tid; t < nseg * DPC; t += 256) {
        const int seg = t / DPC, p = t - seg * DPC;
        const int xa = seg * seglen, xb = min(xa + seglen, nout);
        if (xa >= xb) continue;
        const uint32_t* Pd = P + p;
        u16x2_t sum = {0, 0};
        for (int u = 0; u <= BW; u++) sum += __builtin_bit_cast(u16x2_t, Pd[(size_t)(xa + u) * PP]);
        uint32_t* o = (uint32_t*)(dst + (size_t)xa * g.D) + p;
        *o = __builtin_bit_cast(uint32_t, sum);
        for (int xo = xa + 1; xo < xb; xo++) {
            sum += __builtin_bit_cast(u16x2_t, Pd[(size_t)(xo + BW) * PP]) - __builtin_bit_cast(u16x2_t, Pd[(size_t)(xo - 1) * PP]);
            o += g.D / 2;
            *o = __builtin_bit_cast(uint32_t, sum);
        }
    }
}

// Vertical box + P2 offset + the bottom-row rule, in segments of kVsumRows rows per thread
// (each segment starts from its own window sum; rows y >= 1 with y + SH2 >= H repeat the
// value of row max(H - SH2 - 1, 0) in MODE_SGBM, or are P2 in MODE_HH). A thread owns two
// adjacent disparities (one u32 of the row: width1 * D is even), int sums per half (the
// overflow flag needs the true value), one u32 load per row and window edge, one u32 store.
// SGM_OCV_COL0_LEGACY (OpenCV 3.x, `for (x = D; ...)`): column 0 keeps its row-0 value for
// y >= 1 (MODE_SGBM's single C row) or the P2 initialisation (MODE_HH's per-row C).
// Overflow flag (Geom::wide == 2): a C' above g.ovf_thr (32767: int16 volumes no longer exact
// for the scalar branch; 32767 - P2 for SIMD_SAT, where (short)(minLr + P2) could wrap), or a
// horizontal sum that left int16 (its u16 word has the sign bit: every true sum is >= 0).
#ifndef SGM_VSUM_ROWS
#define SGM_VSUM_ROWS 64
#endif
constexpr int kVsumRows = SGM_VSUM_ROWS;
__global__ __launch_bounds__(256) void k_ocv_vsum_seg(const int16_t* __restrict__ hs, Geom g, int fullDP,
                                                      int16_t* __restrict__ C)
{
    const int i = blockIdx.x * 256 + threadIdx.x;         // pair index in a row
    const size_t rs = (size_t)g.width1 * g.D / 2;          // u32 per row
    if (i >= (int)rs) return;
    const uint32_t* h32 = (const uint32_t*)hs;
    uint32_t* C32 = (uint32_t*)C;
    const int H = g.H, SH2 = g.SH2;
    const int y0 = blockIdx.y * kVsumRows, y1 = min(H, y0 + kVsumRows);
    auto lo16 = [](uint32_t w) { return (int)(int16_t)(uint16_t)w; };
    auto hi16 = [](uint32_t w) { return (int)w >> 16; };
    uint32_t signs = 0;                                    // OR of every loaded sum word
    auto window = [&](int y, int& s0, int& s1) {
        s0 = 0; s1 = 0;
        for (int k = y - SH2; k <= y + SH2; k++) {
            const uint32_t w = h32[(size_t)min(max(k, 0), H - 1) * rs + i];
            s0 += lo16(w); s1 += hi16(w);
            signs |= w;
        }
    };
    bool ovf = false;                                      // a C' above ovf_thr (Geom::wide == 2)
    const int ylast = max(H - SH2 - 1, 0);                 // last row whose window is recomputed
    const bool tail = y1 - 1 >= 1 && y1 - 1 + SH2 >= H;    // the segment reaches the repeated rows
    int rep0 = g.P2, rep1 = g.P2;
    if (!fullDP && tail) { int t0, t1; window(ylast, t0, t1); rep0 += t0; rep1 += t1; }
    // column 0 under COL0_LEGACY: every row y >= 1 holds z (row 0's value, or P2 in MODE_HH)
    const bool c0 = (g.compat & SGM_OCV_COL0_LEGACY) && i < g.D / 2;
    int z0 = g.P2, z1 = g.P2;
    if (c0 && !fullDP) { int t0, t1; window(0, t0, t1); z0 += t0; z1 += t1; }
    int s0, s1;
    window(y0, s0, s1);
    // rows in chunks of 8: the chunk's 16 entering / leaving rows are loaded together (clamped
    // rows, used only where the window slides), so a thread keeps 16 loads in flight
    constexpr int U = 8;
    for (int yb = y0; yb < y1; yb += U) {
        uint32_t ha[U], hb[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int y = min(yb + u, y1 - 1);
            ha[u] = h32[(size_t)min(y + SH2, H - 1) * rs + i];
            hb[u] = h32[(size_t)max(y - SH2 - 1, 0) * rs + i];
            signs |= ha[u];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int y = yb + u;
            if (y >= y1) break;                            // uniform over the block
            int v0, v1;
            if (y == 0 || y + SH2 < H) {
                if (y > y0) { s0 += lo16(ha[u]) - lo16(hb[u]); s1 += hi16(ha[u]) - hi16(hb[u]); }
                v0 = g.P2 + s0; v1 = g.P2 + s1;
            } else {
                v0 = rep0; v1 = rep1;
            }
            if (c0 && y > 0) { v0 = z0; v1 = z1; }
            ovf |= max(v0, v1) > g.ovf_thr;
            C32[(size_t)y * rs + i] = ((uint32_t)v0 & 0xFFFFu) | ((uint32_t)v1 << 16);
        }
    }
    ovf |= (signs & 0x80008000u) != 0;
    if (g.wide == 2 && g.ovf) {                            // one atomic per wave that saw one
        const uint64_t b = __ballot(ovf);
        if (b && (int)(threadIdx.x & 63) == __builtin_ctzll(b)) atomicOr(g.ovf, 1);
    }
}

// ---- SGM_OCV_SIMD_SAT frames the overflow flag marks: OpenCV's SIMD cost loop, exactly ------
// (gated: each kernel returns at once unless the frame takes the flagged path). The SIMD
// branch saturates the running sums of rows y >= 1 — the horizontal sums of image rows
// k > SH2 ((h - sub) + add) and the vertical update ((Cprev - hsumSub) + hsumAdd) — so a value
// that saturated once changes every later one: sequential sums, one thread per (row, d) or per
// (column, d) pair; rows k <= SH2 and row y = 0 keep the scalar int16 wrap.
// grid-stride over the (x1, y) cells of the frame, block 256 over d
__global__ __launch_bounds__(256) void k_ocv_pixcost_sat(const uint8_t* __restrict__ planes, Geom g,
                                                         int16_t* __restrict__ cost)
{
    if (!ocv_flagged(g)) return;
    const int n = g.width1 * g.H;
    for (int it = blockIdx.x; it < n; it += gridDim.x) {
        const int y = it / g.width1;
        pixcost_cell(planes, g, it - y * g.width1, y, cost);
    }
}

// thread per (image row k, d): the running horizontal box along x
__global__ __launch_bounds__(256) void k_ocv_hsum_sat(const int16_t* __restrict__ pix, Geom g, int16_t* __restrict__ hs)
{
    if (!ocv_flagged(g)) return;
    const int d = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y;
    if (d >= g.D) return;
    const size_t rb = (size_t)k * g.width1 * g.D + d;
    const int W1 = g.width1, SW2 = g.SW2;
    int s = pix[rb] * (SW2 + 1);
    for (int i = 1; i <= SW2; i++) s += pix[rb + (size_t)min(i, W1 - 1) * g.D];
    int h = (int16_t)s;                                   // first column: scalar, int16 store
    hs[rb] = (int16_t)h;
    const bool sat = k > g.SH2;                            // computed for an output row y >= 1
    for (int x = 1; x < W1; x++) {
        const int a = pix[rb + (size_t)min(x + SW2, W1 - 1) * g.D];
        const int b = pix[rb + (size_t)max(x - SW2 - 1, 0) * g.D];
        h = sat ? sat16(sat16(h - b) + a) : (int)(int16_t)(h + a - b);
        hs[rb + (size_t)x * g.D] = (int16_t)h;
    }
}

// thread per (column, d): C' down the rows (OpenCV's row loop with the SIMD vertical update)
__global__ __launch_bounds__(256) void k_ocv_vsum_sat(const int16_t* __restrict__ hs, Geom g, int fullDP,
                                                      int16_t* __restrict__ C)
{
    if (!ocv_flagged(g)) return;
    const size_t rc = (size_t)g.width1 * g.D;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rc) return;
    const int H = g.H, SH2 = g.SH2;
    const bool c0 = (g.compat & SGM_OCV_COL0_LEGACY) && i < (size_t)g.D;
    int c = g.P2;                                          // row 0: P2 + the clamped window (int16 wrap)
    for (int k = -SH2; k <= SH2; k++) c += hs[(size_t)min(max(k, 0), H - 1) * rc + i];
    c = (int16_t)c;
    C[i] = (int16_t)c;
    for (int y = 1; y < H; y++) {
        if (y + SH2 < H) {
            if (!c0) c = sat16(sat16(c - hs[(size_t)max(y - SH2 - 1, 0) * rc + i]) + hs[(size_t)(y + SH2) * rc + i]);
            else if (fullDP) c = g.P2;
        } else if (fullDP) {
            c = g.P2;                                      // MODE_HH: never recomputed, the P2 init
        }                                                  // MODE_SGBM: the last computed row
        C[(size_t)y * rc + i] = (int16_t)c;
    }
}

// ---- the whole cost stage in one pass: pixel cost + vertical box + horizontal box + P2 ------
// (replaces k_ocv_pixhsum + k_ocv_vsum_seg, whose 2 B/cell horizontal-sum volume went to HBM
// and was read back twice: 1.71 GB moved for 0.50 GB of C' at 1080p D=128, PMC r03). The box
// is separable and OpenCV's int16 wrap is arithmetic mod 2^16, so the vertical sums can come
// first: a block owns a tile of XB output columns x DC disparities over a band of rows and walks
// the band's rows (+ SH2 above and below) once. Per row:
//   staging threads (waves 4-7): the BT intervals of the row (k_ocv_prefilter writes them) into LDS in
//       k_ocv_pixhsum's formats (left columns duplicated into both halves of a word, right
//       entries as pair words of adjacent disparities);
//   every thread: the pixel costs of its staged column k and I disparity pairs (packed u16 ops,
//       the left words kept in registers), and its vertical window sums V: V += P - P(row - R),
//       the last R = 2*SH2 + 1 rows of P in registers (the slot is picked by a uniform switch,
//       so every ring slot is a static register); V of the row to LDS;
//   box threads (every wave for R <= 9, else waves 0-3): the horizontal box (2*SW2+1 = R wide:
//       OpenCV's block is square) of the previous row's V: a segment of L output columns per
//       thread and pair, its L + R - 1 window values read from LDS at once (staged columns
//       outside [0, width1) read as the edge column: OpenCV's replicate rule) and slid over in
//       registers, + P2, stored as int16 (u16 wrap = OpenCV's CostType store);
// one barrier per row (staging, V and the box double-buffered). The true sums are exact in u16
// when (2*SW2+1)(2*SH2+1)(2*ftzero+63) <= 65535 (the launcher's condition), so the overflow flag
// of Geom::wide == 2 is max(box) > ovf_thr - P2, as k_ocv_vsum_seg computes it (no horizontal sum
// can leave int16 under that bound). OpenCV's bottom-row rule: the band holding the last computed
// row ylast = max(H - SH2 - 1, 0) also writes the rows below it (its last values in MODE_SGBM, P2
// in MODE_HH); COL0_LEGACY's column is written by k_ocv_col0_legacy afterwards.
// Block ids are dealt XCD-aware: the DC-chunks of one tile (and then the next strip of the band)
// run back to back on one XCD, so the partial lines of their C' rows merge in that L2.
#ifndef SGM_FUSE_NX
#define SGM_FUSE_NX 128          // A/B: staged columns per block (256: 1024-thread blocks, one per CU)
#endif
constexpr int kFuseNX = SGM_FUSE_NX;      // staged columns per block: 4 threads per column
constexpr int kFuseThreads = 4 * kFuseNX;
constexpr int kFuseHalf = kFuseThreads / 2;   // waves 0 .. W/2 - 1: box (R > 9); the rest: staging
__host__ __device__ inline int fuse_xb(const Geom& g) { return kFuseNX - 2 * g.SW2; }
#ifndef SGM_FUSE_RB2
#define SGM_FUSE_RB2 1           // A/B: two rows per barrier for boxes wider than 9 (0: one)
#endif
// rows per barrier: RB rows of pixel costs, boxes and staging between two barriers, the box RB
// rows behind the pixel costs and the staging RB rows ahead, over 2 * RB LDS buffers each
__host__ __device__ constexpr int fuse_rb(int R) { return (R > 9 && SGM_FUSE_RB2 != 0) ? 2 : 1; }
#ifndef SGM_FUSE_RING8
#define SGM_FUSE_RING8 1         // the pixel-cost ring as bytes (half the registers)
#endif
#ifndef SGM_FUSE_RING0_LDS
#define SGM_FUSE_RING0_LDS 1     // boxes wider than 9: ring slot 0 kept in LDS (hipcc had spilled it to scratch)
#endif
// words of LDS that hold ring slot 0 (R > 9): one per ring register of every thread
__host__ __device__ constexpr int fuse_ring0_words(int r, int dpc)
{
    // RQ ring registers per thread: I = dpc / 4 disparity pairs, two per register as bytes (SGM_FUSE_RING8)
    return (SGM_FUSE_RING0_LDS != 0 && r > 9) ? (SGM_FUSE_RING8 != 0 ? dpc / 8 : dpc / 4) * kFuseThreads : 0;
}
struct FuseGeo {
    int DC, M, MH;
    __host__ __device__ FuseGeo(int dpc) {
        DC = 2 * dpc;
        M = ((kFuseNX + DC) & ~1) + 2;
        MH = M / 2;
        // 32 pairs per block: the odd-entry half starts at MH = 101 (not 97), which makes the
        // pixel-cost reads of a 32-lane half hit 32 distinct banks (2-way before: SQ_LDS_BANK_CONFLICT
        // 44 % of the LDS cycles at 1080p block 5, profiles/r04_ocv_cost_pmc_fused_final_1080p.txt)
        if (dpc == 32) MH += ((5 - MH % 8) + 8) % 8;
    }
    __host__ __device__ int stage_words() const { return 6 * kFuseNX + 14 * MH; }
    // + ring slot 0 in LDS for boxes wider than 9 (fuse_ring0_words)
    __host__ __device__ size_t lds_bytes(int dpc, int rb, int r = 0) const {
        return (size_t)4 * 2 * rb * (stage_words() + kFuseNX * dpc) + (size_t)4 * fuse_ring0_words(r, dpc);
    }
};
struct FuseGrid {
    int strips, bands, chunks, band_rows, ncomp, total, per_xcd;
};
constexpr uint32_t kFuseDrop = 0x80000000u;      // a byte offset past every C' row descriptor's range
// TRK: what the overflow flag tracks (ocv_fuse_track): 0 nothing (no gate), 1 the max of C' itself
// (box + P2 below 2^16 whatever the pixels; P2 taken off at the end), 2 the max of C' - P2
template <int R, int DPC, int I, int TRK>
// A/B knobs of k_ocv_cost_fused, defaults as measured (profiles/r04_ocv_cost_ring_ab_v2.jsonl; cost stage,
// 1080p block 5 / the shipped 2448x2048 D=480 block 21): the ring as bytes 0.234 -> 0.231 / 3.17 -> 3.01 ms,
// plus <= 128 VGPRs asked for R > 9 (two blocks per CU at 36 B of spills) -> 2.86 ms; the box reads issued
// before the pixel costs instead of after the V store: 3.73 ms at R = 21 (the window registers live across
// the pixel-cost phase), no gain at R = 5
#ifndef SGM_FUSE_BOX_EARLY
#define SGM_FUSE_BOX_EARLY 0     // the box reads issued before the pixel costs (else after the V store)
#endif
#ifndef SGM_FUSE_NB_WIDE
#define SGM_FUSE_NB_WIDE kFuseHalf   // A/B: box threads for R > 9 (kFuseThreads: every wave)
#endif
#ifndef SGM_FUSE_RKOFF
#define SGM_FUSE_RKOFF 1         // the right-entry LDS base kept opaque (read2 immediates, no add per read)
#endif
#ifndef SGM_FUSE_BUFST
#define SGM_FUSE_BUFST 9         // C' stores through a row descriptor (scalar offsets, no per-store VALU) for
                                 // boxes up to this size (1080p block 5: 0.221 -> 0.217 ms; the shipped
                                 // block 21: 2.00 -> 2.05 ms, so not there; profiles/r05_ocv_pk_cost_ab.jsonl)
#endif
#ifndef SGM_FUSE_DPC16_PART
#define SGM_FUSE_DPC16_PART 1    // 16 pairs per block row (a partial last chunk) for D % 32 == 16, D >= 256
#endif
#ifndef SGM_FUSE_LDS_PIPE
#define SGM_FUSE_LDS_PIPE 1      // a pair's right entries read from LDS one pair ahead: 1 for boxes wider than
#endif                           // 9 (already at 128 VGPRs: shipped block 21 cost 1.856 -> 1.838 ms), 2 always
                                 // (1080p block 5: 128 -> 155 VGPRs, one block per CU, 0.206 -> 0.256 ms;
                                 // profiles/r06_ocv_cost_pipe_ab.jsonl), 0 never
#ifndef SGM_FUSE_WPE
#define SGM_FUSE_WPE -1          // waves per SIMD asked of the compiler (4: <= 128 VGPRs); -1: 4 for R > 9
#endif
__global__ __launch_bounds__(kFuseThreads) __attribute__((amdgpu_waves_per_eu(SGM_FUSE_WPE < 0 ? (R > 9 ? 4 : 1) : SGM_FUSE_WPE)))
void k_ocv_cost_fused(const uint32_t* __restrict__ bt, Geom g, int fullDP,
                                                                 FuseGrid fg, int16_t* __restrict__ C)
{
    // every Geom / FuseGrid field the kernel reads, as scalars: a by-value struct that any
    // lambda captures by reference is otherwise given an address (copied to scratch)
    const int gW = g.W, gH = g.H, gD = g.D, gP2 = g.P2, gw1 = g.width1, gminD = g.minD, gminX1 = g.minX1;
    const int gSW2 = g.SW2, gSH2 = g.SH2, gcompat = g.compat, govf_thr = g.ovf_thr;
    int* const govf = g.ovf;
    const int fg_strips = fg.strips, fg_chunks = fg.chunks, fg_band_rows = fg.band_rows, fg_ncomp = fg.ncomp;
    const int fg_total = fg.total, fg_per_xcd = fg.per_xcd;
    static_assert(DPC / I * kFuseNX == kFuseThreads, "4 threads per staged column");
    static_assert(R <= 21, "ring slots: cases 0..20 below");
    constexpr int TPC = DPC / I;
    extern __shared__ uint32_t lds_fuse[];
    const FuseGeo fz(DPC);
    const int DC = fz.DC, M = fz.M, MH = fz.MH, NX = kFuseNX;
    const int SW2 = gSW2, SH2 = gSH2, XB = NX - 2 * SW2;
    // XCD-aware deal: XCD x = blockIdx.x % 8 runs logical tiles x * per_xcd, x * per_xcd + 1, ...
    const int lid = (blockIdx.x & 7) * fg_per_xcd + (blockIdx.x >> 3);
    if (lid >= fg_total) return;
    const int chunk = lid % fg_chunks, tile = lid / fg_chunks;
    const int strip = tile % fg_strips, band = tile / fg_strips;
    const int x0 = strip * XB, d0 = chunk * DC;
    const int y0 = band * fg_band_rows, y1 = min(fg_ncomp, y0 + fg_band_rows);
    const int nv = (y1 - y0) + 2 * SH2;                      // rows of P the band needs
    const int t = threadIdx.x;
    constexpr int RB = fuse_rb(R), NBUF = 2 * RB;
    uint32_t* S0 = lds_fuse;                                 // staging, NBUF buffers
    uint32_t* V0 = lds_fuse + NBUF * fz.stage_words();       // V rows [NX][DPC], NBUF buffers
    auto Sbuf = [&](int r) { return S0 + (r % NBUF) * fz.stage_words(); };
    const int xs = gminX1 + x0 - SW2;                       // staged column k <-> image x = xs + k
    const int xr0 = xs - gminD - (d0 + DC - 1);             // right entry r <-> xr0 + r
    const size_t plane = (size_t)gW * gH;
    // staging (waves 4-7, beside the box of waves 0-3): entry st of the 2 * NX left entries (one
    // each) and entries st, st + kFuseHalf of the 2 * NRr right ones; the bt words of row v + 2 are
    // loaded while row v + 1's are written to LDS, so a global load's latency spans a whole phase
    const int st = t - kFuseHalf;
    const int NRr = NX + DC - 1;
    const int cl = st >= NX, kl = st - cl * NX;
    const int cr0 = st >= NRr, r0 = st - cr0 * NRr;
    static_assert(2 * kFuseNX <= kFuseHalf, "one staging thread per left entry");
    const bool has1 = st + kFuseHalf < 2 * NRr;
    const int cr1 = st + kFuseHalf >= NRr, r1 = st + kFuseHalf - cr1 * NRr;
    // 32-bit element offsets off the uniform base (4 planes < 2^32 elements: the launcher's
    // condition), one register each instead of a 64-bit pointer
    const uint32_t oL = (uint32_t)(cl * plane) + (uint32_t)min(max(xs + kl, 0), gW - 1);
    const uint32_t oR0 = (uint32_t)((2 + cr0) * plane) + (uint32_t)min(max(xr0 + r0, 0), gW - 1);
    const uint32_t oR1 = (uint32_t)((2 + cr1) * plane) + (uint32_t)min(max(xr0 + r1, 0), gW - 1);
    uint32_t wl = 0, wr0 = 0, wr1 = 0;
    auto stage_load = [&](int v) {
        const uint32_t ro = (uint32_t)(min(max(y0 - SH2 + v, 0), gH - 1) * gW);
        wl = bt[oL + ro];
        wr0 = bt[oR0 + ro];
        wr1 = has1 ? bt[oR1 + ro] : 0u;
    };
    auto put_right = [&](uint16_t* Rh, int c, int r, uint32_t w) {
        const int j = M - 1 - r;
        uint16_t* lo16 = Rh + 2 * (7 * ((j & 1) * MH + (j >> 1)) + 3 * c);
        uint16_t* hi16 = Rh + 2 * (7 * (((j - 1) & 1) * MH + ((j - 1) >> 1)) + 3 * c) + 1;
        const uint16_t v = w & 0xFF, lo = (w >> 8) & 0xFF, hi = (w >> 16) & 0xFF;
        lo16[0] = v; lo16[2] = lo; lo16[4] = hi;
        hi16[0] = v; hi16[2] = lo; hi16[4] = hi;
    };
    auto stage_store = [&](uint32_t* S) {
        uint32_t* o = S + 6 * kl + 3 * cl;
        o[0] = (wl & 0xFFu) * 0x10001u; o[1] = ((wl >> 8) & 0xFFu) * 0x10001u; o[2] = ((wl >> 16) & 0xFFu) * 0x10001u;
        uint16_t* Rh = (uint16_t*)(S + 6 * NX);
        put_right(Rh, cr0, r0, wr0);
        if (has1) put_right(Rh, cr1, r1, wr1);
    };
    // P + ring + V: staged column kc, pairs tq*I .. tq*I + I - 1; the last R rows of P in
    // registers, slot v mod R picked by a uniform switch (static register indices, one copy of
    // the row code)
    const int kc = t / TPC, tq = t % TPC;
    // the thread's first right-entry word of staging buffer 0 (loop-invariant, kept opaque so the
    // per-row reads are one base add + ds_read2 immediates, not one add per read: the folded
    // 6*NX*4-byte constant had pushed every read2 offset out of its 1020-byte range)
    int rk_off = 6 * NX + 7 * (((M - DC - kc + 2 * tq * I) & 1) * MH + ((M - DC - kc + 2 * tq * I) >> 1));
    if constexpr (SGM_FUSE_RKOFF != 0) asm volatile("" : "+v"(rk_off));
    // kRing8: a pixel cost is <= 2*ftzero + 63 <= 255 (the launcher's condition), so the ring
    // keeps bytes, two disparity pairs per register
    constexpr bool kRing8 = SGM_FUSE_RING8 != 0;
    constexpr bool kEarly = SGM_FUSE_BOX_EARLY != 0;
    constexpr int RQ = kRing8 ? I / 2 : I;
    uint32_t ring[RQ][R];
    uint32_t Vs[I];
#pragma unroll
    for (int q = 0; q < I; q++) Vs[q] = 0;
#pragma unroll
    for (int q = 0; q < RQ; q++)
#pragma unroll
        for (int s2 = 0; s2 < R; s2++) ring[q][s2] = 0;
    // ring slot 0 in LDS for wide boxes (each thread its own words: no barrier; read and written
    // once every R rows): at <= 128 VGPRs hipcc spilled that slot to scratch, whose reload put a
    // vmcnt(0) wait (the row's C' stores and BT loads) into every R-th row
    constexpr bool kRing0Lds = fuse_ring0_words(R, DPC) > 0;
    uint32_t* ring0 = lds_fuse + NBUF * fz.stage_words() + NBUF * kFuseNX * DPC + t;
    if constexpr (kRing0Lds) {
#pragma unroll
        for (int q = 0; q < RQ; q++) ring0[q * kFuseThreads] = 0;
    }
    auto sat = [](u16x2_t a, u16x2_t b) { return __builtin_elementwise_sub_sat(a, b); };
    auto wd = [](const uint32_t* p, int o) { return __builtin_bit_cast(u16x2_t, p[o]); };
    // box: thread (segment, pair); NB box threads, L outputs per segment, the NL = L + R - 1
    // window values of a segment read from LDS at once (one wait, not one per output)
    constexpr int NB = R <= 9 ? kFuseThreads : SGM_FUSE_NB_WIDE;   // every wave for small boxes, else waves 0-3
    constexpr int NSEG = NB / DPC;
    constexpr int L = (kFuseNX - (R - 1) + NSEG - 1) / NSEG;
    constexpr int NL = L + R - 1;
    const int nout = min(XB, gw1 - x0);
    const int klo = max(SW2 - x0, 0), khi = min(gw1 - 1 - x0 + SW2, NX - 1);
    const bool edge = klo > 0 || khi < NX - 1;               // uniform: strips at the frame's sides
    const int bp = t % DPC, bseg = t / DPC;
    const int xa = bseg * L, xb = min(xa + L, nout);
    // the last chunk of a frame whose D is not a multiple of DC holds pairs past D: computed
    // (their right entries clamp inside the row) but never stored nor flagged
    const bool pok = d0 + 2 * bp < gD;
    u16x2_t bmax = {0, 0};                                   // flag: the largest box sum seen
    const bool col0 = (gcompat & SGM_OCV_COL0_LEGACY) && x0 == 0;
    const u16x2_t p2v = {(unsigned short)gP2, (unsigned short)gP2};
    uint32_t* C32 = (uint32_t*)C;
    const size_t rowC = (size_t)gw1 * gD / 2;         // u32 per C' row
    const bool last_band = y1 == fg_ncomp;
    int v_cur = 0;                                           // the row of the loop below
    if (t >= kFuseHalf) {
        for (int r = 0; r < RB && r < nv; r++) {
            stage_load(r);
            stage_store(Sbuf(r));
        }
        if (RB < nv) stage_load(RB);
    }
    __syncthreads();
    auto box_load = [&](u16x2_t (&w)[NL]) __attribute__((always_inline)) {
        const uint32_t* Vp = V0 + ((v_cur - RB) % NBUF) * NX * DPC + bp;
        if (edge) {                                          // staged columns outside the frame: the edge column
#pragma unroll
            for (int i = 0; i < NL; i++) w[i] = wd(Vp, min(max(xa + i, klo), khi) * DPC);
        } else {
#pragma unroll
            for (int i = 0; i < NL; i++) {
                // only the last segment's window passes the staged row (L * NSEG >= XB)
                const int k = i > NX - 1 - (NSEG - 1) * L ? min(xa + i, NX - 1) : xa + i;
                w[i] = wd(Vp, k * DPC);
            }
        }
    };
    int slot = 0;
    for (int v = 0; v < nv + RB; v++) {
        v_cur = v;
        uint32_t* S = Sbuf(v);
        // the box of row v - RB (its V written RB iterations ago, a barrier between)
        const bool dobox = t < NB && v >= RB && v - RB >= 2 * SH2 && xa < xb;
        u16x2_t w[NL];
        if constexpr (kEarly)
            if (dobox) box_load(w);
        if (v < nv) {
            const uint32_t* Lk = S + 6 * kc;
            u16x2_t u[2], ulo[2], uhi[2];
#pragma unroll
            for (int c = 0; c < 2; c++) { u[c] = wd(Lk, 3 * c); ulo[c] = wd(Lk, 3 * c + 1); uhi[c] = wd(Lk, 3 * c + 2); }
            const uint32_t* Rk = S + rk_off;
            uint32_t P[I];
            // kPipe (SGM_FUSE_LDS_PIPE): the right entries of pair q + 1 read from LDS before pair
            // q's arithmetic (else hipcc issues each pair's reads just before their use)
            constexpr bool kPipe = SGM_FUSE_LDS_PIPE == 2 || (SGM_FUSE_LDS_PIPE == 1 && R > 9);
            u16x2_t rw[2][6];
            auto rload = [&](int q, u16x2_t (&r)[6]) {
#pragma unroll
                for (int k = 0; k < 6; k++) r[k] = wd(Rk, 7 * q + k);
            };
            if constexpr (kPipe) {
                rload(0, rw[0]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int q = 0; q < I; q++) {
                if constexpr (kPipe) {
                    if (q + 1 < I) rload(q + 1, rw[(q + 1) & 1]);
                    __builtin_amdgcn_sched_barrier(0);
                } else {
                    rload(q, rw[q & 1]);
                }
                const u16x2_t (&r)[6] = rw[q & 1];
                u16x2_t m[2];
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    const u16x2_t vv = r[3 * c], v0 = r[3 * c + 1], v1 = r[3 * c + 2];
                    const u16x2_t c0 = __builtin_elementwise_max(sat(u[c], v1), sat(v0, u[c]));
                    const u16x2_t c1 = __builtin_elementwise_max(sat(vv, uhi[c]), sat(ulo[c], vv));
                    m[c] = __builtin_elementwise_min(c0, c1);
                }
                P[q] = __builtin_bit_cast(uint32_t, m[0] + (m[1] >> (u16x2_t){2, 2}));
                if constexpr (kPipe) __builtin_amdgcn_sched_barrier(0);
            }
            auto upd = [&](auto ss) {
                constexpr int s2 = decltype(ss)::value;
                auto vupd = [&](int q, uint32_t old) {
                    Vs[q] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, Vs[q]) + __builtin_bit_cast(u16x2_t, P[q]) -
                                                         __builtin_bit_cast(u16x2_t, old));
                };
                if constexpr (kRing8) {
#pragma unroll
                    for (int h = 0; h < RQ; h++) {
                        const uint32_t o = (kRing0Lds && s2 == 0) ? ring0[h * kFuseThreads] : ring[h][s2];
                        vupd(2 * h, __builtin_amdgcn_perm(o, o, 0x0C010C00u));       // bytes 0, 1 -> u16 lanes
                        vupd(2 * h + 1, __builtin_amdgcn_perm(o, o, 0x0C030C02u));   // bytes 2, 3
                        const uint32_t nw = __builtin_amdgcn_perm(P[2 * h + 1], P[2 * h], 0x06040200u);
                        if (kRing0Lds && s2 == 0) ring0[h * kFuseThreads] = nw;
                        else ring[h][s2] = nw;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < I; q++) {
                        vupd(q, (kRing0Lds && s2 == 0) ? ring0[q * kFuseThreads] : ring[q][s2]);
                        if (kRing0Lds && s2 == 0) ring0[q * kFuseThreads] = P[q];
                        else ring[q][s2] = P[q];
                    }
                }
            };
            switch (slot) {
#define SGM_RING_CASE(n) case n: if constexpr (n < R) upd(std::integral_constant<int, n>{}); break;
            SGM_RING_CASE(0) SGM_RING_CASE(1) SGM_RING_CASE(2) SGM_RING_CASE(3) SGM_RING_CASE(4) SGM_RING_CASE(5)
            SGM_RING_CASE(6) SGM_RING_CASE(7) SGM_RING_CASE(8) SGM_RING_CASE(9) SGM_RING_CASE(10) SGM_RING_CASE(11)
            SGM_RING_CASE(12) SGM_RING_CASE(13) SGM_RING_CASE(14) SGM_RING_CASE(15) SGM_RING_CASE(16)
            SGM_RING_CASE(17) SGM_RING_CASE(18) SGM_RING_CASE(19) SGM_RING_CASE(20)
#undef SGM_RING_CASE
            default: break;
            }
            slot = slot + 1 == R ? 0 : slot + 1;
            if (v >= 2 * SH2) {
                uint32_t* Vout = V0 + (v % NBUF) * NX * DPC + kc * DPC + tq * I;
                // exactly the thread's I words (I = 2 at DPC = 8: one 8-byte store, 8-byte aligned)
                if constexpr (I % 4 == 0) {
#pragma unroll
                    for (int q = 0; q < I; q += 4) *(uint4*)(Vout + q) = make_uint4(Vs[q], Vs[q + 1], Vs[q + 2], Vs[q + 3]);
                } else {
                    static_assert(I % 2 == 0, "pairs of words per thread");
#pragma unroll
                    for (int q = 0; q < I; q += 2) *(uint2*)(Vout + q) = make_uint2(Vs[q], Vs[q + 1]);
                }
            }
        }
        if (dobox) {                                         // the box of row v - RB
            const int y = y0 + (v - RB) - 2 * SH2;
            const bool tail = last_band && y == fg_ncomp - 1;
            if constexpr (!kEarly) box_load(w);
            // the window sum starts at P2, so the slid sum IS C' (mod 2^16, OpenCV's CostType wrap)
            u16x2_t sum = w[0] + p2v;
#pragma unroll
            for (int i = 1; i < R; i++) sum += w[i];
            // 32-bit element offsets off the uniform C' base (C' < 2^32 words: the launcher's
            // condition)
            const uint32_t ob = (uint32_t)y * (uint32_t)rowC + (uint32_t)(((x0 + xa) * gD + d0) / 2 + bp);
            // stores through a descriptor of the row (wave-uniform base, SGPRs): the lane's byte
            // offset in one VGPR and output j's step as the scalar offset, no per-store VALU
            const __amdgpu_buffer_rsrc_t crow = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(C32 + (size_t)y * rowC), 0, (int)(rowC * 4), 0x00020000);
            const uint32_t vb = 4u * (uint32_t)(((x0 + xa) * gD + d0) / 2 + bp);
            if constexpr (R <= SGM_FUSE_BUFST) {
                // branch-free: an output past the segment's end goes to an offset past the range,
                // where the hardware drops it, and the flag's max is a select (1080p block 5 cost
                // 0.210 -> 0.204 ms; at R = 21 the same form measured 2.00 against 1.97 for the
                // branches below, and the branches with descriptor stores 2.02: profiles/
                // r05_ocv_cost_box_ab.jsonl, r05_ocv_cost_box2_ab.jsonl)
                const int nj = xb - xa;                      // outputs of the segment (> 0)
                const bool skip0 = col0 && xa == 0 && y > 0; // COL0_LEGACY's column: not in the flag
#pragma unroll
                for (int j = 0; j < L; j++) {
                    if (j > 0) sum += w[j + R - 1] - w[j - 1];
                    const bool ok = j < nj && pok;
                    if constexpr (TRK != 0) {
                        const u16x2_t cand = __builtin_elementwise_max(bmax, TRK == 1 ? sum : sum - p2v);
                        bmax = (ok && !(j == 0 && skip0)) ? cand : bmax;
                    }
                    __builtin_amdgcn_raw_buffer_store_b32(as_u(sum), crow, ok ? (int)vb : (int)kFuseDrop, j * gD * 2, 0);
                }
            } else {
#pragma unroll
                for (int j = 0; j < L; j++) {
                    if (j > 0) sum += w[j + R - 1] - w[j - 1];
                    if (xa + j < xb && pok) {
                        if constexpr (TRK != 0)
                            if (!(col0 && xa + j == 0 && y > 0))
                                bmax = __builtin_elementwise_max(bmax, TRK == 1 ? sum : sum - p2v);
                        C32[ob + (uint32_t)(j * (gD / 2))] = as_u(sum);
                    }
                }
            }
            if (tail) {                                      // OpenCV's bottom rows: never recomputed
                // (the row's values slid again from the registers: reading the stores back would
                // put a vmcnt(0) wait into every row of the loop)
                sum = w[0] + p2v;
#pragma unroll
                for (int i = 1; i < R; i++) sum += w[i];
                uint32_t* o = C32 + ob;
#pragma unroll
                for (int j = 0; j < L; j++) {
                    if (j > 0) sum += w[j + R - 1] - w[j - 1];
                    const uint32_t c = fullDP ? gP2 * 0x10001u : as_u(sum);
                    if (xa + j < xb && pok)
                        for (int yy = y + 1; yy < gH; yy++) o[(size_t)(yy - y) * rowC] = c;
                    o += gD / 2;
                }
            }
        }
        if (t >= kFuseHalf && v + RB < nv) {
            stage_store(Sbuf(v + RB));
            if (v + RB + 1 < nv) stage_load(v + RB + 1);
        }
        // every write of iteration v is read RB iterations later and every buffer is rewritten
        // 2 * RB iterations after its reads: one barrier per RB iterations orders both
        if ((v + 1) % RB == 0) __syncthreads();
    }
    if (TRK != 0 && govf && t < NB) {
        const int m = max((int)bmax[0], (int)bmax[1]) - (TRK == 1 ? gP2 : 0);
        const bool ovf = m > govf_thr - gP2;
        const uint64_t b = __ballot(ovf);
        if (b && (int)(threadIdx.x & 63) == __builtin_ctzll(b)) atomicOr(govf, 1);
    }
}

// COL0_LEGACY after the fused cost: column x1 = 0 of rows y >= 1 holds row 0's value (MODE_SGBM's
// single C row is never updated there) or the P2 initialisation (MODE_HH)
__global__ __launch_bounds__(256) void k_ocv_col0_legacy(Geom g, int fullDP, int16_t* __restrict__ C)
{
    const int np = g.D / 2;                               // u32 pairs of column 0
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (g.H - 1) * np) return;
    const int y = 1 + i / np, pr = i - (y - 1) * np;
    uint32_t* C32 = (uint32_t*)C;
    C32[(size_t)y * g.width1 * np + pr] = fullDP ? ((uint32_t)g.P2 & 0xFFFFu) * 0x10001u : C32[pr];
}

// The fused cost applies: R = 2*SH2 + 1 <= 21 (the register ring; SH2 <= 10 leaves XB >= 108 of
// the 128 staged columns) and every sum exact in u16.
__host__ inline bool ocv_cost_fusable(const Geom& g)
{
    const long long B = (long long)(2 * g.SW2 + 1) * (2 * g.SH2 + 1) * (2 * g.ftzero + 63);
    const char* e = std::getenv("SGM_OCV_FUSED");
    // default: frames with enough tiles x bands to fill the chip (10^8 cells: C1 measured 0.10
    // fused vs 0.053 ms; 1080p block 5 0.29 vs 0.42, the shipped block-21 config 3.18 vs 3.79 ms,
    // profiles/r04_ocv_cost_box_ab.jsonl)
    const bool dflt = (double)g.width1 * g.H * g.D >= 1e8;
    return g.SH2 <= 10 && g.SW2 == g.SH2 && B <= 65535 && 2 * g.ftzero + 63 <= 255 &&
           (double)g.W * g.H * 4 < 4294967296.0 && (double)g.width1 * g.H * g.D / 2 < 4294967296.0 && g.width1 > 0 && (e ? std::atoi(e) != 0 : dflt);
}

// The SIMD_SAT flagged frames whose horizontal sums cannot saturate: when
// (2*SW2 + 1) * (2*ftzero + 63) <= 32767 every running horizontal sum of the SIMD loop stays in
// int16 (it is a box of pixel costs <= 2*ftzero + 63, and (h - sub) + add never leaves
// [-maxP, 32767]), so the plain horizontal sums hs (k_ocv_pixhsum) ARE the SIMD branch's and only
// the vertical update saturates: C_y = sat(sat(C_{y-1} - hs[y-SH2-1]) + hs[y+SH2]). That chain is
// sequential per (column, d), so a thread owns a pair of adjacent disparities (packed saturating
// i16 ops, v_pk_sub_i16 / v_pk_add_i16 with clamp) and walks every row; the grid covers
// width1 * D / 2 pairs (437 K threads at the shipped 2448x2048 D=480 config). Each hs row is read
// from HBM once, as it enters the window, U rows ahead of the chain, and kept in the thread's
// LDS ring (R = 2*SH2 + 1 slots) until it leaves: 2 B read + 2 B written per cell. The old
// k_ocv_pixcost_sat / k_ocv_hsum_sat / k_ocv_vsum_sat chain (one int16 per thread, no prefetch)
// stays for the configs whose horizontal sums can saturate (boxes wider than ~171 columns).
typedef short s16x2_t __attribute__((ext_vector_type(2)));
__host__ __device__ inline bool ocv_hsum_cannot_saturate(const Geom& g)
{
    return (2 * g.SW2 + 1) * (2 * g.ftzero + 63) <= 32767;
}
__host__ inline int vsum_sat2_unroll(const Geom& g)
{
    const int R = 2 * g.SH2 + 1;
    return R >= 8 ? 8 : R >= 4 ? 4 : R >= 2 ? 2 : 1;
}
template <int U>
__global__ __launch_bounds__(256) void k_ocv_vsum_sat2(const int16_t* __restrict__ hs, Geom g, int fullDP,
                                                       int16_t* __restrict__ C)
{
    if (!ocv_flagged(g)) return;
    extern __shared__ uint32_t ring_sat[];                 // [R][256]: slot s of thread t at s * 256 + t
    const int t = threadIdx.x, i = blockIdx.x * 256 + t;
    const size_t rs = (size_t)g.width1 * g.D / 2;           // u32 pairs per row
    if (i >= (int)rs) return;                               // no barriers below: the ring is per thread
    const uint32_t* h32 = (const uint32_t*)hs;
    uint32_t* C32 = (uint32_t*)C;
    const int H = g.H, SH2 = g.SH2, R = 2 * SH2 + 1;
    uint32_t* ring = ring_sat + t;
    auto lo16 = [](uint32_t w) { return (int)(int16_t)(uint16_t)w; };
    auto hi16 = [](uint32_t w) { return (int)w >> 16; };
    auto S = [](uint32_t w) { return __builtin_bit_cast(s16x2_t, w); };
    // row 0: P2 + the clamped window, int sums wrapped to int16 (the scalar y == 0 loop)
    int s0 = 0, s1 = 0;
    for (int k = 0; k <= SH2; k++) {
        const uint32_t w = h32[(size_t)min(k, H - 1) * rs + i];
        if (k < H) ring[k * 256] = w;                       // rows 0 .. SH2 enter the ring (k < R)
        const int m = k == 0 ? SH2 + 1 : 1;                 // row 0 weighs SH2 + 1 (clamped rows above)
        s0 += m * lo16(w); s1 += m * hi16(w);
    }
    uint32_t c = ((uint32_t)(g.P2 + s0) & 0xFFFFu) | ((uint32_t)(g.P2 + s1) << 16);
    C32[i] = c;
    const bool col0 = (g.compat & SGM_OCV_COL0_LEGACY) && i < g.D / 2;
    const uint32_t p2w = ((uint32_t)g.P2 & 0xFFFFu) * 0x10001u;
    const int ylast = H - SH2 - 1;                           // rows y <= ylast add row y + SH2
    // ring slot of row y - SH2 - 1 (= the slot row y + SH2 takes: they are R rows apart), kept
    // as a running counter (no modulo in the loop); rows y <= SH2 subtract row 0 (slot 0) and
    // add row y + SH2 < R into slot y + SH2
    int q0 = (R - SH2) % R;                                  // its value at y = 1
    for (int yb = 1; yb < H; yb += U) {
        uint32_t add[U], sub[U];
        int slot[U];
#pragma unroll
        for (int u = 0; u < U; u++) {                        // entering rows (clamped: used only if y <= ylast)
            const int y = yb + u;
            int q = q0 + u;
            q = q >= R ? q - R : q;                          // U <= R
            slot[u] = y <= SH2 ? y + SH2 : q;
            add[u] = h32[(size_t)min(y + SH2, H - 1) * rs + i];
            sub[u] = ring[(y <= SH2 ? 0 : q) * 256];         // leaving rows: none of this group's (U <= R)
        }
        q0 += U;
        q0 = q0 >= R ? q0 - R : q0;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int y = yb + u;
            if (y >= H) break;
            if (y <= ylast) {
                if (!col0)
                    c = __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(
                            __builtin_elementwise_sub_sat(S(c), S(sub[u])), S(add[u])));
                else if (fullDP)
                    c = p2w;
                ring[slot[u] * 256] = add[u];
            } else if (fullDP) {
                c = p2w;                                     // MODE_HH: never recomputed, the P2 init
            }                                                // MODE_SGBM: the last computed row
            C32[(size_t)y * rs + i] = c;
        }
    }
}

// DPL consecutive int16 as vector accesses (DPL a power of two <= 32; aligned to min(2*DPL, 16) B)
template <int DPL>
__device__ __forceinline__ void load_i16(const int16_t* p, int16_t (&v)[DPL])
{
    if constexpr (DPL == 1) v[0] = *p;
    else if constexpr (DPL == 2) { const uint32_t w = *(const uint32_t*)p; v[0] = (int16_t)w; v[1] = (int16_t)(w >> 16); }
    else {
        constexpr int NW = DPL / 2;
        uint32_t w[NW];
        if constexpr (DPL == 4) { const uint2 t = *(const uint2*)p; w[0] = t.x; w[1] = t.y; }
        else {
#pragma unroll
            for (int c = 0; c < NW / 4; c++) {
                const uint4 t = ((const uint4*)p)[c];
                w[4 * c] = t.x; w[4 * c + 1] = t.y; w[4 * c + 2] = t.z; w[4 * c + 3] = t.w;
            }
        }
#pragma unroll
        for (int i = 0; i < NW; i++) { v[2 * i] = (int16_t)w[i]; v[2 * i + 1] = (int16_t)(w[i] >> 16); }
    }
}
// nontemporal: the path volumes are streamed once into the WTA
template <int DPL>
__device__ __forceinline__ void store_i16(int16_t* p, const int (&v)[DPL])
{
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    if constexpr (DPL == 1) __builtin_nontemporal_store((int16_t)v[0], p);
    else {
        constexpr int NW = DPL / 2;
        uint32_t w[NW];
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = ((uint32_t)v[2 * i] & 0xFFFFu) | ((uint32_t)v[2 * i + 1] << 16);
        if constexpr (DPL == 2) __builtin_nontemporal_store(w[0], (uint32_t*)p);
        else if constexpr (DPL == 4) __builtin_nontemporal_store((v2u){w[0], w[1]}, (v2u*)p);
        else {
#pragma unroll
            for (int c = 0; c < NW / 4; c++)
                __builtin_nontemporal_store((v4u){w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]}, (v4u*)p + c);
        }
    }
}

// The same through a raw buffer descriptor (32-bit byte offsets; an offset past the
// descriptor's range reads 0 / drops the store: the 32-lane path kernel's masking)
template <int DPL>
__device__ __forceinline__ void bload_i16(__amdgpu_buffer_rsrc_t rs, uint32_t off, int (&v)[DPL])
{
    if constexpr (DPL == 1) {
        v[0] = (int)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
        return;
    }
    uint32_t w[DPL / 2 > 0 ? DPL / 2 : 1];
    if constexpr (DPL == 2) w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    else if constexpr (DPL == 4) { const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0); w[0] = t[0]; w[1] = t[1]; }
    else {
#pragma unroll
        for (int c = 0; c < DPL / 8; c++) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * c, 0, 0);
            w[4 * c] = t[0]; w[4 * c + 1] = t[1]; w[4 * c + 2] = t[2]; w[4 * c + 3] = t[3];
        }
    }
#pragma unroll
    for (int i = 0; i < DPL / 2; i++) { v[2 * i] = (int)(int16_t)w[i]; v[2 * i + 1] = (int)w[i] >> 16; }
}
template <int DPL>
__device__ __forceinline__ void bstore_i16(__amdgpu_buffer_rsrc_t rs, uint32_t off, const int (&v)[DPL])
{
    constexpr int aux = 2;                               // nt: streamed once into the WTA
    if constexpr (DPL == 1) {
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v[0], rs, off, 0, aux);
        return;
    }
    uint32_t w[DPL / 2 > 0 ? DPL / 2 : 1];
#pragma unroll
    for (int i = 0; i < DPL / 2; i++) w[i] = ((uint32_t)v[2 * i] & 0xFFFFu) | ((uint32_t)v[2 * i + 1] << 16);
    if constexpr (DPL == 2) __builtin_amdgcn_raw_buffer_store_b32(w[0], rs, off, 0, aux);
    else if constexpr (DPL == 4) {
        typedef unsigned int v2u __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, rs, off, 0, aux);
    } else {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int c = 0; c < DPL / 8; c++)
            __builtin_amdgcn_raw_buffer_store_b128((v4u){w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]}, rs,
                                                   off + 16 * c, 0, aux);
    }
}

// Path volumes hold VT per cell: int16 (CostType, exact whenever no path cost can leave
// int16) or int32 (Geom::wide: the cost volume itself may wrap, and OpenCV adds the int
// path costs, not their CostType copies, into S). N dwords per lane for int32.
template <int N>
__device__ __forceinline__ void store_dw(uint32_t* p, const uint32_t (&w)[N])
{
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    if constexpr (N == 1) __builtin_nontemporal_store(w[0], p);
    else if constexpr (N == 2) __builtin_nontemporal_store((v2u){w[0], w[1]}, (v2u*)p);
    else {
#pragma unroll
        for (int c = 0; c < N / 4; c++)
            __builtin_nontemporal_store((v4u){w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]}, (v4u*)p + c);
    }
}
template <int N>
__device__ __forceinline__ void bstore_dw(__amdgpu_buffer_rsrc_t rs, uint32_t off, const uint32_t (&w)[N])
{
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    if constexpr (N == 1) __builtin_amdgcn_raw_buffer_store_b32(w[0], rs, off, 0, 2);
    else if constexpr (N == 2) __builtin_amdgcn_raw_buffer_store_b64((v2u){w[0], w[1]}, rs, off, 0, 2);
    else {
#pragma unroll
        for (int c = 0; c < N / 4; c++)
            __builtin_amdgcn_raw_buffer_store_b128((v4u){w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]}, rs,
                                                   off + 16 * c, 0, 2);
    }
}
template <typename VT, int DPL>
__device__ __forceinline__ void store_vals(VT* p, const int (&v)[DPL])
{
    if constexpr (sizeof(VT) == 2) store_i16<DPL>((int16_t*)p, v);
    else store_dw<DPL>((uint32_t*)p, (const uint32_t (&)[DPL])v);
}
template <typename VT, int DPL>
__device__ __forceinline__ void bstore_vals(__amdgpu_buffer_rsrc_t rs, uint32_t off, const int (&v)[DPL])
{
    if constexpr (sizeof(VT) == 2) bstore_i16<DPL>(rs, off, v);
    else bstore_dw<DPL>(rs, off, (const uint32_t (&)[DPL])v);
}
template <typename VT, int DPL>
__device__ __forceinline__ void load_vals(const VT* p, int (&v)[DPL])
{
    if constexpr (sizeof(VT) == 2) {
        int16_t t[DPL];
        load_i16<DPL>((const int16_t*)p, t);
#pragma unroll
        for (int k = 0; k < DPL; k++) v[k] = t[k];
    } else if constexpr (DPL == 1) {
        v[0] = *(const int*)p;
    } else if constexpr (DPL == 2) {
        const int2 t = *(const int2*)p;
        v[0] = t.x; v[1] = t.y;
    } else {
#pragma unroll
        for (int c = 0; c < DPL / 4; c++) {
            const int4 t = ((const int4*)p)[c];
            v[4 * c] = t.x; v[4 * c + 1] = t.y; v[4 * c + 2] = t.z; v[4 * c + 3] = t.w;
        }
    }
}

// Deficit planes (Geom::evol). In the plain int16 regime a path cost is L = C' - e with
// e = (minLp + P2) - min(Lp(d), Lp(d -+ 1) + P1, minLp + P2) in [0, P2] (OpenCV's recurrence:
// ocv_step_pk computes e on the way to L), so for P2 <= 511 a volume slot holds e in 9 bits
// instead of L in 16: the D low bytes of a pixel and bit 8 of each as D/8 bytes (in each byte the
// even d of a group of 8 at bits 0-3 and the odd ones at bits 4-7, the order the packed pairs
// give), 9/8 B per cell instead of 2 written by the paths and read by the WTA; the readers load C'
// beside them and rebuild L exactly. Two layouts (Geom::evol): 1 = one record per pixel
// (9D/8 rounded up to 16 B: a path step writes one contiguous run), 2 = a byte plane then a bit
// plane (D % 128 == 0: each pixel's low bytes are whole 128-B lines).
struct EvLayout {
    uint32_t ls, hs;        // bytes per pixel of the low bytes / of the bits
    size_t hb;              // offset of pixel 0's bits in the slot
};
__host__ __device__ inline int evol_rs(int D) { return (9 * D / 8 + 15) & ~15; }
__host__ __device__ inline EvLayout evol_layout(const Geom& g)
{
    if (g.evol == 2) return EvLayout{(uint32_t)g.D, (uint32_t)g.D / 8, (size_t)g.width1 * g.H * g.D};
    const uint32_t rs = (uint32_t)evol_rs(g.D);
    return EvLayout{rs, rs, (size_t)g.D};
}
__device__ __forceinline__ int evol_pos(int d) { return ((d & 1) << 2) | ((d & 7) >> 1); }
// N consecutive e from d0 (a multiple of N): lo = the low byte of d0, hi = the bit byte holding
// d0's bit
template <int N>
__device__ __forceinline__ void load_e(const uint8_t* lo, const uint8_t* hi, int d0, int (&e)[N])
{
    uint32_t w[(N + 3) / 4];
    if constexpr (N == 1) w[0] = *lo;
    else if constexpr (N == 2) w[0] = *(const uint16_t*)lo;
    else if constexpr (N == 4) w[0] = *(const uint32_t*)lo;
    else if constexpr (N == 8) { const uint2 t = *(const uint2*)lo; w[0] = t.x; w[1] = t.y; }
    else {
#pragma unroll
        for (int c = 0; c < N / 16; c++) {
            const uint4 t = ((const uint4*)lo)[c];
            w[4 * c] = t.x; w[4 * c + 1] = t.y; w[4 * c + 2] = t.z; w[4 * c + 3] = t.w;
        }
    }
    uint32_t h;                                          // bit planes are only 2-B aligned for N = 32
    if constexpr (N <= 8) h = *hi;
    else if constexpr (N == 16) h = *(const uint16_t*)hi;
    else h = (uint32_t)((const uint16_t*)hi)[0] | ((uint32_t)((const uint16_t*)hi)[1] << 16);
#pragma unroll
    for (int k = 0; k < N; k++) {
        const int pos = N >= 8 ? evol_pos(k) + 8 * (k / 8) : evol_pos(d0 + k);
        e[k] = (int)(((w[k / 4] >> (8 * (k % 4))) & 0xFFu) | (((h >> pos) & 1u) << 8));
    }
}

// OpenCV recurrence of one cell with int16 storage semantics, for a path line held by LPL
// lanes (16: one row of the wave; 32: two rows) — lane p: d = p*DPL .. p*DPL + DPL - 1.
// Entries with d >= D hold kMaxCost (OpenCV's Lr[-1] / Lr[D] = MAX_COST padding).
template <int LPL>
__device__ __forceinline__ int line_shr1(int v, int p)
{
    if constexpr (LPL == 16) return (int)row_shr1((uint32_t)v, (uint32_t)kMaxCost);
    if constexpr (LPL == 64) return __builtin_amdgcn_update_dpp(kMaxCost, v, 0x138, 0xf, 0xf, false);   // lane 0: old
    const int t = __builtin_amdgcn_update_dpp(kMaxCost, v, 0x138, 0xf, 0xf, false);   // wave_shr:1
    return p == 0 ? kMaxCost : t;                      // lane 32 must not see lane 31 (the other line)
}
template <int LPL>
__device__ __forceinline__ int line_shl1(int v, int p)
{
    if constexpr (LPL == 16) return (int)row_shl1((uint32_t)v, (uint32_t)kMaxCost);
    if constexpr (LPL == 64) return __builtin_amdgcn_update_dpp(kMaxCost, v, 0x130, 0xf, 0xf, false);   // lane 63: old
    const int t = __builtin_amdgcn_update_dpp(kMaxCost, v, 0x130, 0xf, 0xf, false);   // wave_shl:1
    return p == LPL - 1 ? kMaxCost : t;
}
// Lout: the CostType (int16) path costs, the recurrence's state; Lraw: the int values
// OpenCV adds into S (equal to Lout unless a cost left int16).
// SAT (SGM_OCV_SIMD_SAT in the overflow regime): the SIMD recurrence, all in saturating int16 —
// Lp(d +- 1) + P1 saturated, delta = (short)(minLr + P2) (wraps), L = sat(sat(min - delta) + C);
// Lout = Lraw = L and the min is over the int16 values.
template <int DPL, int LPL, bool SAT = false>
__device__ __forceinline__ int ocv_step(const int (&Cp)[DPL], const int (&Lp)[DPL], int mLp, bool pv, int p,
                                        const Geom& g, int (&Lout)[DPL], int (&Lraw)[DPL])
{
    const int fromLeft = line_shr1<LPL>(Lp[DPL - 1], p);
    const int fromRight = line_shl1<LPL>(Lp[0], p);
    const int lp_min = pv ? mLp : 0;
    const int delta = SAT ? (int)(int16_t)(lp_min + g.P2) : lp_min + g.P2;
    int lmin = 1 << 30;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
        const int d = p * DPL + k;
        int a = pv ? Lp[k] : 0;
        int lm1 = k > 0 ? Lp[k - 1] : fromLeft;
        int lp1 = k < DPL - 1 ? Lp[k + 1] : fromRight;
        if (!pv) { lm1 = d > 0 ? 0 : kMaxCost; lp1 = d < g.D - 1 ? 0 : kMaxCost; }
        int v;
        if constexpr (SAT) {
            const int m = min(min(a, sat16(lm1 + g.P1)), min(sat16(lp1 + g.P1), delta));
            v = sat16(sat16(m - delta) + Cp[k]);
        } else {
            v = Cp[k] + min(a, min(lm1 + g.P1, min(lp1 + g.P1, delta))) - delta;
        }
        Lout[k] = d < g.D ? (int)(int16_t)v : kMaxCost;   // Lr is CostType (int16)
        Lraw[k] = d < g.D ? v : kMaxCost;
        if (d < g.D) lmin = min(lmin, v);                  // minL over the int values
    }
    return lmin;
}

// signed min over the LPL lanes of each line (16: a row; 32: a row pair joined by
// v_permlane16_swap; 64: the wave, halves joined by v_permlane32_swap), result in every
// lane of the line
template <int LPL>
__device__ __forceinline__ int line_min_i32(int v)
{
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true));     // quad_perm [1,0,3,2]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true));     // quad_perm [2,3,0,1]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xf, 0xf, true));    // row_ror:4
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, true));    // row_ror:8
    if constexpr (LPL >= 32) {
        const auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);   // rows (0,1), (2,3) exchanged
        v = min((int)sw[0], (int)sw[1]);
    }
    if constexpr (LPL == 64) {
        const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);   // halves exchanged
        v = min((int)sw[0], (int)sw[1]);
    }
    return v;
}

// buffer offset of a dropped store: past every buffer range the buffer path is used for
constexpr uint32_t kBufDrop = 0xFFFFFF00u;

// a 64-bit value the caller knows to be wave-uniform, stated so (kept in SGPRs)
__device__ __forceinline__ long long lane64(long long v, int lane)   // lane `lane`'s v, wave-uniform
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((unsigned long long)v >> 32), lane);
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ long long uni64(long long v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}

#ifndef SGM_OCV_VWTA_PK
#define SGM_OCV_VWTA_PK 1  // k_ocv_vwta_pk for the plain int16 regime with uniqueness < 100
#endif
#ifndef SGM_OCV_ILV
#define SGM_OCV_ILV 1  // k_ocv_paths: the directions' blocks dealt round-robin for 64-lane lines (env SGM_OCV_ILV overrides)
#endif
#ifndef SGM_OCV_VWTA_PK_EV5
#define SGM_OCV_VWTA_PK_EV5 1  // k_ocv_vwta_pk also for MODE_SGBM when the volumes are deficit records
#endif
#ifndef SGM_OCV_VWTA_PK_MIND
#define SGM_OCV_VWTA_PK_MIND 4  // k_ocv_vwta_pk from this many values per lane: 4 (128 < D <= 256, deficit
                                // records in half groups) against the int kernel, frame ms: 12 MP D=256 MODE_HH
                                // 25.4 -> 23.95, MODE_SGBM 17.48 -> 16.18, 1080p D=256 MODE_HH 4.22 -> 4.17
                                // (profiles/r06_ocv_vwta_pk4_ab.jsonl)
#endif
#ifndef SGM_OCV_VWTA_PK_PF
#define SGM_OCV_VWTA_PK_PF 0  // k_ocv_vwta_pk steps in flight (0: by shape)
#endif
#ifndef SGM_OCV_PK_PF
#define SGM_OCV_PK_PF 16   // packed path lines: cost rows in flight for up to 4 dwords per lane (4 for 8, 2 for 16)
#endif
#ifndef SGM_OCV_PK_PF16
#define SGM_OCV_PK_PF16 12 // packed 16-lane path lines of <= 8 values: cost rows in flight
#endif
#ifndef SGM_OCV_PK_PF8
#define SGM_OCV_PK_PF8 8   // packed 64-lane path lines of 16 values: cost rows in flight
#endif
#ifndef SGM_OCV_PK
#define SGM_OCV_PK 1       // the plain int16 path recurrence in packed u16 pairs (0: one int per value)
#endif
// The plain (non-SAT) int16 regime of the path recurrence in packed u16 pairs. There every
// C' lies in [P2, 32767] (box sum + P2, no cost left int16: the gate's condition), so with
// delta = minLp + P2 the candidates Lp, Lp(d -+ 1) + P1 and delta stay below 65536 (P1, P2 <=
// 32768: the launcher's condition) and OpenCV's C + min(...) - delta = C - (delta - min(...))
// never leaves [0, 32767]: the u16 halves are exactly OpenCV's int values and its CostType
// copies. A lane's DPL values are DPL / 2 dwords as loaded from C' and stored to the volume
// (no unpacking), the neighbours two alignbits of adjacent pairs and one DPP per lane edge.
template <int LPL>
__device__ __forceinline__ uint32_t line_shr1_u(uint32_t v, int p)      // lane p <- p - 1; line start: 0xFFFFFFFF
{
    if constexpr (LPL == 16) return row_shr1(v, 0xFFFFFFFFu);
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x138, 0xf, 0xf, false);
    return (LPL == 64 || p != 0) ? t : 0xFFFFFFFFu;
}
template <int LPL>
__device__ __forceinline__ uint32_t line_shl1_u(uint32_t v, int p)      // lane p <- p + 1; line end: 0xFFFFFFFF
{
    if constexpr (LPL == 16) return row_shl1(v, 0xFFFFFFFFu);
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x130, 0xf, 0xf, false);
    return (LPL == 64 || p != LPL - 1) ? t : 0xFFFFFFFFu;
}
// One step: L2 (the previous L of the lane's pairs) -> the new L; returns the lane's min over
// its valid d (entries with d >= D are forced to kMaxCost = 32767 by imask, as OpenCV pads).
template <int DPL, int LPL>
__device__ __forceinline__ uint32_t ocv_step_pk(const uint32_t (&C2)[DPL / 2], uint32_t (&L2)[DPL / 2], uint32_t delta2,
                                                uint32_t P1P1, const uint32_t (&imask)[DPL / 2], int p,
                                                uint32_t* E2 = nullptr)   // E2: the deficits e = C' - L
{
    constexpr int M = DPL / 2;
    uint32_t q[M];
#pragma unroll
    for (int i = 0; i < M; i++) q[i] = pk_add(L2[i], P1P1);
    const uint32_t X = line_shr1_u<LPL>(q[M - 1], p), Y = line_shl1_u<LPL>(q[0], p);
    uint32_t Op = alignbit16(q[0], X);                   // (q(d - 1), q(d)) of pair 0
    uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < M; i++) {
        const uint32_t On = (i + 1 < M) ? alignbit16(q[i + 1], q[i]) : alignbit16(Y, q[M - 1]);
        const uint32_t t = pk_min(pk_min(Op, On), pk_min(L2[i], delta2));
        const uint32_t e = pk_sub(delta2, t);
        if (E2) E2[i] = e;
        const uint32_t v = pk_sub(C2[i], e);
        L2[i] = (v & ~imask[i]) | (0x7FFF7FFFu & imask[i]);
        mn = pk_min(mn, L2[i]);
        Op = On;
    }
    return min(mn & 0xFFFFu, mn >> 16);
}
template <int N>
__device__ __forceinline__ void bload_dw(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t (&w)[N])
{
    if constexpr (N == 1) w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    else if constexpr (N == 2) { const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0); w[0] = t[0]; w[1] = t[1]; }
    else {
#pragma unroll
        for (int c = 0; c < N / 4; c++) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * c, 0, 0);
            w[4 * c] = t[0]; w[4 * c + 1] = t[1]; w[4 * c + 2] = t[2]; w[4 * c + 3] = t[3];
        }
    }
}

// One step's deficits of a lane (DPL = 8 or 16 values, DPL / 2 packed pairs) into the deficit
// planes: DPL low bytes at lo_off, DPL bits (evol_pos order) at hi_off; nontemporal, streamed once
// into the WTA
template <int DPL>
__device__ __forceinline__ void evol_store(__amdgpu_buffer_rsrc_t rs, uint32_t lo_off, __amdgpu_buffer_rsrc_t rsh,
                                           uint32_t hi_off, const uint32_t (&E2)[DPL / 2])
{
    static_assert(DPL == 8 || DPL == 16, "one or two groups of 8 deficits per lane");
    constexpr int NG = DPL / 8;
    uint32_t lo[2 * NG], hb = 0;
#pragma unroll
    for (int c = 0; c < NG; c++) {
        lo[2 * c] = __builtin_amdgcn_perm(E2[4 * c + 1], E2[4 * c], 0x06040200u);       // e(d0..d3) low bytes
        lo[2 * c + 1] = __builtin_amdgcn_perm(E2[4 * c + 3], E2[4 * c + 2], 0x06040200u);
        uint32_t t = 0;                                  // pair i: bit 8 of e(2i) -> bit i, of e(2i+1) -> 16 + i
#pragma unroll
        for (int i = 0; i < 4; i++) t |= as_u(as_v2(E2[4 * c + i]) >> (u16x2_t){8, 8}) << i;
        hb |= ((t | (t >> 12)) & 0xFFu) << (8 * c);
    }
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    if constexpr (NG == 1) {
        __builtin_amdgcn_raw_buffer_store_b64((v2u){lo[0], lo[1]}, rs, lo_off, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)hb, rsh, hi_off, 0, 2);
    } else {
        __builtin_amdgcn_raw_buffer_store_b128((v4u){lo[0], lo[1], lo[2], lo[3]}, rs, lo_off, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)hb, rsh, hi_off, 0, 2);
    }
}

// 64 / LPL path lines per wave. Block b of direction dir holds its lines NLW*b .. NLW*b +
// NLW - 1: horizontal (ry == 0) line = row; row sweeps (ry != 0): lines [0, width1) start on
// the first row at that column, the others on the entry column at row offset
// line - width1 + 1. The lines of a block have (nearly) equal lengths; each stores only
// while its own steps last. Fewer, wider lines (LPL 32) shorten each step's instruction
// chain: a line is a sequential walk, and its step latency bounds the kernel.
// REBK: the instantiation for 64-lane lines of 8 values whose volumes pass 4 GB (the step-rebased
// packed form only; kept apart so its descriptors' SGPRs do not weigh on the buffer-offset kernel)
template <int DPL, int LPL, typename VT, bool SAT, bool REBK = false>
__global__ __launch_bounds__(64) void k_ocv_paths(const int16_t* __restrict__ C, VT* __restrict__ vols,
                                                  size_t vol_elems, size_t trash_off, Geom g, int dirmask, int4 nblk0,
                                                  int4 nblk1, int use_buf, int use_pk, int ilv)
{
    if (ocv_gate_skip<SAT || sizeof(VT) == 4>(g)) return;
    const int nb[8] = {nblk0.x, nblk0.y, nblk0.z, nblk0.w, nblk1.x, nblk1.y, nblk1.z, nblk1.w};
    // block -> (direction, group of 4 lines); volume slot = rank of the direction in dirmask.
    // ilv: the directions' blocks dealt round-robin (block b: the (b mod n)-th direction with
    // blocks, its group b / n; groups past a direction's count exit), so the lines of every
    // direction that start together run together
    int b = blockIdx.x, dir = 0, slot = 0;
    if (ilv) {
        int nact = 0, nbd = 0;
        for (int i = 0; i < 8; i++) nact += nb[i] > 0;
        const int k = b % nact;
        b /= nact;
        for (int i = 0, c = 0; i < 8; i++) {
            if (!((dirmask >> i) & 1)) continue;
            if (nb[i] > 0 && c++ == k) { dir = i; nbd = nb[i]; break; }
            slot++;
        }
        if (b >= nbd) return;
    } else {
        for (int i = 0; i < 8; i++) {
            if (!((dirmask >> i) & 1)) continue;
            if (b < nb[i]) { dir = i; break; }
            b -= nb[i];
            slot++;
        }
    }
    // uniform by construction (block-level values); stated, so the volume's buffer descriptor
    // stays in SGPRs (hipcc had lost track after the round-robin deal and wrapped every buffer
    // load and store of the small-D instantiations in a readfirstlane waterfall loop)
    dir = __builtin_amdgcn_readfirstlane(dir);
    slot = __builtin_amdgcn_readfirstlane(slot);
    b = __builtin_amdgcn_readfirstlane(b);
    VT* V = vols + (size_t)slot * vol_elems;
    constexpr int NLW = 64 / LPL;                      // lines per wave
    constexpr bool kRaw = sizeof(VT) == 4;             // store the int path costs (Geom::wide)
    const int lane = threadIdx.x, r = lane / LPL, p = lane % LPL;
    const int rx = dir_rx(dir), ry = dir_ry(dir);
    const int line = NLW * b + r;
    const int nlines = ry == 0 ? g.H : g.width1 + (rx != 0 ? g.H - 1 : 0);
    int x0 = 0, s0 = 0, n = 0;
    if (line < nlines) {
        if (ry == 0) { x0 = rx > 0 ? 0 : g.width1 - 1; s0 = line; n = g.width1; }
        else {
            if (line < g.width1) { x0 = line; s0 = 0; }
            else { x0 = rx > 0 ? 0 : g.width1 - 1; s0 = line - g.width1 + 1; }
            n = g.H - s0;
            if (rx > 0) n = min(n, g.width1 - x0);
            if (rx < 0) n = min(n, x0 + 1);
        }
    }
    int nmax = 0;
#pragma unroll
    for (int w = 0; w < NLW; w++) nmax = max(nmax, __builtin_amdgcn_readlane(n, w * LPL));
    // cell offset of step i = base + i * step (clamped to the line for LPL 16)
    const int ybase = ry >= 0 ? s0 : g.H - 1 - s0;
    const long long cbase = ((long long)ybase * g.width1 + x0) * g.D;
    const long long cstep = ((long long)ry * g.width1 + rx) * g.D;
    const int ilast = max(n - 1, 0);
    auto cell = [&](int i) -> long long { return cbase + (long long)min(i, ilast) * cstep; };
    int Lp[DPL], mLp = 0;
#pragma unroll
    for (int k = 0; k < DPL; k++) Lp[k] = kMaxCost;
    // C of the next PF steps in flight (one global-load latency per PF steps, not per step);
    // one vector load per lane (lanes past D read the last valid group: their C never
    // reaches an entry with d < D): no exec-masked branch around the loads, so the prefetch
    // keeps counted waits
    constexpr int PF = DPL <= 4 ? SGM_OCV_PF : LPL == 32 ? SGM_OCV_PF_WIDE32 : SGM_OCV_PF_WIDE;
    int Cb[PF][DPL];
    const bool lane_act = p * DPL < g.D;
    // 32 values per lane (64-lane lines, D > 1024) with D % 32 = 16: one lane straddles D. It
    // loads from its own first d (its upper 16 values read the next cell: d >= D never reaches
    // a valid entry) and stores only its lower half. Lanes wholly past D load the last group.
    const bool straddle = DPL == 32 && lane_act && p * DPL + DPL > g.D;
    const int dl = lane_act ? p * DPL : g.D - DPL;
    // Straight-line steps (no branch, so hipcc keeps counted vmcnt waits across the loop).
    // The first PF steps are peeled (pv = false only at step 0, a constant elsewhere).
    if constexpr (!SAT && sizeof(VT) == 2 && DPL >= 2) {
        // the plain int16 regime in packed u16 pairs (ocv_step_pk): volumes below 4 GB with 32-bit
        // buffer offsets that move by the step, or — 64-lane lines (one line per wave, so a step's
        // cell is wave-uniform) — any size, each step's descriptors rebased on the step's cell
        // (64-bit scalar arithmetic, lane offsets within the cell): the D > 512 frames (the
        // processing launch's D = 752 has 5.2 GB int16 volumes) keep the packed step and the
        // deficit records. 16 values per lane (512 < D <= 1024) in this kernel; 8 values (256 < D <=
        // 512 on frames past 4 GiB of volume, e.g. 12 MP) in their own instantiation (REBK), because
        // the per-step descriptors of 16 rows in flight cost SGPRs that the buffer-offset form of the
        // same kernel (the shipped D=480 config) would otherwise pay for (105 -> 138 VGPRs); 32 values
        // (D > 1024) have a lane straddling D that would load past its rebased cell. 32-lane lines of
        // 8 values (128 < D <= 256 beside the fused vertical WTA, 12 MP frames past 4 GiB) take the
        // same REBK instantiation with one descriptor per half-wave line.
        if (use_pk && (use_buf || (LPL == 64 && (DPL == 16 || REBK)) || (LPL == 32 && REBK))) {
            constexpr int M = DPL / 2;
            const size_t cells = (size_t)g.width1 * g.H * g.D;
            const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (int)(uint32_t)(cells * 2), 0x00020000);
            const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)V, 0, (int)(uint32_t)(cells * 2), 0x00020000);
            const uint32_t bstep = (uint32_t)(cstep * 2);
            uint32_t ld_b = (uint32_t)((cbase + dl) * 2), st_b = ld_b;
            uint32_t imask[M];
#pragma unroll
            for (int i = 0; i < M; i++)
                imask[i] = (p * DPL + 2 * i < g.D ? 0u : 0xFFFFu) | (p * DPL + 2 * i + 1 < g.D ? 0u : 0xFFFF0000u);
            const uint32_t P1P1 = (uint32_t)g.P1 * 0x10001u, P2 = (uint32_t)g.P2;
            // rows in flight: hipcc waits for all of an iteration's loads at its top (vmcnt(0)), so
            // the iteration is PK_PF steps long: one memory latency per PK_PF steps
            // (1080p D=128 MODE_SGBM paths, M = 4: 0.97 ms unpacked, packed 0.91 / 0.86 / 0.84 at 4 / 8 /
            // 16 rows; the shipped D=480 config, M = 8: 6.20 ms unpacked and at 4 rows, 6.79 at 8;
            // profiles/r05_ocv_pk_ab.jsonl)
            // 16 values per lane on 64-lane lines (512 < D <= 1024, the rebased form): 8 rows
            // (the D=752 config's paths 7.49 -> 7.27 ms MODE_SGBM, 13.29 -> 12.95 MODE_HH; 2 / 3 / 6:
            // 7.48-7.51 / 7.44; profiles/r06_ocv_paths_pf8_ab.jsonl)
            // <= 4 dwords per lane: 16 rows, 12 on 16-lane lines (1080p D=128 paths MODE_SGBM 0.812 ->
            // 0.798 ms, MODE_HH 1.257 -> 1.203; 8 / 24: 0.803 / 0.816, 1.219 / 1.326; the shipped D=480
            // 64-lane lines keep 16: 5.34 against 5.40 / 5.51 at 12 / 8, 5.31 at 24;
            // profiles/r06_ocv_paths_pf_m4_ab.jsonl)
            constexpr int PF = M <= 4 ? (LPL == 16 ? SGM_OCV_PK_PF16 : SGM_OCV_PK_PF)
                             : M <= 8 ? (LPL == 64 ? SGM_OCV_PK_PF8 : 4) : 2;
            // deficits (Geom::evol, 8 or 16 values per lane): the low bytes and the bits of d
            const EvLayout el = evol_layout(g);
            const long long pix0 = (long long)ybase * g.width1 + x0, pstep = (long long)ry * g.width1 + rx;
            uint32_t ev_lo = (uint32_t)(pix0 * el.ls + dl), ev_hi = (uint32_t)(el.hb + pix0 * el.hs + dl / 8);
            const uint32_t ev_step = (uint32_t)(pstep * el.ls), ev_hstep = (uint32_t)(pstep * el.hs);
            // rebased form (REB): the line's cell / pixel of step i (clamped to its last step, so every
            // descriptor base stays inside the volume), stated uniform over the line: the wave's one
            // line (64 lanes), or the two half-wave lines' (32 lanes): one descriptor then spans both
            // lines' cells of the step (adjacent lines of one direction, lengths within a step of each
            // other: a few rows apart at most) and each lane adds its own line's distance from the lower
            constexpr int NH = LPL == 32 ? 2 : 1;
            long long ucb[NH], ucs[NH], upx[NH], ups[NH];
            int ulast[NH];
#pragma unroll
            for (int h = 0; h < NH; h++) {
                ucb[h] = NH == 1 ? uni64(cbase) : lane64(cbase, 32 * h);
                ucs[h] = NH == 1 ? uni64(cstep) : lane64(cstep, 32 * h);
                upx[h] = NH == 1 ? uni64(pix0) : lane64(pix0, 32 * h);
                ups[h] = NH == 1 ? uni64(pstep) : lane64(pstep, 32 * h);
                ulast[h] = NH == 1 ? __builtin_amdgcn_readfirstlane(ilast) : __builtin_amdgcn_readlane(ilast, 32 * h);
            }
            if constexpr (NH == 2) {
                // a second half past the direction's last line (n = 0) follows the first one's line
                if (!__builtin_amdgcn_readlane((int)(line < nlines), 32)) {
                    ucb[1] = ucb[0]; ucs[1] = ucs[0]; upx[1] = upx[0]; ups[1] = ups[0]; ulast[1] = ulast[0];
                }
            }
            const uint32_t cell_bytes = (uint32_t)g.D * 2u;
            // elements a, b (the two half-lines' cells or pixels of a step, `unit` bytes apart) under one
            // descriptor from the lower one to `extra` bytes past the higher; off: the lane's own offset
            auto span = [&](const void* base, long long a, long long b, long long unit, uint32_t extra, uint32_t& off) {
                if constexpr (NH == 1) {                 // one line per wave: the element's own descriptor
                    off = 0;
                    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + a * unit), 0, (int)extra, 0x00020000);
                } else {
                    const long long lo = a < b ? a : b, d = a < b ? b - a : a - b;
                    off = (uint32_t)(((r ? b : a) - lo) * unit);
                    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + lo * unit), 0,
                                                             (int)(uint32_t)(d * unit + extra), 0x00020000);
                }
            };
            auto cell_at = [&](int h, int i) { return ucb[h] + (long long)min(i, ulast[h]) * ucs[h]; };
            auto px_at = [&](int h, int i) { return upx[h] + (long long)min(i, ulast[h]) * ups[h]; };
            auto run = [&](auto evc, auto rebc) {
                constexpr bool EV = decltype(evc)::value;
                constexpr bool REB = decltype(rebc)::value;
                uint32_t C2[PF][M], L2[M];
#pragma unroll
                for (int i = 0; i < M; i++) L2[i] = 0;
                uint32_t delta2 = P2 * 0x10001u;         // the path's first pixel: L = C - P2
                auto loadC = [&](int i, uint32_t (&c)[M]) {
                    if constexpr (REB) {
                        uint32_t off;
                        const auto rs = span(C, cell_at(0, i), cell_at(NH - 1, i), 2, cell_bytes, off);
                        bload_dw<M>(rs, off + (uint32_t)dl * 2u, c);
                    } else {
                        bload_dw<M>(rsC, ld_b, c);
                        ld_b += bstep;
                    }
                };
#pragma unroll
                for (int q = 0; q < PF; q++) loadC(q, C2[q]);
                auto steps = [&](int i0) {
#pragma unroll
                    for (int q = 0; q < PF; q++) {
                        const int i = i0 + q;
                        uint32_t E2[M];
                        const uint32_t lmin = ocv_step_pk<DPL, LPL>(C2[q], L2, delta2, P1P1, imask, p, EV ? E2 : nullptr);
                        const bool ok = lane_act && i < n;
                        if constexpr (EV && REB) {
                            const long long pa = px_at(0, i), pb = px_at(NH - 1, i);
                            uint32_t olo, ohi;
                            const auto rlo = span(V, pa, pb, el.ls, el.ls, olo);
                            const auto rhi = span((const char*)V + el.hb, pa, pb, el.hs, el.hs, ohi);
                            evol_store<DPL>(rlo, ok ? olo + (uint32_t)dl : kBufDrop, rhi, ok ? ohi + (uint32_t)dl / 8u : kBufDrop, E2);
                        } else if constexpr (EV) {
                            evol_store<DPL>(rsV, ok ? ev_lo : kBufDrop, rsV, ok ? ev_hi : kBufDrop, E2);
                            ev_lo += ev_step;
                            ev_hi += ev_hstep;
                        } else {
                            uint32_t so = st_b;
                            auto rsS = rsV;
                            if constexpr (REB) {
                                rsS = span(V, cell_at(0, i), cell_at(NH - 1, i), 2, cell_bytes, so);
                                so += (uint32_t)dl * 2u;
                            }
                            if constexpr (DPL == 32) {   // two halves: the straddling lane drops its upper one
                                bstore_dw<8>(rsS, ok ? so : kBufDrop, *reinterpret_cast<const uint32_t(*)[8]>(&L2[0]));
                                bstore_dw<8>(rsS, ok && !straddle ? so + 32u : kBufDrop,
                                             *reinterpret_cast<const uint32_t(*)[8]>(&L2[8]));
                            } else {
                                bstore_dw<M>(rsS, ok ? so : kBufDrop, L2);
                            }
                        }
                        delta2 = ((uint32_t)line_min_i32<LPL>((int)lmin) + P2) * 0x10001u;
                        loadC(i + PF, C2[q]);
                        st_b += bstep;
                    }
                };
                // longest-remaining-first priority (lr_prio) on lines of <= 4 dwords per lane: the
                // lines that still have the most steps are served first when the frame's waves
                // compete (interleaved A/B, frame ms off -> on: C1 0.199 -> 0.190, 1080p D=128
                // MODE_SGBM 1.389 -> 1.357, MODE_HH 1.937 -> 1.914, 12 MP D=128 MODE_SGBM 8.54 ->
                // 8.31, the shipped D=480 MODE_SGBM 10.31 -> 10.23, MODE_HH 15.59 -> 15.38, 12 MP
                // D=480 25.46 -> 25.22; 8 dwords (D=752 MODE_HH 21.75 -> 21.80) and the int branches
                // (int32 volumes MODE_HH 19.95 -> 20.07) keep it off; profiles/r06_ocv_prio_ab.jsonl)
                constexpr bool kPrio = SGM_OCV_PRIO == 2 || (SGM_OCV_PRIO == 1 && M <= 4);
                for (int i0 = 0; i0 < nmax; i0 += PF) {
                    if (kPrio && (i0 & 15) < PF) lr_prio(nmax - i0, max(g.width1, g.H));
                    steps(i0);
                }
            };
            if constexpr ((LPL == 64 && (DPL == 16 || REBK)) || (LPL == 32 && REBK)) {
                if (!use_buf) {
                    {
                        if (g.evol) {
                            run(std::true_type{}, std::true_type{});
                            return;
                        }
                    }
                    run(std::false_type{}, std::true_type{});
                    return;
                }
            }
            if constexpr (DPL == 8 || DPL == 16) {
                if (g.evol) {
                    run(std::true_type{}, std::false_type{});
                    return;
                }
            }
            run(std::false_type{}, std::false_type{});
            return;
        }
    }
    if (use_buf) {
        // Volumes < 4 GB - 256 B: raw buffer loads and stores with 32-bit byte offsets that just
        // move by the step (mod 2^32); a step past the line's end reads whatever lies there
        // (unused) or 0 past the range, and a store that must not land is sent to kBufDrop,
        // past the range, where the hardware drops it. No clamps, 64-bit address selects or trash slot in the step chain (C1
        // paths 115 -> 90 us: a small frame's line is issue-bound, 61 -> 48 instructions/step).
        const size_t cells = (size_t)g.width1 * g.H * g.D;
        const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (int)(uint32_t)(cells * 2), 0x00020000);
        const __amdgpu_buffer_rsrc_t rsV =
            __builtin_amdgcn_make_buffer_rsrc((void*)V, 0, (int)(uint32_t)(cells * sizeof(VT)), 0x00020000);
        const uint32_t bstep = (uint32_t)(cstep * 2), vstep = (uint32_t)(cstep * (long long)sizeof(VT));
        uint32_t ld_b = (uint32_t)((cbase + dl) * 2), st_b = (uint32_t)((cbase + dl) * (long long)sizeof(VT));
#pragma unroll
        for (int q = 0; q < PF; q++) { bload_i16<DPL>(rsC, ld_b, Cb[q]); ld_b += bstep; }
        auto steps = [&](int i0, auto first) {
#pragma unroll
            for (int q = 0; q < PF; q++) {
                const int i = i0 + q;
                int L[DPL], Lraw[DPL];
                const int lmin = ocv_step<DPL, LPL, SAT>(Cb[q], Lp, mLp, !(decltype(first)::value && q == 0), p, g, L, Lraw);
                const bool ok = lane_act && i < n;
                if constexpr (DPL == 32) {        // two halves: the straddling lane drops its upper one
                    const int (&Vs)[32] = kRaw ? Lraw : L;
                    bstore_vals<VT, 16>(rsV, ok ? st_b : kBufDrop, *reinterpret_cast<const int(*)[16]>(&Vs[0]));
                    bstore_vals<VT, 16>(rsV, ok && !straddle ? st_b + 16u * (uint32_t)sizeof(VT) : kBufDrop,
                                        *reinterpret_cast<const int(*)[16]>(&Vs[16]));
                } else {
                    bstore_vals<VT, DPL>(rsV, ok ? st_b : kBufDrop, kRaw ? Lraw : L);
                }
                mLp = (int)(int16_t)line_min_i32<LPL>(lmin);   // minLr is CostType
#pragma unroll
                for (int k = 0; k < DPL; k++) Lp[k] = L[k];
                bload_i16<DPL>(rsC, ld_b, Cb[q]);
                st_b += vstep;
                ld_b += bstep;
            }
        };
        if (nmax > 0) steps(0, std::true_type{});
        for (int i0 = PF; i0 < nmax; i0 += PF) {
            if (SGM_OCV_PRIO == 2 && (i0 & 15) < PF) lr_prio(nmax - i0, max(g.width1, g.H));
            steps(i0, std::false_type{});
        }
    } else {
        // larger volumes: 64-bit addresses, clamped to the line; steps past a line's end and
        // lanes past D store to a per-lane trash slot after the volumes (vols + trash_off)
        VT* const tr = vols + trash_off + lane * DPL;
        auto load = [&](int (&c)[DPL], long long off) {
            int16_t v[DPL];
            load_i16<DPL>(C + off + dl, v);
#pragma unroll
            for (int k = 0; k < DPL; k++) c[k] = v[k];
        };
#pragma unroll
        for (int q = 0; q < PF; q++) load(Cb[q], cell(q));
        auto steps = [&](int i0, auto first) {
#pragma unroll
            for (int q = 0; q < PF; q++) {
                const int i = i0 + q;
                int L[DPL], Lraw[DPL];
                const int lmin = ocv_step<DPL, LPL, SAT>(Cb[q], Lp, mLp, !(decltype(first)::value && q == 0), p, g, L, Lraw);
                const bool ok = lane_act && i < n;
                if constexpr (DPL == 32) {
                    const int (&Vs)[32] = kRaw ? Lraw : L;
                    store_vals<VT, 16>(ok ? V + cell(i) + dl : tr, *reinterpret_cast<const int(*)[16]>(&Vs[0]));
                    store_vals<VT, 16>(ok && !straddle ? V + cell(i) + dl + 16 : tr + 16,
                                       *reinterpret_cast<const int(*)[16]>(&Vs[16]));
                } else {
                    store_vals<VT, DPL>(ok ? V + cell(i) + dl : tr, kRaw ? Lraw : L);
                }
                mLp = (int)(int16_t)line_min_i32<LPL>(lmin);   // minLr is CostType
#pragma unroll
                for (int k = 0; k < DPL; k++) Lp[k] = L[k];
                load(Cb[q], cell(i + PF));
            }
        };
        if (nmax > 0) steps(0, std::true_type{});
        for (int i0 = PF; i0 < nmax; i0 += PF) {
            if (SGM_OCV_PRIO == 2 && (i0 & 15) < PF) lr_prio(nmax - i0, max(g.width1, g.H));
            steps(i0, std::false_type{});
        }
    }
}

// S of one cell from the direction volumes (slot order: MODE_SGBM dirs 0, 2, 3, 6, 7; MODE_HH
// dirs 0..7), in OpenCV's order. Scalar branch: the int sum of pass 1 (dirs 6, 2, 0, 3 =
// OpenCV's r0..r3) saturated, then the fifth path (MODE_SGBM) or pass 2 (dirs 7, 4, 1, 5),
// saturated. SAT (SIMD branch): S = sat(sat(S + sat(L0 + L1)) + sat(L2 + L3)) per pass, the
// fifth path sat(S + L).
template <int NDIR, bool SAT, int DPL>
__device__ __forceinline__ int ocv_sum(const int (&v)[NDIR][DPL], int k)
{
    if constexpr (SAT) {
        if constexpr (NDIR == 5) {
            const int s1 = sat16(sat16(v[3][k] + v[1][k]) + sat16(v[0][k] + v[2][k]));
            return sat16(s1 + v[4][k]);
        } else {
            const int s1 = sat16(sat16(v[6][k] + v[2][k]) + sat16(v[0][k] + v[3][k]));
            return sat16(sat16(s1 + sat16(v[7][k] + v[4][k])) + sat16(v[1][k] + v[5][k]));
        }
    } else {
        int s1, s2;
        if constexpr (NDIR == 5) {
            s1 = v[0][k] + v[1][k] + v[2][k] + v[3][k];
            s2 = v[4][k];
        } else {
            s1 = v[0][k] + v[2][k] + v[3][k] + v[6][k];
            s2 = v[1][k] + v[4][k] + v[5][k] + v[7][k];
        }
        return sat16(sat16(s1) + s2);
    }
}

// WTA key tie order: the first d (OpenCV 4.x / scalar), or SGM_OCV_LANE_TIE (3.x SSE2 MODE_SGBM:
// lane d mod 8 first, then d) — `bits` = the key's disparity field width
__device__ __forceinline__ int wta_tie(int d, bool lane, int bits) { return lane ? ((d & 7) << (bits - 3)) | (d >> 3) : d; }
__device__ __forceinline__ int wta_untie(int t, bool lane, int bits)
{
    return lane ? ((t & ((1 << (bits - 3)) - 1)) << 3) | (t >> (bits - 3)) : t;
}

// WTA of the OCV modes, one workgroup (4 waves) per image row, 16 lanes per pixel (4 pixels
// per wave-instruction): lane p of a row holds d = p*DPL .. p*DPL + DPL - 1 of its pixel,
// loaded as one DPL-value vector per volume (coalesced). Same decisions as OpenCV's loop
// (SURVEY Appendix A.6): S = the saturating sums in OpenCV's pass order; best = first minimal d through
// one 16-lane min over (S + 32768) * 512 + d; uniqueness per element (S may be any int16
// here); S[best +- 1] through a per-row LDS slice; then the shared disp2 / LR epilogue.
template <int DPL, int NDIR, typename VT, bool SAT, bool EV>
__global__ __launch_bounds__(256) void k_ocv_wta16(const VT* __restrict__ vols, size_t vol_elems, Geom g,
                                                   int16_t* __restrict__ out, size_t out_stride,
                                                   const int16_t* __restrict__ Cv)   // C' (EV: deficit planes)
{
    if (ocv_gate_skip<SAT || sizeof(VT) == 4>(g)) return;
    const bool lanetie = NDIR == 5 && (g.compat & SGM_OCV_LANE_TIE);
    extern __shared__ uint32_t lds_ocv[];
    int16_t* sl = (int16_t*)lds_ocv;                      // 16 lane rows x 16 lanes x DPL S values
    RowLds R((char*)lds_ocv + (size_t)16 * 16 * DPL * 2, g.W);
    const int tid = threadIdx.x, lane = tid & 63, y = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane >> 4, p = lane & 15;
    R.init(g, tid, 256);
    const bool lane_act = p * DPL < g.D;
    const int dl = lane_act ? p * DPL : 0;
    int16_t* srow = sl + (w * 4 + r) * 16 * DPL;
    const int n = g.width1, nq = (n + 3) / 4;
    const size_t row0 = (size_t)y * g.width1 * g.D;
    // pixel 4q + r; the last group reads up to 3 pixels past the row (the next row or the
    // volume slack), results never stored
    auto load = [&](int q, int (&v)[NDIR][DPL]) {
        const size_t cell = row0 + (size_t)(4 * q + r) * g.D + dl;
        if constexpr (EV) {                              // L = C' - e
            int16_t c[DPL];
            load_i16<DPL>(Cv + cell, c);
            const EvLayout el = evol_layout(g);
            const size_t px = (size_t)y * g.width1 + 4 * q + r;
#pragma unroll
            for (int k = 0; k < NDIR; k++) {
                const uint8_t* vb = (const uint8_t*)(vols + (size_t)k * vol_elems);
                int e[DPL];
                load_e<DPL>(vb + px * el.ls + dl, vb + el.hb + px * el.hs + dl / 8, dl, e);
#pragma unroll
                for (int j = 0; j < DPL; j++) v[k][j] = c[j] - e[j];
            }
        } else {
            const VT* base = vols + cell;
#pragma unroll
            for (int k = 0; k < NDIR; k++) load_vals<VT, DPL>(base + (size_t)k * vol_elems, v[k]);
        }
    };
    int nxt[NDIR][DPL];
    load(min(w, nq - 1), nxt);
    for (int q = w; q < nq; q += 4) {
        // S in OpenCV's order of saturating adds: pass 1 (dirs 0, 2, 3, 6: volume slots 0-3
        // for MODE_SGBM, 0, 2, 3, 6 for MODE_HH) is added and saturated, then the fifth path
        // (MODE_SGBM) or pass 2 (MODE_HH) — they differ once sums overflow int16
        int S[DPL];
#pragma unroll
        for (int k = 0; k < DPL; k++) S[k] = ocv_sum<NDIR, SAT>(nxt, k);
        load(min(q + 4, nq - 1), nxt);
        uint32_t km = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < DPL; k++) {
            const int d = p * DPL + k;
            const uint32_t key = ((uint32_t)(S[k] + 32768) << 9) | (uint32_t)wta_tie(d, lanetie, 9);
            km = (lane_act && d < g.D) ? min(km, key) : km;
        }
        const uint32_t kmin = row_min_u32(km);
        const int best = wta_untie((int)(kmin & 511u), lanetie, 9);
        const int minS = (int)(kmin >> 9) - 32768;
        bool hit = false;
#pragma unroll
        for (int k = 0; k < DPL; k++) {
            const int d = p * DPL + k;
            hit |= lane_act && d < g.D && (unsigned)(d - best + 1) > 2u && S[k] * (100 - g.uniq) < minS * 100;
        }
        // every S saturated at MAX_COST: OpenCV's strict `Sval < minS` from minS = MAX_COST
        // never fires, bestDisp stays -1 and the pixel ends up (minD - 1) * 16 = INVALID with
        // no disp2 update, i.e. exactly a uniqueness reject
        const bool rej = row_sum_u32(hit ? 1u : 0u) != 0u || minS >= 32767;
#pragma unroll
        for (int k = 0; k < DPL; k++) srow[p * DPL + k] = (int16_t)S[k];
        const int sm = srow[max(best - 1, 0)], sp = srow[min(best + 1, g.D - 1)];
        const int den = max(sm + sp - 2 * minS, 1);
        const bool use = g.subpix && best > 0 && best < g.D - 1;
        const int d16 = best * 16 + (use ? tdiv_rcp((sm - sp) * 16 + den, 2 * den) : 0) + g.minD * 16;
        const int x1 = 4 * q + r;
        const bool wr = p == 0 && x1 < n;
        const int x = wr ? g.minX1 + x1 : g.W + lane;
        R.bst[x] = (int16_t)(rej ? -1 : best);
        R.mins[x] = (uint16_t)minS;
        R.drow[(wr && !rej) ? x : g.W + lane] = (int16_t)d16;
    }
    row_finish(g, tid, 256, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, out + (size_t)y * out_stride);
}

// N dwords (2N int16) from p
template <int N>
__device__ __forceinline__ void load_dw(const int16_t* p, uint32_t (&w)[N])
{
    if constexpr (N == 1) w[0] = *(const uint32_t*)p;
    else if constexpr (N == 2) { const uint2 t = *(const uint2*)p; w[0] = t.x; w[1] = t.y; }
    else {
#pragma unroll
        for (int c = 0; c < N / 4; c++) {
            const uint4 t = ((const uint4*)p)[c];
            w[4 * c] = t.x; w[4 * c + 1] = t.y; w[4 * c + 2] = t.z; w[4 * c + 3] = t.w;
        }
    }
}

// k_ocv_wta16 in packed u16 pairs for the plain int16 regime (no flagged frame, uniqueness
// ratio < 100), the same rows, lanes and decisions. Every path cost there lies in [0, 32767], so
// OpenCV's S = sat16(sat16(s1) + s2) is min(sum, 32767) in any order: saturating packed i16 adds
// of the loaded dwords. With deficit volumes (EV: L = C' - e, e <= P2 <= 511 <= C') the sum is
// S = min(NDIR * C' - E, 32767) with E = the sum of the NDIR deficits (<= 4088, exact in u16),
// and with C' clamped first to Cc = ceil((32767 + NDIR * P2) / NDIR) (NDIR * Cc <= 36856 in u16)
// the clamp gives the same S: the deficits are summed as raw bytes and bits before any unpacking,
// in an even / odd split of each group of 8 (dword h of a group: (d 4h, d 4h + 2) for the evens,
// (d 4h + 1, d 4h + 3) for the odds), and C' is permuted into that order instead. Entries with
// d >= D are forced to 0xFFFF, above every real S. best and minS from one 16-lane min over
// S << 9 | tie(d); uniqueness as a count (k_ocv_vwta_pk): the number of d with S < T =
// ceil(minS * 100 / (100 - u)) against the count inside {best - 1, best, best + 1}.
#ifndef SGM_OCV_WTA_PK
#define SGM_OCV_WTA_PK 1   // the packed row WTA for the plain int16 regime (0: k_ocv_wta16 everywhere)
#endif
template <int DPL, bool EV>
__device__ __forceinline__ int wta_pk_d(int k, int h)   // d - dl of half h of dword k of a lane
{
    if constexpr (EV) {
        const int gi = k / 4, kk = k % 4;
        return 8 * gi + ((kk & 2) ? 1 : 0) + 4 * (kk & 1) + 2 * h;
    } else {
        return 2 * k + h;
    }
}
template <int DPL, int NDIR, bool EV>
__global__ __launch_bounds__(256) void k_ocv_wta16_pk(const int16_t* __restrict__ vols, size_t vol_elems, Geom g,
                                                      int16_t* __restrict__ out, size_t out_stride,
                                                      const int16_t* __restrict__ Cv)   // C' (EV: deficit planes)
{
    if (ocv_gate_skip<false>(g)) return;
    constexpr int M = DPL / 2;
    static_assert(!EV || DPL == 8 || DPL == 16, "deficit planes: 8 or 16 values per lane");
    constexpr int NG = DPL / 8;                          // EV: groups of 8 per lane
    // raw words per direction: plain M dwords; EV the low-byte dwords, then the bit bytes
    constexpr int NW = EV ? DPL / 4 + 1 : M;
    const bool lanetie = NDIR == 5 && (g.compat & SGM_OCV_LANE_TIE);
    extern __shared__ uint32_t lds_ocv[];
    uint32_t* sl = lds_ocv;                              // 16 lane rows x 16 lanes x M dwords of S
    RowLds R((char*)lds_ocv + (size_t)16 * 16 * DPL * 2, g.W);
    const int tid = threadIdx.x, lane = tid & 63, y = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane >> 4, p = lane & 15;
    R.init(g, tid, 256);
    const bool lane_act = p * DPL < g.D;
    const int dl = lane_act ? p * DPL : 0;
    uint32_t* srow = sl + (w * 4 + r) * 16 * M;
    const int n = g.width1, nq = (n + 3) / 4;
    const size_t row0 = (size_t)y * g.width1 * g.D;
    uint32_t imask[M], tie[M][2];
#pragma unroll
    for (int j = 0; j < M; j++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int d = p * DPL + wta_pk_d<DPL, EV>(j, h);
            tie[j][h] = (uint32_t)wta_tie(d, lanetie, 9);
        }
        const int d0 = p * DPL + wta_pk_d<DPL, EV>(j, 0), d1 = p * DPL + wta_pk_d<DPL, EV>(j, 1);
        imask[j] = (lane_act && d0 < g.D ? 0u : 0xFFFFu) | (lane_act && d1 < g.D ? 0u : 0xFFFF0000u);
    }
    const int kq = 100 - g.uniq;
    const float inv_kq = 1.0f / (float)kq;
    const uint32_t Cc = (uint32_t)((32767 + NDIR * g.P2 + NDIR - 1) / NDIR);
    const uint32_t Cc2 = Cc * 0x10001u;
    const EvLayout el = evol_layout(g);
    // buffer loads with 32-bit byte offsets off wave-uniform descriptors (one per volume slot and
    // one for C'; the launcher's condition: every offset below 2^32), moved by a constant per
    // iteration. Pixel 4q + r; past the last pixel group the loads read the next row or return 0
    // past a range, and the results are never stored.
    const uint32_t vbytes = (uint32_t)min(vol_elems * 2, (size_t)0xFFFFFFFFu);
    __amdgpu_buffer_rsrc_t rsv[NDIR];
#pragma unroll
    for (int s = 0; s < NDIR; s++)
        rsv[s] = __builtin_amdgcn_make_buffer_rsrc((void*)(vols + (size_t)s * vol_elems), 0, (int)vbytes, 0x00020000);
    const uint32_t cbytes = (uint32_t)min((size_t)g.width1 * g.H * g.D * 2, (size_t)0xFFFFFFFFu);
    const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc((void*)Cv, 0, (int)cbytes, 0x00020000);
    const uint32_t px0 = (uint32_t)y * (uint32_t)g.width1 + 4u * (uint32_t)w + (uint32_t)r;
    uint32_t oc = (uint32_t)((row0 + (size_t)(4 * w + r) * g.D + dl) * 2);
    uint32_t olo = EV ? px0 * el.ls + (uint32_t)dl : 0u, ohi = EV ? (uint32_t)el.hb + px0 * el.hs + (uint32_t)dl / 8 : 0u;
    const uint32_t sc = 16u * (uint32_t)g.D * 2u, slo = 16u * el.ls, shi = 16u * el.hs;   // per iteration (4 groups)
    auto load = [&](uint32_t (&c)[M], uint32_t (&v)[NDIR][NW]) {
        bload_dw<M>(rsc, oc, c);
        if constexpr (EV) {
#pragma unroll
            for (int s = 0; s < NDIR; s++) {
                if constexpr (DPL == 8) {
                    const auto t = __builtin_amdgcn_raw_buffer_load_b64(rsv[s], olo, 0, 0);
                    v[s][0] = t[0]; v[s][1] = t[1];
                    v[s][2] = __builtin_amdgcn_raw_buffer_load_b8(rsv[s], ohi, 0, 0);
                } else {
                    const auto t = __builtin_amdgcn_raw_buffer_load_b128(rsv[s], olo, 0, 0);
                    v[s][0] = t[0]; v[s][1] = t[1]; v[s][2] = t[2]; v[s][3] = t[3];
                    v[s][4] = __builtin_amdgcn_raw_buffer_load_b16(rsv[s], ohi, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < NDIR; s++) bload_dw<M>(rsv[s], oc, v[s]);
        }
        oc += sc; olo += slo; ohi += shi;
    };
    uint32_t nc[M], nv[NDIR][NW];
    load(nc, nv);
    for (int q = w; q < nq; q += 4) {
        uint32_t S2[M];
        if constexpr (EV) {
            // the NDIR deficits summed in the split order: low bytes through one perm per dword
            // and half, bit 8 of the evens / odds spread to bytes by one multiply of the nibble
            // (bit i -> bit 8i, the partial products' bits never overlap) and summed as bytes (<= 8)
            uint32_t Alo[M], Hb[2 * NG];
#pragma unroll
            for (int j = 0; j < M; j++) Alo[j] = 0;
#pragma unroll
            for (int j = 0; j < 2 * NG; j++) Hb[j] = 0;
#pragma unroll
            for (int s = 0; s < NDIR; s++) {
#pragma unroll
                for (int gi = 0; gi < NG; gi++) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint32_t wd = nv[s][2 * gi + h];
                        Alo[4 * gi + h] += __builtin_amdgcn_perm(0u, wd, 0x0C020C00u);       // (d 4h, d 4h + 2)
                        Alo[4 * gi + 2 + h] += __builtin_amdgcn_perm(0u, wd, 0x0C030C01u);   // (d 4h + 1, d 4h + 3)
                    }
                    const uint32_t hb = (nv[s][DPL / 4] >> (8 * gi)) & 0xFFu;
                    Hb[2 * gi] += ((hb & 0xFu) * 0x00204081u) & 0x01010101u;   // evens (4 bits: no carries)
                    Hb[2 * gi + 1] += ((hb >> 4) * 0x00204081u) & 0x01010101u;  // odds
                }
            }
#pragma unroll
            for (int gi = 0; gi < NG; gi++) {
                // C' of the group in the split order
                const uint32_t c0 = nc[4 * gi], c1 = nc[4 * gi + 1], c2 = nc[4 * gi + 2], c3 = nc[4 * gi + 3];
                const uint32_t Cs[4] = {__builtin_amdgcn_perm(c1, c0, 0x05040100u), __builtin_amdgcn_perm(c3, c2, 0x05040100u),
                                        __builtin_amdgcn_perm(c1, c0, 0x07060302u), __builtin_amdgcn_perm(c3, c2, 0x07060302u)};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t hb2 = __builtin_amdgcn_perm(0u, Hb[2 * gi + (k >> 1)], (k & 1) ? 0x0C030C02u : 0x0C010C00u);
                    const uint32_t E = Alo[4 * gi + k] + (hb2 << 8);
                    const u16x2_t cm = __builtin_elementwise_min(as_v2(Cs[k]), as_v2(Cc2));
                    const uint32_t s = as_u(cm * (u16x2_t){(unsigned short)NDIR, (unsigned short)NDIR} - as_v2(E));
                    S2[4 * gi + k] = pk_min(s, 0x7FFF7FFFu) | imask[4 * gi + k];
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < M; j++) {
                s16x2_t a = __builtin_bit_cast(s16x2_t, nv[0][j]);
#pragma unroll
                for (int s = 1; s < NDIR; s++) a = __builtin_elementwise_add_sat(a, __builtin_bit_cast(s16x2_t, nv[s][j]));
                S2[j] = __builtin_bit_cast(uint32_t, a) | imask[j];
            }
        }
        load(nc, nv);
        uint32_t km = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < M; j++) {
            const uint32_t klo = ((S2[j] & 0xFFFFu) << 9) | tie[j][0];
            const uint32_t khi = ((S2[j] >> 7) & 0xFFFFFE00u) | tie[j][1];
            km = min(km, min(klo, khi));
        }
        const uint32_t kmin = row_min_u32(km);
        const int best = wta_untie((int)(kmin & 511u), lanetie, 9);
        const int minS = (int)(kmin >> 9);
#pragma unroll
        for (int j = 0; j < M; j++) srow[p * M + j] = S2[j];
        auto s_at = [&](uint32_t d) {                    // S of d from the pixel's LDS slice
            const uint32_t k = d % DPL;
            // EV: u16 index 2j + h of d's half in the split order
            const uint32_t idx = EV ? 8 * (k >> 3) + 4 * (k & 1) + 2 * ((k >> 2) & 1) + ((k >> 1) & 1) : k;
            // read as the u32 it was written as (a u16 view would be an aliasing violation)
            return (int)((srow[(d / DPL) * M + idx / 2] >> (16 * (idx & 1))) & 0xFFFFu);
        };
        const int sm = s_at((uint32_t)max(best - 1, 0)), sp = s_at((uint32_t)min(best + 1, g.D - 1));
        // uniqueness: S * kq < minS * 100 <=> S < T = ceil(minS * 100 / kq) (the quotient from the
        // float reciprocal, then one correction each way; T clamped to 32768 > every real S). Some d
        // outside {best - 1, best, best + 1} qualifies iff the sum of max(T - S, 0) over the pixel
        // exceeds the window's share (census wta_pix16's test; d >= D hold 0xFFFF: no share)
        const int num = minS * 100 + kq - 1;
        int T = (int)((float)num * inv_kq);
        T += (T + 1) * kq <= num ? 1 : 0;
        T -= T * kq > num ? 1 : 0;
        T = min(T, 32768);
        const uint32_t T2 = (uint32_t)T * 0x10001u;
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < M; j++) acc = __builtin_amdgcn_sad_u16(as_u(__builtin_elementwise_sub_sat(as_v2(T2), as_v2(S2[j]))), 0u, acc);
        const int total = (int)row_sum_u32(acc);
        const int win = max(T - minS, 0) + (best > 0 ? max(T - sm, 0) : 0) + (best < g.D - 1 ? max(T - sp, 0) : 0);
        const bool rej = total > win || minS >= 32767;
        // subpixel, branch-free (tdiv_rcp's C truncation with both corrections as selects)
        const int den = max(sm + sp - 2 * minS, 1);
        const bool use = g.subpix && best > 0 && best < g.D - 1;
        const int sn = (sm - sp) * 16 + den, sd = 2 * den;
        int sq = (int)__builtin_truncf((float)sn * __builtin_amdgcn_rcpf((float)sd));
        const int sr = sn - sq * sd;
        sq += sn >= 0 ? (sr >= sd ? 1 : (sr < 0 ? -1 : 0)) : (sr <= -sd ? -1 : (sr > 0 ? 1 : 0));
        const int d16 = best * 16 + (use ? sq : 0) + g.minD * 16;
        const int x1 = 4 * q + r;
        const bool wr = p == 0 && x1 < n;
        const int x = wr ? g.minX1 + x1 : g.W + lane;
        R.bst[x] = (int16_t)(rej ? -1 : best);
        R.mins[x] = (uint16_t)minS;
        R.drow[(wr && !rej) ? x : g.W + lane] = (int16_t)d16;
    }
    row_finish(g, tid, 256, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, out + (size_t)y * out_stride);
}

// WTA of the OCV modes for D > 512 (the node's cfg allows disparity ranges up to 2048):
// one pixel per wave, 64 lanes x 16 disparities per chunk of 1024, chunks in turn. Pass 1
// sums S (OpenCV's saturating order), keeps the key min over (S + 32768) * 2048 + d and
// stores S in the wave's LDS slice; pass 2 reads the slice for the uniqueness test and
// S[best +- 1]. Same decisions and the same disp2 / LR epilogue as k_ocv_wta16.
constexpr int kWta64Chunk = 1024;
template <int NDIR, typename VT, bool SAT>
__global__ __launch_bounds__(256) void k_ocv_wta64(const VT* __restrict__ vols, size_t vol_elems, Geom g,
                                                   int16_t* __restrict__ out, size_t out_stride)
{
    if (ocv_gate_skip<SAT || sizeof(VT) == 4>(g)) return;
    const bool lanetie = NDIR == 5 && (g.compat & SGM_OCV_LANE_TIE);
    constexpr int DPL = kWta64Chunk / 64;
    extern __shared__ uint32_t lds_ocv[];
    const int Dpad = (g.D + kWta64Chunk - 1) / kWta64Chunk * kWta64Chunk;
    const int tid = threadIdx.x, lane = tid & 63, y = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int16_t* srow = (int16_t*)lds_ocv + (size_t)w * Dpad;   // this wave's S slice
    RowLds R((char*)lds_ocv + (size_t)4 * Dpad * 2, g.W);
    R.init(g, tid, 256);
    const int n = g.width1;
    const size_t row0 = (size_t)y * g.width1 * g.D;
    for (int x1 = w; x1 < n; x1 += 4) {
        int km = 0x7FFFFFFF;
        for (int c0 = 0; c0 < g.D; c0 += kWta64Chunk) {
            const int db = c0 + lane * DPL;
            const bool act = db < g.D;
            const VT* base = vols + row0 + (size_t)x1 * g.D + (act ? db : 0);
            int v[NDIR][DPL];
#pragma unroll
            for (int k = 0; k < NDIR; k++) load_vals<VT, DPL>(base + (size_t)k * vol_elems, v[k]);
#pragma unroll
            for (int k = 0; k < DPL; k++) {
                const int S = ocv_sum<NDIR, SAT>(v, k);
                const int d = db + k;
                const int key = ((S + 32768) << 11) | wta_tie(d, lanetie, 11);
                km = (act && d < g.D) ? min(km, key) : km;
                if (act) srow[d] = (int16_t)S;
            }
        }
        const int kmin = wave_min(km);
        const int best = wta_untie(kmin & 2047, lanetie, 11);
        const int minS = (kmin >> 11) - 32768;
        bool hit = false;
        for (int d = lane; d < g.D; d += 64)
            hit |= (unsigned)(d - best + 1) > 2u && (int)srow[d] * (100 - g.uniq) < minS * 100;
        // every S saturated at MAX_COST: OpenCV's bestDisp stays -1 (see k_ocv_wta16)
        const bool rej = __ballot(hit) != 0ull || minS >= 32767;
        const int sm = srow[max(best - 1, 0)], sp = srow[min(best + 1, g.D - 1)];
        const int den = max(sm + sp - 2 * minS, 1);
        const bool use = g.subpix && best > 0 && best < g.D - 1;
        const int d16 = best * 16 + (use ? tdiv_rcp((sm - sp) * 16 + den, 2 * den) : 0) + g.minD * 16;
        const bool wr = lane == 0;
        const int x = wr ? g.minX1 + x1 : g.W + lane;
        R.bst[x] = (int16_t)(rej ? -1 : best);
        R.mins[x] = (uint16_t)minS;
        R.drow[(wr && !rej) ? x : g.W + lane] = (int16_t)d16;
    }
    row_finish(g, tid, 256, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, out + (size_t)y * out_stride);
}

// The vertical path of OpenCV's last group fused with the WTA (`k_ocv_vwta`): MODE_SGBM's ↓
// (dir 0, volume slot 0) or MODE_HH's ↑ (dir 1, slot 1, in pass 2) runs after the other
// directions' volumes are complete. Each wave is one column, its 64 lanes holding the D
// disparities (the WTA's pixel layout), so at every step the wave has L of pixel (x, y) in
// registers: it loads the other NDIR - 1 path costs of (x, y), sums S in OpenCV's saturating
// order (ocv_sum, with its own values in their slot) and runs the pixel's WTA (the decisions of
// k_ocv_wta16: key-min over (S + 32768) << 11 | tie(d), per-element uniqueness, S[best +- 1]
// by readlane). That volume is never written or read: 4 B per cell less for
// int16 volumes. Per-pixel results (d16 | best << 16 | minS << 32, rejected: d16 = invalid,
// best = -1) go to res; k_census_rowfin finishes the rows (disp2 + LR, the shared row_finish).
// A column is a sequential chain of H steps and there are only width1 of them, so this pays
// on tall frames with many columns (the shipped 2448x2048 config), not on small ones.
template <int DPL, int NDIR, typename VT, bool SAT, bool EV>
__global__ __launch_bounds__(64) void k_ocv_vwta(const int16_t* __restrict__ C, const VT* __restrict__ vols,
                                                 size_t vol_elems, Geom g, uint64_t* __restrict__ res, int use_pk)
{
    if (ocv_gate_skip<SAT || sizeof(VT) == 4>(g)) return;
    constexpr int LPL = 64;                            // one column per wave: the line is the wave
    constexpr int F = NDIR == 5 ? 0 : 1;               // the fused direction = its volume slot
    constexpr bool kRaw = sizeof(VT) == 4;             // the volumes hold the int path costs
    // steps whose operands are in flight (fewer for wide lanes: the register file)
    constexpr int PF = DPL <= 8 ? SGM_OCV_VWTA_PF : DPL == 16 ? 2 : 1;
    const int p = threadIdx.x;
    const int x1 = blockIdx.x;
    const bool lanetie = NDIR == 5 && (g.compat & SGM_OCV_LANE_TIE);
    const bool lane_act = p * DPL < g.D;
    const int dl = lane_act ? p * DPL : g.D - DPL;     // lanes past D load the last group
    auto cell = [&](int i) -> size_t {                 // cell of step i (clamped: prefetch past the end)
        const int y = F == 0 ? min(i, g.H - 1) : max(g.H - 1 - i, 0);
        return ((size_t)y * g.width1 + x1) * g.D + dl;
    };
    auto load = [&](int i, int (&c)[DPL], int (&v)[NDIR][DPL]) {
        int16_t t[DPL];
        const size_t ci = cell(i);
        const EvLayout el = evol_layout(g);
        const size_t px = (size_t)(F == 0 ? min(i, g.H - 1) : max(g.H - 1 - i, 0)) * g.width1 + x1;
        load_i16<DPL>(C + ci, t);
#pragma unroll
        for (int k = 0; k < DPL; k++) c[k] = t[k];
#pragma unroll
        for (int s = 0; s < NDIR; s++) {
            if (s == F) continue;
            if constexpr (EV) {                          // L = C' - e (deficit planes)
                const uint8_t* vb = (const uint8_t*)(vols + (size_t)s * vol_elems);
                int e[DPL];
                load_e<DPL>(vb + px * el.ls + dl, vb + el.hb + px * el.hs + dl / 8, dl, e);
#pragma unroll
                for (int k = 0; k < DPL; k++) v[s][k] = c[k] - e[k];
            } else {
                load_vals<VT, DPL>(vols + (size_t)s * vol_elems + ci, v[s]);
            }
        }
    };
    int Lp[DPL], mLp = 0, Cq[PF][DPL], Vq[PF][NDIR][DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) Lp[k] = kMaxCost;
    // the plain int16 regime: the recurrence in packed u16 pairs (ocv_step_pk), the WTA on ints
    // (DPL >= 8 only: the shipped D=480 config 3.55 -> 3.48 ms, while 1080p D=128 MODE_HH, DPL = 2,
    // measured 0.87 -> 0.93 ms; profiles/r05_ocv_pk_ab.jsonl)
    constexpr bool kPk = !SAT && sizeof(VT) == 2 && DPL >= 8 && SGM_OCV_PK != 0;
    constexpr int M2 = DPL >= 2 ? DPL / 2 : 1;
    uint32_t L2[M2], imask2[M2], delta2 = (uint32_t)g.P2 * 0x10001u;
    const uint32_t P1P1 = (uint32_t)g.P1 * 0x10001u;
#pragma unroll
    for (int i = 0; i < M2; i++) {
        L2[i] = 0;
        imask2[i] = (p * DPL + 2 * i < g.D ? 0u : 0xFFFFu) | (p * DPL + 2 * i + 1 < g.D ? 0u : 0xFFFF0000u);
    }
#pragma unroll
    for (int q = 0; q < PF; q++) load(q, Cq[q], Vq[q]);
    // step i: the recurrence (a chain through mLp), then the pixel's WTA, which no later step
    // waits for: S[best +- 1] come from a readlane (best is wave-uniform), so no LDS barrier
    // orders the steps and the WTA of one step overlaps the recurrence of the next
    auto step = [&](int i, int (&Cc)[DPL], int (&V)[NDIR][DPL]) {
        bool done = false;
        if constexpr (kPk) {
            if (use_pk) {                              // (the path's first pixel: L2 = 0, delta = P2)
                uint32_t C2[M2];
#pragma unroll
                for (int j = 0; j < M2; j++) C2[j] = ((uint32_t)Cc[2 * j] & 0xFFFFu) | ((uint32_t)Cc[2 * j + 1] << 16);
                const uint32_t lmin = ocv_step_pk<DPL, LPL>(C2, L2, delta2, P1P1, imask2, p);
                delta2 = ((uint32_t)line_min_i32<LPL>((int)lmin) + (uint32_t)g.P2) * 0x10001u;
#pragma unroll
                for (int j = 0; j < M2; j++) {
                    V[F][2 * j] = (int)(L2[j] & 0xFFFFu);
                    V[F][2 * j + 1] = (int)(L2[j] >> 16);
                }
                done = true;
            }
        }
        if (!done) {
            int L[DPL], Lraw[DPL];
            const int lmin = ocv_step<DPL, LPL, SAT>(Cc, Lp, mLp, i > 0, p, g, L, Lraw);
            mLp = (int)(int16_t)line_min_i32<LPL>(lmin);   // minLr is CostType
#pragma unroll
            for (int k = 0; k < DPL; k++) {
                Lp[k] = L[k];
                V[F][k] = kRaw ? Lraw[k] : L[k];           // what the volume would have held
            }
        }
        int S[DPL];
        int km = 0x7FFFFFFF;                           // keys < 2^27: signed min
#pragma unroll
        for (int k = 0; k < DPL; k++) {
            S[k] = ocv_sum<NDIR, SAT>(V, k);
            const int d = p * DPL + k;
            const int key = ((S[k] + 32768) << 11) | wta_tie(d, lanetie, 11);
            km = (lane_act && d < g.D) ? min(km, key) : km;
        }
        const int kmin = __builtin_amdgcn_readfirstlane(line_min_i32<LPL>(km));
        const int best = wta_untie(kmin & 2047, lanetie, 11);
        const int minS = (kmin >> 11) - 32768;
#if SGM_OCV_VWTA_THR
        // uniqueness: S * (100 - u) < minS * 100 is S < T = ceil(minS * 100 / (100 - u)) for
        // u < 100 (one uniform threshold instead of a multiply per value)
        bool hit = false;
        if (g.uniq < 100) {
            const int M = minS * 100, kq = 100 - g.uniq;
            int T = (int)__builtin_ceilf((float)M / (float)kq);
            T -= (T - 1) * kq >= M ? 1 : 0;
            T += T * kq < M ? 1 : 0;
#pragma unroll
            for (int k = 0; k < DPL; k++) {
                const int d = p * DPL + k;
                hit |= lane_act && d < g.D && (unsigned)(d - best + 1) > 2u && S[k] < T;
            }
        } else {
#pragma unroll
            for (int k = 0; k < DPL; k++) {
                const int d = p * DPL + k;
                hit |= lane_act && d < g.D && (unsigned)(d - best + 1) > 2u && S[k] * (100 - g.uniq) < minS * 100;
            }
        }
#else
        bool hit = false;
#pragma unroll
        for (int k = 0; k < DPL; k++) {
            const int d = p * DPL + k;
            hit |= lane_act && d < g.D && (unsigned)(d - best + 1) > 2u && S[k] * (100 - g.uniq) < minS * 100;
        }
#endif
        // every S saturated at MAX_COST: bestDisp stays -1 in OpenCV (see k_ocv_wta16)
        const bool rej = __ballot(hit) != 0ull || minS >= 32767;
        auto s_at = [&](int d) {                       // S[d] of the pixel (d wave-uniform)
            const int kk = d % DPL, ln = d / DPL;
#if SGM_OCV_VWTA_RL
            // one readlane per element, the element picked among the scalars: a select over the
            // S registers themselves is folded into an indexed load, which puts S in LDS
            int v = __builtin_amdgcn_readlane(S[0], ln);
#pragma unroll
            for (int k = 1; k < DPL; k++) {
                const int r = __builtin_amdgcn_readlane(S[k], ln);
                v = kk == k ? r : v;
            }
            return v;
#else
            int v = S[0];
#pragma unroll
            for (int k = 1; k < DPL; k++) v = kk == k ? S[k] : v;
            return __builtin_amdgcn_readlane(v, ln);
#endif
        };
        const int sm = s_at(max(best - 1, 0)), sp = s_at(min(best + 1, g.D - 1));
        const int den = max(sm + sp - 2 * minS, 1);
        const bool use = g.subpix && best > 0 && best < g.D - 1;
        const int d16 = best * 16 + (use ? tdiv_rcp((sm - sp) * 16 + den, 2 * den) : 0) + g.minD * 16;
        const int y = F == 0 ? i : g.H - 1 - i;
        const uint64_t v = (uint64_t)(uint16_t)(rej ? g.invalid : d16) |
                           ((uint64_t)(uint16_t)(rej ? -1 : best) << 16) | ((uint64_t)(uint16_t)minS << 32);
        if (p == 0 && i < g.H) __builtin_nontemporal_store(v, res + (size_t)y * g.W + g.minX1 + x1);
    };
    for (int i0 = 0; i0 < g.H; i0 += PF) {
#pragma unroll
        for (int q = 0; q < PF; q++) {
            int Cc[DPL], V[NDIR][DPL];
#pragma unroll
            for (int k = 0; k < DPL; k++) {
                Cc[k] = Cq[q][k];
#pragma unroll
                for (int s = 0; s < NDIR; s++) V[s][k] = Vq[q][s][k];
            }
            load(i0 + q + PF, Cq[q], Vq[q]);           // operands of step i + PF
            step(i0 + q, Cc, V);
        }
    }
}

// ------------------------------------------------------------------------------------
static int dpl_for(int D) { return D <= 16 ? 1 : D <= 32 ? 2 : D <= 64 ? 4 : D <= 128 ? 8 : D <= 256 ? 16 : 32; }

// C' of the frame into bufA (bufB: scratch, the horizontal sums). SIMD_SAT frames that take
// the flagged kernels (Geom::wide != 0 and the overflow flag) get the exact SIMD cost written
// over it, by kernels that return at once on the other frames: the vertical SIMD update over
// the plain horizontal sums (k_ocv_vsum_sat2) when those cannot saturate, else the sequential
// chain (pixel costs -> bufA, horizontal sums -> bufB, C' -> bufA).
// Disparity pairs per block row (DC = 2 * DPC disparities): 32 only for R <= 9 (its I = 8
// pairs per thread keep 8 R-slot rings in registers), else 16, or 8 (I = 2: 95 VGPRs at R = 21
// against 165 for 16, i.e. two blocks per CU instead of one); SGM_FUSE_DPC forces one.
static int fuse_dpc(const Geom& g)
{
    const int R = 2 * g.SH2 + 1;
    // D % 32 == 16 from D = 256 on: 16 pairs with a half-empty last chunk (<= 6 % of the pixel-cost
    // work wasted) beat 8 pairs, whose blocks stage the same BT rows for half the disparities (the
    // processing launch's D = 752 block 21: profiles/r06_ocv_cost_dpc_ab.jsonl)
    int dpc = (R <= 9 && g.D % 64 == 0) ? 32 : (g.D % 32 == 0 || (g.D >= 256 && SGM_FUSE_DPC16_PART)) ? 16 : 8;
    if (const char* e = std::getenv("SGM_FUSE_DPC")) {
        const int f = std::atoi(e);
        if ((f == 32 && R <= 9 && g.D % 64 == 0) || f == 16 || f == 8) dpc = f;
    }
    return dpc;
}

// The overflow flag's tracking (k_ocv_cost_fused's TRK): none without the gate (Geom::wide != 2);
// the max of C' when box + P2 stays below 2^16 for any pixels (a pixel cost is <= 2*ftzero + 63),
// so the slid sum that starts at P2 is compared as it is stored; else the max of C' - P2
static int ocv_fuse_track(const Geom& g)
{
    if (g.wide != 2) return 0;
    const long long B = (long long)(2 * g.SW2 + 1) * (2 * g.SH2 + 1) * (2 * g.ftzero + 63);
    return B + g.P2 <= 65535 ? 1 : 2;
}

template <int R, int TRK>
static void launch_cost_fused_rt(const uint32_t* bt, const Geom& g, int fullDP, const FuseGrid& fg, int16_t* C,
                                 hipStream_t st)
{
    const dim3 grid(fg.per_xcd * 8), block(kFuseThreads);
    const int dpc = fuse_dpc(g);
    if constexpr (R <= 9) {
        if (dpc == 32) {
            hipLaunchKernelGGL((k_ocv_cost_fused<R, 32, 8, TRK>), grid, block, FuseGeo(32).lds_bytes(32, fuse_rb(R), R), st, bt, g,
                               fullDP, fg, C);
            return;
        }
    }
    // blocks above 64 KB of LDS (R > 9: two rows per barrier plus ring slot 0) ask for it
    auto allow = [](const void* k, size_t lds) {
        if (lds > 65536) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    };
    if (dpc == 16) {
        const size_t lds = FuseGeo(16).lds_bytes(16, fuse_rb(R), R);
        allow(reinterpret_cast<const void*>(&k_ocv_cost_fused<R, 16, 4, TRK>), lds);
        hipLaunchKernelGGL((k_ocv_cost_fused<R, 16, 4, TRK>), grid, block, lds, st, bt, g, fullDP, fg, C);
    } else {
        const size_t lds = FuseGeo(8).lds_bytes(8, fuse_rb(R), R);
        allow(reinterpret_cast<const void*>(&k_ocv_cost_fused<R, 8, 2, TRK>), lds);
        hipLaunchKernelGGL((k_ocv_cost_fused<R, 8, 2, TRK>), grid, block, lds, st, bt, g, fullDP, fg, C);
    }
}

template <int R>
static void launch_cost_fused_r(const uint32_t* bt, const Geom& g, int fullDP, const FuseGrid& fg, int16_t* C,
                                hipStream_t st)
{
    switch (ocv_fuse_track(g)) {
    case 0: launch_cost_fused_rt<R, 0>(bt, g, fullDP, fg, C, st); break;
    case 1: launch_cost_fused_rt<R, 1>(bt, g, fullDP, fg, C, st); break;
    default: launch_cost_fused_rt<R, 2>(bt, g, fullDP, fg, C, st); break;
    }
}

static FuseGrid fuse_grid(const Geom& g)
{
    FuseGrid fg{};
    const int dpc = fuse_dpc(g);
    const int XB = fuse_xb(g);
    fg.strips = (g.width1 + XB - 1) / XB;
    fg.chunks = (g.D + 2 * dpc - 1) / (2 * dpc);   // the last one partly past D when 2 * dpc does not divide D
    fg.ncomp = std::max(g.H - g.SH2 - 1, 0) + 1;             // rows 0 .. ylast are computed
    const long long tiles = (long long)fg.strips * fg.chunks;
    // bands: about four rounds of blocks over the chip's slots (two 512-thread blocks per CU, every
    // instantiation at <= 128 VGPRs), bands of about max(64, 8*SH2) rows or more so the 2*SH2
    // warm-up rows stay a small share. Measured (profiles/r04_ocv_cost_rows_ab.jsonl): the shipped block-21
    // config 2.43 ms at the earlier ~ncomp*tiles/1024 rows (507: 1275 blocks, 2.5 rounds) against
    // 2.06 at 256 rows (2040 blocks), 2.10-2.11 at 128-160; 1080p block 5 best at 64 rows
    // slot count of the calling thread's current device, cached per device (launches run from
    // several host threads at once: per-device atomics, each written with the same value)
    static std::atomic<int> slots_of[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    int slots = dev < 64 ? slots_of[dev].load(std::memory_order_relaxed) : 0;
    if (!slots) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        slots = (2 * 128 / kFuseNX) * cus;             // 512-thread blocks: two per CU
        if (dev < 64) slots_of[dev].store(slots, std::memory_order_relaxed);
    }
    const int min_rows = std::max(64, 8 * g.SH2);
    const long long nb = std::max<long long>(1, std::min<long long>((4LL * slots + tiles / 2) / std::max(tiles, 1LL),
                                                                    (fg.ncomp + min_rows - 1) / min_rows));
    const char* e = std::getenv("SGM_FUSE_ROWS");
    fg.band_rows = e ? std::max(std::atoi(e), 1) : (int)((fg.ncomp + nb - 1) / nb);
    fg.bands = (fg.ncomp + fg.band_rows - 1) / fg.band_rows;
    fg.total = (int)(tiles * fg.bands);
    fg.per_xcd = (fg.total + 7) / 8;
    return fg;
}

// C' of the frame into bufA (bufB: scratch, the horizontal sums of the unfused kernels).
// Default: k_ocv_prefilter (with the BT planes) + k_ocv_cost_fused (+ k_ocv_col0_legacy) when ocv_cost_fusable, else
// k_ocv_pixhsum (or k_ocv_pixcost + k_ocv_hsum) + k_ocv_vsum_seg. SIMD_SAT frames that take the
// flagged kernels (Geom::wide != 0 and the overflow flag) get the exact SIMD cost written over
// it, by kernels that return at once on the other frames: the vertical SIMD update over the
// plain horizontal sums (k_ocv_vsum_sat2; after the fused cost, a gated k_ocv_pixhsum makes
// those sums first) when the horizontal sums cannot saturate, else the sequential chain
// (pixel costs -> bufA, horizontal sums -> bufB, C' -> bufA).
// The frame's cost stage takes k_ocv_cost_fused (and so reads the packed BT planes after the
// prefilter planes): the workspace layout reserves those 16 B/px only then.
// wide == 1 with SIMD_SAT: every launch after the cost reads the SIMD cost, the plain C' is never used.
bool ocv_cost_takes_fused(const Geom& g)
{
    const bool simd_only = g.wide == 1 && (g.compat & SGM_OCV_SIMD_SAT);
    return !simd_only && ocv_cost_fusable(g);
}

hipError_t launch_ocv_cost(const uint8_t* L, const uint8_t* R, size_t stride, const Geom& g, int fullDP,
                           uint8_t* planes, int16_t* bufA, int16_t* bufB, hipStream_t st)
{
    const size_t lds = pix_lds_bytes(g);
    const bool simd_only = g.wide == 1 && (g.compat & SGM_OCV_SIMD_SAT);
    const bool fused = ocv_cost_takes_fused(g);
    uint32_t* bt = fused ? (uint32_t*)(planes + ocv_planes_bytes(g.W, g.H)) : nullptr;
    hipLaunchKernelGGL(k_ocv_prefilter, dim3((g.W + 1023) / 1024, g.H, 2), dim3(256), 0, st, L, R, stride, g.W, g.H,
                       g.ftzero, planes, bt);
    const bool sat2 = g.wide && (g.compat & SGM_OCV_SIMD_SAT) && ocv_hsum_cannot_saturate(g) && lds <= 64 * 1024 &&
                      (size_t)(2 * g.SH2 + 1) * 256 * 4 <= 64 * 1024 && !std::getenv("SGM_OCV_SAT_SEQ");
    if (simd_only) {
        if (sat2) {                    // the horizontal sums for k_ocv_vsum_sat2
            const int XB = pix_xb(g), DC = pix_dc(g);
            hipLaunchKernelGGL(k_ocv_pixhsum<true>, dim3((g.width1 + XB - 1) / XB, g.H, (g.D + DC - 1) / DC), dim3(256),
                               lds, st, planes, g, bufB);
        }
    } else if (fused) {
        const FuseGrid fg = fuse_grid(g);
        switch (g.SH2) {
        case 0: launch_cost_fused_r<1>(bt, g, fullDP, fg, bufA, st); break;
        case 1: launch_cost_fused_r<3>(bt, g, fullDP, fg, bufA, st); break;
        case 2: launch_cost_fused_r<5>(bt, g, fullDP, fg, bufA, st); break;
        case 3: launch_cost_fused_r<7>(bt, g, fullDP, fg, bufA, st); break;
        case 4: launch_cost_fused_r<9>(bt, g, fullDP, fg, bufA, st); break;
        case 5: launch_cost_fused_r<11>(bt, g, fullDP, fg, bufA, st); break;
        case 6: launch_cost_fused_r<13>(bt, g, fullDP, fg, bufA, st); break;
        case 7: launch_cost_fused_r<15>(bt, g, fullDP, fg, bufA, st); break;
        case 8: launch_cost_fused_r<17>(bt, g, fullDP, fg, bufA, st); break;
        case 9: launch_cost_fused_r<19>(bt, g, fullDP, fg, bufA, st); break;
        default: launch_cost_fused_r<21>(bt, g, fullDP, fg, bufA, st); break;
        }
        if ((g.compat & SGM_OCV_COL0_LEGACY) && g.H > 1)
            hipLaunchKernelGGL(k_ocv_col0_legacy, dim3(((g.H - 1) * (g.D / 2) + 255) / 256), dim3(256), 0, st, g, fullDP,
                               bufA);
        if (sat2) {                    // the flagged frames' horizontal sums for k_ocv_vsum_sat2
            const int XB = pix_xb(g), DC = pix_dc(g);
            hipLaunchKernelGGL(k_ocv_pixhsum<true>, dim3((g.width1 + XB - 1) / XB, g.H, (g.D + DC - 1) / DC), dim3(256),
                               lds, st, planes, g, bufB);
        }
    } else {
        if (lds <= 64 * 1024) {
            const int XB = pix_xb(g), DC = pix_dc(g);
            hipLaunchKernelGGL(k_ocv_pixhsum<false>, dim3((g.width1 + XB - 1) / XB, g.H, (g.D + DC - 1) / DC), dim3(256),
                               lds, st, planes, g, bufB);
        } else {            // very wide boxes x wide ranges: the unfused pair (no LDS staging)
            hipLaunchKernelGGL(k_ocv_pixcost, dim3(g.width1, g.H), dim3(256), 0, st, planes, g, bufA);
            hipLaunchKernelGGL(k_ocv_hsum, dim3((g.D + 255) / 256, g.H), dim3(256), 0, st, bufA, g, bufB);
        }
        hipLaunchKernelGGL(k_ocv_vsum_seg, dim3((g.width1 * g.D / 2 + 255) / 256, (g.H + kVsumRows - 1) / kVsumRows),
                           dim3(256), 0, st, bufB, g, fullDP, bufA);
    }
    if (g.wide && (g.compat & SGM_OCV_SIMD_SAT)) {
        const size_t rc = (size_t)g.width1 * g.D;
        if (sat2) {
            const size_t ring = (size_t)(2 * g.SH2 + 1) * 256 * 4;
            const dim3 grid((unsigned)((rc / 2 + 255) / 256));
            switch (vsum_sat2_unroll(g)) {
            case 8: hipLaunchKernelGGL(k_ocv_vsum_sat2<8>, grid, dim3(256), ring, st, bufB, g, fullDP, bufA); break;
            case 4: hipLaunchKernelGGL(k_ocv_vsum_sat2<4>, grid, dim3(256), ring, st, bufB, g, fullDP, bufA); break;
            case 2: hipLaunchKernelGGL(k_ocv_vsum_sat2<2>, grid, dim3(256), ring, st, bufB, g, fullDP, bufA); break;
            default: hipLaunchKernelGGL(k_ocv_vsum_sat2<1>, grid, dim3(256), ring, st, bufB, g, fullDP, bufA); break;
            }
        } else {
            hipLaunchKernelGGL(k_ocv_pixcost_sat, dim3(std::min(g.width1 * g.H, 8192)), dim3(256), 0, st, planes, g, bufA);
            hipLaunchKernelGGL(k_ocv_hsum_sat, dim3((g.D + 255) / 256, g.H), dim3(256), 0, st, bufA, g, bufB);
            hipLaunchKernelGGL(k_ocv_vsum_sat, dim3((unsigned)((rc + 255) / 256)), dim3(256), 0, st, bufB, g, fullDP, bufA);
        }
    }
    return hipGetLastError();
}

// vols: the direction volumes (vol_elems apart) followed by >= 64 * 32 VT of trash slots
// skipdir >= 0: that direction keeps its volume slot but launches no blocks (k_ocv_vwta runs it)
template <int DPL, int LPL, typename VT, bool SAT>
static hipError_t launch_ocv_paths_l(const int16_t* C, void* vols_, size_t cells, const Geom& g, int dirmask,
                               hipStream_t st, int skipdir)
{
    VT* vols = (VT*)vols_;
    const size_t vol_elems = ocv_vol_elems(cells, sizeof(VT));
    int ndir = 0;
    for (int i = 0; i < 8; i++) ndir += (dirmask >> i) & 1;
    const size_t trash_off = (size_t)ndir * vol_elems;
    int nb[8], total = 0, nact = 0, nbmax = 0;
    for (int i = 0; i < 8; i++) {
        nb[i] = 0;
        if (!((dirmask >> i) & 1)) continue;
        const int lines = dir_ry(i) == 0 ? g.H : g.width1 + (dir_rx(i) != 0 ? g.H - 1 : 0);
        nb[i] = i == skipdir ? 0 : (lines + 64 / LPL - 1) / (64 / LPL);
        total += nb[i];
        nact += nb[i] > 0;
        nbmax = std::max(nbmax, nb[i]);
    }
    // directions dealt round-robin for 64-lane lines (one line per wave, D > 256): the diagonal
    // lines that start on the top row together read each C' row at about the same time, the
    // second read served by the caches (the shipped 2448x2048 D=480 MODE_SGBM paths 5.30 -> 4.16 ms,
    // MODE_HH 9.78 -> 9.57; 1080p D=128, 16-lane lines: 0.81 -> 0.83 and 1.16 -> 1.22, so not there;
    // profiles/r05_ocv_ilv_ab.jsonl). SGM_OCV_ILV=0 / 1 forces it.
    const char* ie = getenv("SGM_OCV_ILV");
    const int ilv = (ie ? atoi(ie) != 0 : SGM_OCV_ILV != 0 && LPL == 64) && nact > 1;
    if (ilv) total = nact * nbmax;
    const int4 a = make_int4(nb[0], nb[1], nb[2], nb[3]), b = make_int4(nb[4], nb[5], nb[6], nb[7]);
    // 32-bit buffer offsets when a volume ends below kBufDrop (the shipped 2448x2048 D=480
    // config's int16 volumes are 3.6 GB; SGM_OCV_NO_BUF=1 forces the 64-bit path)
    const int use_buf = (size_t)g.width1 * g.H * g.D * sizeof(VT) < (size_t)kBufDrop && !getenv("SGM_OCV_NO_BUF");
    // packed u16 recurrence: the plain int16 regime with P1, P2 <= 32768 (SGM_OCV_PK=0 at build time: ints)
    const int use_pk = SGM_OCV_PK != 0 && !SAT && sizeof(VT) == 2 && g.P1 <= 32768 && g.P2 <= 32768;
    // the plain kernel writes deficit records only on its packed branch (8 or 16 values per lane,
    // buffer offsets or 64-lane rebased descriptors); ocv_evol_mode decided g.evol from the same conditions, and the WTA reads
    // deficits whenever it is set: refuse a frame where the two disagree rather than hand the WTA
    // int16 L volumes it would read as deficits (flagged kernels ignore evol and write full volumes)
    if (!SAT && sizeof(VT) == 2 && g.evol &&
        !((DPL == 8 || DPL == 16) && use_pk && (use_buf || LPL == 64 || (LPL == 32 && DPL == 8))))
        return hipErrorInvalidValue;
    if (total <= 0) return hipSuccess;
    if constexpr ((LPL == 64 || LPL == 32) && DPL == 8 && !SAT && sizeof(VT) == 2) {
        if (!use_buf && use_pk) {     // volumes past 4 GB: the rebased packed form (k_ocv_paths REBK)
            hipLaunchKernelGGL((k_ocv_paths<DPL, LPL, VT, SAT, true>), dim3(total), dim3(64), 0, st, C, vols, vol_elems,
                               trash_off, g, dirmask, a, b, use_buf, use_pk, ilv);
            return hipSuccess;
        }
    }
    hipLaunchKernelGGL((k_ocv_paths<DPL, LPL, VT, SAT>), dim3(total), dim3(64), 0, st, C, vols, vol_elems, trash_off, g,
                       dirmask, a, b, use_buf, use_pk, ilv);
    return hipSuccess;
}

// the plain kernels (wide != 1) and the flagged ones (wide != 0): int32 volumes for the scalar
// branch, saturating int16 over the SIMD cost (Csat) for SIMD_SAT; with wide == 2 the one not
// matching the frame's flag exits at once
template <int DPL, int LPL>
static hipError_t launch_ocv_paths_v(const int16_t* C, const int16_t* Csat, void* vols, size_t cells, const Geom& g,
                                     int dirmask, hipStream_t st, int skipdir)
{
    if (g.wide != 1) {
        const hipError_t e = launch_ocv_paths_l<DPL, LPL, int16_t, false>(C, vols, cells, g, dirmask, st, skipdir);
        if (e != hipSuccess) return e;
    }
    if (g.wide == 0) return hipSuccess;
    if (g.compat & SGM_OCV_SIMD_SAT) return launch_ocv_paths_l<DPL, LPL, int16_t, true>(Csat, vols, cells, g, dirmask, st, skipdir);
    return launch_ocv_paths_l<DPL, LPL, int32_t, false>(C, vols, cells, g, dirmask, st, skipdir);
}

// Lanes per path line. A line is a sequential walk, so a launch with few lines is bound by
// the latency of one step: 32 lanes halve the step's chain (D/32 cells per lane) at the
// cost of a permlane16_swap and two masks per step. With enough lines to fill the SIMDs
// the 16-lane step, fewer instructions per cell, wins (MI355X: C1 640x480 D=64 0.36 vs
// 0.39-0.42 ms per frame; 1920x1080 D=128 3.24 vs 2.85 ms). SGM_OCV_LPL=16|32 forces one.
constexpr int kOcvWideLineWaves = 1536;     // 16-lane waves below which 32 lanes pay
#ifndef SGM_OCV_LPL_MID
#define SGM_OCV_LPL_MID 64                  // lanes per line for 256 < D <= 512 (32 or 64: the shipped D=480
                                            // MODE_SGBM paths 5.96 -> 5.63 ms, MODE_HH 11.2 -> 10.0, profiles/r05_ocv_lpl64_ab.jsonl)
#endif
// fused_v: the frame's vertical direction runs in the fused vertical WTA (skipdir >= 0)
static int ocv_lanes_per_line(const Geom& g, int dirmask, bool fused_v)
{
    if (g.D <= 32) return 16;
    if (g.D > 512) return 64;       // a line per wave: 16 or 32 values per lane (D <= 2048)
    if (g.D > 256) return SGM_OCV_LPL_MID;   // 16 lanes x DPL 32 would straddle D when D % 32 = 16, and
                                    // its 32-value step is slower anyway (the shipped 2448x2048
                                    // D=480 config, MODE_SGBM paths: 17.4 ms vs 8.8 ms); 64 lanes
                                    // of 8 values beat 32 of 16 once the packed step keeps 16 rows
                                    // in flight (5.63 vs 5.96 ms)
    if (const char* e = getenv("SGM_OCV_LPL")) return atoi(e) == 32 ? 32 : 16;
    // 128 < D <= 256 beside the fused vertical WTA (int16 L volumes either way): 32 lanes of 8
    // values, the packed step's 4-dword shape (16 rows in flight, the wave priority), instead of
    // 16 lanes of 16 (interleaved A/B, frame ms: 1080p D=256 MODE_HH 5.51 -> 4.48, 12 MP D=256
    // MODE_HH 29.4 -> 27.0, MODE_SGBM 19.53 -> 18.86); with the row WTA the 16-lane lines write
    // deficit records at 16 values per lane and stay ahead (1080p D=256 MODE_SGBM 2.44 vs 2.51;
    // profiles/r06_ocv_lpl32_d256_ab.jsonl)
    if (fused_v && g.D > 128) return 32;
    int waves = 0;
    for (int i = 0; i < 8; i++)
        if ((dirmask >> i) & 1)
            waves += ((dir_ry(i) == 0 ? g.H : g.width1 + (dir_rx(i) != 0 ? g.H - 1 : 0)) + 3) / 4;
    return waves < kOcvWideLineWaves ? 32 : 16;
}

// the values per lane launch_ocv_paths picks for the frame
static int ocv_paths_dpl(const Geom& g, int dirmask, bool fused_v)
{
    const int D = g.D, lpl = ocv_lanes_per_line(g, dirmask, fused_v);
    if (lpl == 64) return D <= 512 ? 8 : D <= 1024 ? 16 : 32;
    if (lpl == 32) return D <= 64 ? 2 : D <= 128 ? 4 : D <= 256 ? 8 : 16;
    return dpl_for(D);
}

// Deficits (Geom::evol, load_e) for the plain kernels of a frame: P2 <= 511 (e in 9 bits), the
// packed paths step (P1 <= 32768) with buffer offsets or 64-lane rebased descriptors, 8 or 16
// values per path lane (whole groups of 8 per lane), D <= 512 (the row WTA k_ocv_wta16 or the
// fused vertical WTA read them) or D <= 1024 under the fused vertical WTA. Returns
// the layout (1 records, 2 planes for D % 128 == 0) or 0; SGM_OCV_EVOL=0 (environment or build
// macro) keeps int16 L volumes, =1 / =2 forces a layout.
#ifndef SGM_OCV_EVOL
#define SGM_OCV_EVOL 1
#endif
#ifndef SGM_OCV_EVOL_VW_MIND
#define SGM_OCV_EVOL_VW_MIND 128   // beside the fused vertical WTA, deficits only for D above this: at
#endif                             // 128 < D <= 256 the 32-lane path lines of 8 values write them (1080p D=256
                                   // MODE_HH paths 2.45 -> 2.11 ms, frame 4.49 -> 4.25; the fused kernel reads
                                   // them in the same time; profiles/r06_ocv_evol_d256_ab.jsonl)
int ocv_evol_mode(const Geom& g, int dirmask, int skipdir)
{
    if (SGM_OCV_EVOL == 0 || SGM_OCV_PK == 0) return 0;
    const char* e = std::getenv("SGM_OCV_EVOL");       // 0 off, 1 / 2 force a layout
    if (e && std::atoi(e) == 0) return 0;
    if (g.wide == 1 || g.P2 > 511 || g.P1 > 32768 || g.D > 1024 || g.width1 <= 0) return 0;
    const int pmask = skipdir >= 0 ? dirmask & ~(1 << skipdir) : dirmask;
    const int dpl = ocv_paths_dpl(g, pmask, skipdir >= 0);
    if (dpl != 8 && dpl != 16) return 0;
    // 32-bit buffer offsets, or 64-lane lines / 32-lane lines of 8 values (rebased per step, any size)
    const int lpl = ocv_lanes_per_line(g, pmask, skipdir >= 0);
    const bool reb = lpl == 64 || (lpl == 32 && dpl == 8);
    if (!reb && ((size_t)g.width1 * g.H * g.D * 2 >= (size_t)kBufDrop || std::getenv("SGM_OCV_NO_BUF"))) return 0;
    // D > 512: only the fused vertical WTA reads deficits (the row WTA k_ocv_wta64 reads int16 L)
    if (g.D > 512 && skipdir < 0) return 0;
    // the fused vertical WTA reads them from 4 or more values per lane (D > 128): with 2 the byte and
    // bit loads per direction cost more than they save (1080p D=128 MODE_HH 2.48 -> 2.95 ms)
    if (skipdir >= 0 && g.D <= SGM_OCV_EVOL_VW_MIND) return 0;
    if (e && (std::atoi(e) == 1 || std::atoi(e) == 2)) return std::atoi(e);
    return g.D % 128 == 0 ? 2 : 1;
}

hipError_t launch_ocv_paths(const int16_t* C, const int16_t* Csat, void* vols, size_t cells, const Geom& g,
                            int dirmask, hipStream_t st, int skipdir)
{
    const int D = g.D;
    hipError_t e = hipSuccess;
    const int lpl = ocv_lanes_per_line(g, skipdir >= 0 ? dirmask & ~(1 << skipdir) : dirmask, skipdir >= 0);
    if (lpl == 64) {
        if (D <= 512) e = launch_ocv_paths_v<8, 64>(C, Csat, vols, cells, g, dirmask, st, skipdir);
        else if (D <= 1024) e = launch_ocv_paths_v<16, 64>(C, Csat, vols, cells, g, dirmask, st, skipdir);
        else e = launch_ocv_paths_v<32, 64>(C, Csat, vols, cells, g, dirmask, st, skipdir);
    } else if (lpl == 32) {
        if (D <= 64) e = launch_ocv_paths_v<2, 32>(C, Csat, vols, cells, g, dirmask, st, skipdir);
        else if (D <= 128) e = launch_ocv_paths_v<4, 32>(C, Csat, vols, cells, g, dirmask, st, skipdir);
        else if (D <= 256) e = launch_ocv_paths_v<8, 32>(C, Csat, vols, cells, g, dirmask, st, skipdir);
        else e = launch_ocv_paths_v<16, 32>(C, Csat, vols, cells, g, dirmask, st, skipdir);
    } else {
        switch (dpl_for(D)) {
        case 1: e = launch_ocv_paths_v<1, 16>(C, Csat, vols, cells, g, dirmask, st, skipdir); break;
        case 2: e = launch_ocv_paths_v<2, 16>(C, Csat, vols, cells, g, dirmask, st, skipdir); break;
        case 4: e = launch_ocv_paths_v<4, 16>(C, Csat, vols, cells, g, dirmask, st, skipdir); break;
        case 8: e = launch_ocv_paths_v<8, 16>(C, Csat, vols, cells, g, dirmask, st, skipdir); break;
        default: e = launch_ocv_paths_v<16, 16>(C, Csat, vols, cells, g, dirmask, st, skipdir); break;   // D <= 256 here
        }
    }
    return e != hipSuccess ? e : hipGetLastError();
}

template <int DPL, typename VT, bool SAT, bool EV>
static void launch_ocv_wta_e(const int16_t* C, const void* vols, size_t cells, int ndir, const Geom& g, int16_t* out,
                             size_t out_stride, hipStream_t st)
{
    const size_t vol_elems = ocv_vol_elems(cells, sizeof(VT));
    const size_t lds = (size_t)16 * 16 * DPL * 2 + RowLds::bytes(g.W);
    const VT* v = (const VT*)vols;
    if constexpr (!SAT && sizeof(VT) == 2 && DPL >= 2 && DPL <= 16 && (!EV || DPL >= 8)) {
        // the plain int16 regime, packed (k_ocv_wta16_pk; 32-bit buffer offsets: slots below 4 GB)
        if (SGM_OCV_WTA_PK != 0 && g.uniq < 100 && vol_elems * 2 < (size_t)kBufDrop) {
            if (ndir == 8)
                hipLaunchKernelGGL((k_ocv_wta16_pk<DPL, 8, EV>), dim3(g.H), dim3(256), lds, st, (const int16_t*)v,
                                   vol_elems, g, out, out_stride, C);
            else
                hipLaunchKernelGGL((k_ocv_wta16_pk<DPL, 5, EV>), dim3(g.H), dim3(256), lds, st, (const int16_t*)v,
                                   vol_elems, g, out, out_stride, C);
            return;
        }
    }
    if (ndir == 8)
        hipLaunchKernelGGL((k_ocv_wta16<DPL, 8, VT, SAT, EV>), dim3(g.H), dim3(256), lds, st, v, vol_elems, g, out,
                           out_stride, C);
    else
        hipLaunchKernelGGL((k_ocv_wta16<DPL, 5, VT, SAT, EV>), dim3(g.H), dim3(256), lds, st, v, vol_elems, g, out,
                           out_stride, C);
}
template <int DPL, typename VT, bool SAT>
static void launch_ocv_wta_dpl(const int16_t* C, const void* vols, size_t cells, int ndir, const Geom& g, int16_t* out,
                               size_t out_stride, hipStream_t st)
{
    if constexpr (!SAT && sizeof(VT) == 2) {
        if (g.evol) {
            launch_ocv_wta_e<DPL, VT, SAT, true>(C, vols, cells, ndir, g, out, out_stride, st);
            return;
        }
    }
    launch_ocv_wta_e<DPL, VT, SAT, false>(C, vols, cells, ndir, g, out, out_stride, st);
}

template <typename VT, bool SAT>
static void launch_ocv_wta_t(const int16_t* C, const void* vols, size_t cells, int ndir, const Geom& g, int16_t* out,
                             size_t out_stride, hipStream_t st)
{
    const int D = g.D;
    if (D > 512) {
        const size_t vol_elems = ocv_vol_elems(cells, sizeof(VT));
        const size_t lds = (size_t)4 * ((D + kWta64Chunk - 1) / kWta64Chunk * kWta64Chunk) * 2 + RowLds::bytes(g.W);
        const VT* v = (const VT*)vols;
        if (ndir == 8)
            hipLaunchKernelGGL((k_ocv_wta64<8, VT, SAT>), dim3(g.H), dim3(256), lds, st, v, vol_elems, g, out, out_stride);
        else
            hipLaunchKernelGGL((k_ocv_wta64<5, VT, SAT>), dim3(g.H), dim3(256), lds, st, v, vol_elems, g, out, out_stride);
        return;
    }
    if (D <= 32) launch_ocv_wta_dpl<2, VT, SAT>(C, vols, cells, ndir, g, out, out_stride, st);
    else if (D <= 64) launch_ocv_wta_dpl<4, VT, SAT>(C, vols, cells, ndir, g, out, out_stride, st);
    else if (D <= 128) launch_ocv_wta_dpl<8, VT, SAT>(C, vols, cells, ndir, g, out, out_stride, st);
    else if (D <= 256) launch_ocv_wta_dpl<16, VT, SAT>(C, vols, cells, ndir, g, out, out_stride, st);
    else launch_ocv_wta_dpl<32, VT, SAT>(C, vols, cells, ndir, g, out, out_stride, st);
}

// vols: int16 volumes (wide 0), the flagged kind (wide 1: int32, or saturating int16 under
// SIMD_SAT), or a region sized for the larger, read as the one the cost kernel's overflow
// flag selects (wide 2); cells = width1 * H * D per volume
hipError_t launch_ocv_wta(const int16_t* C, const void* vols, size_t cells, int ndir, const Geom& g, int16_t* out,
                          size_t out_stride, hipStream_t st)
{
    if (g.wide != 1) launch_ocv_wta_t<int16_t, false>(C, vols, cells, ndir, g, out, out_stride, st);
    if (g.wide == 0) return hipGetLastError();
    Geom gf = g;
    gf.evol = 0;                                         // the flagged kernels keep full volumes
    if (g.compat & SGM_OCV_SIMD_SAT) launch_ocv_wta_t<int16_t, true>(C, vols, cells, ndir, gf, out, out_stride, st);
    else launch_ocv_wta_t<int32_t, false>(C, vols, cells, ndir, gf, out, out_stride, st);
    return hipGetLastError();
}

// k_ocv_vwta in packed u16 pairs for the plain int16 regime (the step of ocv_step_pk; no flagged
// frame, uniqueness ratio < 100). Every path cost there lies in [0, 32767], so OpenCV's S =
// sat16(sat16(s1) + s2) is min(sum, 32767) in any order: saturating packed i16 adds of the
// loaded dwords. Entries with d >= D are forced to 0xFFFF after the sum, above every real S.
// The WTA decisions are k_ocv_vwta's: best and minS from one 64-lane min over
// S << 11 | tie(d) (first minimal d, or the 3.x lane rule); uniqueness as a count — the number
// of d with S < T = ceil(minS * 100 / (100 - u)) over the line (packed saturating subtract, a
// per-lane sum, one 64-lane reduction) against the count inside {best - 1, best, best + 1}
// (from minS and the two neighbours the subpixel step reads anyway): a d outside the window
// qualifies iff the first exceeds the second.
template <int LPL>
__device__ __forceinline__ int line_sum_i32(int v)
{
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true);     // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true);     // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xf, 0xf, true);    // row_ror:4
    v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, true);    // row_ror:8
    if constexpr (LPL >= 32) {
        const auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = (int)sw[0] + (int)sw[1];
    }
    if constexpr (LPL == 64) {
        const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        v = (int)sw[0] + (int)sw[1];
    }
    return v;
}
// The packed pairs of the lane's deficits (Geom::evol) from its raw loads: w[0 .. M/2) the byte
// plane's dwords, w[M/2] the bit-plane bytes (DPL = 8 or 16; DPL = 4: half a group, hsh = 2 for
// its upper half, whose bits sit two places up in each nibble)
template <int M>
__device__ __forceinline__ void evol_pairs(const uint32_t (&w)[M], uint32_t (&e2)[M], int hsh = 0)
{
    if constexpr (M == 2) {
        const uint32_t h2 = (((w[1] & 0xFFu) >> hsh) * 0x1001u) & 0x000F000Fu;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const uint32_t lo2 = __builtin_amdgcn_perm(0u, w[0], i ? 0x0C030C02u : 0x0C010C00u);
            e2[i] = ((h2 << (8 - i)) & 0x01000100u) | lo2;
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < M / 4; c++) {
        // evens of the group at bits 0-3, odds at bits 16-19
        const uint32_t hb = (w[M / 2] >> (8 * c)) & 0xFFu;
        const uint32_t h2 = (hb * 0x1001u) & 0x000F000Fu;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t lo2 = __builtin_amdgcn_perm(0u, w[2 * c + i / 2], (i & 1) ? 0x0C030C02u : 0x0C010C00u);
            e2[4 * c + i] = ((h2 << (8 - i)) & 0x01000100u) | lo2;
        }
    }
}
template <int DPL, int NDIR, bool EV>
__global__ __launch_bounds__(64) void k_ocv_vwta_pk(const int16_t* __restrict__ C, const int16_t* __restrict__ vols,
                                                    size_t vol_elems, Geom g, uint64_t* __restrict__ res)
{
    if (ocv_gate_skip<false>(g)) return;
    constexpr int LPL = 64, M = DPL / 2;
    constexpr int F = NDIR == 5 ? 0 : 1;               // the fused direction = its volume slot
    // steps in flight: a column is one latency-bound chain (width1 waves, ~2 per SIMD), and the
    // packed operands are half the registers of k_ocv_vwta's ints. 16 values per lane (D > 512):
    // 8 steps of MODE_HH operands are 512 VGPRs (904 B/lane of scratch: the D=752 processing
    // config's kernel 21.3 ms), 2 or 4 steps fit (7.85 ms; profiles/r06_ocv_d752_vwta_ab.jsonl); with
    // deficit records MODE_HH keeps 2 (5.67 ms against 7.4-7.6 at 3-4) and MODE_SGBM takes 4 (4.36-4.39
    // against 4.52-4.54 at 2; profiles/r06_ocv_d752_vwta_pf_ab.jsonl). 8 values per lane: MODE_HH over
    // deficit records 4 (the shipped D=480 frame's kernel 4.77 -> 3.68 ms), else 8 (MODE_SGBM 2.95
    // against 3.04 at 4, 2.99 at 6; profiles/r06_ocv_cost_ring0_vwta_pf_ab.jsonl)
    // 4 values per lane (128 < D <= 256): 6 steps (frame ms of the fused kernel at 2 / 4 / 6 / 8 / 12: 12 MP
    // D=256 MODE_SGBM 5.81 / 5.22 / 5.22 / 5.62 / 6.03, MODE_HH 6.71 / 7.07 / 7.21 / - / 10.48, 1080p D=256
    // MODE_HH 1.55-1.72 / 1.57-1.70 / 1.35 / - / 1.89; profiles/r06_ocv_vwta_pk4_pf_ab.jsonl)
    constexpr int PF = SGM_OCV_VWTA_PK_PF > 0 ? SGM_OCV_VWTA_PK_PF
                       : DPL == 4                 ? 6
                       : DPL >= 32                ? 1
                       : DPL >= 16                ? (NDIR == 5 ? 4 : 2)
                       : (NDIR == 8 && EV)        ? 4
                                                  : 8;
    const int p = threadIdx.x;
    const int x1 = blockIdx.x;
    const bool lanetie = NDIR == 5 && (g.compat & SGM_OCV_LANE_TIE);
    const bool lane_act = p * DPL < g.D;
    const int dl = lane_act ? p * DPL : g.D - DPL;     // lanes past D load the last group
    auto cell = [&](int i) -> size_t {
        const int y = F == 0 ? min(i, g.H - 1) : max(g.H - 1 - i, 0);
        return ((size_t)y * g.width1 + x1) * g.D + dl;
    };
    static_assert(!EV || DPL == 4 || DPL == 8 || DPL == 16, "deficit planes: 4, 8 or 16 values per lane");
    auto load = [&](int i, uint32_t (&c)[M], uint32_t (&v)[NDIR][M]) {
        const size_t o = cell(i);
        load_dw<M>(C + o, c);
        const EvLayout el = evol_layout(g);
        const size_t px = (size_t)(F == 0 ? min(i, g.H - 1) : max(g.H - 1 - i, 0)) * g.width1 + x1;
#pragma unroll
        for (int s = 0; s < NDIR; s++) {
            if (s == F) continue;
            if constexpr (EV) {                          // raw: byte-plane dwords, then the bit-plane bytes
                const uint8_t* vb = (const uint8_t*)(vols + (size_t)s * vol_elems);
                const uint8_t* lo = vb + px * el.ls + dl;
                const uint8_t* hi = vb + el.hb + px * el.hs + dl / 8;
                if constexpr (DPL == 4) {
                    v[s][0] = *(const uint32_t*)lo;
                    v[s][1] = *hi;
                } else if constexpr (DPL == 8) {
                    const uint2 t = *(const uint2*)lo;
                    v[s][0] = t.x; v[s][1] = t.y;
                    v[s][2] = *hi;
                } else {
                    const uint4 t = *(const uint4*)lo;
                    v[s][0] = t.x; v[s][1] = t.y; v[s][2] = t.z; v[s][3] = t.w;
                    v[s][4] = *(const uint16_t*)hi;
                }
            } else {
                load_dw<M>(vols + (size_t)s * vol_elems + o, v[s]);
            }
        }
    };
    uint32_t imask[M], tie[M][2];
#pragma unroll
    for (int j = 0; j < M; j++) {
        const int d = p * DPL + 2 * j;
        imask[j] = (d < g.D ? 0u : 0xFFFFu) | (d + 1 < g.D ? 0u : 0xFFFF0000u);
        tie[j][0] = (uint32_t)wta_tie(d, lanetie, 11);
        tie[j][1] = (uint32_t)wta_tie(d + 1, lanetie, 11);
    }
    const uint32_t P1P1 = (uint32_t)g.P1 * 0x10001u, P2 = (uint32_t)g.P2;
    // uniqueness threshold divisor (u < 100: the launcher's condition)
    const int kq = 100 - g.uniq;
    uint32_t L2[M], delta2 = P2 * 0x10001u;            // the path's first pixel: L = C - P2
#pragma unroll
    for (int j = 0; j < M; j++) L2[j] = 0;
    uint32_t Cq[PF][M], Vq[PF][NDIR][M];
#pragma unroll
    for (int q = 0; q < PF; q++) load(q, Cq[q], Vq[q]);
    auto step = [&](int i, const uint32_t (&Cc)[M], const uint32_t (&V)[NDIR][M]) {
        const uint32_t lmin = ocv_step_pk<DPL, LPL>(Cc, L2, delta2, P1P1, imask, p);
        delta2 = ((uint32_t)line_min_i32<LPL>((int)lmin) + P2) * 0x10001u;
        uint32_t S2[M], Lv[NDIR][M];                    // the other directions' L of the cell
#pragma unroll
        for (int s = 0; s < NDIR; s++) {
            if (s == F) continue;
            if constexpr (EV) {
                uint32_t e2[M];
                evol_pairs<M>(V[s], e2, (dl & 4) >> 1);
#pragma unroll
                for (int j = 0; j < M; j++) Lv[s][j] = pk_sub(Cc[j], e2[j]);
            } else {
#pragma unroll
                for (int j = 0; j < M; j++) Lv[s][j] = V[s][j];
            }
        }
        int km = 0x7FFFFFFF;
#pragma unroll
        for (int j = 0; j < M; j++) {
            s16x2_t a = __builtin_bit_cast(s16x2_t, L2[j]);
#pragma unroll
            for (int s = 0; s < NDIR; s++)
                if (s != F) a = __builtin_elementwise_add_sat(a, __builtin_bit_cast(s16x2_t, Lv[s][j]));
            S2[j] = __builtin_bit_cast(uint32_t, a) | imask[j];
            const int klo = (int)(((S2[j] & 0xFFFFu) << 11) | tie[j][0]);
            const int khi = (int)(((S2[j] >> 16) << 11) | tie[j][1]);
            km = min(km, min(klo, khi));
        }
        const int kmin = __builtin_amdgcn_readfirstlane(line_min_i32<LPL>(km));
        const int best = wta_untie(kmin & 2047, lanetie, 11);
        const int minS = kmin >> 11;
        // S of d (wave-uniform): one readlane per register of the lane holding d, then a select
        auto s_at = [&](int d) {
            const int ln = d / DPL, k = d % DPL, jj = k >> 1;
            uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)S2[0], ln);
#pragma unroll
            for (int j = 1; j < M; j++) {
                const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)S2[j], ln);
                v = jj == j ? r : v;
            }
            return (int)((k & 1) ? v >> 16 : v & 0xFFFFu);
        };
        const int sm = s_at(max(best - 1, 0)), sp = s_at(min(best + 1, g.D - 1));
        // uniqueness: S * kq < minS * 100 <=> S < T = ceil(minS * 100 / kq); T clamped to 32768
        // (every real S is <= 32767, and d >= D holds 0xFFFF)
        const int Mq = minS * 100;
        const int T = min((Mq + kq - 1) / kq, 32768);
        const uint32_t T2 = (uint32_t)T * 0x10001u;
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < M; j++) {
            const uint32_t t = as_u(__builtin_elementwise_sub_sat(as_v2(T2), as_v2(S2[j])));   // > 0 where S < T
            acc = pk_add(acc, pk_min(t, 0x00010001u));
        }
        const int total = line_sum_i32<LPL>((int)((acc & 0xFFFFu) + (acc >> 16)));
        const int inwin = (best >= 1 && sm < T ? 1 : 0) + (minS < T ? 1 : 0) + (best + 1 < g.D && sp < T ? 1 : 0);
        const bool rej = __builtin_amdgcn_readfirstlane(total) > inwin || minS >= 32767;
        const int den = max(sm + sp - 2 * minS, 1);
        const bool use = g.subpix && best > 0 && best < g.D - 1;
        const int d16 = best * 16 + (use ? tdiv_rcp((sm - sp) * 16 + den, 2 * den) : 0) + g.minD * 16;
        const int y = F == 0 ? i : g.H - 1 - i;
        const uint64_t v = (uint64_t)(uint16_t)(rej ? g.invalid : d16) |
                           ((uint64_t)(uint16_t)(rej ? -1 : best) << 16) | ((uint64_t)(uint16_t)minS << 32);
        if (p == 0 && i < g.H) __builtin_nontemporal_store(v, res + (size_t)y * g.W + g.minX1 + x1);
    };
    for (int i0 = 0; i0 < g.H; i0 += PF) {
#pragma unroll
        for (int q = 0; q < PF; q++) {
            uint32_t Cc[M], V[NDIR][M];
#pragma unroll
            for (int j = 0; j < M; j++) {
                Cc[j] = Cq[q][j];
#pragma unroll
                for (int s = 0; s < NDIR; s++) V[s][j] = Vq[q][s][j];
            }
            load(i0 + q + PF, Cq[q], Vq[q]);           // operands of step i + PF
            step(i0 + q, Cc, V);
        }
    }
}

// Fused vertical path + WTA (k_ocv_vwta): one 64-lane line (a column) per wave, DPL = D / 64
// rounded up to a power of two; the plain and the flagged kinds as for the paths.
template <int DPL, int NDIR, typename VT, bool SAT>
static void launch_ocv_vwta_l(const int16_t* C, const void* vols, size_t cells, const Geom& g, uint64_t* res,
                              hipStream_t st)
{
    const size_t vol_elems = ocv_vol_elems(cells, sizeof(VT));
    const int use_pk = SGM_OCV_PK != 0 && !SAT && sizeof(VT) == 2 && g.P1 <= 32768 && g.P2 <= 32768;
    // everything packed (k_ocv_vwta_pk) for MODE_HH at >= 8 values per lane: the shipped D=480
    // config's fused kernel 5.67 -> 5.27 ms with 8 steps in flight; MODE_SGBM (3.47 vs 3.53-3.60)
    // and 1080p MODE_HH (0.87 vs 0.90-0.94) keep k_ocv_vwta (profiles/r05_ocv_vwta_pk_ab.jsonl):
    // the kernel streams its volumes near the read peak, and fewer instructions help only where
    // the operands of more steps fit in flight
    if constexpr (!SAT && sizeof(VT) == 2 && DPL >= SGM_OCV_VWTA_PK_MIND) {
        if (use_pk && g.uniq < 100 && SGM_OCV_VWTA_PK != 0 && (NDIR == 8 || (g.evol && SGM_OCV_VWTA_PK_EV5))) {
            if constexpr (DPL <= 16) {
                if (g.evol) {
                    hipLaunchKernelGGL((k_ocv_vwta_pk<DPL, NDIR, true>), dim3(g.width1), dim3(64), 0, st, C,
                                       (const int16_t*)vols, vol_elems, g, res);
                    return;
                }
            }
            hipLaunchKernelGGL((k_ocv_vwta_pk<DPL, NDIR, false>), dim3(g.width1), dim3(64), 0, st, C, (const int16_t*)vols,
                               vol_elems, g, res);
            return;
        }
    }
    if constexpr (!SAT && sizeof(VT) == 2 && DPL <= 16) {
        if (g.evol) {
            hipLaunchKernelGGL((k_ocv_vwta<DPL, NDIR, VT, SAT, true>), dim3(g.width1), dim3(64), 0, st, C, (const VT*)vols,
                               vol_elems, g, res, use_pk);
            return;
        }
    }
    hipLaunchKernelGGL((k_ocv_vwta<DPL, NDIR, VT, SAT, false>), dim3(g.width1), dim3(64), 0, st, C, (const VT*)vols,
                       vol_elems, g, res, use_pk);
}
template <int DPL, int NDIR>
static void launch_ocv_vwta_v(const int16_t* C, const int16_t* Csat, const void* vols, size_t cells, const Geom& g,
                              uint64_t* res, hipStream_t st)
{
    if (g.wide != 1) launch_ocv_vwta_l<DPL, NDIR, int16_t, false>(C, vols, cells, g, res, st);
    if (g.wide == 0) return;
    if (g.compat & SGM_OCV_SIMD_SAT) launch_ocv_vwta_l<DPL, NDIR, int16_t, true>(Csat, vols, cells, g, res, st);
    else launch_ocv_vwta_l<DPL, NDIR, int32_t, false>(C, vols, cells, g, res, st);
}
template <int NDIR>
static void launch_ocv_vwta_n(const int16_t* C, const int16_t* Csat, const void* vols, size_t cells, const Geom& g,
                              uint64_t* res, hipStream_t st)
{
    const int D = g.D;
    if (D <= 64) launch_ocv_vwta_v<1, NDIR>(C, Csat, vols, cells, g, res, st);
    else if (D <= 128) launch_ocv_vwta_v<2, NDIR>(C, Csat, vols, cells, g, res, st);
    else if (D <= 256) launch_ocv_vwta_v<4, NDIR>(C, Csat, vols, cells, g, res, st);
    else if (D <= 512) launch_ocv_vwta_v<8, NDIR>(C, Csat, vols, cells, g, res, st);
    else if (D <= 1024) launch_ocv_vwta_v<16, NDIR>(C, Csat, vols, cells, g, res, st);
    else launch_ocv_vwta_v<32, NDIR>(C, Csat, vols, cells, g, res, st);
}
// the vertical direction of the last group (MODE_SGBM: dir 0, MODE_HH: dir 1) fused with the
// WTA; its volume slot is never written (launch_ocv_paths with skipdir = ocv_vwta_dir(ndir))
int ocv_vwta_dir(int ndir) { return ndir == 8 ? 1 : 0; }
hipError_t launch_ocv_vwta(const int16_t* C, const int16_t* Csat, const void* vols, size_t cells, int ndir,
                           const Geom& g, uint64_t* res, hipStream_t st)
{
    if (g.width1 <= 0) return hipSuccess;
    if (ndir == 8) launch_ocv_vwta_n<8>(C, Csat, vols, cells, g, res, st);
    else launch_ocv_vwta_n<5>(C, Csat, vols, cells, g, res, st);
    return hipGetLastError();
}

}  // namespace sgm
