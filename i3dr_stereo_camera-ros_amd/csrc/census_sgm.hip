// census_sgm.hip — north-star census-SGM kernels for gfx950 (SGM_MODE_CENSUS8).
//
// Spec: SURVEY.md Appendix B (build-defined; CPU definition oracle/sgm_oracle.c
// `census_step`/`census_path`/`wta_pixel`). Pipeline per frame:
//   k_census9x7       L,R u8        -> census codes u64 (2 x W x H)
//   k_census_paths16  codes         -> 8 u8 path volumes [H][width1][D], all directions in
//                                      one launch (6 row sweeps + 2 horizontal scans)
//   k_census_wta      8 volumes     -> S = sum of the 8 paths, WTA, uniqueness, subpixel,
//                                      disp2 and LR check (one workgroup per row)
// The matching cost popcount(cL ^ cR) is recomputed on the fly in every path (never
// stored); S never touches HBM.
#include "sgm_device.h"

#include <atomic>
#include <string>

#ifndef SGM_WPE
#define SGM_WPE 4          // minimum waves per SIMD of the path kernels (register budget)
#endif
#ifndef SGM_WPE32
#define SGM_WPE32 4        // the same for 32 disparities per lane (D > 256; 2: C5 single frame 27.4 vs 23.9 ms)
#endif
#ifndef SGM_NT_STORE
#define SGM_NT_STORE 1     // path volumes written with nontemporal stores (0: plain)
#endif
#ifndef SGM_NT_LOAD
#define SGM_NT_LOAD 1      // WTA volume loads with the nt cache policy (0: default)
#endif
#ifndef SGM_EXP
#define SGM_EXP 0          // timing-only experiments (results invalid): bit 0 row segments from row 0,
                           // bit 1 dir-1 volume stores to the trash slot, bit 2 WTA reads 7 volumes
#endif
#if SGM_EXP != 0 && !defined(SGM_EXPERIMENT_BUILD)
#error "SGM_EXP builds give invalid results: define SGM_EXPERIMENT_BUILD as well (never in a release build)"
#endif
#ifndef SGM_LRPRIO_HW
#define SGM_LRPRIO_HW 37   // a horizontal-scan step in row-sweep steps, x/64
#endif
#ifndef SGM_LRPRIO_DIAG
#define SGM_LRPRIO_DIAG 64 // a diagonal row-sweep step in vertical row-sweep steps, x/64
#endif
#ifndef SGM_UPWTA_PRIO
#define SGM_UPWTA_PRIO 0   // s_setprio of the up+WTA blocks (0: default priority)
#endif
#ifndef SGM_ROWS_LPL8
#define SGM_ROWS_LPL8 0    // 1: row sweeps with 8 lanes per path line for D <= 256 (RowsCfg; measured slower)
#endif
#ifndef SGM_P32
#define SGM_P32 1          // D > 256: 32-lane path lines of 16 disparities per lane (0: 16 lanes x 32, LineCfg)
#endif

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace sgm {

// ------------------------------------------------------------------------------------
// 9x7 census code of the pixel whose 9 x 7 window starts at byte tx of row ty of an LDS tile
// (pitch a multiple of 4). Each window row is three aligned u32 reads and two alignbytes; the
// 62 bits are produced from the highest down, each compare's result shifted into the code
// (2 VALU per bit: byte compare, shift-add), instead of a u8 LDS read, compare, 64-bit shift
// and or per bit. Bit order: LSB-first raster over the window, centre skipped.
// ------------------------------------------------------------------------------------
// acc = 2 * acc + (byte b of w < c): an SDWA byte compare into vcc and an add-with-carry
// (b is a constant once the window loops are unrolled)
#define SGM_CENSUS_BIT(B)                                                              \
    asm("v_cmp_lt_u32_sdwa vcc, %1, %2 src0_sel:BYTE_" #B " src1_sel:DWORD\n\t"      \
        "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc"                                       \
        : "+v"(acc) : "v"(w), "v"(c) : "vcc")
__device__ __forceinline__ void census_bit(uint32_t& acc, uint32_t w, uint32_t c, int b)
{
    switch (b) {
    case 0: SGM_CENSUS_BIT(0); break;
    case 1: SGM_CENSUS_BIT(1); break;
    case 2: SGM_CENSUS_BIT(2); break;
    default: SGM_CENSUS_BIT(3); break;
    }
}
#undef SGM_CENSUS_BIT

template <int PITCH>
__device__ __forceinline__ uint64_t census_code_lds(const uint8_t* tile, int ty, int tx)
{
    static_assert(PITCH % 4 == 0, "u32 rows");
    const uint32_t* t32 = (const uint32_t*)tile + (PITCH / 4) * ty + (tx >> 2);
    const int sb = tx & 3;
    const uint32_t c = tile[(ty + 3) * PITCH + tx + 4];
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int dy = 6; dy >= 0; dy--) {
        const uint32_t* r = t32 + (PITCH / 4) * dy;
        const uint32_t w0 = r[0], w1 = r[1], w2 = r[2];
        const uint32_t a0 = __builtin_amdgcn_alignbyte(w1, w0, sb);   // window bytes 0..3
        const uint32_t a1 = __builtin_amdgcn_alignbyte(w2, w1, sb);   // 4..7
        const uint32_t a2 = __builtin_amdgcn_alignbyte(w2, w2, sb);   // 8 (low byte)
#pragma unroll
        for (int dx = 8; dx >= 0; dx--) {
            if (dy == 3 && dx == 4) continue;
            const int k = dy * 9 + dx - (dy * 9 + dx > 31 ? 1 : 0);    // bit index
            const uint32_t w = dx < 4 ? a0 : dx < 8 ? a1 : a2;
            if (k >= 32) census_bit(hi, w, c, dx & 3);
            else census_bit(lo, w, c, dx & 3);
        }
    }
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// 9x7 census: one thread per pixel, a 10 x 72 byte LDS tile per 64 x 4 pixel block.
// blockIdx.z selects the image (0 = left, 1 = right).
__global__ __launch_bounds__(256) void k_census9x7(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                   size_t stride, int W, int H,
                                                   uint64_t* __restrict__ cL, uint64_t* __restrict__ cR)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[10 * 72];
    const uint8_t* img = blockIdx.z ? R : L;
    uint64_t* out = blockIdx.z ? cR : cL;
    const int x0 = blockIdx.x * 64, y0 = blockIdx.y * 4;
    for (int i = threadIdx.x; i < 10 * 72; i += 256) {
        int ty = i / 72, tx = i - ty * 72;
        int yy = min(max(y0 + ty - 3, 0), H - 1), xx = min(max(x0 + tx - 4, 0), W - 1);
        tile[i] = img[(size_t)yy * stride + xx];
    }
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int x = x0 + tx, y = y0 + ty;
    if (x >= W || y >= H) return;
    out[(size_t)y * W + x] = census_code_lds<72>(tile, ty, tx);
}

// ====================================================================================
// P16 path engine. A path line owns one 16-lane row of a wave: lane p holds disparities
// d = p*DPL .. p*DPL + DPL-1 (DPL = D_pad/16, D_pad = 16*DPL >= D), two per 32-bit
// register as packed u16 (v_pk_*_u16). The recurrence is kept in relative form
//     L(d)  = C(d) + min(L'(d), min(L'(d-1), L'(d+1)) + P1, P2),   L' = Lprev - min Lprev
// which equals SGM's C + min(Lp, Lp+-1 + P1, minLp + P2) - minLp exactly (all values
// <= 255 because C <= 62 and P2 <= 193). min over D is a 4-step DPP reduction inside the
// row; the d-1 / d+1 neighbours are v_alignbit of adjacent registers plus one row_shr /
// row_shl DPP for the lane boundary. Values are kept as biased-f16 bit patterns (see
// p16_step) so that one v_pk_minimum3_f16 does two of the mins; entries with d >= D are
// forced to a large finite pattern.
//
// Memory-op discipline: gfx950 counts loads and stores on one in-order vmcnt and hipcc
// only emits counted waits when every path through a loop body issues the same VMEM ops.
// So loops issue a fixed sequence: clamped prefetches, and cells that must not be written
// (outside the image, d >= D, padding steps) go to a per-volume trash slot.
// ====================================================================================
// DPL consecutive u8 costs of one lane (the P16 layout of a volume pixel) as dwords
template <int DPL>
__device__ __forceinline__ void wload(const uint8_t* src, uint32_t (&wd)[(DPL + 3) / 4])
{
    if constexpr (DPL == 2) { wd[0] = *(const uint16_t*)src; }
    else if constexpr (DPL == 4) { wd[0] = *(const uint32_t*)src; }
    else if constexpr (DPL == 8) { const uint2 v = *(const uint2*)src; wd[0] = v.x; wd[1] = v.y; }
    else {
#pragma unroll
        for (int q = 0; q < DPL / 16; q++) {
            const uint4 v = ((const uint4*)src)[q];
            wd[4 * q] = v.x; wd[4 * q + 1] = v.y; wd[4 * q + 2] = v.z; wd[4 * q + 3] = v.w;
        }
    }
}

// the same from a raw buffer (base wave-uniform, byte offset off per lane)
template <int DPL>
__device__ __forceinline__ void wload_buf(const uint8_t* base, uint32_t off, uint32_t (&wd)[(DPL + 3) / 4])
{
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFFF, 0x00020000);
    constexpr int aux = SGM_NT_LOAD ? 2 : 0;           // 2: nt (streamed once)
    if constexpr (DPL == 2) { wd[0] = __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, aux); }
    else if constexpr (DPL == 4) { wd[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, aux); }
    else if constexpr (DPL == 8) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, aux);
        wd[0] = v[0]; wd[1] = v[1];
    } else {
#pragma unroll
        for (int q = 0; q < DPL / 16; q++) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * q, 0, aux);
            wd[4 * q] = v[0]; wd[4 * q + 1] = v[1]; wd[4 * q + 2] = v[2]; wd[4 * q + 3] = v[3];
        }
    }
}

// dst_hi: where bytes 16..31 go when DPL == 32 (D not a multiple of 32 leaves the lane that
// straddles D half valid: its upper half must go to the trash slot, not the next pixel)
template <int DPL>
__device__ __forceinline__ void store_pairs(uint8_t* dst, uint8_t* dst_hi, const uint32_t (&L)[DPL / 2])
{
    // (lo, hi) u16 pairs with values <= 255 -> DPL consecutive bytes
    if constexpr (DPL == 2) {
        const uint16_t v = (uint16_t)__builtin_amdgcn_perm(0u, L[0], 0x0c0c0200u);
        if constexpr (SGM_NT_STORE) __builtin_nontemporal_store(v, (uint16_t*)dst);
        else *(uint16_t*)dst = v;
    } else if constexpr (DPL == 4) {
        const uint32_t v = __builtin_amdgcn_perm(L[1], L[0], 0x06040200u);
        if constexpr (SGM_NT_STORE) __builtin_nontemporal_store(v, (uint32_t*)dst);
        else *(uint32_t*)dst = v;
    } else if constexpr (DPL == 8) {
        typedef unsigned int v2u __attribute__((ext_vector_type(2)));
        const v2u v = {__builtin_amdgcn_perm(L[1], L[0], 0x06040200u), __builtin_amdgcn_perm(L[3], L[2], 0x06040200u)};
        if constexpr (SGM_NT_STORE) __builtin_nontemporal_store(v, (v2u*)dst);
        else *(v2u*)dst = v;
    } else {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < DPL / 16; q++) {
            const v4u v = {__builtin_amdgcn_perm(L[8 * q + 1], L[8 * q + 0], 0x06040200u),
                           __builtin_amdgcn_perm(L[8 * q + 3], L[8 * q + 2], 0x06040200u),
                           __builtin_amdgcn_perm(L[8 * q + 5], L[8 * q + 4], 0x06040200u),
                           __builtin_amdgcn_perm(L[8 * q + 7], L[8 * q + 6], 0x06040200u)};
            v4u* d = (v4u*)(q == 0 ? dst : dst_hi);
            if constexpr (SGM_NT_STORE) __builtin_nontemporal_store(v, d);
            else *d = v;
        }
    }
}

// Path-cost arithmetic in the "biased f16" domain. A cost v in [0, 1024) is held as the u16
// bit pattern kBase + v (kBase = 0x6400 = f16 1024.0). In that binade the f16 ulp is 1, so
//  * the bit pattern is exactly the f16 value 1024 + v: f16 min/minimum3 on patterns = integer
//    min on v (v_pk_minimum3_f16 gives a packed 3-way min in one instruction), and
//  * integer adds/subtracts of small amounts on the pattern (v_pk_add_u16, v_bcnt's
//    accumulator) are exact, and the low byte of a pattern is v itself (v <= 255).
// "Infinite" entries (d >= D, lane edges) are kInfP = 0x7000 (f16 8192): finite, so no NaN
// can appear, and above every real value (<= kBase + 255 + P1 + 62).
constexpr uint32_t kBaseP = 0x6400u, kBaseP2 = 0x64006400u;
constexpr uint32_t kInfP = 0x7000u, kInfP2 = 0x70007000u;

__device__ __forceinline__ uint32_t pk_min3_p(uint32_t a, uint32_t b, uint32_t c)
{
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    const h2_t r = __builtin_elementwise_minimum(
        __builtin_elementwise_minimum(__builtin_bit_cast(h2_t, a), __builtin_bit_cast(h2_t, b)), __builtin_bit_cast(h2_t, c));
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_max(as_v2(a), as_v2(b))); }

// popcount(x) + acc (v_bcnt_u32_b32 with accumulator). Inline asm keeps the accumulator
// chain as written: hipcc otherwise re-associates the adds into extra v_add3 / v_add_lshl.
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
// acc + Hamming(a, b) of two 64-bit census codes: 2 xor + 2 bcnt
__device__ __forceinline__ uint32_t ham_acc(uint64_t a, uint64_t b, uint32_t acc)
{
    const uint64_t x = a ^ b;
    return bcnt_acc((uint32_t)(x >> 32), bcnt_acc((uint32_t)x, acc));
}

// packed u16 helpers of the WTA: per-half shift and saturating subtract
__device__ __forceinline__ uint32_t pk_shl(uint32_t a, int sh)
{
    return as_u(as_v2(a) << (u16x2_t){(unsigned short)sh, (unsigned short)sh});
}
__device__ __forceinline__ uint32_t pk_subs(uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_sub_sat(as_v2(a), as_v2(b))); }
// Relative state of a line from its absolute costs: Lr = Labs - min over the line's D
// (LPL lanes per line: 16 = a whole 16-lane row, 8 = one parity of a row, see p16_rows)
template <int DPL, int LPL = 16>
__device__ __forceinline__ void p16_relative(const uint32_t (&Labs)[DPL / 2], uint32_t (&Lr)[DPL / 2])
{
    constexpr int M = DPL / 2;
    uint32_t mn = Labs[0];
#pragma unroll
    for (int i = 1; i < M; i += 2) mn = (i + 1 < M) ? pk_min3_p(mn, Labs[i], Labs[i + 1]) : pk_min(mn, Labs[i]);
    mn = line_min_u32<LPL>(pk_min(mn, alignbit16(mn, mn)));   // (min, min) in every lane of the line
    uint32_t off = mn - kBaseP2;                          // pattern(L) - off = pattern(L - min)
    asm("" : "+v"(off));                                  // keep (Labs - off): not (Labs - mn) + kBase
    // A plain 32-bit subtract is the packed one here (no borrow crosses the halves: every
    // half of Labs is >= min >= kBase), and v_sub_u32 issues at twice v_pk_sub_u16's rate.
#pragma unroll
    for (int i = 0; i < M; i++) Lr[i] = Labs[i] - off;
}

// One recurrence step of the lane's pairs, costs computed on the fly:
//   L(d) = C(d) + min(Lr(d), Lr(d-1) + P1, Lr(d+1) + P1, P2),  C(d) = Hamming(cl, crk(d))
// Lr: relative state (patterns) in/out. Labs: absolute L (patterns) out.
// Per pair: q = Lr + P1 (1), neighbour align (1), minimum3 (1), min P2 (1), 4 xor + 4 bcnt
// + 1 shift-add for the two costs (the low cost rides on v_bcnt's accumulator), 1/2 for the
// min reduction, 1 subtract.
// LPL = 8: the line's lanes are every other lane of a 16-lane row, so the neighbouring lane
// of the same line is 2 lanes away (row_shr:2 / row_shl:2; both lines' edge lanes read kInf).
// LPL = 32: a line is a row pair; the neighbours cross the row boundary (line32_shr1/shl1).
template <int DPL, bool EXACT, int LPL = 16, typename F>
__device__ __forceinline__ void p16_step(uint32_t (&Lr)[DPL / 2], uint64_t cl, F crk, uint32_t P1P1, uint32_t P2P2,
                                         const uint32_t (&imask)[DPL / 2], uint32_t (&Labs)[DPL / 2])
{
    constexpr int M = DPL / 2;
    constexpr int SH = LPL == 8 ? 2 : 1;
    uint32_t q[M];
#pragma unroll
    for (int i = 0; i < M; i++) q[i] = Lr[i] + P1P1;      // = pk_add: halves <= kInfP | kBaseP, no carry
    // previous lane: its .hi is q(d0 - 1); next lane: its .lo is q(d0 + DPL)
    const uint32_t X = LPL == 32 ? line32_shr1(q[M - 1], kInfP2) : row_shr_n<SH>(q[M - 1], kInfP2);
    const uint32_t Y = LPL == 32 ? line32_shl1(q[0], kInfP2) : row_shl_n<SH>(q[0], kInfP2);
    uint32_t Oprev = alignbit16(q[0], X);                 // (q(d-1), q(d)) for pair 0
#pragma unroll
    for (int i = 0; i < M; i++) {
        const uint32_t Onext = (i + 1 < M) ? alignbit16(q[i + 1], q[i]) : alignbit16(Y, q[M - 1]);
        const uint32_t t = pk_min(pk_min3_p(Oprev, Onext, Lr[i]), P2P2);
        const uint32_t c1 = ham_acc(cl, crk(2 * i + 1), 0u);
        uint32_t L = ham_acc(cl, crk(2 * i), t) + (c1 << 16);
        if (!EXACT) L = pk_max(L, imask[i]);
        Labs[i] = L;
        Oprev = Onext;
    }
    p16_relative<DPL, LPL>(Labs, Lr);
}

// imask: kInfP in the halves with d >= D (0 elsewhere); start: the relative state of a
// path's first pixel (L = C): kBase, or kInfP | kBase for d >= D.
template <int DPL, bool EXACT>
__device__ __forceinline__ void make_imask(int p, int D, uint32_t (&imask)[DPL / 2], uint32_t (&start)[DPL / 2])
{
#pragma unroll
    for (int i = 0; i < DPL / 2; i++) {
        const int d = p * DPL + 2 * i;
        imask[i] = EXACT ? 0u : ((d < D ? 0u : kInfP) | (d + 1 < D ? 0u : kInfP << 16));
        start[i] = imask[i] | kBaseP2;
    }
}

// Row-band exact tile mode (sgm_match_tiled_exact): a band's row sweeps continue the lines
// of its neighbours. bnd[0] holds the last row of the band above for the downward
// directions 0, 2, 3 (slots 0, 1, 2), bnd[1] the first row of the band below for the upward
// directions 1, 4, 5; each slot is width1 * D u8 costs in volume order, bnd_slot bytes
// apart. Null: the band edge is the image edge (lines start there).
struct PathLaunch16 {
    int xb_lo[6];        // row sweeps: first base column of the direction
    const uint8_t* bnd[2];
    size_t bnd_slot;
};
__host__ __device__ constexpr int bnd_slot_of(int dir) { return dir <= 1 ? 0 : (dir == 2 || dir == 4 ? 1 : 2); }
// Work list entry (one per workgroup): dir << 24 | frame-in-group << 22 | local block.
__host__ __device__ constexpr uint32_t path_item(int dir, int lb, int f = 0)
{
    return ((uint32_t)dir << 24) | ((uint32_t)f << 22) | (uint32_t)lb;
}

// wave-uniform pick from a kernel-argument array without dynamic indexing (no scratch)
template <typename T>
__device__ __forceinline__ T pick4(const T (&a)[kMaxGroup], int f)
{
    return f == 0 ? a[0] : f == 1 ? a[1] : f == 2 ? a[2] : a[3];
}

constexpr int kWG = 256;          // 4 waves

// Lanes per path line of a launch whose 16-lane layout would hold DPL16 disparities per lane.
// D > 256 (DPL16 = 32) runs 32-lane lines of 16 disparities per lane: the 16-lane form's 32
// values per lane held the kernel at 128 VGPRs (4 waves/SIMD) and made each step one long
// dependent chain; 32-lane lines keep the D <= 256 register budget at the price of one
// cross-row select per neighbour exchange and a permlane16 swap in the min over D.
template <int DPL16>
struct LineCfg {
    static constexpr int LPL = (DPL16 == 32 && SGM_P32) ? 32 : 16;
    static constexpr int DPL = DPL16 * 16 / LPL;       // disparities per lane
    static constexpr int HROWS = 4 * (64 / LPL);       // image rows per horizontal-scan workgroup
};

// ---------------------------------------------------------------- horizontal scans ----
// Scalar operands per step come from 16-step chunks held one value per lane (lane j of a
// row holds step j) and are broadcast inside the row with ds_swizzle. The right-code
// window slides by one column per step through a rotating register file (no moves).
struct HChunk16 {
    uint64_t cl, inj;
};

// entries of chunk `chunk` for the 16 lanes of a row (i16 = lane within the row); LPL: lanes
// per line (the window spans LPL * DPL disparities)
template <int DPL, int DX, int LPL>
__device__ __forceinline__ HChunk16 hload16(const uint64_t* cLr, const uint64_t* cRr, const Geom& g, int chunk,
                                            int i16)
{
    const int i = chunk * 16 + i16;
    const int x = DX > 0 ? g.minX1 + i : g.maxX1 - 1 - i;
    HChunk16 c;
    c.cl = cLr[min(max(x, 0), g.W - 1)];
    const int xr = DX > 0 ? x + 1 - g.minD : x - g.minD - LPL * DPL;   // code entering the window
    c.inj = cRr[min(max(xr, 0), g.W - 1)];
    return c;
}

// One image row per path line (LPL = 16: four lines per wave; 32: two, each a row pair of
// lanes), rows y0 + line. With 32-lane lines both rows of a line load the same chunk
// entries, so the per-row broadcasts serve the whole line.
template <int DPL, bool EXACT, int DX, bool PRIO = false, int LPL = 16>
__device__ __forceinline__ void p16_horiz(const uint64_t* __restrict__ cL, const uint64_t* __restrict__ cR,
                                          uint8_t* __restrict__ V, uint8_t* __restrict__ trash, const Geom& g,
                                          int y0)
{
    static_assert(LPL == 16 || LPL == 32, "horizontal scans: 16- or 32-lane lines");
    constexpr int M = DPL / 2;
    constexpr int U = DPL > 16 ? DPL : 16;       // unroll: window rotation period and chunk size
    const int lane = threadIdx.x & 63;
    const int r = lane / LPL, p = lane % LPL;
    const int y = y0 + r;
    const bool rowok = y < g.H;
    const int yc = min(y, g.H - 1);
    const uint64_t* cLr = cL + (size_t)yc * g.W;
    const uint64_t* cRr = cR + (size_t)yc * g.W;
    uint32_t imask[M], start[M];
    make_imask<DPL, EXACT>(p, g.D, imask, start);
    const uint32_t P1P1 = (uint32_t)g.P1 * 0x10001u, P2P2 = ((uint32_t)g.P2 + kBaseP) * 0x10001u;
    const int n = g.width1;
    const int xfirst = DX > 0 ? g.minX1 : g.maxX1 - 1;
    uint64_t cr[DPL];                             // physical window registers
#pragma unroll
    for (int k = 0; k < DPL; k++) cr[k] = cRr[min(max(xfirst - g.minD - p * DPL - k, 0), g.W - 1)];
    uint32_t Lr[M];
#pragma unroll
    for (int i = 0; i < M; i++) Lr[i] = start[i];
    uint8_t* rowbase = V + (size_t)yc * g.width1 * g.D + p * DPL;
    uint8_t* tr = trash + lane * DPL;
    const bool lane_ok = rowok && (EXACT || p * DPL < g.D);
    const bool hi_ok = EXACT || p * DPL + 16 < g.D;            // DPL == 32 only
    HChunk16 cur = hload16<DPL, DX, LPL>(cLr, cRr, g, 0, lane & 15);
    HChunk16 nxt = cur;
    for (int b = 0; b * U < n; b++) {
        if constexpr (PRIO) lr_prio(((n - b * U) * SGM_LRPRIO_HW) >> 6, g.H);   // a scan step ~0.58 row steps
        static_for<0, U>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            if constexpr (t % 16 == 0) nxt = hload16<DPL, DX, LPL>(cLr, cRr, g, (b * U + t) / 16 + 1, lane & 15);
            const int i = b * U + t;
            const uint64_t cl = row_bcast_u64<t % 16>(cur.cl);
            const uint64_t inj = row_bcast_u64<t % 16>(cur.inj);
            // logical window index k lives in physical register (k - t) (DX>0) / (k + t) (DX<0)
            uint32_t Labs[M];
            p16_step<DPL, EXACT, LPL>(Lr, cl, [&](int k) { return cr[DX > 0 ? ((k - t) % DPL + DPL) % DPL : (k + t) % DPL]; },
                                      P1P1, P2P2, imask, Labs);
            const int x1 = DX > 0 ? i : n - 1 - i;
            const bool ok = lane_ok && i < n;
            uint8_t* dst = ok ? rowbase + (size_t)x1 * g.D : tr;
            store_pairs<DPL>(dst, (ok && hi_ok) ? dst + 16 : tr + 16, Labs);
            if constexpr (DX > 0) {
                constexpr int ph = ((DPL - 1 - t) % DPL + DPL) % DPL;
                cr[ph] = LPL == 32 ? line32_shr1_u64(cr[ph], inj) : row_shr1_u64(cr[ph], inj);
            } else {
                constexpr int ph = t % DPL;
                cr[ph] = LPL == 32 ? line32_shl1_u64(cr[ph], inj) : row_shl1_u64(cr[ph], inj);
            }
            if constexpr (t % 16 == 15) cur = nxt;
        });
    }
}

// ---------------------------------------------------------------- row sweeps ----------
// Workgroup = 4 waves of 64 / LPL lines each (NL = 256 / LPL adjacent lines). LPL = 16: a
// line is one 16-lane row (slot j = 4*wave + row). LPL = 8: a 16-lane row holds two lines,
// interleaved by lane parity (lane = 2*p + line), so a line's d-neighbour lanes are 2 apart
// and its min over D stays inside the parity (p16_step, line_min_u32); slot j =
// 8*wave + 2*row + parity. LPL = 32: a line is a row pair (slot j = 2*wave + half). Each step the WG stages the row's right-code segment
// (LPL*DPL + NL - 1 codes) and the NL left codes in LDS, double-buffered, one barrier per
// step. The segment is padded so that the lanes' strided window reads spread over the
// banks (LPL 16 and 32: one code per 16, a lane stride of 17 codes; LPL 8: four codes per
// 32, a lane stride of 36 codes = 8 banks, conflict-free for the four lines of a 32-lane half).
template <int DPL, int LPL>
struct RowSeg {
    static constexpr int NL = kWG / LPL;                     // lines per workgroup
    static constexpr int NSEG = LPL * DPL + NL - 1;
    static constexpr int NPAD = LPL >= 16 ? NSEG + NSEG / 16 + 1 : NSEG + 4 * (NSEG / 32) + 4;
    static constexpr int NTOT = NSEG + NL;                   // codes staged per step
    static constexpr int NLOAD = (NTOT + kWG - 1) / kWG;     // per thread
    static constexpr int BUF = NPAD + NL + kWG;              // + cL + dummy slots
    static __device__ __forceinline__ int phys(int e) { return LPL >= 16 ? e + (e >> 4) : e + 4 * (e >> 5); }
};
// row-sweep geometry for a 16-lane DPL: LineCfg's lines, or with SGM_ROWS_LPL8 D <= 256
// sweeps with 8 lanes per line (twice the disparities per lane: the per-step overhead and the
// row's code reads are shared by 32 lines; measured slower)
template <int DPL16>
struct RowsCfg {
#if SGM_ROWS_LPL8
    static constexpr int LPL = DPL16 <= 16 ? 8 : LineCfg<DPL16>::LPL;
#else
    static constexpr int LPL = LineCfg<DPL16>::LPL;
#endif
    static constexpr int DPL = DPL16 * 16 / LPL;
    static constexpr int NL = kWG / LPL;
};

// The code images have kCodeMargin readable codes before and after them (workspace
// layout), and the codes outside [0, W) of a row feed only lines or lanes whose results go
// to the trash slot, so each lane keeps ONE byte offset for the whole sweep and a step moves
// the wave-uniform base (SGPR base + VGPR offset loads, no per-step VALU).
template <int DPL, int LPL>
using SegRegs = uint64_t[RowSeg<DPL, LPL>::NLOAD];     // one step's staged codes per thread
template <int DPL, int LPL>
struct SegAddr {
    uint32_t off[RowSeg<DPL, LPL>::NLOAD];   // byte offsets from the step base
    const char* lo;                          // min(cL, cR) - bias codes
};
template <int DPL, int LPL>
__device__ __forceinline__ SegAddr<DPL, LPL> seg_addr(const uint64_t* cL, const uint64_t* cR, const Geom& g, int tid)
{
    using RS = RowSeg<DPL, LPL>;
    SegAddr<DPL, LPL> a;
    const uint64_t* base = cL < cR ? cL : cR;
    const int bias = LPL * DPL + max(g.minD, 0);        // makes every lane offset >= 0
    a.lo = (const char*)base - (size_t)8 * bias;
#pragma unroll
    for (int m = 0; m < RS::NLOAD; m++) {
        const int q = min(tid + m * kWG, RS::NTOT - 1);
        const int rel = q < RS::NSEG ? (int)(cR - base) + q - g.minD - LPL * DPL + 1 : (int)(cL - base) + (q - RS::NSEG);
        a.off[m] = (uint32_t)(8 * (rel + bias));
    }
    return a;
}
template <int DPL, int LPL>
__device__ __forceinline__ void seg_load(SegRegs<DPL, LPL>& v, const SegAddr<DPL, LPL>& a,
                                         const Geom& g, int rx, int ry, int xb, int s)
{
    const int y = ry > 0 ? s : g.H - 1 - s;
    const int yc = (SGM_EXP & 1) ? 0 : min(max(y, 0), g.H - 1);
    const char* sb = a.lo + (size_t)8 * ((size_t)yc * g.W + (xb + rx * s));   // wave-uniform
#pragma unroll
    for (int m = 0; m < RowSeg<DPL, LPL>::NLOAD; m++) v[m] = *(const uint64_t*)(sb + a.off[m]);
}

template <int DPL, int LPL>
__device__ __forceinline__ void seg_store(uint64_t* buf, const SegRegs<DPL, LPL>& v, int tid)
{
    using RS = RowSeg<DPL, LPL>;
#pragma unroll
    for (int m = 0; m < RS::NLOAD; m++) {
        const int q0 = tid + m * kWG;
        const int at = q0 < RS::NSEG ? RS::phys(q0) : (q0 < RS::NTOT ? RS::NPAD + (q0 - RS::NSEG) : RS::NPAD + RS::NL + tid);
        buf[at] = v[m];
    }
}

// Relative state of a line continued from a neighbouring band: the u8 costs Lprev stored
// for its predecessor pixel (src: the lane's DPL bytes) -> Lprev - min Lprev. Every lane of
// the line takes part (line-wide min); the caller selects per line.
template <int DPL, bool EXACT, int LPL>
__device__ __forceinline__ void p16_seed(const uint8_t* src, const uint32_t (&imask)[DPL / 2], uint32_t (&Lr)[DPL / 2])
{
    uint32_t wd[(DPL + 3) / 4], Labs[DPL / 2];
    wload<DPL>(src, wd);
#pragma unroll
    for (int i = 0; i < DPL / 2; i++) {
        const uint32_t pr = __builtin_amdgcn_perm(0u, wd[i / 2], (i & 1) ? 0x0c030c02u : 0x0c010c00u);
        Labs[i] = pr | kBaseP2;                           // bytes -> biased-f16 patterns
        if (!EXACT) Labs[i] = pk_max(Labs[i], imask[i]);
    }
    p16_relative<DPL, LPL>(Labs, Lr);
}

// The last sweep fused with the WTA (census_fused16 "up+WTA" blocks): the upward vertical
// sweep (dir 1) of a frame whose other seven volumes are complete; at each step every line
// holds L_1(x, y, .) in the WTA's 16-lanes-per-pixel layout, adds the seven stored costs of
// (x, y) and runs the WTA of that pixel, so volume 1 is never written or read. The per-pixel
// results (d16 | best << 16 | minS << 32; rejected: d16 = invalid, best = -1) go to res[y][x];
// k_census_rowfin does disp2 + LR of each row from them.
struct UpWta {
    const uint8_t* vols;     // the frame's volume set: direction v at vols + v * vol_bytes
    size_t vol_bytes;
    uint64_t* res;           // [H][W] results + 64 trash slots
};
struct WtaPix { int best, minS, d16; bool rej; };   // one pixel's WTA result (wta_pix16)
template <int DPL, bool EXACT>
__device__ __forceinline__ WtaPix wta_pix16(const uint32_t (&E)[(DPL + 3) / 4], const uint32_t (&O)[(DPL + 3) / 4],
                                            int p, const Geom& g, float inv_u, uint32_t* srow);
template <int DPL, bool EXACT>
__device__ __forceinline__ void wta_emask(int p, const Geom& g, uint32_t (&emaskE)[(DPL + 3) / 4],
                                          uint32_t (&emaskO)[(DPL + 3) / 4]);
// LDS of an up+WTA block: the row sweep's code buffers, then 16 lines x 32 x NWD S dwords
template <int DPL>
__host__ __device__ constexpr size_t upwta_lds_bytes() { return (size_t)8 * 2 * RowSeg<DPL, 16>::BUF + (size_t)16 * 32 * ((DPL + 3) / 4) * 4; }

// NL lines of direction dir starting at base column xb (DPL disparities per lane, LPL
// lanes per line; lds: 2 * RowSeg<DPL, LPL>::BUF codes).
template <int DPL, bool EXACT, int LPL, bool FUSE = false, bool PRIO = false>
__device__ __forceinline__ void p16_rows(const uint64_t* __restrict__ cL, const uint64_t* __restrict__ cR,
                                         uint8_t* __restrict__ V, uint8_t* __restrict__ trash, const Geom& g, int dir,
                                         int xb, const PathLaunch16& pl, uint64_t* lds, const UpWta& uw = UpWta{})
{
    static_assert(!FUSE || LPL == 16, "up+WTA blocks use 16 lanes per line (the WTA layout)");
    using RS = RowSeg<DPL, LPL>;
    constexpr int M = DPL / 2;
    constexpr int NL = RS::NL;
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int r = lane >> 4;
    const int p = LPL == 32 ? lane & 31 : LPL == 16 ? lane & 15 : (lane & 15) >> 1;    // lane within the line
    const int j = LPL == 32 ? 2 * w + (lane >> 5) : LPL == 16 ? 4 * w + r : 8 * w + 2 * r + (lane & 1);   // slot (line)
    const int rx = dir_rx(dir), ry = dir_ry(dir);
    int s0, s1;
    if (rx == 0) { s0 = 0; s1 = g.H; }
    else if (rx > 0) { s0 = max(0, g.minX1 - xb - (NL - 1)); s1 = min(g.H, g.maxX1 - xb); }
    else { s0 = max(0, xb - g.maxX1 + 1); s1 = min(g.H, xb + NL - g.minX1); }
    if (s0 >= s1) return;                          // uniform over the workgroup
    uint32_t imask[M], start[M];
    make_imask<DPL, EXACT>(p, g.D, imask, start);
    const uint32_t P1P1 = (uint32_t)g.P1 * 0x10001u, P2P2 = ((uint32_t)g.P2 + kBaseP) * 0x10001u;
    uint32_t Lr[M];
#pragma unroll
    for (int i = 0; i < M; i++) Lr[i] = start[i];
    bool pv = false;
    const uint8_t* bnd = pl.bnd[ry > 0 ? 0 : 1];
    if (bnd && s0 == 0) {                          // exact tile mode: continue the band above / below
        const int x = xb + j, xp = x - rx;         // the line's pixel at step 0 and its predecessor
        const bool cont = x >= g.minX1 && x < g.maxX1 && xp >= g.minX1 && xp < g.maxX1;
        const int xs = min(max(xp, g.minX1), g.maxX1 - 1) - g.minX1;
        uint32_t Ls[M];
        p16_seed<DPL, EXACT, LPL>(bnd + bnd_slot_of(dir) * pl.bnd_slot + (size_t)xs * g.D + p * DPL, imask, Ls);
#pragma unroll
        for (int i = 0; i < M; i++) Lr[i] = cont ? Ls[i] : Lr[i];
        pv = cont;
    }
    const bool lane_act = EXACT || p * DPL < g.D;
    const bool hi_ok = EXACT || p * DPL + 16 < g.D;            // DPL == 32 only
    // stores: the step's row base is wave-uniform (64-bit, scalar math); lanes add a 32-bit
    // offset inside the row (< width1 * D), or go to their trash slot
    uint8_t* const tr = trash + (tid & 63) * DPL;
    const int e_hi = j + (LPL - p) * DPL - 1;      // segment index of the lane's k = 0 code

    // Segments are staged in LDS (double buffer, one barrier per step) from registers loaded
    // 3 steps ahead: the counted vmcnt wait for a segment then leaves the stores of the last
    // three steps in flight (gfx950 retires loads and stores on one in-order counter).
    uint64_t* buf0 = lds;
    uint64_t* buf1 = lds + RS::BUF;
    uint64_t R0[RS::NLOAD], R1[RS::NLOAD], R2[RS::NLOAD], R3[RS::NLOAD];
    const SegAddr<DPL, LPL> sa = seg_addr<DPL, LPL>(cL, cR, g, tid);
    seg_load<DPL, LPL>(R0, sa, g, rx, ry, xb, s0);
    seg_store<DPL, LPL>(buf0, R0, tid);
    seg_load<DPL, LPL>(R1, sa, g, rx, ry, xb, min(s0 + 1, s1 - 1));
    seg_load<DPL, LPL>(R2, sa, g, rx, ry, xb, min(s0 + 2, s1 - 1));
    seg_load<DPL, LPL>(R3, sa, g, rx, ry, xb, min(s0 + 3, s1 - 1));
    __syncthreads();

    // up+WTA (FUSE): the seven other volumes of the line's pixel, loaded one step ahead
    constexpr int NWD = (DPL + 3) / 4;
    uint32_t vw[7][NWD], emaskE[NWD], emaskO[NWD];
    uint32_t* srow = (uint32_t*)(lds + 2 * RS::BUF) + j * 32 * NWD;
    const float inv_u = 1.0f / (float)max(100 - g.uniq, 1);
    const uint32_t voff = (uint32_t)((min(max(xb + j, g.minX1), g.maxX1 - 1) - g.minX1) * g.D + (lane_act ? p * DPL : 0));
    auto vload = [&](int s) {
        const uint8_t* rb = uw.vols + (size_t)max(g.H - 1 - s, 0) * g.width1 * g.D;   // wave-uniform
#pragma unroll
        for (int k = 0; k < 7; k++) wload_buf<DPL>(rb + (size_t)(k == 0 ? 0 : k + 1) * uw.vol_bytes, voff, vw[k]);
    };
    if constexpr (FUSE) {
        wta_emask<DPL, EXACT>(p, g, emaskE, emaskO);
        vload(s0);
    }
    auto step = [&](int s, const uint64_t* bufc) {
        const int x = xb + j + rx * s;
        const bool valid = s < s1 && x >= g.minX1 && x < g.maxX1;
        const int y = ry > 0 ? s : g.H - 1 - s;
        const uint64_t cl = bufc[RS::NPAD + j];
        uint32_t Labs[M];
        uint32_t E[NWD], O[NWD];
        if constexpr (FUSE) {       // this step's seven costs, then the next step's loads
#pragma unroll
            for (int jj = 0; jj < NWD; jj++) {
                uint32_t e = 0, o = 0;
#pragma unroll
                for (int k = 0; k < 7; k++) {
                    e += vw[k][jj] & 0x00FF00FFu;
                    o += __builtin_amdgcn_perm(0u, vw[k][jj], 0x0c030c01u);
                }
                asm("" : "+v"(e), "+v"(o));     // the sums, not 14 extracted words, stay live
                E[jj] = e;
                O[jj] = o;
            }
        }
        // path start (first valid pixel of the line): L = C. The P2 cap of the recurrence is
        // lowered to "0" (kBase), which clamps every candidate: one select per step.
        const uint32_t P2x = pv ? P2P2 : kBaseP2;
        if constexpr (FUSE) __builtin_amdgcn_sched_barrier(0);
        p16_step<DPL, EXACT, LPL>(Lr, cl, [&](int k) { return bufc[RS::phys(e_hi - k)]; }, P1P1, P2x, imask, Labs);
        if constexpr (FUSE) {
            __builtin_amdgcn_sched_barrier(0);
            // + L_1: the low byte of each biased-f16 pattern (pair i holds d = 2i, 2i + 1)
#pragma unroll
            for (int jj = 0; jj < NWD; jj++) {
                const uint32_t a = Labs[2 * jj], b = 2 * jj + 1 < M ? Labs[2 * jj + 1] : 0u;
                E[jj] = (E[jj] + __builtin_amdgcn_perm(b, a, 0x0c040c00u)) | emaskE[jj];
                O[jj] = (O[jj] + __builtin_amdgcn_perm(b, a, 0x0c060c02u)) | emaskO[jj];
            }
            // the next step's loads: in flight during this step's WTA (not during the sweep step,
            // whose temporaries they would otherwise share the register file with)
            vload(s + 1);
            __builtin_amdgcn_sched_barrier(0);
            const WtaPix px = wta_pix16<DPL, EXACT>(E, O, p, g, inv_u, srow);
            const uint64_t v = (uint64_t)(uint16_t)(px.rej ? g.invalid : px.d16) |
                               ((uint64_t)(uint16_t)(px.rej ? -1 : px.best) << 16) | ((uint64_t)(uint16_t)px.minS << 32);
            // lane 0 of each line stores its pixel; the other lanes' stores go past the row
            // descriptor's range, where the hardware drops them (no branch, and no trash slot:
            // 60 of 64 lanes storing into one shared 512-B slot every step made all the frames'
            // up+WTA waves contend on the same lines — 3 frames per launch ran 5x slower)
            const __amdgpu_buffer_rsrc_t rr =
                __builtin_amdgcn_make_buffer_rsrc((void*)(uw.res + (size_t)y * g.W), 0, g.W * 8, 0x00020000);
            typedef unsigned int v2u __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), rr,
                                                  (valid && p == 0) ? (uint32_t)x * 8u : 0x80000000u, 0, 2);
        } else {
            const bool ok = valid && lane_act && !((SGM_EXP & 2) && dir == 1);
            uint8_t* const vrow = V + (size_t)min(max(y, 0), g.H - 1) * g.width1 * g.D;
            uint8_t* const dst = ok ? vrow + (uint32_t)((x - g.minX1) * g.D + p * DPL) : tr;
            store_pairs<DPL>(dst, (ok && hi_ok) ? dst + 16 : tr + 16, Labs);
        }
        pv = valid;
    };
    // step s reads buf[s & 1] (holding segment s), then segment s + 1 (register set
    // (s + 1) % 4) goes to buf[(s + 1) & 1] and set s % 4 is reloaded with segment s + 4
    auto body = [&](int s, const uint64_t* bcur, uint64_t* bnext, uint64_t (&Rnext)[RS::NLOAD],
                    uint64_t (&Rfree)[RS::NLOAD]) {
        seg_load<DPL, LPL>(Rfree, sa, g, rx, ry, xb, min(s + 4, s1 - 1));
        step(s, bcur);
        seg_store<DPL, LPL>(bnext, Rnext, tid);
        __syncthreads();
    };
    for (int s = s0; s < s1; s += 4) {
        if constexpr (PRIO) lr_prio(rx != 0 ? ((s1 - s) * SGM_LRPRIO_DIAG) >> 6 : s1 - s, g.H);
        body(s, buf0, buf1, R1, R0);
        body(s + 1, buf1, buf0, R2, R1);
        body(s + 2, buf0, buf1, R3, R2);
        body(s + 3, buf1, buf0, R0, R3);
    }
}

// One work-list entry: the lines of one block of one direction of one frame (LineCfg<DPL>::HROWS
// rows for the horizontal scans, RowsCfg<DPL>::NL columns for the row sweeps; lds: rows_lds_codes).
template <int DPL>
__host__ __device__ constexpr int rows_lds_codes() { return 2 * RowSeg<RowsCfg<DPL>::DPL, RowsCfg<DPL>::LPL>::BUF; }

template <int DPL, bool EXACT, bool PRIO = false>
__device__ __forceinline__ void paths_block16(const PathFrames& pf, size_t vol_bytes, size_t trash_off,
                                              const Geom& g, const PathLaunch16& pl, uint32_t it, uint64_t* lds)
{
    using RC = RowsCfg<DPL>;
    using HC = LineCfg<DPL>;
    const int dir = (int)(it >> 24);
    const int f = (int)((it >> 22) & 3u);
    const int lb = (int)(it & 0x3FFFFFu);
    if (f >= pf.n || ((pf.skip_dirs >> dir) & 1u)) return;    // uniform over the workgroup
    const uint64_t* cL = pick4(pf.cL, f);
    const uint64_t* cR = pick4(pf.cR, f);
    uint8_t* V = pick4(pf.vols, f) + (size_t)dir * vol_bytes;
    uint8_t* trash = V + trash_off;
    const int y0 = lb * HC::HROWS + (64 / HC::LPL) * (threadIdx.x >> 6);
    if (dir == 6) p16_horiz<HC::DPL, EXACT, 1, PRIO, HC::LPL>(cL, cR, V, trash, g, y0);
    else if (dir == 7) p16_horiz<HC::DPL, EXACT, -1, PRIO, HC::LPL>(cL, cR, V, trash, g, y0);
    else p16_rows<RC::DPL, EXACT, RC::LPL, false, PRIO>(cL, cR, V, trash, g, dir, pl.xb_lo[dir] + lb * RC::NL, pl, lds);
}

// SGM_TRACE debug timeline: one 4 x u64 record per wave {tag | blockIdx << 32, XCC_ID << 32 |
// HW_ID, start, end} (s_memrealtime, 100 MHz)
__device__ __forceinline__ void trace_record(uint64_t* trace, uint64_t tag, uint64_t t0)
{
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));     // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // XCC_ID
    uint64_t* r = trace + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4;
    r[0] = tag | ((uint64_t)blockIdx.x << 32); r[1] = ((uint64_t)xcc << 32) | hw; r[2] = t0; r[3] = t1;
}

template <int DPL, bool EXACT>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(DPL >= 32 && !SGM_P32 ? SGM_WPE32 : SGM_WPE)))
void k_census_paths16(PathFrames pf, size_t vol_bytes, size_t trash_off, Geom g, PathLaunch16 pl,
                      const uint32_t* __restrict__ items, uint64_t* __restrict__ trace)
{
    __shared__ uint64_t lds[rows_lds_codes<DPL>()];
    const uint64_t t0 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    paths_block16<DPL, EXACT, true>(pf, vol_bytes, trash_off, g, pl, items[blockIdx.x], lds);
    if (trace && (threadIdx.x & 63) == 0)        // debug timeline (SGM_TRACE): one record per wave
        trace_record(trace, items[blockIdx.x], t0);
}

// ====================================================================================
// Sum of the 8 path volumes + WTA + uniqueness + subpixel + disp2 + LR check.
// One workgroup (4 waves) per image row. 16 lanes per pixel (the P16 layout of the path
// engine): each wave-instruction covers 4 consecutive pixels, lane p of a row holds
// d = p*DPL .. p*DPL + DPL-1, loaded as one DPL-byte vector per volume (coalesced).
//  * S = sum of 8 u8 volumes in SWAR u16 pairs: even bytes (w & 0x00FF00FF) and odd bytes
//    (perm) accumulate separately, <= 8*255 per half, so 32-bit adds never carry over.
//  * best and minS in ONE 16-lane min-reduction over key = S*512 + d (first minimal d).
//  * uniqueness: a second key-min over d outside [best-1, best+1].
//  * S[best-1], S[best+1] for the subpixel fit: read back from a per-row LDS slice.
// Results go to the row's LDS arrays; row_finish() does disp2 (LDS atomics) + LR + store.
// ====================================================================================
// LDS bytes of one WTA row: the per-row S slices share their space with RowLds::key (the
// slices are dead before row_finish), then the rest of RowLds
template <int DPL>
__host__ __device__ constexpr size_t wta_key_bytes(int W)
{
    // per lane 2 * NWD dwords of packed S (NWD = (DPL + 3) / 4)
    return (size_t)kWG * 8 * ((DPL + 3) / 4) > (size_t)4 * W ? (size_t)kWG * 8 * ((DPL + 3) / 4) : (size_t)4 * W;
}
template <int DPL>
__host__ __device__ constexpr size_t wta_lds_bytes(int W) { return wta_key_bytes<DPL>(W) + RowLds::rest_bytes(W); }

// WTA of the 4 pixels a wave holds (one per 16-lane row, lane p: d = p*DPL ..), from their
// S in packed u16 pairs: E[j] = (S[4j], S[4j+2]), O[j] = (S[4j+1], S[4j+3]); halves past D or
// past the lane's DPL hold 0xFFFF. srow: the row's LDS slice (16 lanes x 2 * NWD dwords).
template <int DPL, bool EXACT>
__device__ __forceinline__ WtaPix wta_pix16(const uint32_t (&E)[(DPL + 3) / 4], const uint32_t (&O)[(DPL + 3) / 4],
                                            int p, const Geom& g, float inv_u, uint32_t* srow)
{
    constexpr int NWD = (DPL + 3) / 4;
    // packed-key geometry: lane-local index k in the low KB bits of a 16-bit key
    constexpr int KB = DPL > 16 ? 5 : 4;
    constexpr uint32_t KMASK = (1u << KB) - 1;
    // ---- (minS, best): packed 16-bit keys S << KB | k, one 16-lane min over S*512 + d ----
    uint32_t km = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < NWD; j++) {
        const uint32_t ke = pk_shl(E[j], KB) | (((uint32_t)(4 * j + 2) << 16) | (uint32_t)(4 * j));
        const uint32_t ko = pk_shl(O[j], KB) | (((uint32_t)(4 * j + 3) << 16) | (uint32_t)(4 * j + 1));
        km = pk_min(km, pk_min(ke, ko));
    }
    km = pk_min(km, alignbit16(km, km)) & 0xFFFFu;      // lane min key (low half)
    const uint32_t kmin = row_min_u32(((km >> KB) << 9) | (uint32_t)(p * DPL + (int)(km & KMASK)));
    WtaPix r;
    const int best = (int)(kmin & 511u);
    const int minS = (int)(kmin >> 9);
    // ---- the row's packed S slice in LDS (S[best +- 1] for subpixel and uniqueness) ----
#pragma unroll
    for (int j = 0; j < NWD; j++) { srow[p * 2 * NWD + j] = E[j]; srow[p * 2 * NWD + NWD + j] = O[j]; }
    auto s_at = [&](int d) {
        const int kk = d % DPL;
        const uint32_t v = srow[(d / DPL) * 2 * NWD + (kk & 1) * NWD + (kk >> 2)];
        return (int)((v >> (16 * ((kk >> 1) & 1))) & 0xFFFFu);
    };
    const int sm = s_at(max(best - 1, 0)), sp = s_at(min(best + 1, 16 * DPL - 1));
    // ---- uniqueness: reject if some d outside [best-1, best+1] has S*(100-u) < minS*100.
    // For u < 100 that is S <= thr = (minS*100 - 1) / (100 - u); with T = thr + 1 the sum of
    // max(T - S, 0) over the row exceeds its window part exactly when such a d exists. For
    // u >= 100 every d qualifies when minS > 0, and for u > 100, minS == 0 those with S > 0
    // (the count of S == 0 outside the window is the same sum with T = 1).
    int T = 0;
    if (g.uniq < 100) {
        if (minS > 0) {
            const int num = minS * 100 - 1, den = 100 - g.uniq;
            int q = (int)((float)num * inv_u);
            q += (q + 1) * den <= num ? 1 : 0;
            q -= q * den > num ? 1 : 0;
            T = min(q + 1, 8 * 255 + 1);      // S <= 8 * 255: keeps the u16 sums exact
        }
    } else {
        T = (minS == 0 && g.uniq > 100) ? 1 : 0;
    }
    const uint32_t TT = (uint32_t)T * 0x10001u;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < NWD; j++) acc += pk_subs(TT, E[j]) + pk_subs(TT, O[j]);   // halves <= 2 * NWD * 2041: no carry
    const int tot = (int)row_sum_u32(__builtin_amdgcn_sad_u16(acc, 0u, 0u));
    const int win = max(T - minS, 0) + (best > 0 ? max(T - sm, 0) : 0) + (best < g.D - 1 ? max(T - sp, 0) : 0);
    int outside = tot - win;
    if (g.uniq >= 100) {
        const int nwin = 1 + (best > 0 ? 1 : 0) + (best < g.D - 1 ? 1 : 0);
        outside = minS > 0 ? g.D - nwin : (g.uniq > 100 ? (g.D - nwin) - outside : 0);
    }
    r.rej = outside > 0;
    const int den = max(sm + sp - 2 * minS, 1);
    const bool use = g.subpix && best > 0 && best < g.D - 1;
    r.d16 = best * 16 + (use ? tdiv_rcp((sm - sp) * 16 + den, 2 * den) : 0) + g.minD * 16;
    r.best = best;
    r.minS = minS;
    return r;
}

// 0xFFFF in the S halves of a lane that hold k >= DPL or d >= D (the E / O split above)
template <int DPL, bool EXACT>
__device__ __forceinline__ void wta_emask(int p, const Geom& g, uint32_t (&emaskE)[(DPL + 3) / 4],
                                          uint32_t (&emaskO)[(DPL + 3) / 4])
{
#pragma unroll
    for (int j = 0; j < (DPL + 3) / 4; j++) {
        auto bad = [&](int k) { return k >= DPL || (!EXACT && p * DPL + k >= g.D); };
        emaskE[j] = (bad(4 * j) ? 0xFFFFu : 0u) | (bad(4 * j + 2) ? 0xFFFF0000u : 0u);
        emaskO[j] = (bad(4 * j + 1) ? 0xFFFFu : 0u) | (bad(4 * j + 3) ? 0xFFFF0000u : 0u);
    }
}

// One image row y (one workgroup). lds: wta_lds_bytes<DPL>(W) bytes.
template <int DPL, bool EXACT, typename OutT = int16_t>
__device__ __forceinline__ void wta_row16(const uint8_t* __restrict__ vols, size_t vol_bytes, const Geom& g,
                                          OutT* __restrict__ out, size_t out_stride, int y, uint32_t* lds)
{
    constexpr int NWD = (DPL + 3) / 4;            // dwords per lane per volume
    uint32_t* sl = lds;                           // 4 waves x 4 rows x 16 lanes x 2*NWD packed S dwords
    RowLds R(lds, (char*)lds + wta_key_bytes<DPL>(g.W), g.W);   // R.key aliases sl
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);     // wave index (uniform: SGPR)
    const int r = lane >> 4, p = lane & 15;
    R.init(g, tid, kWG, false);
    const bool lane_act = EXACT || p * DPL < g.D;
    // wave-uniform 64-bit volume row base (a C5 volume is 5.5 GB) + 32-bit lane offsets:
    // SGPR-base + VGPR-offset addressing
    const size_t row0 = (size_t)y * g.width1 * g.D;
    const uint32_t off0 = (uint32_t)(lane_act ? p * DPL : 0);
    uint32_t* srow = sl + (w * 4 + r) * 32 * NWD;     // 16 lanes x 2 * NWD dwords
    uint32_t emaskE[NWD], emaskO[NWD];            // 0xFFFF in halves with k >= DPL or d >= D
    wta_emask<DPL, EXACT>(p, g, emaskE, emaskO);
    const float inv_u = 1.0f / (float)max(100 - g.uniq, 1);
    const int n = g.width1;
    const int nq = (n + 3) / 4;
    // pixel 4q + r: the group's base is wave-uniform, the lane keeps one offset. The last
    // group reads up to 3 pixels past the row (the next row, or the volume's trash slot
    // after the last row); their results are never stored.
    // Buffer loads (one descriptor per volume from the wave-uniform group base, the lane's
    // offset in a VGPR): no per-lane 64-bit address arithmetic.
    const uint32_t loff = off0 + (uint32_t)(r * g.D);
    auto load = [&](int q, uint32_t (&v)[8][NWD]) {
        const uint8_t* rowq = vols + row0 + (size_t)(4 * q) * g.D;
#pragma unroll
        for (int vv = 0; vv < 8; vv++) {
            if ((SGM_EXP & 4) && vv == 1) { for (int j = 0; j < NWD; j++) v[vv][j] = 0; continue; }
            wload_buf<DPL>(rowq + (size_t)vv * vol_bytes, loff, v[vv]);
        }
    };
    // S in u16 pairs (wta_pix16). The next pixel group's loads are summed at the end of an
    // iteration, so only one set of raw volume words is live.
    uint32_t E[NWD], O[NWD];
    auto sum8 = [&](const uint32_t (&v)[8][NWD]) {
#pragma unroll
        for (int j = 0; j < NWD; j++) {
            uint32_t e = 0, o = 0;
#pragma unroll
            for (int vv = 0; vv < 8; vv++) {
                e += v[vv][j] & 0x00FF00FFu;
                o += __builtin_amdgcn_perm(0u, v[vv][j], 0x0c030c01u);
            }
            E[j] = e | emaskE[j];
            O[j] = o | emaskO[j];
        }
    };
    uint32_t nxt[8][NWD];
    load(min(w, nq - 1), nxt);
    sum8(nxt);
    for (int q = w; q < nq; q += 4) {
        load(min(q + 4, nq - 1), nxt);
        const WtaPix px = wta_pix16<DPL, EXACT>(E, O, p, g, inv_u, srow);
        // ---- results: lane 0 of each row writes its pixel, the others hit dummy slots ----
        const int x1 = 4 * q + r;
        const bool wr = p == 0 && x1 < n;
        const int x = wr ? g.minX1 + x1 : g.W + lane;
        R.bst[x] = (int16_t)(px.rej ? -1 : px.best);
        R.mins[x] = (uint16_t)px.minS;
        R.drow[(wr && !px.rej) ? x : g.W + lane] = (int16_t)px.d16;
        sum8(nxt);
    }
    R.init_key(g, tid, kWG);                      // the S slices are dead: key takes their space
    row_finish(g, tid, kWG, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, out + (size_t)y * out_stride);
}

// block b: row b % H of frame b / H
template <int DPL, bool EXACT>
__device__ __forceinline__ void wta_block16(const WtaFrames& wf, size_t vol_bytes, const Geom& g, size_t out_stride,
                                            int b, uint32_t* lds)
{
    const int f = b / g.H;
    wta_row16<DPL, EXACT>(pick4(wf.vols, f), vol_bytes, g, pick4(wf.out, f), out_stride, b - f * g.H, lds);
}

template <int DPL, bool EXACT>
__global__ __launch_bounds__(kWG) void k_census_wta16(WtaFrames wf, size_t vol_bytes, Geom g, size_t out_stride)
{
    extern __shared__ uint32_t lds_dyn[];
    wta_block16<DPL, EXACT>(wf, vol_bytes, g, out_stride, blockIdx.x, lds_dyn);
}

// The same for one frame whose rows go out as float (the node's CV_32FC1) straight into a host
// buffer mapped into the device's address space: the row stores cross PCIe while the other rows'
// volume reads run, instead of a to-float kernel and an 8 MB copy after the frame (the node's
// host call, matcherOpenCVSGBM.cpp:34 / generate_disparity.cpp:350-357).
template <int DPL, bool EXACT>
__global__ __launch_bounds__(kWG) void k_census_wta16f(WtaFrames wf, size_t vol_bytes, Geom g)
{
    extern __shared__ uint32_t lds_dyn[];
    wta_row16<DPL, EXACT, float>(wf.vols[0], vol_bytes, g, wf.outf[0], wf.outf_stride, blockIdx.x, lds_dyn);
}

// ------------------------------------------------------------------------------------
// Frame pipelining: one launch runs the path sweeps of a group of frames (VALU-bound) and
// the WTA rows of the previous group (HBM-bound). Blocks [0, n_items) walk the path work
// list (longest first, frames interleaved: more blocks than resident slots, so the
// hardware dispatcher balances the CUs), the blocks after them are WTA rows, which fill
// the CUs the path sweeps' tail leaves idle (measured at C3 for one frame: WTA first
// 2.02 ms, interleaved 1.97, evenly from 30 % 1.92, last 1.71).
// ------------------------------------------------------------------------------------
// Census of the next group in the same launch: 64 x 32 pixel blocks (a 38 x 72 byte LDS
// tile, 8 pixels per thread), dispatched after every path and WTA block, so they run in
// the tail where CUs idle. Images are blocks [0, 2n): frame i left = 2i, right = 2i+1.
constexpr int kCensusRows = 32;

__device__ __forceinline__ void census_block(const CensusFrames& cf, int W, int H, int b, uint8_t* tile)
{
    const int bx = (W + 63) / 64, per_img = bx * ((H + kCensusRows - 1) / kCensusRows);
    const int img = b / per_img, r = b - img * per_img;
    const int f = img >> 1, by = r / bx;
    const uint8_t* src = (img & 1) ? pick4(cf.R, f) : pick4(cf.L, f);
    uint64_t* out = (img & 1) ? pick4(cf.cR, f) : pick4(cf.cL, f);
    const int x0 = (r - by * bx) * 64, y0 = by * kCensusRows;
    constexpr int TH = kCensusRows + 6;
    if (cf.rect.tab) {      // rectify on the fly: tile = remap(raw) at the clamped positions
        // (selects, not a dynamic index: that would copy the kernel argument to scratch)
        const float* mx = (img & 1) ? cf.rect.map[2] : cf.rect.map[0];
        const float* my = (img & 1) ? cf.rect.map[3] : cf.rect.map[1];
        uint8_t* rect = (img & 1) ? pick4(cf.rectR, f) : pick4(cf.rectL, f);
        for (int i = threadIdx.x; i < TH * 72; i += kWG) {
            const int ty = i / 72, tx = i - ty * 72;
            const int yy = min(max(y0 + ty - 3, 0), H - 1), xx = min(max(x0 + tx - 4, 0), W - 1);
            const size_t m = (size_t)yy * cf.rect.map_stride + xx;
            const uint8_t v = remap_cubic_px(src, cf.stride, cf.rect.src_w, cf.rect.src_h, mx[m], my[m], cf.rect.tab);
            tile[i] = v;
            // each rectified pixel is written by the one block whose interior holds it
            if (rect && ty >= 3 && ty < 3 + kCensusRows && tx >= 4 && tx < 68 && y0 + ty - 3 < H && x0 + tx - 4 < W)
                rect[(size_t)yy * cf.rect_stride + xx] = v;
        }
    } else {
        for (int i = threadIdx.x; i < TH * 72; i += kWG) {
            const int ty = i / 72, tx = i - ty * 72;
            const int yy = min(max(y0 + ty - 3, 0), H - 1), xx = min(max(x0 + tx - 4, 0), W - 1);
            tile[i] = src[(size_t)yy * cf.stride + xx];
        }
    }
    __syncthreads();
    const int tx = threadIdx.x & 63, x = x0 + tx;
    if (x >= W) return;
    for (int ty = threadIdx.x >> 6; ty < kCensusRows; ty += kWG / 64) {
        const int y = y0 + ty;
        if (y >= H) break;
        out[(size_t)y * W + x] = census_code_lds<72>(tile, ty, tx);
    }
}

// census (optionally rectifying) of all frames of cf on its own: one block per 64 x 32 tile
__global__ __launch_bounds__(kWG) void k_census_tiles(CensusFrames cf, int W, int H)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[(kCensusRows + 6) * 72];
    census_block(cf, W, H, blockIdx.x, tile);
}

// blocks: [0, n_items) path items of pf | H * wf.n WTA rows of wf | census blocks of cf.
// wta_rows = 0: wf is served by up+WTA items (dir 8) of the work list instead of WTA rows.
template <int DPL, bool EXACT>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(DPL >= 32 ? SGM_WPE32 : SGM_WPE)))
void k_census_fused16(PathFrames pf, WtaFrames wf, CensusFrames cf, size_t vol_bytes, size_t trash_off, Geom g,
                      PathLaunch16 pl, const uint32_t* __restrict__ items, int n_items, size_t out_stride,
                      int period16, int wta_rows, uint64_t* __restrict__ trace)
{
    extern __shared__ uint64_t lds_dyn64[];
    const uint64_t t0 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const int b = blockIdx.x;
    const int n_wta = wta_rows ? g.H * wf.n : 0;
    // paths and WTA blocks merged: among the first b+1 blocks, wcount(b) are WTA rows
    // (one in period16/16 blocks, period16 = 0: all WTA rows after the paths)
    auto wcount = [&](int bb) {
        int w = period16 > 0 ? min((bb + 1) * 16 / period16, n_wta) : 0;
        return max(w, bb + 1 - n_items);
    };
    int kind = 2, idx = b - n_items - n_wta;
    if (b < n_items + n_wta) {
        const int w = wcount(b);
        const bool is_wta = w > (b > 0 ? wcount(b - 1) : 0);
        kind = is_wta ? 1 : 0;
        idx = is_wta ? w - 1 : b - w;
    }
    if (kind == 0) {
        const uint32_t it = items[idx];
        if constexpr (DPL > 16) {           // D > 256: no up+WTA items (host layout)
            paths_block16<DPL, EXACT>(pf, vol_bytes, trash_off, g, pl, it, lds_dyn64);
        } else if ((it >> 24) == 8u) {      // up+WTA of frame f of wf
            using RC = RowsCfg<DPL>;
            const int f = (int)((it >> 22) & 3u);
            if (f < wf.n) {
#if SGM_UPWTA_PRIO
                __builtin_amdgcn_s_setprio(SGM_UPWTA_PRIO);   // the launch's longest blocks
#endif
                const UpWta uw{pick4(wf.vols, f), vol_bytes, pick4(wf.res, f)};
                p16_rows<DPL, EXACT, 16, true>(pick4(wf.cL, f), pick4(wf.cR, f), nullptr, nullptr, g, 1,
                                               pl.xb_lo[1] + (int)(it & 0x3FFFFFu) * 16, pl, lds_dyn64, uw);
            }
        } else {
            paths_block16<DPL, EXACT>(pf, vol_bytes, trash_off, g, pl, it, lds_dyn64);
        }
    } else if (kind == 1) {
        wta_block16<DPL, EXACT>(wf, vol_bytes, g, out_stride, idx, (uint32_t*)lds_dyn64);
    } else {
        census_block(cf, g.W, g.H, idx, (uint8_t*)lds_dyn64);
    }
    if (trace && (threadIdx.x & 63) == 0)         // debug timeline (SGM_TRACE), kind in bits 62-63
        trace_record(trace, (kind == 0 ? items[idx] : 0u) | ((uint64_t)kind << 62), t0);
}

// disp2 + LR check + store of one row from the up+WTA results: block b = row b % H of frame
// b / H of wf (wf.res in, wf.out written)
__global__ __launch_bounds__(kWG) void k_census_rowfin(WtaFrames wf, Geom g, size_t out_stride)
{
    extern __shared__ uint32_t lds_dyn[];
    const int f = blockIdx.x / g.H, y = blockIdx.x - f * g.H;
    const uint64_t* res = pick4(wf.res, f) + (size_t)y * g.W;
    RowLds R(lds_dyn, g.W);
    R.init(g, threadIdx.x, kWG, true);
    for (int x = g.minX1 + threadIdx.x; x < g.maxX1; x += kWG) {
        const uint64_t v = __builtin_nontemporal_load(res + x);
        R.drow[x] = (int16_t)(uint16_t)v;
        R.bst[x] = (int16_t)(uint16_t)(v >> 16);
        R.mins[x] = (uint16_t)(v >> 32);
    }
    row_finish(g, threadIdx.x, kWG, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, pick4(wf.out, f) + (size_t)y * out_stride);
}

// ------------------------------------------------------------------------------------
// host-side launchers
// ------------------------------------------------------------------------------------
hipError_t launch_census(const uint8_t* L, const uint8_t* R, size_t stride, int W, int H, uint64_t* cL,
                         uint64_t* cR, hipStream_t st)
{
    dim3 grid((W + 63) / 64, (H + 3) / 4, R ? 2 : 1);
    hipLaunchKernelGGL(k_census9x7, grid, dim3(256), 0, st, L, R, stride, W, H, cL, cR);
    return hipGetLastError();
}

static int dpl16_for(int D) { return D <= 32 ? 2 : D <= 64 ? 4 : D <= 128 ? 8 : D <= 256 ? 16 : 32; }
// lines per row-sweep workgroup (RowsCfg<DPL>::NL of the launch's DPL)
static int rows_lines(int D)
{
    switch (dpl16_for(D)) {
    case 2: return RowsCfg<2>::NL;
    case 4: return RowsCfg<4>::NL;
    case 8: return RowsCfg<8>::NL;
    case 16: return RowsCfg<16>::NL;
    default: return RowsCfg<32>::NL;
    }
}
// image rows per horizontal-scan workgroup (LineCfg<DPL>::HROWS of the launch's DPL)
static int hscan_rows(int D) { return dpl16_for(D) == 32 ? LineCfg<32>::HROWS : LineCfg<16>::HROWS; }

PathLaunch16 make_path_launch16(const Geom& g)
{
    PathLaunch16 pl{};
    for (int dir = 0; dir < 6; dir++) pl.xb_lo[dir] = g.minX1 - (dir_rx(dir) > 0 ? g.H - 1 : 0);
    return pl;
}

// Work list of one paths launch for a group of `group` frames: every 16-line block of
// every direction in dir_mask (bit d: direction d) of every frame, longest first with
// the frames of equal-length blocks adjacent, dealt in a snake over rounds of n_slots
// workgroups (consecutive workgroup ids go to different CUs, so each CU mixes long and
// short work; with group > 1 there are more blocks than resident slots and the dispatcher
// hands the short ones to whichever CUs drain first).
// up_group > 0 adds the up+WTA blocks (dir code 8, the dir-1 column blocks) of that many
// frames of the launch's WTA group, first: they are the longest.
int census_path_items(const Geom& g, unsigned dir_mask, int n_slots, int group, uint32_t* out, int cap, int up_group)
{
    struct Item { int len; uint32_t code; };
    std::vector<Item> v;
    const PathLaunch16 pl = make_path_launch16(g);
    group = std::min(std::max(group, 1), kMaxGroup);
    up_group = std::min(std::max(up_group, 0), kMaxGroup);
    {
        const int NL = 16;                 // up+WTA blocks: 16-lane lines (the WTA layout), 16 per block
        const int nb = (g.maxX1 - pl.xb_lo[1] + NL - 1) / NL;
        for (int b = 0; b < nb; b++)
            for (int f = 0; f < up_group; f++) v.push_back({4 * g.H + 4 * g.W, path_item(8, b, f)});
    }
    for (int dir = 0; dir < 8; dir++) {
        if (!((dir_mask >> dir) & 1u)) continue;
        if (dir >= 6) {
            const int nb = (g.H + hscan_rows(g.D) - 1) / hscan_rows(g.D);
            for (int b = 0; b < nb; b++)
                for (int f = 0; f < group; f++) v.push_back({g.width1, path_item(dir, b, f)});
            continue;
        }
        const int rx = dir_rx(dir);
        const int hi = g.maxX1 + (rx < 0 ? g.H - 1 : 0);
        const int NL = rows_lines(g.D);
        const int nb = (hi - pl.xb_lo[dir] + NL - 1) / NL;
        for (int b = 0; b < nb; b++) {
            const int xb = pl.xb_lo[dir] + b * NL;
            int s0, s1;      // same step range as p16_rows
            if (rx == 0) { s0 = 0; s1 = g.H; }
            else if (rx > 0) { s0 = std::max(0, g.minX1 - xb - (NL - 1)); s1 = std::min(g.H, g.maxX1 - xb); }
            else { s0 = std::max(0, xb - g.maxX1 + 1); s1 = std::min(g.H, xb + NL - g.minX1); }
            for (int f = 0; f < group; f++) v.push_back({std::max(s1 - s0, 0), path_item(dir, b, f)});
        }
    }
    const int n = (int)v.size();
    if (!out) return n;
    if (n > cap) return -1;
    std::stable_sort(v.begin(), v.end(), [](const Item& a, const Item& b) { return a.len > b.len; });
    n_slots = std::max(n_slots, 1);
    for (int k = 0; k < n; k++) {
        const int round = k / n_slots, i = k % n_slots;
        const int in_round = std::min(n_slots, n - round * n_slots);
        out[round * n_slots + ((round & 1) ? in_round - 1 - i : i)] = v[k].code;
    }
    return n;
}

// SGM_TRACE=<file>: debug timeline of path / fused launches (one record per wave), written
// after a synchronise by trace_dump. Never set in production runs.
static uint64_t* trace_buffer(int n_blocks)
{
    static uint64_t* trace = nullptr;
    static size_t trace_n = 0;
    if (!getenv("SGM_TRACE")) return nullptr;
    if (trace_n < (size_t)n_blocks * 16) {
        if (trace) (void)hipFree(trace);
        trace_n = (size_t)n_blocks * 16;
        if (hipMalloc(&trace, trace_n * 8) != hipSuccess) { trace = nullptr; trace_n = 0; }
    }
    if (trace) (void)hipMemset(trace, 0, (size_t)n_blocks * 16 * 8);
    return trace;
}

static void trace_dump(uint64_t* tr, int n_blocks, hipStream_t st)
{
    if (!tr) return;
    std::vector<uint64_t> h((size_t)n_blocks * 16);
    if (hipStreamSynchronize(st) == hipSuccess &&
        hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
        // the first '%d' in the name is replaced by the dump number (one file per traced
        // launch); the value is never used as a format string
        static std::atomic<int> n_dump{0};
        const std::string pat = getenv("SGM_TRACE");
        const size_t at = pat.find("%d");
        const std::string name = at == std::string::npos
                                     ? pat
                                     : pat.substr(0, at) + std::to_string(n_dump++) + pat.substr(at + 2);
        FILE* f = fopen(name.c_str(), "wb");
        if (f) { fwrite(h.data(), 8, h.size(), f); fclose(f); }
    }
}

template <int DPL>
static void launch_paths_dpl(const PathFrames& pf, size_t vol_bytes, size_t trash_off, const Geom& g,
                             const PathLaunch16& pl, const uint32_t* items, int n_items, hipStream_t st)
{
    uint64_t* tr = trace_buffer(n_items);
    dim3 grid(n_items), block(kWG);
    if (g.D == 16 * DPL)
        hipLaunchKernelGGL((k_census_paths16<DPL, true>), grid, block, 0, st, pf, vol_bytes, trash_off, g, pl, items,
                           tr);
    else
        hipLaunchKernelGGL((k_census_paths16<DPL, false>), grid, block, 0, st, pf, vol_bytes, trash_off, g, pl, items,
                           tr);
    trace_dump(tr, n_items, st);
}

// Path sweeps of the frames in pf (codes -> volumes). Each volume slice is vol_bytes long:
// H*width1*D cells followed by a trash slot. items: device copy of census_path_items().
// bnd_down / bnd_up (exact tile mode, may be null): see PathLaunch16.
hipError_t launch_census_paths(const PathFrames& pf, size_t vol_bytes, const Geom& g, const uint32_t* items,
                               int n_items, hipStream_t st, const uint8_t* bnd_down, const uint8_t* bnd_up,
                               size_t bnd_slot)
{
    if (n_items <= 0) return hipSuccess;
    PathLaunch16 pl = make_path_launch16(g);
    pl.bnd[0] = bnd_down;
    pl.bnd[1] = bnd_up;
    pl.bnd_slot = bnd_slot;
    const size_t trash_off = (size_t)g.H * g.width1 * g.D;
    switch (dpl16_for(g.D)) {
    case 2: launch_paths_dpl<2>(pf, vol_bytes, trash_off, g, pl, items, n_items, st); break;
    case 4: launch_paths_dpl<4>(pf, vol_bytes, trash_off, g, pl, items, n_items, st); break;
    case 8: launch_paths_dpl<8>(pf, vol_bytes, trash_off, g, pl, items, n_items, st); break;
    case 16: launch_paths_dpl<16>(pf, vol_bytes, trash_off, g, pl, items, n_items, st); break;
    default: launch_paths_dpl<32>(pf, vol_bytes, trash_off, g, pl, items, n_items, st); break;
    }
    return hipGetLastError();
}

template <int DPL>
static void launch_wta_dpl(const WtaFrames& wf, size_t vol_bytes, const Geom& g, size_t out_stride, hipStream_t st)
{
    dim3 grid(g.H * wf.n), block(kWG);
    const size_t lds = wta_lds_bytes<DPL>(g.W);
    if (wf.outf[0]) {                  // one frame, float rows into a mapped host buffer
        if (g.D == 16 * DPL)
            hipLaunchKernelGGL((k_census_wta16f<DPL, true>), dim3(g.H), block, lds, st, wf, vol_bytes, g);
        else
            hipLaunchKernelGGL((k_census_wta16f<DPL, false>), dim3(g.H), block, lds, st, wf, vol_bytes, g);
        return;
    }
    if (g.D == 16 * DPL)
        hipLaunchKernelGGL((k_census_wta16<DPL, true>), grid, block, lds, st, wf, vol_bytes, g, out_stride);
    else
        hipLaunchKernelGGL((k_census_wta16<DPL, false>), grid, block, lds, st, wf, vol_bytes, g, out_stride);
}

// WTA + LR of the frames in wf (volumes -> disparity).
hipError_t launch_census_wta(const WtaFrames& wf, size_t vol_bytes, const Geom& g, size_t out_stride, hipStream_t st)
{
    switch (dpl16_for(g.D)) {
    case 2: launch_wta_dpl<2>(wf, vol_bytes, g, out_stride, st); break;
    case 4: launch_wta_dpl<4>(wf, vol_bytes, g, out_stride, st); break;
    case 8: launch_wta_dpl<8>(wf, vol_bytes, g, out_stride, st); break;
    case 16: launch_wta_dpl<16>(wf, vol_bytes, g, out_stride, st); break;
    default: launch_wta_dpl<32>(wf, vol_bytes, g, out_stride, st); break;
    }
    return hipGetLastError();
}

template <int DPL>
static void launch_fused_dpl(const PathFrames& pf, const WtaFrames& wf, const CensusFrames& cf, size_t vol_bytes,
                             size_t trash_off, const Geom& g, const PathLaunch16& pl, const uint32_t* items,
                             int n_items, size_t out_stride, bool up_wta, hipStream_t st)
{
    const int n_census = ((g.W + 63) / 64) * ((g.H + kCensusRows - 1) / kCensusRows) * 2 * cf.n;
    dim3 grid(n_items + (up_wta ? 0 : g.H * wf.n) + n_census), block(kWG);
    const size_t lds = std::max({up_wta ? upwta_lds_bytes<DPL>() : wta_lds_bytes<DPL>(g.W),
                                 sizeof(uint64_t) * rows_lds_codes<DPL>(), (size_t)(kCensusRows + 6) * 72});
    uint64_t* tr = trace_buffer((int)grid.x);
    // WTA rows interleaved one per 2.5 blocks (C3 sweeps, first build: after the paths 554
    // pairs/s, 1/2 498, 1/2.5 578, 1/2.75 580, 1/3 577, 1/3.5 574; with nontemporal volumes,
    // two interleaved rounds: 1/2.25 655-658, 1/2.5 660-663, 1/2.75 641-657, 1/3.25 649-652,
    // 1/4 621-635): the memory-bound rows co-run with the VALU-bound sweeps on ~1 slot in 3
    // instead of waiting for the sweeps' tail
    static const int period = getenv("SGM_WTA_PERIOD") ? (int)(16 * atof(getenv("SGM_WTA_PERIOD"))) : 40;
    if (g.D == 16 * DPL)
        hipLaunchKernelGGL((k_census_fused16<DPL, true>), grid, block, lds, st, pf, wf, cf, vol_bytes, trash_off, g,
                           pl, items, n_items, out_stride, period, up_wta ? 0 : 1, tr);
    else
        hipLaunchKernelGGL((k_census_fused16<DPL, false>), grid, block, lds, st, pf, wf, cf, vol_bytes, trash_off, g,
                           pl, items, n_items, out_stride, period, up_wta ? 0 : 1, tr);
    trace_dump(tr, (int)grid.x, st);
}

hipError_t launch_census_tiles(const CensusFrames& cf, int W, int H, hipStream_t st)
{
    const int n = ((W + 63) / 64) * ((H + kCensusRows - 1) / kCensusRows) * 2 * cf.n;
    if (n > 0) hipLaunchKernelGGL(k_census_tiles, dim3(n), dim3(kWG), 0, st, cf, W, H);
    return hipGetLastError();
}

// One launch: path sweeps of the frames in pf (items), WTA of the frames in wf (the previous
// group) and census of the frames in cf (the next group). Any of the three may be empty
// (n_items = 0, wf.n = 0, cf.n = 0). All volume sets have the same geometry. up_wta: the
// work list carries up+WTA items for wf (its dir-1 sweeps; wf.res receives the results, and
// launch_census_rowfin finishes the rows) instead of WTA rows.
hipError_t launch_census_fused(const PathFrames& pf, const WtaFrames& wf, const CensusFrames& cf, size_t vol_bytes,
                               const Geom& g, const uint32_t* items, int n_items, size_t out_stride, bool up_wta,
                               hipStream_t st)
{
    const PathLaunch16 pl = make_path_launch16(g);
    const size_t trash_off = (size_t)g.H * g.width1 * g.D;
    switch (dpl16_for(g.D)) {
    case 2: launch_fused_dpl<2>(pf, wf, cf, vol_bytes, trash_off, g, pl, items, n_items, out_stride, up_wta, st); break;
    case 4: launch_fused_dpl<4>(pf, wf, cf, vol_bytes, trash_off, g, pl, items, n_items, out_stride, up_wta, st); break;
    case 8: launch_fused_dpl<8>(pf, wf, cf, vol_bytes, trash_off, g, pl, items, n_items, out_stride, up_wta, st); break;
    case 16: launch_fused_dpl<16>(pf, wf, cf, vol_bytes, trash_off, g, pl, items, n_items, out_stride, up_wta, st); break;
    default: launch_fused_dpl<32>(pf, wf, cf, vol_bytes, trash_off, g, pl, items, n_items, out_stride, up_wta, st); break;
    }
    return hipGetLastError();
}

// disp2 + LR + store of every row of the frames in wf from their up+WTA results
hipError_t launch_census_rowfin(const WtaFrames& wf, const Geom& g, size_t out_stride, hipStream_t st)
{
    if (wf.n > 0)
        hipLaunchKernelGGL(k_census_rowfin, dim3(g.H * wf.n), dim3(kWG), RowLds::bytes(g.W), st, wf, g, out_stride);
    return hipGetLastError();
}

}  // namespace sgm
