// census_sgm.hip — north-star census-SGM kernels for gfx950 (SGM_MODE_CENSUS8).
//
// Spec: SURVEY.md Appendix B (build-defined; CPU definition oracle/sgm_oracle.c
// `census_step`/`census_path`/`wta_pixel`). Pipeline per frame:
//   k_census9x7      L,R u8            -> census codes u64 (2 x W x H)
//   k_census_paths   codes             -> 7 u8 path volumes [H][width1][D] (dirs 0..6)
//   k_census_final   codes + 7 volumes -> dir 7 (r = (-1,0)) fused with the 8-way sum,
//                                         WTA, uniqueness, subpixel, disp2 and LR check
// The matching cost popcount(cL ^ cR) is recomputed on the fly in every path (never
// stored); S = sum of the 8 paths never touches HBM.
#include "sgm_device.h"

namespace sgm {

// ------------------------------------------------------------------------------------
// 9x7 census: one thread per pixel, a 10 x 72 byte LDS tile per 64 x 4 pixel block.
// blockIdx.z selects the image (0 = left, 1 = right).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_census9x7(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                   size_t stride, int W, int H,
                                                   uint64_t* __restrict__ cL, uint64_t* __restrict__ cR)
{
    __shared__ uint8_t tile[10][72];
    const uint8_t* img = blockIdx.z ? R : L;
    uint64_t* out = blockIdx.z ? cR : cL;
    const int x0 = blockIdx.x * 64, y0 = blockIdx.y * 4;
    for (int i = threadIdx.x; i < 10 * 72; i += 256) {
        int ty = i / 72, tx = i - ty * 72;
        int yy = min(max(y0 + ty - 3, 0), H - 1), xx = min(max(x0 + tx - 4, 0), W - 1);
        tile[ty][tx] = img[(size_t)yy * stride + xx];
    }
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int x = x0 + tx, y = y0 + ty;
    if (x >= W || y >= H) return;
    const int c = tile[ty + 3][tx + 4];
    uint64_t code = 0;
    int bit = 0;
#pragma unroll
    for (int dy = 0; dy < 7; dy++) {
#pragma unroll
        for (int dx = 0; dx < 9; dx++) {
            if (dy == 3 && dx == 4) continue;
            code |= (uint64_t)(tile[ty + dy][tx + dx] < c) << bit;
            bit++;
        }
    }
    out[(size_t)y * W + x] = code;
}

// ------------------------------------------------------------------------------------
// Path recurrence of one cell for the DPL disparities of this lane.
//   L(d) = C(d) + min(Lp(d), Lp(d-1)+P1, Lp(d+1)+P1, minLp+P2) - minLp
// Lanes with d >= D hold kInf. `cost[k]` = popcount(cL ^ cR(x - minD - d)).
// ------------------------------------------------------------------------------------
template <int DPL>
__device__ __forceinline__ int path_step(const int (&cost)[DPL], const int (&Lp)[DPL], int mLp, bool pv,
                                         int lane, int D, int P1, int P2, int (&Lout)[DPL])
{
    const int fromLeft = dpp_shr1(Lp[DPL - 1], kInf);   // Lp(d-1) for k = 0
    const int fromRight = dpp_shl1(Lp[0], kInf);        // Lp(d+1) for k = DPL-1
    const int q = mLp + P2;
    int lmin = kInf;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
        const int lm1 = k > 0 ? Lp[k - 1] : fromLeft;
        const int lp1 = k < DPL - 1 ? Lp[k + 1] : fromRight;
        int t = min(lm1, lp1) + P1;
        t = min(min(Lp[k], t), q);
        int v = pv ? cost[k] + t - mLp : cost[k];
        v = (lane * DPL + k) < D ? v : kInf;
        Lout[k] = v;
        lmin = min(lmin, v);
    }
    return lmin;
}

struct PathLaunch {
    int blk_start[8];   // first block of dir i (dirs 0..6), blk_start[7] = total
    int xb_lo[6];       // first line base column of row-sweep dir i
};

constexpr int kG = 4;       // adjacent lines (columns) per wave in the row sweeps
constexpr int kChunk = 16;  // steps per unrolled chunk of the horizontal scans

// Memory-op discipline (why the loops look the way they do): gfx950 counts loads AND
// stores on one in-order vmcnt. hipcc only emits counted waits (vmcnt(N)) when every path
// through the loop body issues the same VMEM ops in the same order; a conditional store
// or prefetch makes it fall back to vmcnt(0), i.e. one full memory round trip per step.
// So every loop body below issues an unconditional, fixed sequence: prefetches use clamped
// indices, and cells that must not be written (outside the image, lanes with d >= D,
// padding steps) store into a per-volume trash slot instead of branching around the store.

// Per-step inputs of a row sweep: the lane's window of right codes (DPL + kG - 1 values
// cover its DPL disparities for the kG adjacent columns) and the kG left codes (scalar).
template <int DPL>
struct RowIn {
    uint64_t cr[DPL + kG - 1];
    uint64_t cl[kG];
};

template <int DPL>
__device__ __forceinline__ void row_load(RowIn<DPL>& in, const uint64_t* __restrict__ cL,
                                         const uint64_t* __restrict__ cR, const Geom& g, int rx, int ry, int xb,
                                         int s, int lane)
{
    const int y = ry > 0 ? s : g.H - 1 - s;
    const uint64_t* cLr = cL + (size_t)y * g.W;
    const uint64_t* cRr = cR + (size_t)y * g.W;
    const int xs = xb + rx * s;
    const int jb = xs - g.minD - lane * DPL - (DPL - 1);
#pragma unroll
    for (int m = 0; m < DPL + kG - 1; m++) in.cr[m] = cRr[min(max(jb + m, 0), g.W - 1)];
#pragma unroll
    for (int j = 0; j < kG; j++) in.cl[j] = cLr[min(max(xs + j, 0), g.W - 1)];
}

template <int DPL>
struct RowState {
    int Lp[kG][DPL];
    int mLp[kG];
    bool pv[kG];
};

template <int DPL>
__device__ __forceinline__ void row_step(const RowIn<DPL>& in, RowState<DPL>& st, uint8_t* __restrict__ V,
                                         uint8_t* __restrict__ trash, const Geom& g, int rx, int ry, int xb, int s,
                                         int s1, int lane)
{
    using VT = typename LaneVec<DPL>::T;
    const int y = ry > 0 ? s : g.H - 1 - s;
    const int xs = xb + rx * s;
    const bool active = lane * DPL < g.D;
#pragma unroll
    for (int j = 0; j < kG; j++) {
        const int x = xs + j;
        const bool valid = s < s1 && x >= g.minX1 && x < g.maxX1;        // wave-uniform
        int cost[DPL], L[DPL];
#pragma unroll
        for (int k = 0; k < DPL; k++) cost[k] = popc64(in.cl[j] ^ in.cr[j - k + DPL - 1]);
        const int lmin = path_step<DPL>(cost, st.Lp[j], st.mLp[j], st.pv[j], lane, g.D, g.P1, g.P2, L);
        uint8_t* dst = (valid && active) ? V + ((size_t)y * g.width1 + (x - g.minX1)) * g.D + lane * DPL
                                         : trash + lane * DPL;
        *(VT*)dst = pack_u8<DPL>(L);
        st.mLp[j] = wave_min(lmin);
#pragma unroll
        for (int k = 0; k < DPL; k++) st.Lp[j][k] = L[k];
        st.pv[j] = valid;
    }
}

// Row sweep (dirs 0..5, ry != 0): the wave owns kG adjacent lines; line j at step s sits
// at column xb + j + rx*s of row y(s). All D of each cell live in the wave. The inputs of
// step s+1 are loaded (ping-pong registers) while step s computes.
template <int DPL>
__device__ __forceinline__ void row_sweep(const uint64_t* __restrict__ cL, const uint64_t* __restrict__ cR,
                                          uint8_t* __restrict__ V, uint8_t* __restrict__ trash, const Geom& g,
                                          int dir, int xb)
{
    const int lane = threadIdx.x;
    const int rx = dir_rx(dir), ry = dir_ry(dir);
    int s0, s1;
    if (rx == 0) { s0 = 0; s1 = g.H; }
    else if (rx > 0) { s0 = max(0, g.minX1 - xb - (kG - 1)); s1 = min(g.H, g.maxX1 - xb); }
    else { s0 = max(0, xb - g.maxX1 + 1); s1 = min(g.H, xb + kG - g.minX1); }
    if (s0 >= s1) return;
    RowState<DPL> st;
#pragma unroll
    for (int j = 0; j < kG; j++) {
        st.pv[j] = false;
        st.mLp[j] = 0;
#pragma unroll
        for (int k = 0; k < DPL; k++) st.Lp[j][k] = kInf;
    }
    RowIn<DPL> A, B;
    row_load<DPL>(A, cL, cR, g, rx, ry, xb, s0, lane);
    for (int s = s0; s < s1; s += 2) {
        row_load<DPL>(B, cL, cR, g, rx, ry, xb, min(s + 1, s1 - 1), lane);
        row_step<DPL>(A, st, V, trash, g, rx, ry, xb, s, s1, lane);
        row_load<DPL>(A, cL, cR, g, rx, ry, xb, min(s + 2, s1 - 1), lane);
        row_step<DPL>(B, st, V, trash, g, rx, ry, xb, s + 1, s1, lane);
    }
}

// Scalar operands of a horizontal scan, kChunk steps per vector load: lane j (< kChunk)
// holds the left code and the window-entry right code of step (kChunk*chunk + j); step i
// reads them with readlane, so no scalar-load latency sits on the recurrence chain.
struct HChunk {
    uint64_t cl, inc;
};

__device__ __forceinline__ HChunk hchunk_load(const uint64_t* cLr, const uint64_t* cRr, const Geom& g, int dirx,
                                              int chunk, int lane, int DPLx64)
{
    const int i = chunk * kChunk + (lane & (kChunk - 1));
    HChunk c;
    if (dirx > 0) {   // x ascending from minX1; inc = code entering for step i + 1
        const int x = g.minX1 + i;
        c.cl = cLr[min(x, g.W - 1)];
        c.inc = cRr[min(max(x + 1 - g.minD, 0), g.W - 1)];
    } else {          // x descending from maxX1 - 1
        const int x = g.maxX1 - 1 - i;
        c.cl = cLr[min(max(x, 0), g.W - 1)];
        c.inc = cRr[min(max(x - g.minD - DPLx64, 0), g.W - 1)];
    }
    return c;
}

// Horizontal sweep, dir 6 (r = (1,0)): one wave per row, x ascending. The right-code
// window slides by one column per step: lane l takes lane l-1's oldest code (DPP),
// lane 0 takes cR(x + 1 - minD).
template <int DPL>
__device__ __forceinline__ void horiz_sweep(const uint64_t* __restrict__ cL, const uint64_t* __restrict__ cR,
                                            uint8_t* __restrict__ V, uint8_t* __restrict__ trash, const Geom& g,
                                            int y)
{
    using VT = typename LaneVec<DPL>::T;
    const int lane = threadIdx.x;
    const bool active = lane * DPL < g.D;
    const uint64_t* cLr = cL + (size_t)y * g.W;
    const uint64_t* cRr = cR + (size_t)y * g.W;
    uint64_t cr[DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) cr[k] = cRr[max(g.minX1 - g.minD - lane * DPL - k, 0)];
    int Lp[DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) Lp[k] = kInf;
    int mLp = 0;
    bool pv = false;
    uint8_t* row = V + (size_t)y * g.width1 * g.D + lane * DPL;
    uint8_t* tr = trash + lane * DPL;
    const int n = g.width1;
    HChunk cur = hchunk_load(cLr, cRr, g, 1, 0, lane, 64 * DPL);
    for (int c = 0; c * kChunk < n; c++) {
        const HChunk nxt = hchunk_load(cLr, cRr, g, 1, c + 1, lane, 64 * DPL);
#pragma unroll
        for (int j = 0; j < kChunk; j++) {
            const int i = c * kChunk + j;
            const uint64_t cl = readlane64(cur.cl, j);
            const uint64_t inc = readlane64(cur.inc, j);
            int cost[DPL], L[DPL];
#pragma unroll
            for (int k = 0; k < DPL; k++) cost[k] = popc64(cl ^ cr[k]);
            const int lmin = path_step<DPL>(cost, Lp, mLp, pv, lane, g.D, g.P1, g.P2, L);
            *(VT*)((active && i < n) ? row + (size_t)i * g.D : tr) = pack_u8<DPL>(L);
            mLp = wave_min(lmin);
#pragma unroll
            for (int k = 0; k < DPL; k++) Lp[k] = L[k];
            pv = true;
            const uint64_t nw = dpp_shr1_u64(cr[DPL - 1], inc);
#pragma unroll
            for (int k = DPL - 1; k > 0; k--) cr[k] = cr[k - 1];
            cr[0] = nw;
        }
        cur = nxt;
    }
}

template <int DPL>
__global__ __launch_bounds__(64) void k_census_paths(const uint64_t* __restrict__ cL, const uint64_t* __restrict__ cR,
                                                     uint8_t* __restrict__ vols, size_t vol_bytes, size_t trash_off,
                                                     Geom g, PathLaunch pl)
{
    const int b = blockIdx.x;
    int dir = 0;
#pragma unroll
    for (int i = 1; i < 7; i++) dir += b >= pl.blk_start[i] ? 1 : 0;
    const int lb = b - pl.blk_start[dir];
    uint8_t* V = vols + (size_t)dir * vol_bytes;
    uint8_t* trash = V + trash_off;
    if (dir < 6) row_sweep<DPL>(cL, cR, V, trash, g, dir, pl.xb_lo[dir] + lb * kG);
    else horiz_sweep<DPL>(cL, cR, V, trash, g, lb);
}

// ------------------------------------------------------------------------------------
// Final pass: dir 7 (r = (-1,0), x descending) + S = L7 + sum of the 7 stored volumes,
// WTA of kU pixels at a time (branch-free, wta_batch), then the row epilogue (disp2 via
// LDS atomics, LR check, store). One wave per row. The 7 volume reads run kPF steps
// ahead in a register ring; the scalar operands come from kChunk-step vector chunks.
// ------------------------------------------------------------------------------------
constexpr int kPF = 8;
constexpr int kU = 4;

template <int DPL>
__global__ __launch_bounds__(64) void k_census_final(const uint64_t* __restrict__ cL, const uint64_t* __restrict__ cR,
                                                     const uint8_t* __restrict__ vols, size_t vol_bytes, Geom g,
                                                     int16_t* __restrict__ out, size_t out_stride)
{
    using VT = typename LaneVec<DPL>::T;
    extern __shared__ uint32_t lds_final[];
    RowLds R(lds_final, g.W);
    const int lane = threadIdx.x;
    const int y = blockIdx.x;
    const bool active = lane * DPL < g.D;
    R.init(g, lane);

    const uint64_t* cLr = cL + (size_t)y * g.W;
    const uint64_t* cRr = cR + (size_t)y * g.W;
    const uint8_t* vrow = vols + (size_t)y * g.width1 * g.D + (active ? lane * DPL : 0);
    const int n = g.width1;
    uint64_t cr[DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) cr[k] = cRr[max(g.maxX1 - 1 - g.minD - lane * DPL - k, 0)];
    int Lp[DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) Lp[k] = kInf;
    int mLp = 0;
    bool pv = false;

    VT buf[kPF][7];
#pragma unroll
    for (int u = 0; u < kPF; u++)
#pragma unroll
        for (int r = 0; r < 7; r++)
            buf[u][r] = *(const VT*)(vrow + (size_t)r * vol_bytes + (size_t)(n - 1 - min(u, n - 1)) * g.D);
    HChunk cur = hchunk_load(cLr, cRr, g, -1, 0, lane, 64 * DPL);

    static_assert(kChunk % kPF == 0 && kPF % kU == 0, "chunk layout");
    for (int c = 0; c * kChunk < n; c++) {
        const HChunk nxt = hchunk_load(cLr, cRr, g, -1, c + 1, lane, 64 * DPL);
#pragma unroll
        for (int q = 0; q < kChunk / kU; q++) {
            int S[kU][DPL];
            int xs[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int j = q * kU + u;            // step within the chunk
                const int slot = j % kPF;             // ring slot (static)
                const int i = c * kChunk + j;
                xs[u] = g.maxX1 - 1 - i;
                VT v[7];
#pragma unroll
                for (int r = 0; r < 7; r++) v[r] = buf[slot][r];
                const int ip = min(i + kPF, n - 1);
#pragma unroll
                for (int r = 0; r < 7; r++)
                    buf[slot][r] = *(const VT*)(vrow + (size_t)r * vol_bytes + (size_t)(n - 1 - ip) * g.D);
                // ---- dir 7 recurrence ----
                const uint64_t cl = readlane64(cur.cl, j);
                const uint64_t inc = readlane64(cur.inc, j);
                int cost[DPL], L[DPL];
#pragma unroll
                for (int k = 0; k < DPL; k++) cost[k] = popc64(cl ^ cr[k]);
                const int lmin = path_step<DPL>(cost, Lp, mLp, pv, lane, g.D, g.P1, g.P2, L);
                mLp = wave_min(lmin);
#pragma unroll
                for (int k = 0; k < DPL; k++) Lp[k] = L[k];
                pv = true;
                const uint64_t nw = dpp_shl1_u64(cr[0], inc);            // slide the window to x-1
#pragma unroll
                for (int k = 0; k < DPL - 1; k++) cr[k] = cr[k + 1];
                cr[DPL - 1] = nw;
                // ---- S = L7 + 7 stored paths ----
#pragma unroll
                for (int k = 0; k < DPL; k++) {
                    int sum = L[k];
#pragma unroll
                    for (int r = 0; r < 7; r++) sum += (int)((v[r] >> (8 * k)) & 0xFF);
                    S[u][k] = active && (lane * DPL + k) < g.D ? sum : kInf;
                }
            }
            const int nvalid = min(max(n - (c * kChunk + q * kU), 0), kU);
            wta_batch<DPL, kU>(S, lane, xs, nvalid, g, R.drow, R.bst, R.mins);
        }
        cur = nxt;
    }
    row_finish(g, lane, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, out + (size_t)y * out_stride);
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

static int dpl_for(int D) { return D <= 64 ? 1 : D <= 128 ? 2 : D <= 256 ? 4 : 8; }

PathLaunch make_path_launch(const Geom& g, int only_dir)
{
    PathLaunch pl{};
    int acc = 0;
    for (int dir = 0; dir < 7; dir++) {
        pl.blk_start[dir] = acc;
        int nb = 0;
        if (dir < 6) {
            const int rx = dir_rx(dir);
            const int lo = g.minX1 - (rx > 0 ? g.H - 1 : 0);
            const int hi = g.maxX1 + (rx < 0 ? g.H - 1 : 0);
            pl.xb_lo[dir] = lo;
            nb = (hi - lo + kG - 1) / kG;
        } else {
            nb = g.H;
        }
        if (only_dir >= 0 && dir != only_dir) nb = 0;
        acc += nb;
    }
    pl.blk_start[7] = acc;
    return pl;
}

// Each volume slice is vol_bytes long: H*width1*D cells followed by a kTrashBytes trash
// slot (see the memory-op discipline note above).
hipError_t launch_census_paths(const uint64_t* cL, const uint64_t* cR, uint8_t* vols, size_t vol_bytes,
                               const Geom& g, int only_dir, hipStream_t st)
{
    PathLaunch pl = make_path_launch(g, only_dir);
    if (pl.blk_start[7] == 0) return hipSuccess;
    const size_t trash_off = (size_t)g.H * g.width1 * g.D;
    dim3 grid(pl.blk_start[7]), block(64);
    switch (dpl_for(g.D)) {
    case 1: hipLaunchKernelGGL(k_census_paths<1>, grid, block, 0, st, cL, cR, vols, vol_bytes, trash_off, g, pl); break;
    case 2: hipLaunchKernelGGL(k_census_paths<2>, grid, block, 0, st, cL, cR, vols, vol_bytes, trash_off, g, pl); break;
    case 4: hipLaunchKernelGGL(k_census_paths<4>, grid, block, 0, st, cL, cR, vols, vol_bytes, trash_off, g, pl); break;
    default: hipLaunchKernelGGL(k_census_paths<8>, grid, block, 0, st, cL, cR, vols, vol_bytes, trash_off, g, pl); break;
    }
    return hipGetLastError();
}

hipError_t launch_census_final(const uint64_t* cL, const uint64_t* cR, const uint8_t* vols, size_t vol_bytes,
                               const Geom& g, int16_t* out, size_t out_stride, hipStream_t st)
{
    dim3 grid(g.H), block(64);
    const size_t lds = RowLds::bytes(g.W);
    switch (dpl_for(g.D)) {
    case 1: hipLaunchKernelGGL(k_census_final<1>, grid, block, lds, st, cL, cR, vols, vol_bytes, g, out, out_stride); break;
    case 2: hipLaunchKernelGGL(k_census_final<2>, grid, block, lds, st, cL, cR, vols, vol_bytes, g, out, out_stride); break;
    case 4: hipLaunchKernelGGL(k_census_final<4>, grid, block, lds, st, cL, cR, vols, vol_bytes, g, out, out_stride); break;
    default: hipLaunchKernelGGL(k_census_final<8>, grid, block, lds, st, cL, cR, vols, vol_bytes, g, out, out_stride); break;
    }
    return hipGetLastError();
}

}  // namespace sgm
