// ocv_sgm.hip — OpenCV-StereoSGBM-compatible modes on gfx950 (SGM_MODE_OCV_SGBM5 / _HH8).
//
// Bit-exact with the CPU restatement oracle/sgm_oracle.c `ocv_match` (which follows
// OpenCV's sequential raster loop); here every stage is re-expressed in parallel form:
//   k_ocv_prefilter  Sobel-x prefilter + raw channel, columns 0 / W-1 forced to ftzero
//   k_ocv_pixcost    Birchfield-Tomasi cost of both channels (raw >> 2), int16 [H][w1][D]
//   k_ocv_hsum       horizontal SAD box, replicate clamp to [0, width1)        (exact)
//   k_ocv_vsum       vertical box + P2 offset + OpenCV's bottom-row quirk:
//                    rows with y + SH2 >= H are never recomputed (MODE_SGBM keeps the
//                    last computed row, MODE_HH keeps the P2 initialisation)
//   k_ocv_paths      each direction independently (L depends only on its own path);
//                    int16 storage of L and minL as OpenCV's CostType
//   k_ocv_wta        S = saturate(sum of L) (all L >= 0 inside the parity domain, so the
//                    saturating order is irrelevant) + the shared WTA / LR row code.
// Parity domain: SAD + 2*P2 <= 32767 (always true for block <= 15 at the node defaults).
#include "sgm_device.h"

namespace sgm {

constexpr int kMaxCost = 32767;

__global__ __launch_bounds__(256) void k_ocv_prefilter(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                       size_t stride, int W, int H, int ftzero,
                                                       uint8_t* __restrict__ planes /* 4 x W x H */)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const int img = blockIdx.z;
    const uint8_t* src = img ? R : L;
    uint8_t* pf = planes + (size_t)(2 * img) * W * H;
    uint8_t* raw = planes + (size_t)(2 * img + 1) * W * H;
    const size_t o = (size_t)y * W + x;
    if (x == 0 || x == W - 1) { pf[o] = (uint8_t)ftzero; raw[o] = (uint8_t)ftzero; return; }
    const uint8_t* r = src + (size_t)y * stride;
    const uint8_t* n = y > 0 ? r - stride : r;
    const uint8_t* s = y < H - 1 ? r + stride : r;
    const int v = (r[x + 1] - r[x - 1]) * 2 + n[x + 1] - n[x - 1] + s[x + 1] - s[x - 1];
    pf[o] = (uint8_t)(min(max(v, -ftzero), ftzero) + ftzero);
    raw[o] = r[x];
}

__device__ __forceinline__ void bt_lohi(const uint8_t* a, int x, int W, int& u, int& lo, int& hi)
{
    u = a[x];
    const int ul = x > 0 ? (u + a[x - 1]) / 2 : u;
    const int ur = x < W - 1 ? (u + a[x + 1]) / 2 : u;
    lo = min(min(ul, ur), u);
    hi = max(max(ul, ur), u);
}

// grid (width1, H), block 256 over d
__global__ __launch_bounds__(256) void k_ocv_pixcost(const uint8_t* __restrict__ planes, Geom g,
                                                     int16_t* __restrict__ cost)
{
    const int x1 = blockIdx.x, y = blockIdx.y;
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

// thread per (x1, d): running vertical box along y, C' = P2 + SAD with the bottom-row rule
__global__ __launch_bounds__(256) void k_ocv_vsum(const int16_t* __restrict__ hs, Geom g, int fullDP,
                                                  int16_t* __restrict__ C)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= g.width1 * g.D) return;
    const size_t rowStride = (size_t)g.width1 * g.D;
    const int H = g.H, SH2 = g.SH2;
    int s = hs[i] * (SH2 + 1);
    for (int k = 1; k <= SH2; k++) s += hs[(size_t)min(k, H - 1) * rowStride + i];
    int last = g.P2 + s;
    C[i] = (int16_t)last;
    for (int y = 1; y < H; y++) {
        int v;
        if (y + SH2 < H) {
            s += hs[(size_t)(y + SH2) * rowStride + i] - hs[(size_t)max(y - SH2 - 1, 0) * rowStride + i];
            v = g.P2 + s;
            last = v;
        } else {
            v = fullDP ? g.P2 : last;
        }
        C[(size_t)y * rowStride + i] = (int16_t)v;
    }
}

// OpenCV recurrence of one cell with int16 storage semantics. Lanes/entries with d >= D
// hold kMaxCost (acts as OpenCV's Lr[-1] / Lr[D] = MAX_COST padding).
template <int DPL>
__device__ __forceinline__ int ocv_step(const int (&Cp)[DPL], const int (&Lp)[DPL], int mLp, bool pv, int lane,
                                        const Geom& g, int (&Lout)[DPL])
{
    const int fromLeft = dpp_shr1(Lp[DPL - 1], kMaxCost);
    const int fromRight = dpp_shl1(Lp[0], kMaxCost);
    const int lp_min = pv ? mLp : 0;
    const int delta = lp_min + g.P2;
    int lmin = 1 << 30;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
        const int d = lane * DPL + k;
        int a = pv ? Lp[k] : 0;
        int lm1 = k > 0 ? Lp[k - 1] : fromLeft;
        int lp1 = k < DPL - 1 ? Lp[k + 1] : fromRight;
        if (!pv) { lm1 = d > 0 ? 0 : kMaxCost; lp1 = d < g.D - 1 ? 0 : kMaxCost; }
        const int v = Cp[k] + min(a, min(lm1 + g.P1, min(lp1 + g.P1, delta))) - delta;
        Lout[k] = d < g.D ? (int)(int16_t)v : kMaxCost;   // Lr is CostType (int16)
        if (d < g.D) lmin = min(lmin, v);                  // minL over the int values
    }
    return lmin;
}

// One wave per line. Row sweeps (ry != 0): line = (column at step 0) for every line
// start; horizontal (ry == 0): line = row.
template <int DPL>
__global__ __launch_bounds__(64) void k_ocv_paths(const int16_t* __restrict__ C, int16_t* __restrict__ vols,
                                                  size_t vol_elems, Geom g, int dirmask, int4 nblk0, int4 nblk1)
{
    const int nb[8] = {nblk0.x, nblk0.y, nblk0.z, nblk0.w, nblk1.x, nblk1.y, nblk1.z, nblk1.w};
    // block -> (direction, line); volume slot = rank of the direction in dirmask
    int b = blockIdx.x, dir = 0, slot = 0;
    for (int i = 0; i < 8; i++) {
        if (!((dirmask >> i) & 1)) continue;
        if (b < nb[i]) { dir = i; break; }
        b -= nb[i];
        slot++;
    }
    int16_t* V = vols + (size_t)slot * vol_elems;
    const int lane = threadIdx.x;
    const int rx = dir_rx(dir), ry = dir_ry(dir);
    int Lp[DPL], mLp = 0;
    bool pv = false;
#pragma unroll
    for (int k = 0; k < DPL; k++) Lp[k] = kMaxCost;
    if (ry == 0) {
        const int y = b;
        for (int i = 0; i < g.width1; i++) {
            const int x1 = rx > 0 ? i : g.width1 - 1 - i;
            const size_t o = ((size_t)y * g.width1 + x1) * g.D;
            int Cp[DPL], L[DPL];
#pragma unroll
            for (int k = 0; k < DPL; k++) { const int d = lane * DPL + k; Cp[k] = d < g.D ? C[o + d] : 0; }
            const int lmin = ocv_step<DPL>(Cp, Lp, mLp, pv, lane, g, L);
#pragma unroll
            for (int k = 0; k < DPL; k++) { const int d = lane * DPL + k; if (d < g.D) V[o + d] = (int16_t)L[k]; }
            mLp = (int)(int16_t)wave_min(lmin);           // minLr is CostType
#pragma unroll
            for (int k = 0; k < DPL; k++) Lp[k] = L[k];
            pv = true;
        }
        return;
    }
    // line start: b < width1 -> starts on the first row at column b; else starts on the
    // entry column (x1 = 0 for rx > 0, width1 - 1 for rx < 0) at row offset b - width1 + 1
    int x1, s0;
    if (b < g.width1) { x1 = b; s0 = 0; }
    else { x1 = rx > 0 ? 0 : g.width1 - 1; s0 = b - g.width1 + 1; }
    for (int s = s0; s < g.H; s++) {
        if (x1 < 0 || x1 >= g.width1) break;
        const int y = ry > 0 ? s : g.H - 1 - s;
        const size_t o = ((size_t)y * g.width1 + x1) * g.D;
        int Cp[DPL], L[DPL];
#pragma unroll
        for (int k = 0; k < DPL; k++) { const int d = lane * DPL + k; Cp[k] = d < g.D ? C[o + d] : 0; }
        const int lmin = ocv_step<DPL>(Cp, Lp, mLp, pv, lane, g, L);
#pragma unroll
        for (int k = 0; k < DPL; k++) { const int d = lane * DPL + k; if (d < g.D) V[o + d] = (int16_t)L[k]; }
        mLp = (int)(int16_t)wave_min(lmin);
#pragma unroll
        for (int k = 0; k < DPL; k++) Lp[k] = L[k];
        pv = true;
        x1 += rx;
    }
}

// one wave per row: S = saturate(sum L) then the shared batched WTA + row epilogue
template <int DPL>
__global__ __launch_bounds__(64) void k_ocv_wta(const int16_t* __restrict__ vols, size_t vol_elems, int ndir, Geom g,
                                                int16_t* __restrict__ out, size_t out_stride)
{
    extern __shared__ uint32_t lds_ocv[];
    RowLds R(lds_ocv, g.W);
    const int lane = threadIdx.x, y = blockIdx.x;
    R.init(g, lane, 64);
    for (int i0 = 0; i0 < g.width1; i0 += 4) {
        int S[4][DPL], xs[4], nvalid = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int x1 = g.width1 - 1 - (i0 + u);
            xs[u] = x1 + g.minX1;
#pragma unroll
            for (int k = 0; k < DPL; k++) S[u][k] = 1 << 20;
            if (x1 < 0) continue;
            nvalid = u + 1;
            const size_t o = ((size_t)y * g.width1 + x1) * g.D;
#pragma unroll
            for (int k = 0; k < DPL; k++) {
                const int d = lane * DPL + k;
                if (d >= g.D) continue;
                int s = 0;
                for (int r = 0; r < ndir; r++) s += vols[(size_t)r * vol_elems + o + d];
                S[u][k] = min(max(s, -32768), kMaxCost);
            }
        }
        wta_batch<DPL, 4>(S, lane, xs, nvalid, g, R.drow, R.bst, R.mins);
    }
    row_finish(g, lane, 64, R.drow, R.bst, R.mins, R.key, (int16_t*)R.mins, out + (size_t)y * out_stride);
}

// ------------------------------------------------------------------------------------
static int dpl_for(int D) { return D <= 64 ? 1 : D <= 128 ? 2 : D <= 256 ? 4 : 8; }

hipError_t launch_ocv_cost(const uint8_t* L, const uint8_t* R, size_t stride, const Geom& g, int fullDP,
                           uint8_t* planes, int16_t* bufA, int16_t* bufB, hipStream_t st)
{
    hipLaunchKernelGGL(k_ocv_prefilter, dim3((g.W + 255) / 256, g.H, 2), dim3(256), 0, st, L, R, stride, g.W, g.H,
                       g.ftzero, planes);
    hipLaunchKernelGGL(k_ocv_pixcost, dim3(g.width1, g.H), dim3(256), 0, st, planes, g, bufA);
    hipLaunchKernelGGL(k_ocv_hsum, dim3((g.D + 255) / 256, g.H), dim3(256), 0, st, bufA, g, bufB);
    hipLaunchKernelGGL(k_ocv_vsum, dim3((g.width1 * g.D + 255) / 256), dim3(256), 0, st, bufB, g, fullDP, bufA);
    return hipGetLastError();
}

hipError_t launch_ocv_paths(const int16_t* C, int16_t* vols, size_t vol_elems, const Geom& g, int dirmask,
                            hipStream_t st)
{
    int nb[8], total = 0;
    for (int i = 0; i < 8; i++) {
        nb[i] = 0;
        if (!((dirmask >> i) & 1)) continue;
        nb[i] = dir_ry(i) == 0 ? g.H : g.width1 + (dir_rx(i) != 0 ? g.H - 1 : 0);
        total += nb[i];
    }
    int4 a = make_int4(nb[0], nb[1], nb[2], nb[3]), b = make_int4(nb[4], nb[5], nb[6], nb[7]);
    switch (dpl_for(g.D)) {
    case 1: hipLaunchKernelGGL(k_ocv_paths<1>, dim3(total), dim3(64), 0, st, C, vols, vol_elems, g, dirmask, a, b); break;
    case 2: hipLaunchKernelGGL(k_ocv_paths<2>, dim3(total), dim3(64), 0, st, C, vols, vol_elems, g, dirmask, a, b); break;
    case 4: hipLaunchKernelGGL(k_ocv_paths<4>, dim3(total), dim3(64), 0, st, C, vols, vol_elems, g, dirmask, a, b); break;
    default: hipLaunchKernelGGL(k_ocv_paths<8>, dim3(total), dim3(64), 0, st, C, vols, vol_elems, g, dirmask, a, b); break;
    }
    return hipGetLastError();
}

hipError_t launch_ocv_wta(const int16_t* vols, size_t vol_elems, int ndir, const Geom& g, int16_t* out,
                          size_t out_stride, hipStream_t st)
{
    const size_t lds = RowLds::bytes(g.W);
    switch (dpl_for(g.D)) {
    case 1: hipLaunchKernelGGL(k_ocv_wta<1>, dim3(g.H), dim3(64), lds, st, vols, vol_elems, ndir, g, out, out_stride); break;
    case 2: hipLaunchKernelGGL(k_ocv_wta<2>, dim3(g.H), dim3(64), lds, st, vols, vol_elems, ndir, g, out, out_stride); break;
    case 4: hipLaunchKernelGGL(k_ocv_wta<4>, dim3(g.H), dim3(64), lds, st, vols, vol_elems, ndir, g, out, out_stride); break;
    default: hipLaunchKernelGGL(k_ocv_wta<8>, dim3(g.H), dim3(64), lds, st, vols, vol_elems, ndir, g, out, out_stride); break;
    }
    return hipGetLastError();
}

}  // namespace sgm
