// post.hip — post filters of StereoSGBMImpl::compute:
//   medianBlur(disp, disp, 3)                  -> k_median3 (int16, replicate border)
//   filterSpeckles(disp, newVal, size, diff)   -> union-find connected components
// Both are O(W*H) and bit-exact with oracle/sgm_oracle.c (sgmref_median3 /
// sgmref_filter_speckles). Speckle regions are the 4-connected components of the graph
// {p : disp(p) != newVal} with an edge p~q iff |disp(p) - disp(q)| <= maxDiff; a region
// of <= maxSize pixels becomes newVal. Component membership is order-independent, so a
// parallel union-find reproduces OpenCV's sequential flood fill exactly.
#include "sgm_device.h"

namespace sgm {

__device__ __forceinline__ void sort2(int& a, int& b) { int t = min(a, b); b = max(a, b); a = t; }

// median of the 3x3 neighbourhood of (x, y), replicate border
__device__ __forceinline__ int median9(const int16_t* __restrict__ src, size_t sstride, int x, int y, int W, int H)
{
    int p[9];
    int n = 0;
#pragma unroll
    for (int dy = -1; dy <= 1; dy++) {
        const int16_t* r = src + (size_t)min(max(y + dy, 0), H - 1) * sstride;
#pragma unroll
        for (int dx = -1; dx <= 1; dx++) p[n++] = r[min(max(x + dx, 0), W - 1)];
    }
    // Paeth's 19-exchange median-of-9 network
    sort2(p[1], p[2]); sort2(p[4], p[5]); sort2(p[7], p[8]);
    sort2(p[0], p[1]); sort2(p[3], p[4]); sort2(p[6], p[7]);
    sort2(p[1], p[2]); sort2(p[4], p[5]); sort2(p[7], p[8]);
    sort2(p[0], p[3]); sort2(p[5], p[8]); sort2(p[4], p[7]);
    sort2(p[3], p[6]); sort2(p[1], p[4]); sort2(p[2], p[5]);
    sort2(p[4], p[7]); sort2(p[4], p[2]); sort2(p[6], p[4]);
    sort2(p[4], p[2]);
    return p[4];
}

__global__ __launch_bounds__(256) void k_median3(const int16_t* __restrict__ src, size_t sstride,
                                                 int16_t* __restrict__ dst, size_t dstride, int W, int H)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    dst[(size_t)y * dstride + x] = (int16_t)median9(src, sstride, x, y, W, H);
}

hipError_t launch_median3(const int16_t* src, size_t sstride, int16_t* dst, size_t dstride, int W, int H,
                          hipStream_t st)
{
    dim3 grid((W + 63) / 64, (H + 3) / 4);
    hipLaunchKernelGGL(k_median3, grid, dim3(256), 0, st, src, sstride, dst, dstride, W, H);
    return hipGetLastError();
}

// ---------------------------------------------------------------- speckle filter ----
// Invariant: lab[i] <= i and lab[i] is in i's component, so every chain ends at a root
// and any (possibly stale) read is still a valid ancestor. Path halving writes go through
// atomicMin so they can never overwrite a smaller link made concurrently on another XCD.
__device__ __forceinline__ int uf_find_halve(int* __restrict__ lab, int x)
{
    int p = lab[x];
    while (p != x) {
        const int q = lab[p];
        if (q != p) atomicMin(&lab[x], q);
        x = p;
        p = q;
    }
    return x;
}

// Read-only find (after the union phase has completed: a kernel boundary away).
__device__ __forceinline__ int uf_root(const int* __restrict__ lab, int x)
{
    int p = lab[x];
    while (p != x) { x = p; p = lab[x]; }
    return x;
}

__device__ __forceinline__ void uf_union(int* __restrict__ lab, int a, int b)
{
    for (;;) {
        a = uf_find_halve(lab, a);
        b = uf_find_halve(lab, b);
        if (a == b) return;
        if (a < b) { int t = a; a = b; b = t; }          // link the larger root under the smaller
        const int old = atomicMin(&lab[a], b);
        if (old == a) return;
        a = old;
    }
}

// Phase 1, one 64 x 16 tile per block: union-find of the tile's own edges in LDS (local
// index = ty * 64 + tx, same order as the global raster index), then every pixel's global
// label = the global index of its tile-local root (<= its own index: the invariant holds).
constexpr int kSpkTW = 64, kSpkTH = 16;
__device__ __forceinline__ int luf_find(int* l, int x)
{
    int p = l[x];
    while (p != x) { const int q = l[p]; if (q != p) atomicMin(&l[x], q); x = p; p = q; }
    return x;
}
__device__ __forceinline__ void luf_union(int* l, int a, int b)
{
    for (;;) {
        a = luf_find(l, a);
        b = luf_find(l, b);
        if (a == b) return;
        if (a < b) { int t = a; a = b; b = t; }
        const int old = atomicMin(&l[a], b);
        if (old == a) return;
        a = old;
    }
}
// med (optional): the unfiltered disparity; the tile then applies medianBlur(3) itself, writes
// the filtered values to d and labels them (one launch less than median + speckle)
__global__ __launch_bounds__(256) void k_spk_tile(const int16_t* __restrict__ med, size_t mstride, int16_t* d,
                                                  size_t stride, int W, int H, int newVal, int maxDiff,
                                                  int* __restrict__ lab, int* __restrict__ cnt)
{
    __shared__ int l[kSpkTW * kSpkTH];
    __shared__ int lcnt[kSpkTW * kSpkTH];
    __shared__ int16_t v[kSpkTW * kSpkTH];
    const int x0 = blockIdx.x * kSpkTW, y0 = blockIdx.y * kSpkTH;
    for (int i = threadIdx.x; i < kSpkTW * kSpkTH; i += 256) {
        const int x = x0 + (i & (kSpkTW - 1)), y = y0 + i / kSpkTW;
        int dv = newVal;
        if (x < W && y < H) {
            if (med) {
                dv = median9(med, mstride, x, y, W, H);
                d[(size_t)y * stride + x] = (int16_t)dv;
            } else {
                dv = d[(size_t)y * stride + x];
            }
        }
        v[i] = (int16_t)dv;
        l[i] = dv != newVal ? i : -1;
        lcnt[i] = 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kSpkTW * kSpkTH; i += 256) {
        const int tx = i & (kSpkTW - 1), ty = i / kSpkTW;
        const int a = v[i];
        if (a == newVal) continue;
        if (tx + 1 < kSpkTW) { const int q = v[i + 1]; if (q != newVal && abs(a - q) <= maxDiff) luf_union(l, i, i + 1); }
        if (ty + 1 < kSpkTH) { const int q = v[i + kSpkTW]; if (q != newVal && abs(a - q) <= maxDiff) luf_union(l, i, i + kSpkTW); }
    }
    __syncthreads();
    // tile-local roots and component sizes (LDS atomics); each local root's pixel carries its
    // tile size in cnt, every other pixel 0
    for (int i = threadIdx.x; i < kSpkTW * kSpkTH; i += 256) {
        const int x = x0 + (i & (kSpkTW - 1)), y = y0 + i / kSpkTW;
        if (l[i] < 0 || x >= W || y >= H) continue;
        int r = i;
        while (l[r] != r) r = l[r];
        atomicAdd(&lcnt[r], 1);
        lab[y * W + x] = (y0 + r / kSpkTW) * W + x0 + (r & (kSpkTW - 1));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kSpkTW * kSpkTH; i += 256) {
        const int x = x0 + (i & (kSpkTW - 1)), y = y0 + i / kSpkTW;
        if (x >= W || y >= H) continue;
        if (l[i] < 0) lab[y * W + x] = -1;
        cnt[y * W + x] = l[i] == i ? lcnt[i] : 0;
    }
}

// Phase 2: the edges that cross tile borders (right column and bottom row of each tile),
// merged with the global union-find. Along a border, consecutive edges mostly join the
// same pair of tile-local components: an edge whose (label, label) pair equals the previous
// edge's is already covered by that edge's union (labels are read before any union of this
// block; any label read is a valid ancestor, so equal pairs mean the same two sets).
__global__ __launch_bounds__(256) void k_spk_border(const int16_t* __restrict__ d, size_t stride, int W, int H,
                                                    int newVal, int maxDiff, int* __restrict__ lab)
{
    __shared__ int pa[kSpkTH + kSpkTW], pb[kSpkTH + kSpkTW];
    const int x0 = blockIdx.x * kSpkTW, y0 = blockIdx.y * kSpkTH;
    const int t = threadIdx.x;
    constexpr int NE = kSpkTH + kSpkTW;
    int x = 0, y = 0, dx = 0, dy = 0;
    bool e = false;
    if (t < kSpkTH) { x = x0 + kSpkTW - 1; y = y0 + t; dx = 1; }                   // right edge
    else if (t < NE) { x = x0 + t - kSpkTH; y = y0 + kSpkTH - 1; dy = 1; }          // bottom edge
    if (t < NE && x + dx < W && y + dy < H && x < W && y < H) {
        const int a = d[(size_t)y * stride + x], q = d[(size_t)(y + dy) * stride + x + dx];
        e = a != newVal && q != newVal && abs(a - q) <= maxDiff;
    }
    if (t < NE) {
        pa[t] = e ? lab[y * W + x] : -1;
        pb[t] = e ? lab[(y + dy) * W + x + dx] : -1;
    }
    __syncthreads();
    if (!e) return;
    if (t != 0 && t != kSpkTH && pa[t - 1] == pa[t] && pb[t - 1] == pb[t]) return;
    uf_union(lab, y * W + x, (y + dy) * W + x + dx);
}

// After the union phase (a kernel boundary away): every label is pointed straight at its
// root (concurrent rewrites only ever replace a label by one of its ancestors, so the chains
// other threads are walking stay valid), and each tile-local root that is not the global
// root adds its tile size (k_spk_tile) to the global root's counter: one atomic per
// tile-local component, not per pixel. Only "size <= maxSize" is ever asked, so a counter
// already past maxSize takes no more adds (a count stays exact while it is <= maxSize).
__global__ __launch_bounds__(256) void k_spk_count(int W, int H, int maxSize, int* __restrict__ lab,
                                                   int* __restrict__ cnt)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H || lab[i] < 0) return;
    const int root = uf_root(lab, i);
    lab[i] = root;
    const int own = cnt[i];                        // > 0: i is a tile-local root
    if (own > 0 && root != i &&
        __hip_atomic_load(&cnt[root], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= maxSize)
        atomicAdd(&cnt[root], own);
}

__global__ __launch_bounds__(256) void k_spk_apply(int16_t* __restrict__ d, size_t stride, int W, int H, int newVal,
                                                   int maxSize, const int* __restrict__ lab,
                                                   const int* __restrict__ cnt)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    const int root = lab[i];
    if (root >= 0 && cnt[root] <= maxSize) {
        const int y = i / W, x = i - y * W;
        d[(size_t)y * stride + x] = (int16_t)newVal;
    }
}

// med != nullptr: medianBlur(3) of med into d first, inside the tile kernel
hipError_t launch_speckle(const int16_t* med, size_t mstride, int16_t* d, size_t stride, int W, int H, int newVal,
                          int maxSize, int maxDiff, int* lab, int* cnt, hipStream_t st)
{
    const int n = W * H;
    dim3 grid((n + 255) / 256), block(256);
    const dim3 tiles((W + kSpkTW - 1) / kSpkTW, (H + kSpkTH - 1) / kSpkTH);
    hipLaunchKernelGGL(k_spk_tile, tiles, block, 0, st, med, mstride, d, stride, W, H, newVal, maxDiff, lab, cnt);
    hipLaunchKernelGGL(k_spk_border, tiles, block, 0, st, d, stride, W, H, newVal, maxDiff, lab);
    hipLaunchKernelGGL(k_spk_count, grid, block, 0, st, W, H, maxSize, lab, cnt);
    hipLaunchKernelGGL(k_spk_apply, grid, block, 0, st, d, stride, W, H, newVal, maxSize, lab, cnt);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_fill16(int16_t* __restrict__ d, size_t stride, int W, int H, int v)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < W && y < H) d[(size_t)y * stride + x] = (int16_t)v;
}

hipError_t launch_fill16(int16_t* d, size_t stride, int W, int H, int v, hipStream_t st)
{
    hipLaunchKernelGGL(k_fill16, dim3((W + 255) / 256, H), dim3(256), 0, st, d, stride, W, H, v);
    return hipGetLastError();
}

// disparity_lr.convertTo(CV_32FC1) on the device (abstractStereoMatcher.cpp:49, matcherOpenCVSGBM.cpp:34):
// exact, every int16 is a float. Row strides in elements.
__global__ __launch_bounds__(256) void k_to_f32(const int16_t* __restrict__ s, size_t ss, float* __restrict__ d, size_t ds,
                                                int W)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < W) d[(size_t)y * ds + x] = (float)s[(size_t)y * ss + x];
}

hipError_t launch_to_f32(const int16_t* s, size_t ss, float* d, size_t ds, int W, int H, hipStream_t st)
{
    hipLaunchKernelGGL(k_to_f32, dim3((W + 255) / 256, H), dim3(256), 0, st, s, ss, d, ds, W);
    return hipGetLastError();
}

}  // namespace sgm
