// HBM bandwidth probe (gfx950): streaming read-only (sum), write-only and copy over a
// buffer much larger than the 256 MiB MALL. Reports the best of several runs in GB/s.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, size_t n, unsigned* out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ p, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4((unsigned)i, 0, 0, 0);
}
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

int main()
{
    const size_t bytes = 4ull << 30;
    const size_t n = bytes / 16;
    uint4 *a, *b;
    unsigned* o;
    (void)hipMalloc(&a, bytes); (void)hipMalloc(&b, bytes); (void)hipMalloc(&o, 4);
    (void)hipMemset(a, 1, bytes); (void)hipMemset(b, 2, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int grid : {1024, 2048, 4096, 8192}) {
        float best[3] = {1e9f, 1e9f, 1e9f};
        for (int r = 0; r < 5; r++) {
            float ms;
            (void)hipEventRecord(e0); hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, o); (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1); best[0] = ms < best[0] ? ms : best[0];
            (void)hipEventRecord(e0); hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, b, n); (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1); best[1] = ms < best[1] ? ms : best[1];
            (void)hipEventRecord(e0); hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n / 2); (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1); best[2] = ms < best[2] ? ms : best[2];
        }
        printf("grid %5d: read %.0f GB/s  write %.0f GB/s  copy %.0f GB/s (read+write bytes)\n", grid,
               bytes / best[0] / 1e6, bytes / best[1] / 1e6, bytes / best[2] / 1e6);
    }
    return 0;
}
