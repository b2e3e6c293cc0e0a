// VALU issue-rate microbenchmark (gfx950): cycles per wave64 instruction per SIMD for the
// instruction kinds the path engine uses. Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)
template <int KIND>
__global__ __launch_bounds__(256) void k(unsigned* out, int iters, unsigned c)
{
    unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#define X(OPS) asm volatile(OPS : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
            if constexpr (KIND == 0) X("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8")
            if constexpr (KIND == 1) X("v_bcnt_u32_b32 %0, %0, %8\n v_bcnt_u32_b32 %1, %1, %8\n v_bcnt_u32_b32 %2, %2, %8\n v_bcnt_u32_b32 %3, %3, %8\n v_bcnt_u32_b32 %4, %4, %8\n v_bcnt_u32_b32 %5, %5, %8\n v_bcnt_u32_b32 %6, %6, %8\n v_bcnt_u32_b32 %7, %7, %8")
            if constexpr (KIND == 2) X("v_pk_min_u16 %0, %0, %8\n v_pk_min_u16 %1, %1, %8\n v_pk_min_u16 %2, %2, %8\n v_pk_min_u16 %3, %3, %8\n v_pk_min_u16 %4, %4, %8\n v_pk_min_u16 %5, %5, %8\n v_pk_min_u16 %6, %6, %8\n v_pk_min_u16 %7, %7, %8")
            if constexpr (KIND == 3) X("v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %8\n v_pk_add_u16 %2, %2, %8\n v_pk_add_u16 %3, %3, %8\n v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %8\n v_pk_add_u16 %6, %6, %8\n v_pk_add_u16 %7, %7, %8")
            if constexpr (KIND == 4) X("v_alignbit_b32 %0, %0, %8, 16\n v_alignbit_b32 %1, %1, %8, 16\n v_alignbit_b32 %2, %2, %8, 16\n v_alignbit_b32 %3, %3, %8, 16\n v_alignbit_b32 %4, %4, %8, 16\n v_alignbit_b32 %5, %5, %8, 16\n v_alignbit_b32 %6, %6, %8, 16\n v_alignbit_b32 %7, %7, %8, 16")
            if constexpr (KIND == 5) X("v_mov_b32_dpp %0, %0 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %1, %1 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %2, %2 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %3, %3 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %4, %4 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %5, %5 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %6, %6 row_shr:1 bound_ctrl:1\n v_mov_b32_dpp %7, %7 row_shr:1 bound_ctrl:1")
            if constexpr (KIND == 6) X("v_pk_minimum3_f16 %0, %0, %8, %1\n v_pk_minimum3_f16 %1, %1, %8, %2\n v_pk_minimum3_f16 %2, %2, %8, %3\n v_pk_minimum3_f16 %3, %3, %8, %4\n v_pk_minimum3_f16 %4, %4, %8, %5\n v_pk_minimum3_f16 %5, %5, %8, %6\n v_pk_minimum3_f16 %6, %6, %8, %7\n v_pk_minimum3_f16 %7, %7, %8, %0")
            if constexpr (KIND == 7) X("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8")
            if constexpr (KIND == 8) X("v_perm_b32 %0, %0, %8, %1\n v_perm_b32 %1, %1, %8, %2\n v_perm_b32 %2, %2, %8, %3\n v_perm_b32 %3, %3, %8, %4\n v_perm_b32 %4, %4, %8, %5\n v_perm_b32 %5, %5, %8, %6\n v_perm_b32 %6, %6, %8, %7\n v_perm_b32 %7, %7, %8, %0")
            if constexpr (KIND == 9) X("v_min_u32 %0, %0, %8\n v_min_u32 %1, %1, %8\n v_min_u32 %2, %2, %8\n v_min_u32 %3, %3, %8\n v_min_u32 %4, %4, %8\n v_min_u32 %5, %5, %8\n v_min_u32 %6, %6, %8\n v_min_u32 %7, %7, %8")
            if constexpr (KIND == 10) X("v_min3_u32 %0, %0, %8, %1\n v_min3_u32 %1, %1, %8, %2\n v_min3_u32 %2, %2, %8, %3\n v_min3_u32 %3, %3, %8, %4\n v_min3_u32 %4, %4, %8, %5\n v_min3_u32 %5, %5, %8, %6\n v_min3_u32 %6, %6, %8, %7\n v_min3_u32 %7, %7, %8, %0")
            if constexpr (KIND == 11) X("v_lshl_or_b32 %0, %0, 16, %8\n v_lshl_or_b32 %1, %1, 16, %8\n v_lshl_or_b32 %2, %2, 16, %8\n v_lshl_or_b32 %3, %3, 16, %8\n v_lshl_or_b32 %4, %4, 16, %8\n v_lshl_or_b32 %5, %5, 16, %8\n v_lshl_or_b32 %6, %6, 16, %8\n v_lshl_or_b32 %7, %7, 16, %8")
            if constexpr (KIND == 12) X("v_min_u32_dpp %0, %0, %0 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %1, %1, %1 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %2, %2, %2 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %3, %3, %3 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %4, %4, %4 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %5, %5, %5 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %6, %6, %6 row_shr:1 bound_ctrl:1\n v_min_u32_dpp %7, %7, %7 row_shr:1 bound_ctrl:1")
            if constexpr (KIND == 13) X("v_pk_sub_u16 %0, %0, %8\n v_pk_sub_u16 %1, %1, %8\n v_pk_sub_u16 %2, %2, %8\n v_pk_sub_u16 %3, %3, %8\n v_pk_sub_u16 %4, %4, %8\n v_pk_sub_u16 %5, %5, %8\n v_pk_sub_u16 %6, %6, %8\n v_pk_sub_u16 %7, %7, %8")
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}

template <int KIND>
void run(const char* name, unsigned* d, int wps)
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
    const int iters = 2000;
    const int blocks = ncu * wps;          // 256 threads = 4 waves = 1 per SIMD per block
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, 10, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double instr_per_simd = (double)wps * iters * 16 * 8;     // wave-instructions per SIMD
    const double cyc = ms * 1e-3 * clk * 1e3;
    printf("%-22s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (clock %d MHz, %.3f ms)\n", name, wps,
           cyc / instr_per_simd, clk / 1000, ms);
}

int main()
{
    unsigned* d;
    hipMalloc(&d, 256 * 256 * 64 * 4);
    for (int w : {1, 2, 4, 8}) {
        run<0>("v_xor_b32", d, w);
        run<1>("v_bcnt_u32_b32", d, w);
        run<2>("v_pk_min_u16", d, w);
        run<3>("v_pk_add_u16", d, w);
        run<13>("v_pk_sub_u16", d, w);
        run<4>("v_alignbit_b32", d, w);
        run<5>("v_mov_b32_dpp", d, w);
        run<12>("v_min_u32_dpp", d, w);
        run<6>("v_pk_minimum3_f16", d, w);
        run<7>("v_add_u32", d, w);
        run<8>("v_perm_b32", d, w);
        run<9>("v_min_u32", d, w);
        run<10>("v_min3_u32", d, w);
        run<11>("v_lshl_or_b32", d, w);
    }
    return 0;
}
