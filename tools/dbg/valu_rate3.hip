#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k0(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_bcnt_u32_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_bcnt_u32_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n v_bcnt_u32_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_bcnt_u32_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k1(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_min_u16 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_pk_min_u16 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_pk_min_u16 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_pk_min_u16 %6, %6, %8\n v_add_u32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k2(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_min_u16 %0, %0, %8\n v_min_u16 %1, %1, %8\n v_pk_min_u16 %2, %2, %8\n v_min_u16 %3, %3, %8\n v_pk_min_u16 %4, %4, %8\n v_min_u16 %5, %5, %8\n v_pk_min_u16 %6, %6, %8\n v_min_u16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k3(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_mov_b32_sdwa %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n v_mov_b32_sdwa %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k4(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_u16_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_min_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k5(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_add_u16_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_add_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k6(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_or_b32_sdwa %0, %0, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %1, %1, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %2, %2, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %3, %3, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %4, %4, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %5, %5, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %6, %6, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n v_or_b32_sdwa %7, %7, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k7(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_lshlrev_b16 %0, 1, %0\n v_lshlrev_b16 %1, 1, %1\n v_lshlrev_b16 %2, 1, %2\n v_lshlrev_b16 %3, 1, %3\n v_lshlrev_b16 %4, 1, %4\n v_lshlrev_b16 %5, 1, %5\n v_lshlrev_b16 %6, 1, %6\n v_lshlrev_b16 %7, 1, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k8(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_lshrrev_b32 %0, %8, %0\n v_lshrrev_b32 %1, %8, %1\n v_lshrrev_b32 %2, %8, %2\n v_lshrrev_b32 %3, %8, %3\n v_lshrrev_b32 %4, %8, %4\n v_lshrrev_b32 %5, %8, %5\n v_lshrrev_b32 %6, %8, %6\n v_lshrrev_b32 %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k9(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_lshlrev_b32 %0, %8, %0\n v_lshlrev_b32 %1, %8, %1\n v_lshlrev_b32 %2, %8, %2\n v_lshlrev_b32 %3, %8, %3\n v_lshlrev_b32 %4, %8, %4\n v_lshlrev_b32 %5, %8, %5\n v_lshlrev_b32 %6, %8, %6\n v_lshlrev_b32 %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k10(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k11(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_mad_u32_u24 %0, %0, %8, %0\n v_mad_u32_u24 %1, %1, %8, %1\n v_mad_u32_u24 %2, %2, %8, %2\n v_mad_u32_u24 %3, %3, %8, %3\n v_mad_u32_u24 %4, %4, %8, %4\n v_mad_u32_u24 %5, %5, %8, %5\n v_mad_u32_u24 %6, %6, %8, %6\n v_mad_u32_u24 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k12(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_max_u16 %0, %0, %8\n v_max_u16 %1, %1, %8\n v_max_u16 %2, %2, %8\n v_max_u16 %3, %3, %8\n v_max_u16 %4, %4, %8\n v_max_u16 %5, %5, %8\n v_max_u16 %6, %6, %8\n v_max_u16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k13(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_sub_u16 %0, %0, %8\n v_sub_u16 %1, %1, %8\n v_sub_u16 %2, %2, %8\n v_sub_u16 %3, %3, %8\n v_sub_u16 %4, %4, %8\n v_sub_u16 %5, %5, %8\n v_sub_u16 %6, %6, %8\n v_sub_u16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k14(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_u32_dpp %0, %0, %0 row_shr:1 bound_ctrl:1\n v_add_u32 %1, %1, %8\n v_min_u32_dpp %2, %2, %2 row_shr:1 bound_ctrl:1\n v_add_u32 %3, %3, %8\n v_min_u32_dpp %4, %4, %4 row_shr:1 bound_ctrl:1\n v_add_u32 %5, %5, %8\n v_min_u32_dpp %6, %6, %6 row_shr:1 bound_ctrl:1\n v_add_u32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k15(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 bound_ctrl:1\n v_xor_b32 %1, %1, %8\n v_mov_b32_dpp %2, %2 row_shr:1 bound_ctrl:1\n v_xor_b32 %3, %3, %8\n v_mov_b32_dpp %4, %4 row_shr:1 bound_ctrl:1\n v_xor_b32 %5, %5, %8\n v_mov_b32_dpp %6, %6 row_shr:1 bound_ctrl:1\n v_xor_b32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k16(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_u16_dpp %0, %0, %0 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %1, %1, %1 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %2, %2, %2 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %3, %3, %3 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %4, %4, %4 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %5, %5, %5 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %6, %6, %6 row_shr:1 bound_ctrl:1\n v_min_u16_dpp %7, %7, %7 row_shr:1 bound_ctrl:1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k17(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_minimum3_f16 %0, %0, %8, %0\n v_xor_b32 %1, %1, %8\n v_pk_minimum3_f16 %2, %2, %8, %2\n v_xor_b32 %3, %3, %8\n v_pk_minimum3_f16 %4, %4, %8, %4\n v_xor_b32 %5, %5, %8\n v_pk_minimum3_f16 %6, %6, %8, %6\n v_xor_b32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k18(unsigned* out, int iters, unsigned c) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_bcnt_u32_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_and_b32 %2, %2, %8\n v_bcnt_u32_b32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_and_b32 %5, %5, %8\n v_bcnt_u32_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
typedef void (*K)(unsigned*, int, unsigned);
int main() { unsigned* d; (void)hipMalloc(&d, 256*256*64*4); int ncu = 0, clk = 0;
 (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0); (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
 K ks[] = {k0, k1, k2, k3, k4, k5, k6, k7, k8, k9, k10, k11, k12, k13, k14, k15, k16, k17, k18};
 const char* nm[] = {"mix bcnt+xor", "mix pkmin+add", "mix pkmin+minu16", "v_mov_b32_sdwa w1", "v_min_u16_sdwa hi", "v_add_u16_sdwa hi", "v_or_b32_sdwa", "v_lshlrev_b16", "v_lshrrev_b32 c", "v_lshlrev_b32 v", "v_mul_u32_u24", "v_mad_u32_u24", "v_max_u16", "v_sub_u16", "v_min_u32_dpp+fast", "v_mov_dpp+xor", "v_min_u16_dpp", "v_pk_min3f16+xor", "bcnt+xor+xor"};
 hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
 for (int i = 0; i < (int)(sizeof(ks)/sizeof(ks[0])); i++) { for (int w : {4}) {
   const int iters = 1000;
   hipLaunchKernelGGL(ks[i], dim3(ncu * w), dim3(256), 0, 0, d, 10, 1u);
   (void)hipEventRecord(a); hipLaunchKernelGGL(ks[i], dim3(ncu * w), dim3(256), 0, 0, d, iters, 1u); (void)hipEventRecord(b);
   (void)hipEventSynchronize(b); float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
   printf("%-20s waves/SIMD %d: %.2f cyc/wave-instr/SIMD\n", nm[i], w, ms * 1e-3 * clk * 1e3 / ((double)w * iters * 16 * 8)); } }
 return 0; }