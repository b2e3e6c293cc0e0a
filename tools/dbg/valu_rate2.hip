#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k0(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_and_b32 %0, %0, %8\n v_and_b32 %1, %1, %8\n v_and_b32 %2, %2, %8\n v_and_b32 %3, %3, %8\n v_and_b32 %4, %4, %8\n v_and_b32 %5, %5, %8\n v_and_b32 %6, %6, %8\n v_and_b32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k1(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_or_b32 %0, %0, %8\n v_or_b32 %1, %1, %8\n v_or_b32 %2, %2, %8\n v_or_b32 %3, %3, %8\n v_or_b32 %4, %4, %8\n v_or_b32 %5, %5, %8\n v_or_b32 %6, %6, %8\n v_or_b32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k2(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_sub_u32 %0, %0, %8\n v_sub_u32 %1, %1, %8\n v_sub_u32 %2, %2, %8\n v_sub_u32 %3, %3, %8\n v_sub_u32 %4, %4, %8\n v_sub_u32 %5, %5, %8\n v_sub_u32 %6, %6, %8\n v_sub_u32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k3(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_max_u32 %0, %0, %8\n v_max_u32 %1, %1, %8\n v_max_u32 %2, %2, %8\n v_max_u32 %3, %3, %8\n v_max_u32 %4, %4, %8\n v_max_u32 %5, %5, %8\n v_max_u32 %6, %6, %8\n v_max_u32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k4(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_i32 %0, %0, %8\n v_min_i32 %1, %1, %8\n v_min_i32 %2, %2, %8\n v_min_i32 %3, %3, %8\n v_min_i32 %4, %4, %8\n v_min_i32 %5, %5, %8\n v_min_i32 %6, %6, %8\n v_min_i32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k5(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_lshlrev_b32 %0, 1, %0\n v_lshlrev_b32 %1, 1, %1\n v_lshlrev_b32 %2, 1, %2\n v_lshlrev_b32 %3, 1, %3\n v_lshlrev_b32 %4, 1, %4\n v_lshlrev_b32 %5, 1, %5\n v_lshlrev_b32 %6, 1, %6\n v_lshlrev_b32 %7, 1, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k6(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_lshrrev_b32 %0, 1, %0\n v_lshrrev_b32 %1, 1, %1\n v_lshrrev_b32 %2, 1, %2\n v_lshrrev_b32 %3, 1, %3\n v_lshrrev_b32 %4, 1, %4\n v_lshrrev_b32 %5, 1, %5\n v_lshrrev_b32 %6, 1, %6\n v_lshrrev_b32 %7, 1, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k7(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k8(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k9(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_fma_f32 %0, %0, %8, %0\n v_fma_f32 %1, %1, %8, %1\n v_fma_f32 %2, %2, %8, %2\n v_fma_f32 %3, %3, %8, %3\n v_fma_f32 %4, %4, %8, %4\n v_fma_f32 %5, %5, %8, %5\n v_fma_f32 %6, %6, %8, %6\n v_fma_f32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k10(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_f32 %0, %0, %8\n v_min_f32 %1, %1, %8\n v_min_f32 %2, %2, %8\n v_min_f32 %3, %3, %8\n v_min_f32 %4, %4, %8\n v_min_f32 %5, %5, %8\n v_min_f32 %6, %6, %8\n v_min_f32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k11(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_add_f16 %0, %0, %8\n v_pk_add_f16 %1, %1, %8\n v_pk_add_f16 %2, %2, %8\n v_pk_add_f16 %3, %3, %8\n v_pk_add_f16 %4, %4, %8\n v_pk_add_f16 %5, %5, %8\n v_pk_add_f16 %6, %6, %8\n v_pk_add_f16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k12(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_min_f16 %0, %0, %8\n v_pk_min_f16 %1, %1, %8\n v_pk_min_f16 %2, %2, %8\n v_pk_min_f16 %3, %3, %8\n v_pk_min_f16 %4, %4, %8\n v_pk_min_f16 %5, %5, %8\n v_pk_min_f16 %6, %6, %8\n v_pk_min_f16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k13(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_fma_f16 %0, %0, %8, %0\n v_pk_fma_f16 %1, %1, %8, %1\n v_pk_fma_f16 %2, %2, %8, %2\n v_pk_fma_f16 %3, %3, %8, %3\n v_pk_fma_f16 %4, %4, %8, %4\n v_pk_fma_f16 %5, %5, %8, %5\n v_pk_fma_f16 %6, %6, %8, %6\n v_pk_fma_f16 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k14(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_add3_u32 %0, %0, %8, %0\n v_add3_u32 %1, %1, %8, %1\n v_add3_u32 %2, %2, %8, %2\n v_add3_u32 %3, %3, %8, %3\n v_add3_u32 %4, %4, %8, %4\n v_add3_u32 %5, %5, %8, %5\n v_add3_u32 %6, %6, %8, %6\n v_add3_u32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k15(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_xad_u32 %0, %0, %8, %0\n v_xad_u32 %1, %1, %8, %1\n v_xad_u32 %2, %2, %8, %2\n v_xad_u32 %3, %3, %8, %3\n v_xad_u32 %4, %4, %8, %4\n v_xad_u32 %5, %5, %8, %5\n v_xad_u32 %6, %6, %8, %6\n v_xad_u32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k16(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_u16 %0, %0, %8\n v_min_u16 %1, %1, %8\n v_min_u16 %2, %2, %8\n v_min_u16 %3, %3, %8\n v_min_u16 %4, %4, %8\n v_min_u16 %5, %5, %8\n v_min_u16 %6, %6, %8\n v_min_u16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k17(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_add_u16 %0, %0, %8\n v_add_u16 %1, %1, %8\n v_add_u16 %2, %2, %8\n v_add_u16 %3, %3, %8\n v_add_u16 %4, %4, %8\n v_add_u16 %5, %5, %8\n v_add_u16 %6, %6, %8\n v_add_u16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k18(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned long long a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(c2));
  }
  out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}
__global__ __launch_bounds__(256) void k19(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n v_mov_b32 %4, %8\n v_mov_b32 %5, %8\n v_mov_b32 %6, %8\n v_mov_b32 %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k20(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_f16 %0, %0, %8\n v_min_f16 %1, %1, %8\n v_min_f16 %2, %2, %8\n v_min_f16 %3, %3, %8\n v_min_f16 %4, %4, %8\n v_min_f16 %5, %5, %8\n v_min_f16 %6, %6, %8\n v_min_f16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k21(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_add_f16 %0, %0, %8\n v_add_f16 %1, %1, %8\n v_add_f16 %2, %2, %8\n v_add_f16 %3, %3, %8\n v_add_f16 %4, %4, %8\n v_add_f16 %5, %5, %8\n v_add_f16 %6, %6, %8\n v_add_f16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k22(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_max3_u32 %0, %0, %8, %0\n v_max3_u32 %1, %1, %8, %1\n v_max3_u32 %2, %2, %8, %2\n v_max3_u32 %3, %3, %8, %3\n v_max3_u32 %4, %4, %8, %4\n v_max3_u32 %5, %5, %8, %5\n v_max3_u32 %6, %6, %8, %6\n v_max3_u32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k23(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_bfe_u32 %0, %0, 8, 8\n v_bfe_u32 %1, %1, 8, 8\n v_bfe_u32 %2, %2, 8, 8\n v_bfe_u32 %3, %3, 8, 8\n v_bfe_u32 %4, %4, 8, 8\n v_bfe_u32 %5, %5, 8, 8\n v_bfe_u32 %6, %6, 8, 8\n v_bfe_u32 %7, %7, 8, 8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k24(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_and_or_b32 %0, %0, %8, %0\n v_and_or_b32 %1, %1, %8, %1\n v_and_or_b32 %2, %2, %8, %2\n v_and_or_b32 %3, %3, %8, %3\n v_and_or_b32 %4, %4, %8, %4\n v_and_or_b32 %5, %5, %8, %5\n v_and_or_b32 %6, %6, %8, %6\n v_and_or_b32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k25(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_or3_b32 %0, %0, %8, %0\n v_or3_b32 %1, %1, %8, %1\n v_or3_b32 %2, %2, %8, %2\n v_or3_b32 %3, %3, %8, %3\n v_or3_b32 %4, %4, %8, %4\n v_or3_b32 %5, %5, %8, %5\n v_or3_b32 %6, %6, %8, %6\n v_or3_b32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k26(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_sad_u32 %0, %0, %8, %0\n v_sad_u32 %1, %1, %8, %1\n v_sad_u32 %2, %2, %8, %2\n v_sad_u32 %3, %3, %8, %3\n v_sad_u32 %4, %4, %8, %4\n v_sad_u32 %5, %5, %8, %5\n v_sad_u32 %6, %6, %8, %6\n v_sad_u32 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k27(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_max_i16 %0, %0, %8\n v_pk_max_i16 %1, %1, %8\n v_pk_max_i16 %2, %2, %8\n v_pk_max_i16 %3, %3, %8\n v_pk_max_i16 %4, %4, %8\n v_pk_max_i16 %5, %5, %8\n v_pk_max_i16 %6, %6, %8\n v_pk_max_i16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k28(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_cvt_f32_u32 %0, %0\n v_cvt_f32_u32 %1, %1\n v_cvt_f32_u32 %2, %2\n v_cvt_f32_u32 %3, %3\n v_cvt_f32_u32 %4, %4\n v_cvt_f32_u32 %5, %5\n v_cvt_f32_u32 %6, %6\n v_cvt_f32_u32 %7, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k29(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_min_u32_e64 %0, %0, %8\n v_min_u32_e64 %1, %1, %8\n v_min_u32_e64 %2, %2, %8\n v_min_u32_e64 %3, %3, %8\n v_min_u32_e64 %4, %4, %8\n v_min_u32_e64 %5, %5, %8\n v_min_u32_e64 %6, %6, %8\n v_min_u32_e64 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k30(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_sub_f32 %0, %0, %8\n v_sub_f32 %1, %1, %8\n v_sub_f32 %2, %2, %8\n v_sub_f32 %3, %3, %8\n v_sub_f32 %4, %4, %8\n v_sub_f32 %5, %5, %8\n v_sub_f32 %6, %6, %8\n v_sub_f32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k31(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_max_f32 %0, %0, %8\n v_max_f32 %1, %1, %8\n v_max_f32 %2, %2, %8\n v_max_f32 %3, %3, %8\n v_max_f32 %4, %4, %8\n v_max_f32 %5, %5, %8\n v_max_f32 %6, %6, %8\n v_max_f32 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k32(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned long long a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4\n v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(c2));
  }
  out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}
__global__ __launch_bounds__(256) void k33(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned long long a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_pk_fma_f32 %0, %0, %4, %0\n v_pk_fma_f32 %1, %1, %4, %1\n v_pk_fma_f32 %2, %2, %4, %2\n v_pk_fma_f32 %3, %3, %4, %3\n v_pk_fma_f32 %0, %0, %4, %0\n v_pk_fma_f32 %1, %1, %4, %1\n v_pk_fma_f32 %2, %2, %4, %2\n v_pk_fma_f32 %3, %3, %4, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(c2));
  }
  out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}
__global__ __launch_bounds__(256) void k34(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_dot2_f32_f16 %0, %0, %8, %0\n v_dot2_f32_f16 %1, %1, %8, %1\n v_dot2_f32_f16 %2, %2, %8, %2\n v_dot2_f32_f16 %3, %3, %8, %3\n v_dot2_f32_f16 %4, %4, %8, %4\n v_dot2_f32_f16 %5, %5, %8, %5\n v_dot2_f32_f16 %6, %6, %8, %6\n v_dot2_f32_f16 %7, %7, %8, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
__global__ __launch_bounds__(256) void k35(unsigned* out, int iters, unsigned c, unsigned long long c2) {
  unsigned v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 + 11, v6 = v0 * 13, v7 = v0 + 15;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++)
      asm volatile("v_max_i16 %0, %0, %8\n v_max_i16 %1, %1, %8\n v_max_i16 %2, %2, %8\n v_max_i16 %3, %3, %8\n v_max_i16 %4, %4, %8\n v_max_i16 %5, %5, %8\n v_max_i16 %6, %6, %8\n v_max_i16 %7, %7, %8" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}
typedef void (*K)(unsigned*, int, unsigned, unsigned long long);
int main() { unsigned* d; (void)hipMalloc(&d, 256*256*64*4); int ncu = 0, clk = 0;
 (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0); (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
 K ks[] = {k0, k1, k2, k3, k4, k5, k6, k7, k8, k9, k10, k11, k12, k13, k14, k15, k16, k17, k18, k19, k20, k21, k22, k23, k24, k25, k26, k27, k28, k29, k30, k31, k32, k33, k34, k35};
 const char* nm[] = {"v_and_b32", "v_or_b32", "v_sub_u32", "v_max_u32", "v_min_i32", "v_lshlrev_b32", "v_lshrrev_b32", "v_cndmask_b32", "v_add_f32", "v_fma_f32", "v_min_f32", "v_pk_add_f16", "v_pk_min_f16", "v_pk_fma_f16", "v_add3_u32", "v_xad_u32", "v_min_u16", "v_add_u16", "v_pk_add_f32", "v_mov_b32", "v_min_f16", "v_add_f16", "v_max3_u32", "v_bfe_u32", "v_and_or_b32", "v_or3_b32", "v_sad_u32", "v_pk_max_i16", "v_cvt_f32_u32", "v_min_u32_e64", "v_sub_f32", "v_max_f32", "v_pk_mul_f32", "v_pk_fma_f32", "v_dot2_f32_f16", "v_max_i16"};
 hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
 for (int i = 0; i < (int)(sizeof(ks)/sizeof(ks[0])); i++) { for (int w : {1, 4}) {
   const int iters = 1000;
   hipLaunchKernelGGL(ks[i], dim3(ncu * w), dim3(256), 0, 0, d, 10, 1u, 1ull);
   (void)hipEventRecord(a); hipLaunchKernelGGL(ks[i], dim3(ncu * w), dim3(256), 0, 0, d, iters, 1u, 1ull); (void)hipEventRecord(b);
   (void)hipEventSynchronize(b); float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
   printf("%-18s waves/SIMD %d: %.2f cyc/wave-instr/SIMD\n", nm[i], w, ms * 1e-3 * clk * 1e3 / ((double)w * iters * 16 * 8)); } }
 return 0; }