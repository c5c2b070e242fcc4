#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k0(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\tv_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k1(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_sub_u32 %0, %0, %8\n\tv_sub_u32 %1, %1, %8\n\tv_sub_u32 %2, %2, %8\n\tv_sub_u32 %3, %3, %8\n\tv_sub_u32 %4, %4, %8\n\tv_sub_u32 %5, %5, %8\n\tv_sub_u32 %6, %6, %8\n\tv_sub_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k2(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_or_b32 %0, %0, %8\n\tv_or_b32 %1, %1, %8\n\tv_or_b32 %2, %2, %8\n\tv_or_b32 %3, %3, %8\n\tv_or_b32 %4, %4, %8\n\tv_or_b32 %5, %5, %8\n\tv_or_b32 %6, %6, %8\n\tv_or_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k3(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_and_b32 %0, %0, %8\n\tv_and_b32 %1, %1, %8\n\tv_and_b32 %2, %2, %8\n\tv_and_b32 %3, %3, %8\n\tv_and_b32 %4, %4, %8\n\tv_and_b32 %5, %5, %8\n\tv_and_b32 %6, %6, %8\n\tv_and_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k4(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_xor_b32 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\tv_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k5(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_lshlrev_b32 %0, 3, %0\n\tv_lshlrev_b32 %1, 3, %1\n\tv_lshlrev_b32 %2, 3, %2\n\tv_lshlrev_b32 %3, 3, %3\n\tv_lshlrev_b32 %4, 3, %4\n\tv_lshlrev_b32 %5, 3, %5\n\tv_lshlrev_b32 %6, 3, %6\n\tv_lshlrev_b32 %7, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k6(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_lshrrev_b32 %0, 3, %0\n\tv_lshrrev_b32 %1, 3, %1\n\tv_lshrrev_b32 %2, 3, %2\n\tv_lshrrev_b32 %3, 3, %3\n\tv_lshrrev_b32 %4, 3, %4\n\tv_lshrrev_b32 %5, 3, %5\n\tv_lshrrev_b32 %6, 3, %6\n\tv_lshrrev_b32 %7, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k7(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_ashrrev_i32 %0, 3, %0\n\tv_ashrrev_i32 %1, 3, %1\n\tv_ashrrev_i32 %2, 3, %2\n\tv_ashrrev_i32 %3, 3, %3\n\tv_ashrrev_i32 %4, 3, %4\n\tv_ashrrev_i32 %5, 3, %5\n\tv_ashrrev_i32 %6, 3, %6\n\tv_ashrrev_i32 %7, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k8(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_min_u32 %0, %0, %8\n\tv_min_u32 %1, %1, %8\n\tv_min_u32 %2, %2, %8\n\tv_min_u32 %3, %3, %8\n\tv_min_u32 %4, %4, %8\n\tv_min_u32 %5, %5, %8\n\tv_min_u32 %6, %6, %8\n\tv_min_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k9(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_max_u32 %0, %0, %8\n\tv_max_u32 %1, %1, %8\n\tv_max_u32 %2, %2, %8\n\tv_max_u32 %3, %3, %8\n\tv_max_u32 %4, %4, %8\n\tv_max_u32 %5, %5, %8\n\tv_max_u32 %6, %6, %8\n\tv_max_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k10(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_max_i32 %0, %0, %8\n\tv_max_i32 %1, %1, %8\n\tv_max_i32 %2, %2, %8\n\tv_max_i32 %3, %3, %8\n\tv_max_i32 %4, %4, %8\n\tv_max_i32 %5, %5, %8\n\tv_max_i32 %6, %6, %8\n\tv_max_i32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k11(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_min_i32 %0, %0, %8\n\tv_min_i32 %1, %1, %8\n\tv_min_i32 %2, %2, %8\n\tv_min_i32 %3, %3, %8\n\tv_min_i32 %4, %4, %8\n\tv_min_i32 %5, %5, %8\n\tv_min_i32 %6, %6, %8\n\tv_min_i32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k12(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_not_b32 %0, %0\n\tv_not_b32 %1, %1\n\tv_not_b32 %2, %2\n\tv_not_b32 %3, %3\n\tv_not_b32 %4, %4\n\tv_not_b32 %5, %5\n\tv_not_b32 %6, %6\n\tv_not_b32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k13(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\tv_mov_b32 %3, %8\n\tv_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\tv_mov_b32 %6, %8\n\tv_mov_b32 %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k14(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_bfrev_b32 %0, %0\n\tv_bfrev_b32 %1, %1\n\tv_bfrev_b32 %2, %2\n\tv_bfrev_b32 %3, %3\n\tv_bfrev_b32 %4, %4\n\tv_bfrev_b32 %5, %5\n\tv_bfrev_b32 %6, %6\n\tv_bfrev_b32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k15(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_ffbh_u32 %0, %0\n\tv_ffbh_u32 %1, %1\n\tv_ffbh_u32 %2, %2\n\tv_ffbh_u32 %3, %3\n\tv_ffbh_u32 %4, %4\n\tv_ffbh_u32 %5, %5\n\tv_ffbh_u32 %6, %6\n\tv_ffbh_u32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k16(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_bcnt_u32_b32 %0, %0, %8\n\tv_bcnt_u32_b32 %1, %1, %8\n\tv_bcnt_u32_b32 %2, %2, %8\n\tv_bcnt_u32_b32 %3, %3, %8\n\tv_bcnt_u32_b32 %4, %4, %8\n\tv_bcnt_u32_b32 %5, %5, %8\n\tv_bcnt_u32_b32 %6, %6, %8\n\tv_bcnt_u32_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k17(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_bfe_u32 %0, %0, 3, 20\n\tv_bfe_u32 %1, %1, 3, 20\n\tv_bfe_u32 %2, %2, 3, 20\n\tv_bfe_u32 %3, %3, 3, 20\n\tv_bfe_u32 %4, %4, 3, 20\n\tv_bfe_u32 %5, %5, 3, 20\n\tv_bfe_u32 %6, %6, 3, 20\n\tv_bfe_u32 %7, %7, 3, 20" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k18(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_bfe_i32 %0, %0, 3, 1\n\tv_bfe_i32 %1, %1, 3, 1\n\tv_bfe_i32 %2, %2, 3, 1\n\tv_bfe_i32 %3, %3, 3, 1\n\tv_bfe_i32 %4, %4, 3, 1\n\tv_bfe_i32 %5, %5, 3, 1\n\tv_bfe_i32 %6, %6, 3, 1\n\tv_bfe_i32 %7, %7, 3, 1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k19(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_bfi_b32 %0, %8, %0, %8\n\tv_bfi_b32 %1, %8, %1, %8\n\tv_bfi_b32 %2, %8, %2, %8\n\tv_bfi_b32 %3, %8, %3, %8\n\tv_bfi_b32 %4, %8, %4, %8\n\tv_bfi_b32 %5, %8, %5, %8\n\tv_bfi_b32 %6, %8, %6, %8\n\tv_bfi_b32 %7, %8, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k20(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_alignbit_b32 %0, %0, %8, 5\n\tv_alignbit_b32 %1, %1, %8, 5\n\tv_alignbit_b32 %2, %2, %8, 5\n\tv_alignbit_b32 %3, %3, %8, 5\n\tv_alignbit_b32 %4, %4, %8, 5\n\tv_alignbit_b32 %5, %5, %8, 5\n\tv_alignbit_b32 %6, %6, %8, 5\n\tv_alignbit_b32 %7, %7, %8, 5" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k21(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_perm_b32 %0, %0, %8, %8\n\tv_perm_b32 %1, %1, %8, %8\n\tv_perm_b32 %2, %2, %8, %8\n\tv_perm_b32 %3, %3, %8, %8\n\tv_perm_b32 %4, %4, %8, %8\n\tv_perm_b32 %5, %5, %8, %8\n\tv_perm_b32 %6, %6, %8, %8\n\tv_perm_b32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k22(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_lshl_or_b32 %0, %0, 2, %8\n\tv_lshl_or_b32 %1, %1, 2, %8\n\tv_lshl_or_b32 %2, %2, 2, %8\n\tv_lshl_or_b32 %3, %3, 2, %8\n\tv_lshl_or_b32 %4, %4, 2, %8\n\tv_lshl_or_b32 %5, %5, 2, %8\n\tv_lshl_or_b32 %6, %6, 2, %8\n\tv_lshl_or_b32 %7, %7, 2, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k23(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_and_or_b32 %0, %0, %8, %8\n\tv_and_or_b32 %1, %1, %8, %8\n\tv_and_or_b32 %2, %2, %8, %8\n\tv_and_or_b32 %3, %3, %8, %8\n\tv_and_or_b32 %4, %4, %8, %8\n\tv_and_or_b32 %5, %5, %8, %8\n\tv_and_or_b32 %6, %6, %8, %8\n\tv_and_or_b32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k24(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_or3_b32 %0, %0, %8, %8\n\tv_or3_b32 %1, %1, %8, %8\n\tv_or3_b32 %2, %2, %8, %8\n\tv_or3_b32 %3, %3, %8, %8\n\tv_or3_b32 %4, %4, %8, %8\n\tv_or3_b32 %5, %5, %8, %8\n\tv_or3_b32 %6, %6, %8, %8\n\tv_or3_b32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k25(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_add3_u32 %0, %0, %8, %8\n\tv_add3_u32 %1, %1, %8, %8\n\tv_add3_u32 %2, %2, %8, %8\n\tv_add3_u32 %3, %3, %8, %8\n\tv_add3_u32 %4, %4, %8, %8\n\tv_add3_u32 %5, %5, %8, %8\n\tv_add3_u32 %6, %6, %8, %8\n\tv_add3_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k26(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_lshl_add_u32 %0, %0, 2, %8\n\tv_lshl_add_u32 %1, %1, 2, %8\n\tv_lshl_add_u32 %2, %2, 2, %8\n\tv_lshl_add_u32 %3, %3, 2, %8\n\tv_lshl_add_u32 %4, %4, 2, %8\n\tv_lshl_add_u32 %5, %5, 2, %8\n\tv_lshl_add_u32 %6, %6, 2, %8\n\tv_lshl_add_u32 %7, %7, 2, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k27(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_min3_u32 %0, %0, %8, %8\n\tv_min3_u32 %1, %1, %8, %8\n\tv_min3_u32 %2, %2, %8, %8\n\tv_min3_u32 %3, %3, %8, %8\n\tv_min3_u32 %4, %4, %8, %8\n\tv_min3_u32 %5, %5, %8, %8\n\tv_min3_u32 %6, %6, %8, %8\n\tv_min3_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k28(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_max3_u32 %0, %0, %8, %8\n\tv_max3_u32 %1, %1, %8, %8\n\tv_max3_u32 %2, %2, %8, %8\n\tv_max3_u32 %3, %3, %8, %8\n\tv_max3_u32 %4, %4, %8, %8\n\tv_max3_u32 %5, %5, %8, %8\n\tv_max3_u32 %6, %6, %8, %8\n\tv_max3_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k29(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_bitop3_b32 %0, %0, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %1, %1, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %2, %2, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %3, %3, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %4, %4, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %5, %5, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %6, %6, %8, %8 bitop3:0x2a\n\tv_bitop3_b32 %7, %7, %8, %8 bitop3:0x2a" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k30(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_dot4_u32_u8 %0, %0, %8, %8\n\tv_dot4_u32_u8 %1, %1, %8, %8\n\tv_dot4_u32_u8 %2, %2, %8, %8\n\tv_dot4_u32_u8 %3, %3, %8, %8\n\tv_dot4_u32_u8 %4, %4, %8, %8\n\tv_dot4_u32_u8 %5, %5, %8, %8\n\tv_dot4_u32_u8 %6, %6, %8, %8\n\tv_dot4_u32_u8 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k31(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mul_lo_u32 %0, %0, %8\n\tv_mul_lo_u32 %1, %1, %8\n\tv_mul_lo_u32 %2, %2, %8\n\tv_mul_lo_u32 %3, %3, %8\n\tv_mul_lo_u32 %4, %4, %8\n\tv_mul_lo_u32 %5, %5, %8\n\tv_mul_lo_u32 %6, %6, %8\n\tv_mul_lo_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k32(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mul_hi_u32 %0, %0, %8\n\tv_mul_hi_u32 %1, %1, %8\n\tv_mul_hi_u32 %2, %2, %8\n\tv_mul_hi_u32 %3, %3, %8\n\tv_mul_hi_u32 %4, %4, %8\n\tv_mul_hi_u32 %5, %5, %8\n\tv_mul_hi_u32 %6, %6, %8\n\tv_mul_hi_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k33(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mul_u32_u24 %0, %0, %8\n\tv_mul_u32_u24 %1, %1, %8\n\tv_mul_u32_u24 %2, %2, %8\n\tv_mul_u32_u24 %3, %3, %8\n\tv_mul_u32_u24 %4, %4, %8\n\tv_mul_u32_u24 %5, %5, %8\n\tv_mul_u32_u24 %6, %6, %8\n\tv_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k34(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mad_u32_u24 %0, %0, %8, %8\n\tv_mad_u32_u24 %1, %1, %8, %8\n\tv_mad_u32_u24 %2, %2, %8, %8\n\tv_mad_u32_u24 %3, %3, %8, %8\n\tv_mad_u32_u24 %4, %4, %8, %8\n\tv_mad_u32_u24 %5, %5, %8, %8\n\tv_mad_u32_u24 %6, %6, %8, %8\n\tv_mad_u32_u24 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k35(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_max_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %1, %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %2, %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %3, %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %4, %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %5, %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %6, %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %7, %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k36(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_add_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %1, %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %2, %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %3, %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %4, %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %5, %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %6, %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32_dpp %7, %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k37(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mov_b32_dpp %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_mov_b32_dpp %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k38(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_max_u32_dpp %0, %0, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %1, %1, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %2, %2, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %3, %3, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %4, %4, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %5, %5, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %6, %6, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_max_u32_dpp %7, %7, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k39(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_cmp_ne_u32 vcc, %0, %8\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc\n\tv_cmp_ne_u32 vcc, %1, %8\n\tv_addc_co_u32 %1, vcc, %1, %1, vcc\n\tv_cmp_ne_u32 vcc, %2, %8\n\tv_addc_co_u32 %2, vcc, %2, %2, vcc\n\tv_cmp_ne_u32 vcc, %3, %8\n\tv_addc_co_u32 %3, vcc, %3, %3, vcc\n\tv_cmp_ne_u32 vcc, %4, %8\n\tv_addc_co_u32 %4, vcc, %4, %4, vcc\n\tv_cmp_ne_u32 vcc, %5, %8\n\tv_addc_co_u32 %5, vcc, %5, %5, vcc\n\tv_cmp_ne_u32 vcc, %6, %8\n\tv_addc_co_u32 %6, vcc, %6, %6, vcc\n\tv_cmp_ne_u32 vcc, %7, %8\n\tv_addc_co_u32 %7, vcc, %7, %7, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k40(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_cmp_ne_u32 s[20:21], %0, %8\n\tv_cndmask_b32 %0, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %1, %8\n\tv_cndmask_b32 %1, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %2, %8\n\tv_cndmask_b32 %2, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %3, %8\n\tv_cndmask_b32 %3, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %4, %8\n\tv_cndmask_b32 %4, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %5, %8\n\tv_cndmask_b32 %5, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %6, %8\n\tv_cndmask_b32 %6, 0, %8, s[20:21]\n\tv_cmp_ne_u32 s[20:21], %7, %8\n\tv_cndmask_b32 %7, 0, %8, s[20:21]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k41(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_min_u32 %0, %0, %8\n\tv_add_u32 %0, %0, %8\n\tv_min_u32 %1, %1, %8\n\tv_add_u32 %1, %1, %8\n\tv_min_u32 %2, %2, %8\n\tv_add_u32 %2, %2, %8\n\tv_min_u32 %3, %3, %8\n\tv_add_u32 %3, %3, %8\n\tv_min_u32 %4, %4, %8\n\tv_add_u32 %4, %4, %8\n\tv_min_u32 %5, %5, %8\n\tv_add_u32 %5, %5, %8\n\tv_min_u32 %6, %6, %8\n\tv_add_u32 %6, %6, %8\n\tv_min_u32 %7, %7, %8\n\tv_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k42(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_sad_u32 %0, %0, %8, %8\n\tv_sad_u32 %1, %1, %8, %8\n\tv_sad_u32 %2, %2, %8, %8\n\tv_sad_u32 %3, %3, %8, %8\n\tv_sad_u32 %4, %4, %8, %8\n\tv_sad_u32 %5, %5, %8, %8\n\tv_sad_u32 %6, %6, %8, %8\n\tv_sad_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k43(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_med3_u32 %0, %0, %8, %8\n\tv_med3_u32 %1, %1, %8, %8\n\tv_med3_u32 %2, %2, %8, %8\n\tv_med3_u32 %3, %3, %8, %8\n\tv_med3_u32 %4, %4, %8, %8\n\tv_med3_u32 %5, %5, %8, %8\n\tv_med3_u32 %6, %6, %8, %8\n\tv_med3_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k44(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_pk_max_u16 %0, %0, %8\n\tv_pk_max_u16 %1, %1, %8\n\tv_pk_max_u16 %2, %2, %8\n\tv_pk_max_u16 %3, %3, %8\n\tv_pk_max_u16 %4, %4, %8\n\tv_pk_max_u16 %5, %5, %8\n\tv_pk_max_u16 %6, %6, %8\n\tv_pk_max_u16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k45(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_cvt_f32_u32 %0, %0\n\tv_cvt_f32_u32 %1, %1\n\tv_cvt_f32_u32 %2, %2\n\tv_cvt_f32_u32 %3, %3\n\tv_cvt_f32_u32 %4, %4\n\tv_cvt_f32_u32 %5, %5\n\tv_cvt_f32_u32 %6, %6\n\tv_cvt_f32_u32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(256) void k46(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_readlane_b32 s20, %0, 5\n\tv_readlane_b32 s20, %1, 5\n\tv_readlane_b32 s20, %2, 5\n\tv_readlane_b32 s20, %3, 5\n\tv_readlane_b32 s20, %4, 5\n\tv_readlane_b32 s20, %5, 5\n\tv_readlane_b32 s20, %6, 5\n\tv_readlane_b32 s20, %7, 5" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory", "s20", "s21", "vcc");
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
int main() {
    int ncu = 0, clk = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    unsigned *out; (void)hipMalloc(&out, (size_t)ncu * 8 * 256 * 4);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int W = 8, iters = 4096, blocks = ncu * W; float ms;
    printf("cycles per wave64 instruction per SIMD, %d waves per SIMD, %d MHz\n", W, clk / 1000);
    k0<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k0<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_add_u32 %0, %0, %8");
    k1<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k1<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_sub_u32 %0, %0, %8");
    k2<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k2<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_or_b32 %0, %0, %8");
    k3<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k3<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_and_b32 %0, %0, %8");
    k4<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k4<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_xor_b32 %0, %0, %8");
    k5<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k5<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_lshlrev_b32 %0, 3, %0");
    k6<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k6<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_lshrrev_b32 %0, 3, %0");
    k7<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k7<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_ashrrev_i32 %0, 3, %0");
    k8<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k8<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_min_u32 %0, %0, %8");
    k9<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k9<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_max_u32 %0, %0, %8");
    k10<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k10<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_max_i32 %0, %0, %8");
    k11<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k11<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_min_i32 %0, %0, %8");
    k12<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k12<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_not_b32 %0, %0");
    k13<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k13<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_mov_b32 %0, %8");
    k14<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k14<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_bfrev_b32 %0, %0");
    k15<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k15<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_ffbh_u32 %0, %0");
    k16<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k16<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_bcnt_u32_b32 %0, %0, %8");
    k17<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k17<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_bfe_u32 %0, %0, 3, 20");
    k18<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k18<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_bfe_i32 %0, %0, 3, 1");
    k19<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k19<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_bfi_b32 %0, %8, %0, %8");
    k20<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k20<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_alignbit_b32 %0, %0, %8, 5");
    k21<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k21<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_perm_b32 %0, %0, %8, %8");
    k22<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k22<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_lshl_or_b32 %0, %0, 2, %8");
    k23<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k23<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_and_or_b32 %0, %0, %8, %8");
    k24<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k24<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_or3_b32 %0, %0, %8, %8");
    k25<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k25<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_add3_u32 %0, %0, %8, %8");
    k26<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k26<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_lshl_add_u32 %0, %0, 2, %8");
    k27<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k27<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_min3_u32 %0, %0, %8, %8");
    k28<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k28<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_max3_u32 %0, %0, %8, %8");
    k29<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k29<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_bitop3_b32 %0, %0, %8, %8 bitop3:0x2a");
    k30<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k30<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_dot4_u32_u8 %0, %0, %8, %8");
    k31<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k31<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_mul_lo_u32 %0, %0, %8");
    k32<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k32<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_mul_hi_u32 %0, %0, %8");
    k33<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k33<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_mul_u32_u24 %0, %0, %8");
    k34<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k34<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_mad_u32_u24 %0, %0, %8, %8");
    k35<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k35<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_max_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
    k36<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k36<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_add_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
    k37<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k37<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_mov_b32_dpp %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
    k38<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k38<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_max_u32_dpp %0, %0, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
    k39<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k39<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 2), "v_cmp_ne_u32 vcc, %0, %8 ; v_addc_co_u32 %0, vcc, %0, %0, vcc");
    k40<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k40<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 2), "v_cmp_ne_u32 s[20:21], %0, %8 ; v_cndmask_b32 %0, 0, %8, s[20:21]");
    k41<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k41<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 2), "v_min_u32 %0, %0, %8 ; v_add_u32 %0, %0, %8");
    k42<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k42<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_sad_u32 %0, %0, %8, %8");
    k43<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k43<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_med3_u32 %0, %0, %8, %8");
    k44<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k44<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_pk_max_u16 %0, %0, %8");
    k45<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k45<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_cvt_f32_u32 %0, %0");
    k46<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k46<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * 1), "v_readlane_b32 s20, %0, 5");
    return 0;
}
