// VALU issue microbenchmark (measurement only): cycles per wave64 VALU instruction per SIMD for
// several instruction forms, with W waves per SIMD (grid of 256 CUs x 4 SIMDs x W waves).  Each
// wave runs 8 independent chains of the instruction in a loop; the kernel time and the instruction
// count give cycles per instruction per SIMD at the given clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHAINS8(INS)                                   \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
                 INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"    \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(b))
#define CHAINS8_DPP(INS, SUF)                          \
    asm volatile(INS " %0, %0, %8 " SUF "\n\t" INS " %1, %1, %8 " SUF "\n\t" INS " %2, %2, %8 " SUF "\n\t" INS " %3, %3, %8 " SUF "\n\t" \
                 INS " %4, %4, %8 " SUF "\n\t" INS " %5, %5, %8 " SUF "\n\t" INS " %6, %6, %8 " SUF "\n\t" INS " %7, %7, %8 " SUF    \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(b))
#define CHAINS8_3(INS)                                 \
    asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t" INS " %3, %3, %8, %8\n\t" \
                 INS " %4, %4, %8, %8\n\t" INS " %5, %5, %8, %8\n\t" INS " %6, %6, %8, %8\n\t" INS " %7, %7, %8, %8"    \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(b))

template <int OP>
__global__ __launch_bounds__(256) void k_issue(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    unsigned long long q0 = a0, q1 = a1, q2 = a2, q3 = a3;
    for (int i = 0; i < iters; ++i) {
        if constexpr (OP == 0) CHAINS8("v_add_u32");
        if constexpr (OP == 1) CHAINS8("v_xor_b32");
        if constexpr (OP == 2) CHAINS8_3("v_add3_u32");
        if constexpr (OP == 3) CHAINS8_3("v_bfe_u32");
        if constexpr (OP == 4) CHAINS8_3("v_min3_u32");
        if constexpr (OP == 5) CHAINS8_3("v_alignbit_b32");
        if constexpr (OP == 6) CHAINS8_DPP("v_max_u32_dpp", "row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
        if constexpr (OP == 7) CHAINS8_3("v_bitop3_b32");
        if constexpr (OP == 8) CHAINS8("v_mul_lo_u32");
        if constexpr (OP == 9) CHAINS8("v_add_f32");
        if constexpr (OP == 10) CHAINS8_3("v_fma_f32");
        if constexpr (OP == 11) CHAINS8("v_pk_add_u16");
        if constexpr (OP == 12) CHAINS8("v_add_u32_e64");
        if constexpr (OP == 13) asm volatile("v_and_b32 %0, 0x55aa55aa, %0\n\tv_and_b32 %1, 0x55aa55aa, %1\n\tv_and_b32 %2, 0x55aa55aa, %2\n\tv_and_b32 %3, 0x55aa55aa, %3\n\tv_and_b32 %4, 0x55aa55aa, %4\n\tv_and_b32 %5, 0x55aa55aa, %5\n\tv_and_b32 %6, 0x55aa55aa, %6\n\tv_and_b32 %7, 0x55aa55aa, %7"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));

        if constexpr (OP == 15) asm volatile("v_lshlrev_b64 %0, 1, %0\n\tv_lshlrev_b64 %1, 1, %1\n\tv_lshlrev_b64 %2, 1, %2\n\tv_lshlrev_b64 %3, 1, %3"
                 : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3));
        if constexpr (OP == 17) { asm volatile("v_bfe_u32 %0, %0, 12, 20\n\tv_bfe_u32 %1, %1, 12, 20\n\tv_bfe_u32 %2, %2, 12, 20\n\tv_bfe_u32 %3, %3, 12, 20\n\tv_bfe_u32 %4, %4, 12, 20\n\tv_bfe_u32 %5, %5, 12, 20\n\tv_bfe_u32 %6, %6, 12, 20\n\tv_bfe_u32 %7, %7, 12, 20" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)); }
        if constexpr (OP == 18) { asm volatile("v_min3_u32 %0, %0, %8, 7\n\tv_min3_u32 %1, %1, %8, 7\n\tv_min3_u32 %2, %2, %8, 7\n\tv_min3_u32 %3, %3, %8, 7\n\tv_min3_u32 %4, %4, %8, 7\n\tv_min3_u32 %5, %5, %8, 7\n\tv_min3_u32 %6, %6, %8, 7\n\tv_min3_u32 %7, %7, %8, 7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(b)); }
        if constexpr (OP == 19) { asm volatile("v_min3_u32 %0, %0, %8, %9\n\tv_min3_u32 %1, %1, %8, %9\n\tv_min3_u32 %2, %2, %8, %9\n\tv_min3_u32 %3, %3, %8, %9\n\tv_min3_u32 %4, %4, %8, %9\n\tv_min3_u32 %5, %5, %8, %9\n\tv_min3_u32 %6, %6, %8, %9\n\tv_min3_u32 %7, %7, %8, %9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(b + 3)); }
        if constexpr (OP == 20) { asm volatile("v_max_u32 %0, %0, %8\n\tv_max_u32 %1, %1, %8\n\tv_max_u32 %2, %2, %8\n\tv_max_u32 %3, %3, %8\n\tv_max_u32 %4, %4, %8\n\tv_max_u32 %5, %5, %8\n\tv_max_u32 %6, %6, %8\n\tv_max_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); }
        if constexpr (OP == 21) { asm volatile("v_lshrrev_b32 %0, 12, %0\n\tv_lshrrev_b32 %1, 12, %1\n\tv_lshrrev_b32 %2, 12, %2\n\tv_lshrrev_b32 %3, 12, %3\n\tv_lshrrev_b32 %4, 12, %4\n\tv_lshrrev_b32 %5, 12, %5\n\tv_lshrrev_b32 %6, 12, %6\n\tv_lshrrev_b32 %7, 12, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)); }
        if constexpr (OP == 22) { asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n\tv_cndmask_b32 %1, %1, %8, vcc\n\tv_cndmask_b32 %2, %2, %8, vcc\n\tv_cndmask_b32 %3, %3, %8, vcc\n\tv_cndmask_b32 %4, %4, %8, vcc\n\tv_cndmask_b32 %5, %5, %8, vcc\n\tv_cndmask_b32 %6, %6, %8, vcc\n\tv_cndmask_b32 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc"); }
        if constexpr (OP == 23) { asm volatile("v_bitop3_b32 %0, %0, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %1, %1, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %2, %2, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %3, %3, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %4, %4, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %5, %5, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %6, %6, %8, 7 bitop3:0x2a\n\tv_bitop3_b32 %7, %7, %8, 7 bitop3:0x2a" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(b)); }
        if constexpr (OP == 16) { CHAINS8("v_add_u32"); CHAINS8_3("v_bfe_u32"); }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)(q0 ^ q1 ^ q2 ^ q3);
}

static const char *names[] = {"v_add_u32", "v_xor_b32", "v_add3_u32", "v_bfe_u32", "v_min3_u32", "v_alignbit_b32",
                              "v_max_u32_dpp", "v_bitop3_b32", "v_mul_lo_u32", "v_add_f32", "v_fma_f32", "v_pk_add_u16", "v_add_u32_e64", "v_and literal", "-", "v_lshlrev_b64 (x4)", "add+bfe (x16)", "bfe v,12,20", "min3 v,s,7", "min3 v,v,v(3 regs)", "v_max_u32 v,v", "lshr 12,v", "cndmask vcc", "bitop3 v,s,7"};

template <int OP>
static float run(unsigned *out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_issue<OP><<<blocks, 256>>>(out, iters);  // warm-up
    hipEventRecord(e0);
    k_issue<OP><<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    int dev = 0, ncu = 0, clk = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
    unsigned *out;
    hipMalloc(&out, (size_t)ncu * 4 * 8 * 256 * 4);
    const int iters = 4096;
    printf("CUs %d, clock %.0f MHz; cycles per wave64 instruction per SIMD (8 chains per wave)\n", ncu, clk / 1e3);
    for (int w : {4, 8}) {
        const int blocks = ncu * w;  // 256 threads = 4 waves, one per SIMD
        auto rep = [&](const char *nm, float ms) {
            const double ins_per_simd = (double)w * iters * 8;
            printf("W=%d %-16s %7.3f ms  %.2f cyc/ins/SIMD\n", w, nm, ms, ms * 1e-3 * clk * 1e3 / ins_per_simd);
        };
        rep(names[0], run<0>(out, blocks, iters));
        rep(names[1], run<1>(out, blocks, iters));
        rep(names[2], run<2>(out, blocks, iters));
        rep(names[3], run<3>(out, blocks, iters));
        rep(names[4], run<4>(out, blocks, iters));
        rep(names[5], run<5>(out, blocks, iters));
        rep(names[6], run<6>(out, blocks, iters));
        rep(names[7], run<7>(out, blocks, iters));
        rep(names[8], run<8>(out, blocks, iters));
        rep(names[9], run<9>(out, blocks, iters));
        rep(names[10], run<10>(out, blocks, iters));
        rep(names[11], run<11>(out, blocks, iters));
        rep(names[12], run<12>(out, blocks, iters));
        rep(names[13], run<13>(out, blocks, iters));
        rep(names[15], run<15>(out, blocks, iters) * 2.0f);  // 4 instructions per iteration: scaled to 8
        rep(names[16], run<16>(out, blocks, iters) * 0.5f);   // 16 per iteration: scaled to 8
        rep(names[17], run<17>(out, blocks, iters));
        rep(names[18], run<18>(out, blocks, iters));
        rep(names[19], run<19>(out, blocks, iters));
        rep(names[20], run<20>(out, blocks, iters));
        rep(names[21], run<21>(out, blocks, iters));
        rep(names[22], run<22>(out, blocks, iters));
        rep(names[23], run<23>(out, blocks, iters));
    }
    hipFree(out);
    return 0;
}
