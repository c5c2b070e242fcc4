# generates op_survey.hip: one kernel per instruction form, 8 independent chains per wave,
# W = 8 waves per SIMD; prints cycles per wave64 instruction per SIMD at the device clock
ops = [
 ("v_add_u32 %0, %0, %8", "v"), ("v_sub_u32 %0, %0, %8", "v"), ("v_or_b32 %0, %0, %8", "v"),
 ("v_and_b32 %0, %0, %8", "v"), ("v_xor_b32 %0, %0, %8", "v"), ("v_lshlrev_b32 %0, 3, %0", ""),
 ("v_lshrrev_b32 %0, 3, %0", ""), ("v_ashrrev_i32 %0, 3, %0", ""), ("v_min_u32 %0, %0, %8", "v"),
 ("v_max_u32 %0, %0, %8", "v"), ("v_max_i32 %0, %0, %8", "v"), ("v_min_i32 %0, %0, %8", "v"),
 ("v_not_b32 %0, %0", ""), ("v_mov_b32 %0, %8", "v"), ("v_bfrev_b32 %0, %0", ""), ("v_ffbh_u32 %0, %0", ""),
 ("v_bcnt_u32_b32 %0, %0, %8", "v"), ("v_bfe_u32 %0, %0, 3, 20", ""), ("v_bfe_i32 %0, %0, 3, 1", ""),
 ("v_bfi_b32 %0, %8, %0, %8", "v"), ("v_alignbit_b32 %0, %0, %8, 5", "v"), ("v_perm_b32 %0, %0, %8, %8", "v"),
 ("v_lshl_or_b32 %0, %0, 2, %8", "v"), ("v_and_or_b32 %0, %0, %8, %8", "v"), ("v_or3_b32 %0, %0, %8, %8", "v"),
 ("v_add3_u32 %0, %0, %8, %8", "v"), ("v_lshl_add_u32 %0, %0, 2, %8", "v"), ("v_min3_u32 %0, %0, %8, %8", "v"),
 ("v_max3_u32 %0, %0, %8, %8", "v"), ("v_bitop3_b32 %0, %0, %8, %8 bitop3:0x2a", "v"),
 ("v_dot4_u32_u8 %0, %0, %8, %8", "v"), ("v_mul_lo_u32 %0, %0, %8", "v"), ("v_mul_hi_u32 %0, %0, %8", "v"),
 ("v_mul_u32_u24 %0, %0, %8", "v"), ("v_mad_u32_u24 %0, %0, %8, %8", "v"),
 ("v_max_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1", "v"),
 ("v_add_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1", "v"),
 ("v_mov_b32_dpp %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1", "v"),
 ("v_max_u32_dpp %0, %0, %8 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1", "v"),
 ("v_cmp_ne_u32 vcc, %0, %8\\n\\tv_addc_co_u32 %0, vcc, %0, %0, vcc", "v"),
 ("v_cmp_ne_u32 s[20:21], %0, %8\\n\\tv_cndmask_b32 %0, 0, %8, s[20:21]", "v"),
 ("v_min_u32 %0, %0, %8\\n\\tv_add_u32 %0, %0, %8", "v"),
 ("v_sad_u32 %0, %0, %8, %8", "v"), ("v_med3_u32 %0, %0, %8, %8", "v"), ("v_pk_max_u16 %0, %0, %8", "v"),
 ("v_cvt_f32_u32 %0, %0", ""), ("v_readlane_b32 s20, %0, 5", ""),
]
hdr = '''#include <hip/hip_runtime.h>
#include <cstdio>
'''
body = []
for i, (ins, _) in enumerate(ops):
    lines = []
    for c in range(8):
        lines.append(ins.replace("%0", f"%{c}"))
    asm = "\\n\\t".join(lines)
    clob = ', "s20", "s21", "vcc"'
    body.append(f'''__global__ __launch_bounds__(256) void k{i}(unsigned *out, int iters) {{
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned b = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i)
        asm volatile("{asm}" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "memory"{clob});
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}}''')
main = ['''int main() {
    int ncu = 0, clk = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    unsigned *out; (void)hipMalloc(&out, (size_t)ncu * 8 * 256 * 4);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int W = 8, iters = 4096, blocks = ncu * W; float ms;
    printf("cycles per wave64 instruction per SIMD, %d waves per SIMD, %d MHz\\n", W, clk / 1000);''']
for i, (ins, _) in enumerate(ops):
    n = ins.count("\\n") + 1
    name = ins.replace("\\n\\t", " ; ").replace('"', "'")
    main.append(f'''    k{i}<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e0); k{i}<<<blocks, 256>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%6.2f  %s\\n", ms * 1e-3 * clk * 1e3 / ((double)W * iters * 8 * {n}), "{name}");''')
main.append("    return 0;\n}")
open("op_survey.hip", "w").write(hdr + "\n".join(body) + "\n" + "\n".join(main) + "\n")
