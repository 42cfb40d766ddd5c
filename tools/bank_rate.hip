// VALU issue cost vs VGPR bank of the source operands (gfx950): 8 independent chains of one
// instruction, sources pinned to registers in the same bank (reg % 4) as the accumulators or in
// different banks. Same grid as tools/instr_rate.hip (8 waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 tools/bank_rate.hip -o build/bank_rate && build/bank_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R8(X) X X X X X X X X
#define BODY(INSN)                                                                       \
    asm volatile("v_mov_b32 v64, %0\n v_mov_b32 v68, %0\n v_mov_b32 v72, %0\n v_mov_b32 v76, %0\n" \
                 "v_mov_b32 v80, %0\n v_mov_b32 v84, %0\n v_mov_b32 v88, %0\n v_mov_b32 v92, %0\n" \
                 "v_mov_b32 v100, %1\n v_mov_b32 v101, %1\n v_mov_b32 v102, %1\n v_mov_b32 v104, %1\n" \
                 "v_mov_b32 v108, %1\n"                                                    \
                 "s_mov_b32 s60, 2048\n"                                                    \
                 "1:\n" R8(INSN) "s_sub_u32 s60, s60, 1\n s_cmp_lg_u32 s60, 0\n s_cbranch_scc1 1b\n" \
                 "v_xor_b32 %0, v64, v68\n v_xor_b32 %0, %0, v72\n v_xor_b32 %0, %0, v76\n"   \
                 "v_xor_b32 %0, %0, v80\n v_xor_b32 %0, %0, v84\n v_xor_b32 %0, %0, v88\n v_xor_b32 %0, %0, v92\n" \
                 : "+v"(x) : "v"(k)                                                         \
                 : "s60", "scc", "v64", "v68", "v72", "v76", "v80", "v84", "v88", "v92", "v100", "v101", \
                   "v102", "v104", "v108", "memory");

#define CH8(OP, A, B) \
    OP " v64, v64, " A ", " B "\n" OP " v68, v68, " A ", " B "\n" OP " v72, v72, " A ", " B "\n" OP " v76, v76, " A ", " B "\n" \
    OP " v80, v80, " A ", " B "\n" OP " v84, v84, " A ", " B "\n" OP " v88, v88, " A ", " B "\n" OP " v92, v92, " A ", " B "\n"
#define CH8_2(OP, A) \
    OP " v64, v64, " A "\n" OP " v68, v68, " A "\n" OP " v72, v72, " A "\n" OP " v76, v76, " A "\n" \
    OP " v80, v80, " A "\n" OP " v84, v84, " A "\n" OP " v88, v88, " A "\n" OP " v92, v92, " A "\n"

#define K(NAME, INSN) \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t k) { uint32_t x = threadIdx.x; BODY(INSN) out[blockIdx.x * 256 + threadIdx.x] = x; }

K(k_bitop3_same, CH8("v_bitop3_b32", "v100", "v104 bitop3:0x96"))
K(k_bitop3_diff, CH8("v_bitop3_b32", "v101", "v102 bitop3:0x96"))
K(k_bitop3_same1, CH8("v_bitop3_b32", "v101", "v104 bitop3:0x96"))
K(k_add_same, CH8_2("v_add_u32", "v100"))
K(k_add_diff, CH8_2("v_add_u32", "v101"))
K(k_perm_same, CH8("v_perm_b32", "v100", "v104"))
K(k_perm_diff, CH8("v_perm_b32", "v101", "v102"))
#define CH8_L(OP, L) \
    OP " v64, " L ", v64\n" OP " v68, " L ", v68\n" OP " v72, " L ", v72\n" OP " v76, " L ", v76\n" \
    OP " v80, " L ", v80\n" OP " v84, " L ", v84\n" OP " v88, " L ", v88\n" OP " v92, " L ", v92\n"
K(k_sub_lit, CH8_L("v_sub_u32", "0x80808080"))
K(k_xor_same, CH8_2("v_xor_b32", "v100"))
K(k_xor_diff, CH8_2("v_xor_b32", "v101"))

typedef void (*kfn)(uint32_t *, uint32_t);
int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct { const char *name; kfn f; } ks[] = {
        {"add_same", k_add_same}, {"add_diff", k_add_diff}, {"xor_same", k_xor_same}, {"xor_diff", k_xor_diff},
        {"sub_lit", k_sub_lit}, {"bitop3_same", k_bitop3_same}, {"bitop3_same1", k_bitop3_same1},
        {"bitop3_diff", k_bitop3_diff}, {"perm_same", k_perm_same}, {"perm_diff", k_perm_diff}};
    for (int i = 0; i < 100; ++i)
        hipLaunchKernelGGL(ks[0].f, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B9u);
    hipDeviceSynchronize();
    for (auto &k : ks) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B9u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        // 8 waves x 2048 iterations x 8 instructions per SIMD; cycles at 2.4 GHz
        printf("%-14s %8.3f ms  %5.2f cyc/wave-instr/SIMD @2.4GHz\n", k.name, best, best * 1e-3 * 2.4e9 / (8.0 * 2048 * 8));
    }
    return 0;
}
