// Issue cost of the packed 16-bit, f16 and lane-swap VALU forms the CNN epilogues could use (gfx950):
// ReLU on packed bf16 (v_pk_max_i16 today), the ReLU' mask (v_pk_min_u16 + v_pk_mul_lo_u16 today),
// their f16-typed packed counterparts, v_cvt_pk_bf16_f32 and the permlane swaps. Each kernel runs
// ITERS x 8 independent chains of one instruction per lane, at 8 waves per SIMD (grid = CUs x 8
// workgroups of 256) and at 1 wave per SIMD (CUs x 1), and prints cycles per wave-instruction per
// SIMD at the clock it ran at (s_memtime / s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 tools/instr_rate16.hip -o build/instr_rate16 && build/instr_rate16
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int ITERS = 4096;

#define CHAINS(OP)                                                                              \
    uint32_t a0 = threadIdx.x * 0x10001u, a1 = a0 ^ 0x00010001u, a2 = a0 ^ 0x00020002u;         \
    uint32_t a3 = a0 ^ 0x00030003u, a4 = a0 ^ 0x00040004u, a5 = a0 ^ 0x00050005u;             \
    uint32_t a6 = a0 ^ 0x00060006u, a7 = a0 ^ 0x00070007u;                                     \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();     \
    for (int it = 0; it < ITERS; ++it) {                                                        \
        OP(a0); OP(a1); OP(a2); OP(a3); OP(a4); OP(a5); OP(a6); OP(a7);                          \
    }                                                                                           \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();     \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;          \
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }

#define OP2(NAME, TXT) \
    __device__ __forceinline__ void NAME(uint32_t &x, uint32_t k) { asm volatile(TXT : "+v"(x) : "v"(k)); }

OP2(o_add, "v_add_u32 %0, %0, %1")
OP2(o_pk_max_i16, "v_pk_max_i16 %0, %0, %1")
OP2(o_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
OP2(o_pk_mul_lo_u16, "v_pk_mul_lo_u16 %0, %0, %1")
OP2(o_pk_max_f16, "v_pk_max_f16 %0, %0, %1")
OP2(o_pk_min_f16, "v_pk_min_f16 %0, %0, %1")
OP2(o_pk_mul_f16, "v_pk_mul_f16 %0, %0, %1")
OP2(o_pk_add_f16, "v_pk_add_f16 %0, %0, %1")
OP2(o_pk_fma_f16, "v_pk_fma_f16 %0, %0, %1, %0")
OP2(o_max_f32, "v_max_f32 %0, %0, %1")
OP2(o_max_i16, "v_max_i16 %0, %0, %1")
OP2(o_cvt_pk_bf16, "v_cvt_pk_bf16_f32 %0, %0, %1")
OP2(o_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x40")
OP2(o_and, "v_and_b32 %0, %0, %1")
OP2(o_permlane16_swap, "v_permlane16_swap_b32 %0, %1")
OP2(o_permlane32_swap, "v_permlane32_swap_b32 %0, %1")

#define KERNEL(NAME)                                                                                \
    __global__ __launch_bounds__(256) void k##NAME(uint32_t *out, uint64_t *clk, uint32_t k)         \
    {                                                                                              \
        auto OPF = [&](uint32_t &x) { NAME(x, k); };                                               \
        CHAINS(OPF)                                                                                \
    }

#define LIST(X) X(o_add) X(o_pk_max_i16) X(o_pk_min_u16) X(o_pk_mul_lo_u16) X(o_pk_max_f16) X(o_pk_min_f16) \
    X(o_pk_mul_f16) X(o_pk_add_f16) X(o_pk_fma_f16) X(o_max_f32) X(o_max_i16) X(o_cvt_pk_bf16) X(o_bitop3) X(o_and) \
    X(o_permlane16_swap) X(o_permlane32_swap)
LIST(KERNEL)

typedef void (*kfn)(uint32_t *, uint64_t *, uint32_t);

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    uint64_t *clk, hclk[2];
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
#define ENT(N) {#N, k##N},
    struct { const char *name; kfn f; } ks[] = {LIST(ENT)};
    for (int i = 0; i < 300; ++i)
        hipLaunchKernelGGL(ks[0].f, dim3(cus * 8), dim3(256), 0, 0, out, clk, 0x3C003C00u);
    hipDeviceSynchronize();
    for (int waves : {8, 1}) {
        const int blocks = cus * waves;   // 256-thread workgroups: one wave per SIMD each
        for (auto &k : ks) {
            float best = 1e30f;
            double ghz = 0;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(a);
                hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 0x3C003C00u);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
                if (ms < best) {
                    best = ms;
                    ghz = (double)hclk[0] / ((double)hclk[1] * 10.0);
                }
            }
            const double cyc = best * 1e-3 * ghz * 1e9 / ((double)waves * ITERS * 8);
            printf("waves/SIMD %d  %-20s %8.3f ms  %5.2f cyc/wave-instr/SIMD  (clock %.2f GHz)\n", waves, k.name + 2,
                   best, cyc, ghz);
        }
    }
    hipFree(out);
    return 0;
}
