// VALU issue cost of the instructions the env step is made of (gfx950).
// Each kernel runs ITERS x 8 independent chains of one instruction kind per lane over a grid
// that fills every SIMD with 8 waves; the time ratio to the v_add_u32 kernel is its cost in
// add-slots, and the absolute rate is printed as cycles per wave-instruction per SIMD at the
// clock the kernel ran at (s_memtime / s_memrealtime stamps, 100 MHz reference).
//   hipcc -O3 --offload-arch=gfx950 tools/instr_rate.hip -o build/instr_rate && build/instr_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

constexpr int ITERS = 4096;

#define CHAINS(OP)                                                          \
    uint32_t a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;        \
    uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;            \
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(a0), "v"(k) : "vcc");    \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    for (int it = 0; it < ITERS; ++it) {                                    \
        OP(a0); OP(a1); OP(a2); OP(a3); OP(a4); OP(a5); OP(a6); OP(a7);      \
    }                                                                       \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }

#define OP2(NAME, TXT) \
    __device__ __forceinline__ void NAME(uint32_t &x, uint32_t k, uint32_t k2) { asm volatile(TXT : "+v"(x) : "v"(k), "v"(k2) : "vcc"); }

OP2(o_add, "v_add_u32 %0, %0, %1")
OP2(o_sub, "v_sub_u32 %0, %0, %1")
OP2(o_and, "v_and_b32 %0, %0, %1")
OP2(o_or, "v_or_b32 %0, %0, %1")
OP2(o_xor, "v_xor_b32 %0, %0, %1")
OP2(o_not, "v_not_b32 %0, %0")
OP2(o_xor3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
OP2(o_bfi, "v_bfi_b32 %0, %0, %1, %2")
OP2(o_perm, "v_perm_b32 %0, %0, %1, %2")
OP2(o_mulhi, "v_mul_hi_u32 %0, %0, %1")
OP2(o_mulu24, "v_mul_u32_u24 %0, %0, %1")
OP2(o_bcnt, "v_bcnt_u32_b32 %0, %0, %1")
OP2(o_cnd, "v_cndmask_b32 %0, %0, %1, vcc")
OP2(o_cmp_cnd, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %0, vcc")
OP2(o_lshl, "v_lshlrev_b32 %0, 3, %0")
OP2(o_lshr, "v_lshrrev_b32 %0, 3, %0")
OP2(o_lshlv, "v_lshlrev_b32 %0, %1, %0")
OP2(o_ashr, "v_ashrrev_i32 %0, 31, %0")
OP2(o_lshl_or, "v_lshl_or_b32 %0, %0, 8, %1")
OP2(o_lshl_add, "v_lshl_add_u32 %0, %0, 8, %1")
OP2(o_and_or, "v_and_or_b32 %0, %0, %1, %2")
OP2(o_or3, "v_or3_b32 %0, %0, %1, %2")
OP2(o_add3, "v_add3_u32 %0, %0, %1, %2")
OP2(o_alignbit, "v_alignbit_b32 %0, %0, %1, 8")
OP2(o_bfe, "v_bfe_u32 %0, %0, 3, 5")
OP2(o_min, "v_min_u32 %0, %0, %1")
OP2(o_max3, "v_max3_u32 %0, %0, %1, %2")
OP2(o_sad, "v_sad_u8 %0, %0, %1, %2")
OP2(o_msad, "v_msad_u8 %0, %0, %1, %2")
OP2(o_pkadd, "v_pk_add_u16 %0, %0, %1")
OP2(o_pkmax, "v_pk_max_u16 %0, %0, %1")
OP2(o_dot4, "v_dot4_u32_u8 %0, %0, %1, %2")
OP2(o_mov, "v_mov_b32 %0, %1")
OP2(o_cmp_vcc, "v_cmp_ne_u32 vcc, %0, %1\n\tv_add_u32 %0, %0, %1")
OP2(o_addco, "v_add_co_u32 %0, vcc, %0, %1")
OP2(o_sdwa_add, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD")
__device__ __forceinline__ void o_cnd64(uint32_t &x, uint32_t k, uint32_t k2)
{
    const uint64_t m = 0x5555555555555555ull ^ k2;
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(k), "s"(m));
}
__device__ __forceinline__ void o_cmp64_cnd64(uint32_t &x, uint32_t k, uint32_t)
{
    uint64_t m;
    asm volatile("v_cmp_gt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(x), "=&s"(m) : "v"(k));
}
OP2(o_sub_lit, "v_sub_u32 %0, 0x80808080, %0")
OP2(o_xad, "v_xad_u32 %0, %0, %1, %2")
OP2(o_add_lshl, "v_add_lshl_u32 %0, %0, %1, 3")
OP2(o_med3, "v_med3_u32 %0, %0, %1, %2")
OP2(o_subrev, "v_subrev_u32 %0, %0, %1")
__device__ __forceinline__ void o_sub_sgpr(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_sub_u32 %0, %1, %0" : "+v"(x) : "s"(__builtin_amdgcn_readfirstlane(k2)));
}
__device__ __forceinline__ void o_bitop3_vvs_s(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xc8" : "+v"(x) : "v"(k), "s"(__builtin_amdgcn_readfirstlane(k2)));
}
__device__ __forceinline__ void o_add_e64_s(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_add_u32_e64 %0, %1, %0" : "+v"(x) : "s"(__builtin_amdgcn_readfirstlane(k2)));
}
__device__ __forceinline__ void o_mad64_s(uint32_t &x, uint32_t k, uint32_t k2)
{
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "s"(__builtin_amdgcn_readfirstlane(k2)) : "vcc");
    x = (uint32_t)(r >> 32);
}
__device__ __forceinline__ void o_xor_inl(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_xor_b32 %0, 64, %0" : "+v"(x));
}
__device__ __forceinline__ void o_mix_sv(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_sub_u32 %0, %1, %0\n\tv_add_u32 %0, %0, %2" : "+v"(x) : "s"(__builtin_amdgcn_readfirstlane(k2)), "v"(k));
}
__device__ __forceinline__ void o_mix_vv(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_sub_u32 %0, %1, %0\n\tv_add_u32 %0, %0, %2" : "+v"(x) : "v"(k2), "v"(k));
}
__device__ __forceinline__ void o_and_sgpr(uint32_t &x, uint32_t k, uint32_t k2)
{
    asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "s"(__builtin_amdgcn_readfirstlane(k2)));
}
OP2(o_and_lit, "v_and_b32 %0, 0x80808080, %0")
OP2(o_bitop3_vvs, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xc8")
__device__ __forceinline__ void o_nop_add(uint32_t &x, uint32_t k, uint32_t)
{
    asm volatile("s_nop 0\n\tv_add_u32 %0, %0, %1" : "+v"(x) : "v"(k));
}
__device__ __forceinline__ void o_mad64(uint32_t &x, uint32_t k, uint32_t)
{
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "v"(k) : "vcc");
    x = (uint32_t)(r >> 32);
}

#define KERNEL(NAME, OP)                                                                    \
    __global__ __launch_bounds__(256) void k##NAME(uint32_t *out, uint64_t *clk, uint32_t k, uint32_t k2) \
    {                                                                                       \
        auto OPF = [&](uint32_t &x) { OP(x, k, k2); };                                       \
        CHAINS(OPF)                                                                         \
    }

#define LIST(X) X(o_add) X(o_sub) X(o_and) X(o_or) X(o_xor) X(o_not) X(o_xor3) X(o_bfi) X(o_perm) X(o_mulhi) \
    X(o_mulu24) X(o_bcnt) X(o_cnd) X(o_cmp_cnd) X(o_lshl) X(o_lshr) X(o_lshlv) X(o_ashr) X(o_lshl_or)         \
    X(o_lshl_add) X(o_and_or) X(o_or3) X(o_add3) X(o_alignbit) X(o_bfe) X(o_min) X(o_max3) X(o_sad) X(o_msad)  \
    X(o_pkadd) X(o_pkmax) X(o_dot4) X(o_mov) X(o_cmp_vcc) X(o_addco) X(o_sdwa_add) X(o_mad64) X(o_cnd64) X(o_cmp64_cnd64) \
    X(o_sub_lit) X(o_and_lit) X(o_bitop3_vvs) X(o_nop_add) X(o_xad) X(o_add_lshl) X(o_med3) X(o_subrev) X(o_sub_sgpr) X(o_and_sgpr) X(o_bitop3_vvs_s) X(o_add_e64_s) X(o_mad64_s) X(o_xor_inl) X(o_mix_sv) X(o_mix_vv)
#define DEF(N) KERNEL(N, N)
LIST(DEF)

typedef void (*kfn)(uint32_t *, uint64_t *, uint32_t, uint32_t);

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 blocks x 4 waves per CU = 8 waves per SIMD
    uint32_t *out;
    uint64_t *clk, hclk[2];
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
#define ENT(N) {#N, k##N},
    struct { const char *name; kfn f; } ks[] = {LIST(ENT)};
    // warm the clocks
    for (int i = 0; i < 200; ++i)
        hipLaunchKernelGGL(ks[0].f, dim3(blocks), dim3(256), 0, 0, out, clk, 0x9E3779B9u, 0x05040302u);
    hipDeviceSynchronize();
    float base = 0;
    for (auto &k : ks) {
        float best = 1e30f;
        double ghz = 0;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 0x9E3779B9u, 0x05040302u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
            if (ms < best) {
                best = ms;
                ghz = (double)hclk[0] / ((double)hclk[1] * 10.0);   // memrealtime ticks at 100 MHz
            }
        }
        if (base == 0)
            base = best;
        // cycles per wave-instruction per SIMD: 8 waves x ITERS x 8 ops share one SIMD
        const double cyc = best * 1e-3 * ghz * 1e9 / (8.0 * ITERS * 8);
        printf("%-12s %8.3f ms  %5.2f x v_add  %5.2f cyc/wave-instr/SIMD  (clock %.2f GHz)\n", k.name + 2, best,
               best / base, cyc, ghz);
    }
    hipFree(out);
    return 0;
}
