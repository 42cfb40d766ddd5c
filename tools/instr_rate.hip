// Relative VALU issue cost of the instructions the env step is made of (gfx950).
// Each kernel runs ITERS x 8 independent chains of one instruction kind per lane over a grid
// that fills every SIMD; the time ratio to the v_add_u32 kernel is its cost in add-slots.
//   hipcc -O3 --offload-arch=gfx950 tools/instr_rate.hip -o build/instr_rate && build/instr_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

#define CHAINS(OP)                                                     \
    uint32_t a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3;   \
    uint32_t a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;       \
    for (int it = 0; it < ITERS; ++it) {                               \
        OP(a0); OP(a1); OP(a2); OP(a3); OP(a4); OP(a5); OP(a6); OP(a7); \
    }                                                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;

#define ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k))
#define XOR3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(k), "v"(k2))
#define PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(k2))
#define MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(k))
#define MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(k))
#define MULU24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(k))
#define BCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(k))
#define CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(k))
#define CMPCND(x)                                                                              \
    asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(x) : "v"(k) : "vcc")
#define CND64(x)                                                                               \
    do {                                                                                       \
        uint64_t m;                                                                            \
        asm volatile("v_cmp_gt_u32 %0, %1, %2" : "=s"(m) : "v"(x), "v"(k));                   \
        asm volatile("v_cndmask_b32 %0, %0, %1, %2\n\tv_cndmask_b32 %0, %0, %1, %2\n\tv_cndmask_b32 %0, %0, %1, %2"   \
                     : "+v"(x) : "v"(k2), "s"(m));                                              \
    } while (0)
#define LSHL(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x))
#define ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(k2))
#define BFE(x) asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(x))
#define ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(k2))
#define MOV(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(k2))
#define MAD64(x)                                                                               \
    do {                                                                                       \
        uint64_t r;                                                                            \
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "v"(k) : "vcc"); \
        x = (uint32_t)(r >> 32) ^ (uint32_t)r;                                                 \
    } while (0)
#define MAD64ONLY(x)                                                                           \
    do {                                                                                       \
        uint64_t r;                                                                            \
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "v"(k) : "vcc"); \
        x = (uint32_t)r;                                                                       \
    } while (0)

#define KERNEL(NAME, OP)                                                        \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t k, uint32_t k2) \
    {                                                                           \
        CHAINS(OP)                                                              \
    }

KERNEL(k_add, ADD)
KERNEL(k_xor3, XOR3)
KERNEL(k_perm, PERM)
KERNEL(k_mullo, MULLO)
KERNEL(k_mulhi, MULHI)
KERNEL(k_mulu24, MULU24)
KERNEL(k_bcnt, BCNT)
KERNEL(k_cnd, CND)
KERNEL(k_mad64, MAD64)
KERNEL(k_cmpcnd, CMPCND)
KERNEL(k_cnd64, CND64)
KERNEL(k_lshl, LSHL)
KERNEL(k_andor, ANDOR)
KERNEL(k_bfe, BFE)
KERNEL(k_add3, ADD3)
KERNEL(k_mad64only, MAD64ONLY)

typedef void (*kfn)(uint32_t *, uint32_t, uint32_t);

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 blocks x 4 waves per CU = 8 waves per SIMD
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct { const char *name; kfn f; int extra; } ks[] = {
        {"v_add_u32", k_add, 0},     {"v_bitop3_b32 (xor3)", k_xor3, 0}, {"v_perm_b32", k_perm, 0},
        {"v_mul_lo_u32", k_mullo, 0}, {"v_mul_hi_u32", k_mulhi, 0}, {"v_mul_u32_u24", k_mulu24, 0},
        {"v_bcnt_u32_b32", k_bcnt, 0}, {"v_cndmask_b32", k_cnd, 0},
        {"v_mad_u64_u32 (+1 xor)", k_mad64, 1}, {"v_mad_u64_u32 (lo only)", k_mad64only, 0},
        {"v_cmp(vcc)+v_cndmask pair", k_cmpcnd, 0}, {"v_cmp(sgpr) + 3 v_cndmask", k_cnd64, 0},
        {"v_lshlrev_b32", k_lshl, 0}, {"v_and_or_b32", k_andor, 0}, {"v_bfe_u32", k_bfe, 0},
        {"v_add3_u32", k_add3, 0},
    };
    float base = 0;
    for (auto &k : ks) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B9u, 0x05040302u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best)
                best = ms;
        }
        if (base == 0)
            base = best;
        const double winstr = (double)blocks * 4 * ITERS * 8;  // wave-instructions of the op
        printf("%-26s %8.3f ms  %6.2f x v_add   %7.2f G wave-instr/s per CU\n", k.name, best, best / base,
               winstr / (best * 1e-3) / cus / 1e9);
    }
    hipFree(out);
    return 0;
}
