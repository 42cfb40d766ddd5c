// MFMA issue vs dependent-accumulation latency on gfx950, one wave per SIMD (256 CUs x 4 waves):
// chains of v_mfma_f32_32x32x16_bf16 / v_mfma_f32_16x16x32_bf16 accumulating into 1, 2 or 4
// independent accumulators (C = previous D of the same accumulator).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_chain.hip -o build/mfma_chain && build/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int N = 2048;

template <int ACC>
__global__ __launch_bounds__(512, 1) void k32(float *out, int n)
{
    bf16x8 a, b;
    for (int j = 0; j < 8; j++) { a[j] = (short)(threadIdx.x + j); b[j] = (short)(threadIdx.x * 3 + j); }
    f32x16 c[ACC];
    for (int q = 0; q < ACC; q++) c[q] = f32x16{};
    for (int i = 0; i < n; i += ACC) {
#pragma unroll
        for (int q = 0; q < ACC; q++)
            c[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[q], 0, 0, 0);
    }
    float s = 0;
    for (int q = 0; q < ACC; q++) for (int r = 0; r < 16; r++) s += c[q][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ACC>
__global__ __launch_bounds__(256, 1) void k16(float *out, int n)
{
    bf16x8 a, b;
    for (int j = 0; j < 8; j++) { a[j] = (short)(threadIdx.x + j); b[j] = (short)(threadIdx.x * 3 + j); }
    f32x4 c[ACC];
    for (int q = 0; q < ACC; q++) c[q] = f32x4{};
    for (int i = 0; i < n; i += ACC) {
#pragma unroll
        for (int q = 0; q < ACC; q++)
            c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[q], 0, 0, 0);
    }
    float s = 0;
    for (int q = 0; q < ACC; q++) for (int r = 0; r < 4; r++) s += c[q][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA + VALU on one SIMD: ROLE 0 = every wave issues its MFMA chain with V independent VALU ops
// after each MFMA; ROLE 1 = waves 0-3 of the 512-thread block run the MFMA chain (4 accumulators),
// waves 4-7 (the second wave of each SIMD) only the V VALU ops per step; ROLE 2 = VALU only.
template <int V>
__device__ __forceinline__ void valu_ops(uint32_t (&x)[8], uint32_t y)
{
#pragma unroll
    for (int v = 0; v < V; v++)
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[v & 7]) : "v"(y));
}

template <int ROLE, int V>
__global__ __launch_bounds__(512, 1) void kmix(float *out, int n)
{
    bf16x8 a, b;
    for (int j = 0; j < 8; j++) { a[j] = (short)(threadIdx.x + j); b[j] = (short)(threadIdx.x * 3 + j); }
    f32x16 c[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
    uint32_t x[8];
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x * (j + 1);
    const uint32_t y = blockIdx.x | 1u;
    const bool valu_wave = (threadIdx.x >> 6) >= 4;
    for (int i = 0; i < n; i += 4) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (ROLE == 0 || (ROLE == 1 && !valu_wave))
                c[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[q], 0, 0, 0);
            if (ROLE == 0 || ROLE == 2 || (ROLE == 1 && valu_wave))
                valu_ops<V>(x, y);
        }
    }
    float s = 0;
    for (int q = 0; q < 4; q++) for (int r = 0; r < 16; r++) s += c[q][r];
    for (int j = 0; j < 8; j++) s += (float)x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char *name, K kern, float *out, int cus, int threads = 256)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), 0, 0, out, N);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    // per SIMD: threads/256 waves each issue N MFMAs
    printf("%-28s %.4f ms  %.1f cycles per MFMA per SIMD @2.4GHz (%d waves/SIMD)\n", name, best,
           best * 1e-3 * 2.4e9 / (N * (threads / 256)), threads / 256);
}

int main()
{
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    hipMalloc(&out, cus * 512 * 4);
    for (int w = 0; w < 20; w++) hipLaunchKernelGGL(k32<4>, dim3(cus), dim3(256), 0, 0, out, N);
    hipDeviceSynchronize();
    run("32x32x16 1 chain", k32<1>, out, cus);
    run("32x32x16 2 chains", k32<2>, out, cus);
    run("32x32x16 4 chains", k32<4>, out, cus);
    run("32x32x16 1 chain x2 waves", k32<1>, out, cus, 512);
    run("32x32x16 2 chains x2 waves", k32<2>, out, cus, 512);
    run("mix: 1 wave MFMA + 0 VALU", kmix<0, 0>, out, cus, 256);
    run("mix: 1 wave MFMA + 4 VALU", kmix<0, 4>, out, cus, 256);
    run("mix: 1 wave MFMA + 8 VALU", kmix<0, 8>, out, cus, 256);
    run("mix: 1 wave MFMA + 16 VALU", kmix<0, 16>, out, cus, 256);
    run("mix: 2 waves MFMA+4 VALU each", kmix<0, 4>, out, cus, 512);
    run("mix: 2 waves MFMA+8 VALU each", kmix<0, 8>, out, cus, 512);
    run("mix: MFMA wave | 8 VALU wave", kmix<1, 8>, out, cus, 512);
    run("mix: MFMA wave | 16 VALU wave", kmix<1, 16>, out, cus, 512);
    run("mix: MFMA wave | 32 VALU wave", kmix<1, 32>, out, cus, 512);
    run("mix: VALU only 8 (1 wave)", kmix<2, 8>, out, cus, 256);
    run("mix: VALU only 16 (1 wave)", kmix<2, 16>, out, cus, 256);
    run("mix: VALU only 16 (2 waves)", kmix<2, 16>, out, cus, 512);
    run("16x16x32 1 chain", k16<1>, out, cus);
    run("16x16x32 2 chains", k16<2>, out, cus);
    run("16x16x32 4 chains", k16<4>, out, cus);
    return 0;
}
