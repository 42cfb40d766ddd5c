// Bandwidth probe: the env step's I/O pattern (16-B board in, 16-B board out, two 1-B planes out
// per board) in place (read and write the same board array) vs ping-pong (read array A, write
// array B, swap every launch). No compute. Back-to-back eager launches, HIP events.
//   hipcc -O3 --offload-arch=gfx950 -o build/pingpong_bw tools/pingpong_bw.hip && build/pingpong_bw
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

// one board pair per lane, like k_step's fast path
__global__ __launch_bounds__(256) void step_io(const int8_t *src, int8_t *dst, int64_t n, uint32_t s, int8_t *act,
                                               uint8_t *done)
{
    const int64_t i = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
    if (i + 1 >= n)
        return;
    uint4 a = *reinterpret_cast<const uint4 *>(src + 16 * i);
    uint4 b = *reinterpret_cast<const uint4 *>(src + 16 * i + 16);
    a.x ^= s;
    b.x ^= s;
    *reinterpret_cast<uint4 *>(dst + 16 * i) = a;
    *reinterpret_cast<uint4 *>(dst + 16 * i + 16) = b;
    *reinterpret_cast<uint16_t *>(act + i) = (uint16_t)(a.y & 0x0303u);
    *reinterpret_cast<uint16_t *>(done + i) = (uint16_t)(b.z & 0x0101u);
}

int main()
{
    const int64_t sizes[] = {1 << 20, 1 << 22, 1 << 24, 1 << 26};
    for (int64_t n : sizes) {
        int8_t *A, *B, *act;
        uint8_t *done;
        CK(hipMalloc(&A, 16 * n));
        CK(hipMalloc(&B, 16 * n));
        CK(hipMalloc(&act, n));
        CK(hipMalloc(&done, n));
        CK(hipMemset(A, 1, 16 * n));
        CK(hipMemset(B, 1, 16 * n));
        const dim3 g((unsigned)((n / 2 + 255) / 256)), blk(256);
        const int reps = n <= (1 << 22) ? 2000 : 200;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int mode = 0; mode < 2; mode++) {
            for (int w = 0; w < reps / 4; w++) {
                const int8_t *src = (mode && (w & 1)) ? B : A;
                int8_t *dst = mode ? ((w & 1) ? A : B) : A;
                hipLaunchKernelGGL(step_io, g, blk, 0, 0, src, dst, n, (uint32_t)w, act, done);
            }
            CK(hipEventRecord(e0, 0));
            for (int w = 0; w < reps; w++) {
                const int8_t *src = (mode && (w & 1)) ? B : A;
                int8_t *dst = mode ? ((w & 1) ? A : B) : A;
                hipLaunchKernelGGL(step_io, g, blk, 0, 0, src, dst, n, (uint32_t)w, act, done);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = 1e3 * ms / reps;
            printf("n=%9lld %-9s %9.3f us/launch  %7.0f GB/s (34 B/board)\n", (long long)n,
                   mode ? "pingpong" : "in-place", us, 34.0 * n / us / 1e3);
        }
        CK(hipFree(A));
        CK(hipFree(B));
        CK(hipFree(act));
        CK(hipFree(done));
    }
    return 0;
}
