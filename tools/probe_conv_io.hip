// Probe: the config-5 conv's memory pattern (r48_conv.hip k_conv3x3) without its MFMAs, to tell
// whether its ~4-4.5 TB/s comes from the access pattern. 256 workgroups x 8 waves (two per SIMD, as
// the conv), a wave per 16-board tile, the tile's 4 input rows in a 4-row register ring refilled one
// row ahead, a dependent VALU chain per output row standing in for its MFMAs, 1-KiB stores per
// instruction (the conv's LDS-staged stores), and optionally a second input stream read in the
// store layout after each row (the SM = 2 epilogue's BN input; EPI = 1), or in the residual add's
// layout (EPI = 2: 8 B per lane per output column and 16-channel pass, the conv's `ad` loads, 16
// boards x 32 B per instruction). Load layouts:
//   H  the conv's: lane (board n = l & 15, g = l >> 4) loads 16 B at board n, cell, channels
//      32 c + 8 g -- every instruction touches 16 half lines (64 B) 2 KiB apart
//   F  the same bytes re-laid so that one instruction reads 1 KiB contiguous (a tiled layout)
// Bytes and instruction counts are the same for H and F. With an argument (any) only the chain-0
// pass runs: the calibration of FETCH_SIZE / WRITE_SIZE for these patterns under rocprofv3 --pmc
// (every dispatch moves a known 134,217,728 bytes per stream).
//   hipcc -O3 --offload-arch=gfx950 -o build/probe_conv_io tools/probe_conv_io.hip && build/probe_conv_io
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

constexpr int kWaves = 8;

template <bool FULL, int EPI>
__global__ __launch_bounds__(64 * kWaves, 1) void conv_io(const uint4 *__restrict__ x, const uint4 *__restrict__ e,
                                                          uint4 *__restrict__ y, int64_t n_tiles, int chain)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n = lane & 15, g = lane >> 4;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t tile = (int64_t)blockIdx.x * kWaves + wave;
    uint4 xr[4][4][2];
    // 16-B unit index of (tile, row R, col, c) for this lane
    auto at = [&](int64_t t, int R, int col, int c) -> int64_t {
        if (FULL)
            return ((t * 16 + 4 * R + col) * 2 + c) * 64 + lane;                  // 1 KiB per (cell, c)
        return ((t * 16 + n) * 16 + 4 * R + col) * 8 + 4 * c + g;               // board n, cell, chunk
    };
    auto load_row = [&](int64_t t, int R) {
#pragma unroll
        for (int col = 0; col < 4; col++)
#pragma unroll
            for (int c = 0; c < 2; c++)
                xr[R][col][c] = x[at(t, R, col, c)];
    };
    float acc = (float)lane;
    if (tile < n_tiles) {
        load_row(tile, 0);
        load_row(tile, 1);
    }
    for (; tile < n_tiles; tile += stride) {
        const int64_t next = tile + stride;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            load_row(r < 2 ? tile : (next < n_tiles ? next : tile), r < 2 ? r + 2 : r - 2);
            __builtin_amdgcn_sched_barrier(0);
            uint32_t h = 0;
#pragma unroll
            for (int dr = -1; dr <= 1; dr++) {
                if (r + dr < 0 || r + dr > 3)
                    continue;
#pragma unroll
                for (int col = 0; col < 4; col++)
#pragma unroll
                    for (int c = 0; c < 2; c++)
                        h ^= xr[r + dr][col][c].x ^ xr[r + dr][col][c].w;
            }
            float v = __uint_as_float((h & 0x007FFFFFu) | 0x3F800000u);
            for (int i = 0; i < chain; i++)          // stands in for the row's MFMAs
                v = __builtin_fmaf(v, 0.999f, acc);
            acc = v;
            // stores of the row: 1 KiB per instruction (two boards' 512-B rows), as the staged conv
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int m = 64 * k + lane, bl = m >> 5, q = m & 31;
                const int64_t o = ((tile * 16 + bl) * 16 + 4 * r) * 8 + q;
                uint4 w = make_uint4(h, __float_as_uint(acc), (uint32_t)k, (uint32_t)r);
                if (EPI == 1) {
                    const uint4 b = e[o];                    // the SM = 2 epilogue's BN-input piece
                    w.x ^= b.x;
                    w.y ^= b.z;
                }
                if (EPI == 2) {                              // the residual add's pieces: 8 B per (col, pass)
                    const uint2 *e2 = reinterpret_cast<const uint2 *>(e);
                    const int col = k & 3, oh = k >> 2;      // 8 of the row's 16 (col, pass) pieces here ...
                    const int64_t b = tile * 16 + n;
                    const int64_t i2 = ((b * 16 + 4 * r + col) * 64 + 16 * oh + 4 * g) / 4;
                    const uint2 p0 = e2[i2], p1 = e2[i2 + 8];  // ... and the other 8 (passes 2, 3)
                    w.x ^= p0.x ^ p1.y;
                }
                y[o] = w;
            }
        }
    }
}

int main(int argc, char **)
{
    const int64_t boards = 1 << 16, n_tiles = boards / 16;
    const size_t bytes = (size_t)boards * 16 * 128;                      // [boards][16 cells][64 bf16]
    uint4 *x[3], *e[3], *y;
    for (int i = 0; i < 3; i++) {                                          // rotate: 3 x 134 MB > Infinity Cache
        CK(hipMalloc(&x[i], bytes));
        CK(hipMalloc(&e[i], bytes));
        CK(hipMemset(x[i], 1, bytes));
        CK(hipMemset(e[i], 2, bytes));
    }
    CK(hipMalloc(&y, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int chains[] = {0, 100, 200, 300};
    const int n_chains = argc > 1 ? 1 : 4;
    for (int ci = 0; ci < n_chains; ci++) {
        const int chain = chains[ci];
        for (int variant = 0; variant < 6; variant++) {
            const bool full = variant & 1;
            const int epi = variant >> 1;
            auto launch = [&](int i) {
                const uint4 *xs = x[i % 3], *es = e[i % 3];
                const dim3 gr(256), bl(64 * kWaves);
                switch (variant) {
                case 0: hipLaunchKernelGGL((conv_io<false, 0>), gr, bl, 0, 0, xs, es, y, n_tiles, chain); break;
                case 1: hipLaunchKernelGGL((conv_io<true, 0>), gr, bl, 0, 0, xs, es, y, n_tiles, chain); break;
                case 2: hipLaunchKernelGGL((conv_io<false, 1>), gr, bl, 0, 0, xs, es, y, n_tiles, chain); break;
                case 3: hipLaunchKernelGGL((conv_io<true, 1>), gr, bl, 0, 0, xs, es, y, n_tiles, chain); break;
                case 4: hipLaunchKernelGGL((conv_io<false, 2>), gr, bl, 0, 0, xs, es, y, n_tiles, chain); break;
                default: hipLaunchKernelGGL((conv_io<true, 2>), gr, bl, 0, 0, xs, es, y, n_tiles, chain);
                }
            };
            for (int i = 0; i < 5; i++)
                launch(i);
            CK(hipDeviceSynchronize());
            const int reps = 30;
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < reps; i++)
                launch(i);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = 1e3 * ms / reps;
            const double moved = (double)bytes * (2 + (epi ? 1 : 0));
            printf("chain %3d  loads %s  %s  %7.1f us  %5.2f TB/s\n", chain, full ? "F (1 KiB/instr)" : "H (conv half lines)",
                   epi == 1 ? "+ epilogue stream (1 KiB)" : epi == 2 ? "+ add stream (8 B/lane) " : "                         ",
                   us, moved / us / 1e6);
        }
    }
    return 0;
}
