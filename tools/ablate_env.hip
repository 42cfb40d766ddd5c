// tools/ablate_env.hip -- where do k_step's cycles go? (standalone, not part of the product)
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o build/ablate tools/ablate_env.hip
// Runs, in one process, interleaved rounds of:
//   roll<R, P>   K steps per launch with boards in VGPRs (compute-bound probe)
//                R = Philox rounds (0 = a 2-multiply hash), P = part: 0 full step, 1 RNG only,
//                2 move only (no spawn / game-over), 3 full step minus game-over
//   copy         same HBM I/O as k_step (16 B in, 16 B out, 1 B action out, 1 B done out), no compute
//   step<R>      the single-step kernel shape at N boards (memory-bound probe)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../rein48_amd/csrc/r48_board.h"

using r48::Board;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <int R>
__device__ __forceinline__ void rng(uint32_t w[4], uint64_t gid, uint32_t step, uint32_t k0, uint32_t k1)
{
    w[0] = (uint32_t)gid;
    w[1] = (uint32_t)(gid >> 32);
    w[2] = step;
    w[3] = 0x2048u;
    if (R == 0) {
        uint32_t x = (uint32_t)gid * 0x9E3779B1u ^ step * 0x85EBCA77u ^ k0;
        x ^= x >> 15;
        x *= 0x2C1B3C6Du;
        x ^= x >> 12;
        w[0] = x;
        w[1] = x * 0x297A2D39u;
        w[2] = w[1] ^ (x >> 7);
        w[3] = w[2] * 0x9E3779B1u;
        return;
    }
#pragma unroll
    for (int i = 0; i < R; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * w[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * w[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ w[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ w[3] ^ k1;
        w[1] = (uint32_t)p1;
        w[3] = (uint32_t)p0;
        w[0] = n0;
        w[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

template <int R, int P>
__global__ __launch_bounds__(256) void roll(int8_t *boards, int64_t n, int K, int8_t *act, uint8_t *done)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    Board b{v.x, v.y, v.z, v.w};
    for (int t = 0; t < K; t++) {
        uint32_t w[4];
        rng<R>(w, (uint64_t)i, (uint32_t)t, 0x2048u, 0x5EEDu);
        const uint32_t a = w[0] >> 30;
        uint32_t d = 0;
        if (P == 0) {
            const r48::StepOut o = r48::step_board<false, false>(b, a, w[1], w[2] < r48::kFourThresh);
            if (o.done)
                r48::reset_board(b, w[3] >> 28, (w[3] & 0x0FFFFFFFu) < r48::kFourThresh28);
            d = o.done;
        } else if (P == 1) {
            b.w0 ^= w[0];
            b.w1 ^= w[1];
            b.w2 ^= w[2];
            b.w3 ^= w[3];
            d = b.w0 & 1u;
        } else if (P == 2) {
            Board L = r48::to_lines(b, a);
            r48::move_lines<false>(L);
            b = r48::from_lines(L, a);
            d = (b.w0 >> 3) & 1u;
        } else {
            Board L = r48::to_lines(b, a);
            const Board L0 = L;
            r48::move_lines<false>(L);
            const bool ch = ((L.w0 ^ L0.w0) | (L.w1 ^ L0.w1) | (L.w2 ^ L0.w2) | (L.w3 ^ L0.w3)) != 0u;
            b = r48::from_lines(L, a);
            const r48::Blanks bl = r48::blanks(b);
            const uint32_t cell = r48::select_blank(bl, r48::mulhi(w[1], bl.n));
            r48::place(b, cell, (w[2] < r48::kFourThresh) ? 2u : 1u, ch);
            d = bl.n == 1u;
            if (d)
                r48::reset_board(b, w[3] >> 28, false);
        }
        act[(int64_t)t * n + i] = (int8_t)a;
        done[(int64_t)t * n + i] = (uint8_t)d;
    }
    *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
}

__global__ __launch_bounds__(256) void copy_like_step(int8_t *boards, int64_t n, uint32_t step, int8_t *act,
                                                       uint8_t *done)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    v.x ^= step;
    *reinterpret_cast<uint4 *>(boards + 16 * i) = v;
    act[i] = (int8_t)(v.y & 3u);
    done[i] = (uint8_t)(v.z & 1u);
}

template <int R>
__global__ __launch_bounds__(256) void step1(int8_t *boards, int64_t n, uint32_t step, int8_t *act, uint8_t *done)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    Board b{v.x, v.y, v.z, v.w};
    uint32_t w[4];
    rng<R>(w, (uint64_t)i, step, 0x2048u, 0x5EEDu);
    const uint32_t a = w[0] >> 30;
    const r48::StepOut o = r48::step_board<false, false>(b, a, w[1], w[2] < r48::kFourThresh);
    if (o.done)
        r48::reset_board(b, w[3] >> 28, (w[3] & 0x0FFFFFFFu) < r48::kFourThresh28);
    *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
    act[i] = (int8_t)a;
    done[i] = (uint8_t)o.done;
}

// B boards per thread: block tile = 256*B boards, board j of thread t = tile + t + 256*j (every
// load/store instruction stays coalesced); all B loads issue before any compute.
template <int R, int B>
__global__ __launch_bounds__(256) void stepB(int8_t *boards, int64_t n, uint32_t step, int8_t *act, uint8_t *done)
{
    const int64_t base = (int64_t)blockIdx.x * 256 * B + threadIdx.x;
    Board b[B];
#pragma unroll
    for (int j = 0; j < B; j++) {
        const int64_t i = base + 256 * j;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (i < n)
            v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
        b[j] = Board{v.x, v.y, v.z, v.w};
    }
#pragma unroll
    for (int j = 0; j < B; j++) {
        const int64_t i = base + 256 * j;
        uint32_t w[4];
        rng<R>(w, (uint64_t)i, step, 0x2048u, 0x5EEDu);
        const uint32_t a = w[0] >> 30;
        const r48::StepOut o = r48::step_board<false, false>(b[j], a, w[1], w[2] < r48::kFourThresh);
        if (o.done)
            r48::reset_board(b[j], w[3] >> 28, (w[3] & 0x0FFFFFFFu) < r48::kFourThresh28);
        if (i < n) {
            *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b[j].w0, b[j].w1, b[j].w2, b[j].w3);
            act[i] = (int8_t)a;
            done[i] = (uint8_t)o.done;
        }
    }
}

// grid-stride over 256-board tiles with the next tile's board prefetched into registers
template <int R>
__global__ __launch_bounds__(256) void stepGS(int8_t *boards, int64_t n, uint32_t step, int8_t *act, uint8_t *done)
{
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i < n)
        v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    for (; i < n; i += stride) {
        const int64_t nx = i + stride;
        uint4 vn = make_uint4(0, 0, 0, 0);
        if (nx < n)
            vn = *reinterpret_cast<const uint4 *>(boards + 16 * nx);
        Board b{v.x, v.y, v.z, v.w};
        uint32_t w[4];
        rng<R>(w, (uint64_t)i, step, 0x2048u, 0x5EEDu);
        const uint32_t a = w[0] >> 30;
        const r48::StepOut o = r48::step_board<false, false>(b, a, w[1], w[2] < r48::kFourThresh);
        if (o.done)
            r48::reset_board(b, w[3] >> 28, (w[3] & 0x0FFFFFFFu) < r48::kFourThresh28);
        *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
        act[i] = (int8_t)a;
        done[i] = (uint8_t)o.done;
        v = vn;
    }
}

// pipelined persistent: grid-stride over FULL 256-board tiles (no per-lane guards, so the
// compiler can count vmcnt exactly), next tile's board prefetched before computing this one.
template <int R>
__global__ __launch_bounds__(256) void stepP(int8_t *boards, int64_t n_tiles, uint32_t step, int8_t *act,
                                             uint8_t *done)
{
    int64_t tile = blockIdx.x;
    const int64_t stride = gridDim.x;
    if (tile >= n_tiles)
        return;
    int64_t i = tile * 256 + threadIdx.x;
    uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    for (;;) {
        const int64_t nt = tile + stride;
        const bool more = nt < n_tiles;
        const int64_t ni = more ? nt * 256 + threadIdx.x : i;
        const uint4 vn = *reinterpret_cast<const uint4 *>(boards + 16 * ni);
        Board b{v.x, v.y, v.z, v.w};
        uint32_t w[4];
        rng<R>(w, (uint64_t)i, step, 0x2048u, 0x5EEDu);
        const uint32_t a = w[0] >> 30;
        const r48::StepOut o = r48::step_board<false, false>(b, a, w[1], w[2] < r48::kFourThresh);
        if (o.done)
            r48::reset_board(b, w[3] >> 28, (w[3] & 0x0FFFFFFFu) < r48::kFourThresh28);
        *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
        act[i] = (int8_t)a;
        done[i] = (uint8_t)o.done;
        if (!more)
            break;
        tile = nt;
        i = ni;
        v = vn;
    }
}

// B boards per thread, straight-line: full tiles take an unguarded path (loads issued back to
// back, board j computed as soon as ITS load is in), only the last partial tile is guarded.
template <int R>
__device__ __forceinline__ void step_one(Board &b, int64_t i, uint32_t step, uint32_t &a, uint32_t &d)
{
    uint32_t w[4];
    rng<R>(w, (uint64_t)i, step, 0x2048u, 0x5EEDu);
    a = w[0] >> 30;
    const r48::StepOut o = r48::step_board<false, false>(b, a, w[1], w[2] < r48::kFourThresh);
    if (o.done)
        r48::reset_board(b, w[3] >> 28, (w[3] & 0x0FFFFFFFu) < r48::kFourThresh28);
    d = o.done;
}

template <int R, int B>
__global__ __launch_bounds__(256) void stepS(int8_t *boards, int64_t n, uint32_t step, int8_t *act, uint8_t *done)
{
    const int64_t base = (int64_t)blockIdx.x * 256 * B + threadIdx.x;
    if ((int64_t)(blockIdx.x + 1) * 256 * B <= n) {
        uint4 v[B];
#pragma unroll
        for (int j = 0; j < B; j++)
            v[j] = *reinterpret_cast<const uint4 *>(boards + 16 * (base + 256 * j));
#pragma unroll
        for (int j = 0; j < B; j++) {
            const int64_t i = base + 256 * j;
            Board b{v[j].x, v[j].y, v[j].z, v[j].w};
            uint32_t a, d;
            step_one<R>(b, i, step, a, d);
            *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
            act[i] = (int8_t)a;
            done[i] = (uint8_t)d;
        }
    } else {
        for (int j = 0; j < B; j++) {
            const int64_t i = base + 256 * j;
            if (i < n) {
                const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
                Board b{v.x, v.y, v.z, v.w};
                uint32_t a, d;
                step_one<R>(b, i, step, a, d);
                *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
                act[i] = (int8_t)a;
                done[i] = (uint8_t)d;
            }
        }
    }
}

template <int R, int T>
__global__ __launch_bounds__(T) void stepT(int8_t *boards, int64_t n, uint32_t step, int8_t *act, uint8_t *done)
{
    const int64_t i = (int64_t)blockIdx.x * T + threadIdx.x;
    if (i >= n)
        return;
    const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    Board b{v.x, v.y, v.z, v.w};
    uint32_t a, d;
    step_one<R>(b, i, step, a, d);
    *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
    act[i] = (int8_t)a;
    done[i] = (uint8_t)d;
}

__global__ __launch_bounds__(256) void copy32(int8_t *boards, int64_t n, uint32_t step, int8_t *, uint8_t *)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    v.x ^= step;
    *reinterpret_cast<uint4 *>(boards + 16 * i) = v;
}

__global__ void init(int8_t *boards, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    uint32_t x = (uint32_t)i * 2654435761u;
    uint32_t w[4];
    for (int k = 0; k < 4; k++) {
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        uint32_t word = 0;
        for (int c = 0; c < 4; c++) {
            const uint32_t e = ((x >> (4 * c)) & 3u) ? 0u : 1u + ((x >> (4 * c + 16)) & 3u);
            word |= e << (8 * c);
        }
        w[k] = word;
    }
    *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(w[0], w[1], w[2], w[3]);
}

struct Timer {
    hipEvent_t a, b;
    Timer()
    {
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
    }
    float ms() const
    {
        float m = 0;
        CK(hipEventElapsedTime(&m, a, b));
        return m;
    }
};

int main(int argc, char **argv)
{
    const int64_t n_small = 1 << 20, n_big = argc > 1 ? atoll(argv[1]) : (1 << 26);
    const int K = 64;
    int8_t *boards, *act;
    uint8_t *done;
    CK(hipMalloc(&boards, 16 * n_big));
    CK(hipMalloc(&act, (size_t)K * n_small > (size_t)n_big ? (size_t)K * n_small : (size_t)n_big));
    CK(hipMalloc(&done, (size_t)K * n_small > (size_t)n_big ? (size_t)K * n_small : (size_t)n_big));
    const dim3 blk(256);
    auto grid = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    hipLaunchKernelGGL(init, grid(n_big), blk, 0, 0, boards, n_big);
    CK(hipDeviceSynchronize());

    struct Case {
        const char *name;
        int64_t n;
        int steps;  // board-steps per launch = n * steps
        void (*launch)(int8_t *, int64_t, int8_t *, uint8_t *, uint32_t);
    };
#define ROLL(R, P)                                                                                            \
    Case{"roll<" #R "," #P ">", n_small, K, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t) {        \
             hipLaunchKernelGGL((roll<R, P>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, n, 64, a, d); \
         }}
#define STEP(R, N)                                                                                            \
    Case{"step1<" #R "> n=" #N, N, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {             \
             hipLaunchKernelGGL((step1<R>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, n, s, a, d);  \
         }}
    std::vector<Case> cases = {
        ROLL(10, 0), ROLL(7, 0), ROLL(0, 0), ROLL(10, 1), ROLL(0, 2), ROLL(0, 3),
        Case{"copy n=big", n_big, 1,
             [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {
                 hipLaunchKernelGGL(copy_like_step, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, n, s, a, d);
             }},
        Case{"copy n=1M", n_small, 1,
             [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {
                 hipLaunchKernelGGL(copy_like_step, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, n, s, a, d);
             }},
    };
#define SB(R, B, NN, LBL)                                                                                  \
    cases.push_back(Case{LBL, NN, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {             \
        hipLaunchKernelGGL((stepB<R, B>), dim3((unsigned)((n + 256 * B - 1) / (256 * B))), dim3(256), 0, 0, b, n, s, \
                           a, d);                                                                             \
    }})
#define GS(R, NN, G, LBL)                                                                                   \
    cases.push_back(Case{LBL, NN, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {             \
        hipLaunchKernelGGL((stepGS<R>), dim3(G), dim3(256), 0, 0, b, n, s, a, d);                              \
    }})
    cases.push_back(Case{"copy32 n=big", n_big, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {
                             hipLaunchKernelGGL(copy32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, n, s, a, d);
                         }});
    cases.push_back(Case{"copy32 n=1M", n_small, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {
                             hipLaunchKernelGGL(copy32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, n, s, a, d);
                         }});
    SB(10, 1, n_big, "stepB<10,1> big");
    SB(10, 2, n_big, "stepB<10,2> big");
    SB(10, 4, n_big, "stepB<10,4> big");
    SB(10, 1, n_small, "stepB<10,1> 1M");
    SB(10, 2, n_small, "stepB<10,2> 1M");
    SB(10, 4, n_small, "stepB<10,4> 1M");
    SB(0, 2, n_small, "stepB<0,2> 1M");
#define SP(R, NN, G, LBL)                                                                                   \
    cases.push_back(Case{LBL, NN, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {             \
        hipLaunchKernelGGL((stepP<R>), dim3(G), dim3(256), 0, 0, b, n / 256, s, a, d);                         \
    }})
    SP(10, n_big, 2048, "stepP<10> g2048 big");
    SP(10, n_small, 2048, "stepP<10> g2048 1M");
    SP(10, n_small, 1024, "stepP<10> g1024 1M");
#define SS(R, B, NN, LBL)                                                                                  \
    cases.push_back(Case{LBL, NN, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {             \
        hipLaunchKernelGGL((stepS<R, B>), dim3((unsigned)((n + 256 * B - 1) / (256 * B))), dim3(256), 0, 0, b, n, s, \
                           a, d);                                                                             \
    }})
    SS(10, 1, n_big, "stepS<10,1> big");
    SS(10, 2, n_big, "stepS<10,2> big");
    SS(10, 4, n_big, "stepS<10,4> big");
    SS(10, 1, n_small, "stepS<10,1> 1M");
    SS(10, 2, n_small, "stepS<10,2> 1M");
    SS(10, 4, n_small, "stepS<10,4> 1M");
#define ST(R, T, NN, LBL)                                                                                  \
    cases.push_back(Case{LBL, NN, 1, [](int8_t *b, int64_t n, int8_t *a, uint8_t *d, uint32_t s) {             \
        hipLaunchKernelGGL((stepT<R, T>), dim3((unsigned)((n + T - 1) / T)), dim3(T), 0, 0, b, n, s, a, d);      \
    }})
    ST(10, 64, n_small, "stepT<10,64> 1M");
    ST(10, 128, n_small, "stepT<10,128> 1M");
    ST(10, 256, n_small, "stepT<10,256> 1M");
    ST(10, 512, n_small, "stepT<10,512> 1M");
    ST(10, 1024, n_small, "stepT<10,1024> 1M");
    ST(10, 512, n_big, "stepT<10,512> big");
    ST(10, 1024, n_big, "stepT<10,1024> big");
    ST(0, 1024, n_small, "stepT<0,1024> 1M");
    GS(10, n_big, 2048, "stepGS<10> g2048 big");
    GS(10, n_small, 2048, "stepGS<10> g2048 1M");
    GS(10, n_small, 1024, "stepGS<10> g1024 1M");
    const int rounds = 5, reps = 20;
    std::vector<std::vector<float>> res(cases.size());
    Timer t;
    uint32_t step = 0;
    for (int r = 0; r < rounds; r++)
        for (size_t c = 0; c < cases.size(); c++) {
            cases[c].launch(boards, cases[c].n, act, done, step++);  // warm
            CK(hipEventRecord(t.a, 0));
            for (int k = 0; k < reps; k++)
                cases[c].launch(boards, cases[c].n, act, done, step++);
            CK(hipEventRecord(t.b, 0));
            CK(hipEventSynchronize(t.b));
            res[c].push_back(t.ms() / reps);
        }
    CK(hipGetLastError());
    // product-style chunk loop: [memset counter] -> fork -> 2 chain graphs -> join, repeated
    {
        hipStream_t user, st[2];
        hipEvent_t fork, join[2];
        CK(hipStreamCreateWithFlags(&user, hipStreamNonBlocking));
        for (int c = 0; c < 2; c++) {
            CK(hipStreamCreateWithFlags(&st[c], hipStreamNonBlocking));
            CK(hipEventCreateWithFlags(&join[c], hipEventDisableTiming));
        }
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        uint32_t *dctr;
        CK(hipMalloc(&dctr, 4));
        const int64_t n = n_small, h = n / 2;
        for (int chunk : {25, 100, 400}) {
            hipGraphExec_t gx[2];
            for (int c = 0; c < 2; c++) {
                hipGraph_t gc;
                CK(hipStreamBeginCapture(st[c], hipStreamCaptureModeThreadLocal));
                for (int k = 0; k < chunk; k++)
                    hipLaunchKernelGGL((stepT<10, 256>), dim3((unsigned)((h + 255) / 256)), dim3(256), 0, st[c],
                                       boards + 16 * h * c, h, (uint32_t)k, act + h * c, done + h * c);
                CK(hipStreamEndCapture(st[c], &gc));
                CK(hipGraphInstantiate(&gx[c], gc, nullptr, nullptr, 0));
            }
            for (int mode = 0; mode < 3; mode++) {  // 0: memset+fork, 1: fork only, 2: no fork (independent)
                const int chunks = 4000 / chunk;
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(t.a, user));
                for (int q = 0; q < chunks; q++) {
                    if (mode == 0)
                        CK(hipMemsetD32Async((hipDeviceptr_t)dctr, q, 1, user));
                    if (mode < 2) {
                        CK(hipEventRecord(fork, user));
                        for (int c = 0; c < 2; c++) CK(hipStreamWaitEvent(st[c], fork, 0));
                    }
                    for (int c = 0; c < 2; c++) CK(hipGraphLaunch(gx[c], st[c]));
                    if (mode < 2)
                        for (int c = 0; c < 2; c++) {
                            CK(hipEventRecord(join[c], st[c]));
                            CK(hipStreamWaitEvent(user, join[c], 0));
                        }
                }
                for (int c = 0; c < 2; c++) {
                    CK(hipEventRecord(join[c], st[c]));
                    CK(hipStreamWaitEvent(user, join[c], 0));
                }
                CK(hipEventRecord(t.b, user));
                CK(hipEventSynchronize(t.b));
                printf("chunk %4d mode %d (%s): %.2f us/step\n", chunk, mode,
                       mode == 0 ? "memset+fork/join" : mode == 1 ? "fork/join" : "no fork", t.ms() * 1e3 / 4000);
            }
        }
    }
    printf("%-22s %12s %14s %10s\n", "case", "ms/launch", "Gboard-steps/s", "GB/s(34B)");
    for (size_t c = 0; c < cases.size(); c++) {
        std::sort(res[c].begin(), res[c].end());
        const float ms = res[c][rounds / 2];
        const double bs = (double)cases[c].n * cases[c].steps / (ms * 1e-3);
        printf("%-22s %12.4f %14.2f %10.1f\n", cases[c].name, ms, bs / 1e9,
               cases[c].steps == 1 ? bs * 34 / 1e9 : 0.0);
    }
    return 0;
}
