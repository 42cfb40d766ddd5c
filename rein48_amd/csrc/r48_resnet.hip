// r48_resnet.hip -- fused ResNet-10 Q-network inference on gfx950 MFMA (BASELINE config 5).
//
// rein48_amd/dqn/nets.py:ResNet10Q in eval mode (BatchNorm folded into the convs on the host,
// rein48_amd/dqn/fused.py:pack_resnet), forward only, for acting on millions of boards:
//   x   = one-hot of the 16 cell exponents (18 planes)
//   h   = relu(conv3x3(x))                                     stem, 18 -> 64
//   4 x h = relu(conv3x3(relu(conv3x3(h))) + h)                basic blocks, 64 -> 64
//   Q   = Wh . flatten(h) + bh                                 head, 1024 -> 4
// and optionally the epsilon-greedy draw of r48_egreedy_actions (same Philox contract).
//
// Orientation (v_mfma_f32_32x32x16_bf16): rows = 32 output channels (two tiles per layer),
// columns = 32 board-positions = 2 boards x 16 cells. Lane l owns column l & 31 (board
// (l & 31) >> 4, cell l & 15) and the half h = l >> 5 of its K range. A layer's 32x32 f32
// accumulators therefore hold each cell's channel vector in that cell's own lanes, and the next
// layer's B operand is built in registers: the 3x3 tap (dr, dc) reads cell p + 4dr + dc, which
// is the lane 4dr + dc further along the same 16-lane DPP row (one board = one DPP row), so a
// tap is a v_mov_b32_dpp row shift with zero fill (cells past the top/bottom edge fall off the
// row) plus a v_cndmask for the left/right edge. No LDS traffic for activations, no lane
// crossing between boards. The k order inside a fragment follows the accumulator layout
// (element j of half h = channel 16s + 8(j>>2) + 4h + (j&3) of k-chunk s); the host packs the
// weight (A) fragments in that order.
// Per column group (2 boards) a 64->64 layer is 9 taps x 4 k-chunks x 2 row tiles = 72 MFMAs;
// each wave carries G column groups (2G boards) so one LDS weight fragment feeds 2G MFMAs.
// Weights: each layer's 72 fragments + its bias (1 KiB each) stream into one of two LDS
// buffers by global_load_lds while the other buffer's layer computes; the workgroup is
// persistent (one per CU, 8 waves) and cycles stem, conv1..conv8 per 32-board tile.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x16 = __attribute__((ext_vector_type(16))) float;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// 8 waves x 2 column groups (two waves per SIMD, so one wave's exposed LDS-read latency runs
// under the other's MFMAs) measured 14.7-14.9 ms per 2^21 boards against 15.5 for 4 waves x 4
// groups and 16.7 for 8 x 1 (bit-identical outputs; tools/exp_resnet_fused.py)
#ifndef R48_RESNET_WAVES
#define R48_RESNET_WAVES 8
#endif
#ifndef R48_RESNET_G
#define R48_RESNET_G 2
#endif
#ifndef R48_RN_ABL   // timing ablations only (wrong results): 1 no per-layer wait/barrier, 2 also no weight
#define R48_RN_ABL 0 // DMA, 3 epilogue = bf16 pack only, 4 no DPP row shifts in the taps
#endif
constexpr int kWaves = R48_RESNET_WAVES;
constexpr int kThreads = 64 * kWaves;
constexpr int G = R48_RESNET_G;                   // column groups (2 boards each) per wave
constexpr int kBoardsPerTile = kWaves * G * 2;    // 32
constexpr int kConvLayers = 8;
constexpr int kStemFrags = 9 * 2 * 2;             // taps x k-chunks (18 planes padded to 32) x row tiles
constexpr int kConvFrags = 9 * 4 * 2;
constexpr int kStemBlock = kStemFrags + 1;        // + bias fragment
constexpr int kConvBlock = kConvFrags + 1;
constexpr int kBufFrags = kConvBlock;             // 73 KiB per LDS buffer
constexpr int kHeadBf16 = 16 * 2 * 4 * 32;        // [cell][half][action][32 channels]
constexpr uint32_t kEgreedyTag = 0xD0Eu;
constexpr int kBlobFrags = kStemBlock + kConvLayers * kConvBlock;

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi)
{
    const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xFFFF0000u); }

// value of cell p + D in the same board (DPP row = 16 lanes), 0 past the row's ends
template <int D>
__device__ __forceinline__ uint32_t cell_shift(uint32_t v)
{
    if constexpr (D == 0)
        return v;
    else if constexpr (D > 0)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + D, 0xF, 0xF, true);   // row_shl: lane i <- i + D
    else
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 - D, 0xF, 0xF, true);   // row_shr: lane i <- i - |D|
}

__device__ __forceinline__ bf16x8 lds_frag(const uint4 *lds, int frag, int lane)
{
    const uint4 v = lds[frag * 64 + lane];
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// tap (DR, DC) of k-chunk s for all column groups: B = the chunk's registers shifted by DR
// grid rows (xs[g][DC + 1] already holds the column-shifted, edge-masked copy), times both
// row tiles -- one pair of LDS weight fragments feeds 2G MFMAs
template <int DR, int DC, int NCH>
__device__ __forceinline__ void tap_mfma(const uint4 *wl, int s, const uint32_t (&xs)[G][3][4], f32x16 (&acc)[G][2],
                                         int lane)
{
    constexpr int t = (DR + 1) * 3 + (DC + 1);
    const bf16x8 A0 = lds_frag(wl, (t * NCH + s) * 2 + 0, lane);
    const bf16x8 A1 = lds_frag(wl, (t * NCH + s) * 2 + 1, lane);
#pragma unroll
    for (int g = 0; g < G; g++) {
        uint32_t r[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            r[q] = R48_RN_ABL == 4 ? xs[g][DC + 1][q] : cell_shift<4 * DR>(xs[g][DC + 1][q]);
        bf16x8 B;
        __builtin_memcpy(&B, r, 16);
        acc[g][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B, acc[g][0], 0, 0, 0);
        acc[g][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B, acc[g][1], 0, 0, 0);
    }
}

// the same tap for ONE column group (the last k-chunk runs group by group)
template <int DR, int DC, int NCH>
__device__ __forceinline__ void tap_mfma1(const uint4 *wl, int s, const uint32_t (&xs)[3][4], f32x16 &a0, f32x16 &a1,
                                          int lane)
{
    constexpr int t = (DR + 1) * 3 + (DC + 1);
    const bf16x8 A0 = lds_frag(wl, (t * NCH + s) * 2 + 0, lane);
    const bf16x8 A1 = lds_frag(wl, (t * NCH + s) * 2 + 1, lane);
    uint32_t r[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
        r[q] = R48_RN_ABL == 4 ? xs[DC + 1][q] : cell_shift<4 * DR>(xs[DC + 1][q]);
    bf16x8 B;
    __builtin_memcpy(&B, r, 16);
    a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B, a1, 0, 0, 0);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

// bias (+ residual) + ReLU of one column group -> packed bf16 activations; SAVE first keeps
// the layer input in res for the block's skip connection
template <bool RESID, bool SAVE>
__device__ __forceinline__ void epilogue1(const f32x16 (&acc)[2], const float *bias, int h, uint32_t (&act)[16],
                                          uint32_t (&res)[16])
{
    if (SAVE) {
#pragma unroll
        for (int k = 0; k < 16; k++)
            res[k] = act[k];
    }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = 8 * (s & 1) + 2 * q;
            // bias of accumulator rows i, i+1: channels 32m + 8(i>>2) + 4h + (i&3), +1
            if (R48_RN_ABL == 3) {
                act[4 * s + q] = pack_bf16x2(acc[s >> 1][i], acc[s >> 1][i + 1]);
                continue;
            }
            const f32x2 bb = *reinterpret_cast<const f32x2 *>(bias + 32 * (s >> 1) + 8 * (i >> 2) + 4 * h + (i & 3));
            f32x2 v = f32x2{acc[s >> 1][i], acc[s >> 1][i + 1]} + bb;
            if (RESID)
                v += f32x2{bf_lo(res[4 * s + q]), bf_hi(res[4 * s + q])};
            // ReLU on the packed bf16 pair as signed int16 (negative bf16 <=> negative int16)
            const i16x2 p = __builtin_bit_cast(i16x2, __builtin_convertvector(v, bf16x2_t));   // one v_cvt_pk_bf16_f32
            act[4 * s + q] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(p, i16x2{0, 0}));
        }
}

// One conv layer: k-chunk by k-chunk, the column-shifted copies x[p-1] (zero on the left edge),
// x[p], x[p+1] (zero on the right edge) of every group are built once and each of the 9 taps
// is then a single DPP row shift by 4dr; then the epilogue (bias, optional residual, ReLU,
// bf16) per group. act[g] is the layer's input and output; SAVE keeps the input in res[g] for
// the block's skip connection. act[g][4s + q] = channels of row tile s >> 1, accumulator
// registers 8(s & 1) + 2q, +1.
// The edge masks are applied as AND with a 0 / all-ones lane mask, never as a select around the
// DPP: the compiler lowers `edge ? 0 : dpp(x)` to an EXEC-masked DPP move, and a DPP read from a
// lane disabled in EXEC returns 0 -- interior cells would lose their edge neighbours.
template <int NCH, bool RESID, bool SAVE>
__device__ __forceinline__ void layer(const uint4 *wl, const float *bias, uint32_t (&act)[G][16],
                                      uint32_t (&res)[G][16], f32x16 (&acc)[G][2], int lane, int h, uint32_t keep_l,
                                      uint32_t keep_r)
{
#pragma unroll
    for (int g = 0; g < G; g++)
        acc[g][0] = acc[g][1] = f32x16{};
#pragma unroll
    for (int s = 0; s < NCH - 1; s++) {
        uint32_t xs[G][3][4];
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t x = act[g][4 * s + q];
                xs[g][0][q] = cell_shift<-1>(x) & keep_l;   // cell p - 1, zero on the left edge
                xs[g][1][q] = x;
                xs[g][2][q] = cell_shift<1>(x) & keep_r;    // cell p + 1, zero on the right edge
            }
        tap_mfma<-1, -1, NCH>(wl, s, xs, acc, lane);
        tap_mfma<-1, 0, NCH>(wl, s, xs, acc, lane);
        tap_mfma<-1, 1, NCH>(wl, s, xs, acc, lane);
        tap_mfma<0, -1, NCH>(wl, s, xs, acc, lane);
        tap_mfma<0, 0, NCH>(wl, s, xs, acc, lane);
        tap_mfma<0, 1, NCH>(wl, s, xs, acc, lane);
        tap_mfma<1, -1, NCH>(wl, s, xs, acc, lane);
        tap_mfma<1, 0, NCH>(wl, s, xs, acc, lane);
        tap_mfma<1, 1, NCH>(wl, s, xs, acc, lane);
    }
    // last k-chunk group by group, each group's epilogue right behind its last MFMAs so the
    // scheduler can run it under the next group's MFMAs
    constexpr int s = NCH - 1;
#pragma unroll
    for (int g = 0; g < G; g++) {
        uint32_t xs[3][4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t x = act[g][4 * s + q];
            xs[0][q] = cell_shift<-1>(x) & keep_l;
            xs[1][q] = x;
            xs[2][q] = cell_shift<1>(x) & keep_r;
        }
        tap_mfma1<-1, -1, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<-1, 0, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<-1, 1, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<0, -1, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<0, 0, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<0, 1, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<1, -1, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<1, 0, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        tap_mfma1<1, 1, NCH>(wl, s, xs, acc[g][0], acc[g][1], lane);
        epilogue1<RESID, SAVE>(acc[g], bias, h, act[g], res[g]);
    }
}

// LDS-DMA of one layer block (frags x 1 KiB) into an LDS buffer: wave w moves fragments w, w+4, ...
__device__ __forceinline__ void stage_block(const uint4 *src, uint4 *dst, int frags, int wave, int lane)
{
    for (int f = wave; f < frags; f += kWaves)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + f * 64 + lane),
                                         (__attribute__((address_space(3))) void *)(dst + f * 64), 16, 0, 0);
}

__device__ __forceinline__ float row16_sum(float x)
{
    // sum over the 16 lanes of a DPP row: quad pairs, quads, half-rows, rows
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));  // row_half_mirror
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));  // row_mirror
    return x;
}

__global__ __launch_bounds__(kThreads, 1) void k_resnet_q(const int8_t *__restrict__ boards, int64_t n,
                                                         const uint4 *__restrict__ blob,
                                                         const uint4 *__restrict__ head_w,
                                                         const float *__restrict__ head_b, float *__restrict__ q_out,
                                                         int8_t *__restrict__ actions, float eps, uint32_t k0,
                                                         uint32_t k1, int64_t gid0, uint32_t ctr)
{
    extern __shared__ uint4 lds[];                  // [2][kBufFrags * 64] weights | head [kHeadBf16 / 8]
    auto buf = [](int i) { return lds + i * (kBufFrags * 64); };
    const uint16_t *head_lds = reinterpret_cast<const uint16_t *>(lds + 2 * kBufFrags * 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, cell = lane & 15;
    const uint32_t keep_l = (lane & 3) == 0 ? 0u : ~0u, keep_r = (lane & 3) == 3 ? 0u : ~0u;
    const int64_t tiles = (n + kBoardsPerTile - 1) / kBoardsPerTile;

    // head weights once per workgroup; first stem block into buffer 0
    for (int i = threadIdx.x; i < kHeadBf16 / 8; i += kThreads)
        lds[2 * kBufFrags * 64 + i] = head_w[i];
    int cur = 0;
    if ((int64_t)blockIdx.x < tiles)
        stage_block(blob, buf(0), kStemBlock, wave, lane);
    const float hb0 = head_b[0], hb1 = head_b[1], hb2 = head_b[2], hb3 = head_b[3];

    uint32_t act[G][16], res[G][16];
    f32x16 acc[G][2];
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const int64_t b0 = tile * kBoardsPerTile + wave * (2 * G);
        // cell exponents of this wave's 8 boards (one byte per lane and group)
        uint32_t e[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int64_t b = b0 + 2 * g + ((lane & 31) >> 4);
            e[g] = b < n ? (uint32_t)(uint8_t)boards[16 * b + cell] : 0xFFu;
        }
        // one-hot B registers of the stem: k-chunk s, element j of half h = plane 16s + 8h + j
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const uint32_t d = e[g] - (uint32_t)(16 * s + 8 * h);
                const uint32_t one = 0x3F80u << (16 * (d & 1u));
#pragma unroll
                for (int q = 0; q < 4; q++)
                    act[g][4 * s + q] = (d < 8u && (d >> 1) == (uint32_t)q) ? one : 0u;
            }
        // ---- stem: its block landed (own DMA + barrier); prefetch conv1 into the other buffer
        __builtin_amdgcn_s_waitcnt(0);                 // vmcnt(0) lgkmcnt(0): this wave's DMA done
        __syncthreads();
        stage_block(blob + kStemBlock * 64, buf(cur ^ 1), kConvBlock, wave, lane);
        layer<2, false, false>(buf(cur), reinterpret_cast<const float *>(buf(cur) + kStemFrags * 64), act, res, acc,
                               lane, h, keep_l, keep_r);
        // ---- 8 convs = 4 basic blocks
        for (int L = 0; L < kConvLayers; ++L) {
            cur ^= 1;
            if (R48_RN_ABL != 1 && R48_RN_ABL != 2) {
                __builtin_amdgcn_s_waitcnt(0);
                __syncthreads();
            }
            // prefetch the next layer, or the next tile's stem
            if (R48_RN_ABL == 2) {
            } else if (L + 1 < kConvLayers)
                stage_block(blob + (kStemBlock + (L + 1) * kConvBlock) * 64, buf(cur ^ 1), kConvBlock, wave, lane);
            else if (tile + gridDim.x < tiles)
                stage_block(blob, buf(cur ^ 1), kStemBlock, wave, lane);
            const float *bias = reinterpret_cast<const float *>(buf(cur) + kConvFrags * 64);
            if ((L & 1) == 0)                        // first conv of a block: keep its input for the skip
                layer<4, false, true>(buf(cur), bias, act, res, acc, lane, h, keep_l, keep_r);
            else
                layer<4, true, false>(buf(cur), bias, act, res, acc, lane, h, keep_l, keep_r);
        }
        // ---- head: per-lane partial dot products over the lane's 32 channels, then sum over the
        // 16 cells (DPP row) and the two halves
        const uint16_t *hw = head_lds + (cell * 2 + h) * 4 * 32;
#pragma unroll
        for (int g = 0; g < G; g++) {
            float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const float lo = bf_lo(act[g][k]), hi = bf_hi(act[g][k]);
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    part[a] += lo * __uint_as_float((uint32_t)hw[a * 32 + 2 * k] << 16);
                    part[a] += hi * __uint_as_float((uint32_t)hw[a * 32 + 2 * k + 1] << 16);
                }
            }
            float qv[4];
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const float r = row16_sum(part[a]);
                qv[a] = r + __shfl_xor(r, 32);
            }
            const int64_t b = b0 + 2 * g + ((lane & 31) >> 4);
            if (lane < 32 && cell == 0 && b < n) {
                const float4 q = make_float4(qv[0] + hb0, qv[1] + hb1, qv[2] + hb2, qv[3] + hb3);
                if (q_out)
                    reinterpret_cast<float4 *>(q_out)[b] = q;
                if (actions) {
                    const uint64_t gid = (uint64_t)(gid0 + b);
                    uint32_t w[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), ctr, kEgreedyTag};
                    r48::philox4x32_10(w, k0, k1);
                    const float u = (float)(w[0] >> 8) * (1.0f / 16777216.0f);
                    uint32_t am = 0;
                    float mx = q.x;
                    if (q.y > mx) { mx = q.y; am = 1; }
                    if (q.z > mx) { mx = q.z; am = 2; }
                    if (q.w > mx) { am = 3; }
                    actions[b] = (int8_t)(u < eps ? (w[1] >> 30) : am);
                }
            }
        }
        cur ^= 1;                                      // the next tile's stem was staged into the other buffer
    }
    __builtin_amdgcn_s_waitcnt(0);                     // no DMA left in flight at exit
}

// ---- weight packing for k_resnet_q (rein48_amd/dqn/fused.py pack_resnet, one launch instead of ~50
// PyTorch ops per repack). ptr[6 L + {0..5}] = conv L's weight [co][ci][3][3], bias [co], BN gamma,
// beta, running mean, running var (gamma NULL: no BN); ptr[54], ptr[55] = head weight [4][1024],
// bias [4]. Folding as ResNet10Q.folded(): s = gamma / sqrt(var + eps), w s, (b - mean) s + beta,
// in f32 with correctly rounded sqrt and division, then bf16 (RNE): the layout is exactly the
// PyTorch packing's; the BN scale may differ from PyTorch's in the last f32 ulp (tests/test_dqn_gpu.py).
__device__ __forceinline__ float bn_scale(const float *const *p, int L, int co, float eps)
{
    const float *g = p[6 * L + 2];
    return g ? __fdiv_rn(g[co], __fsqrt_rn(__fadd_rn(p[6 * L + 5][co], eps))) : 1.0f;
}

__global__ __launch_bounds__(256) void k_resnet_pack(const float *const *__restrict__ p, float eps,
                                                      uint16_t *__restrict__ blob, uint16_t *__restrict__ head_w,
                                                      float *__restrict__ head_b)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;     // bf16 element of the blob
    constexpr int64_t kBlobElems = (int64_t)kBlobFrags * 512;
    if (e < kBlobElems) {
        const int frag = (int)(e / 512), lane = (int)(e % 512) / 8, j = (int)(e % 8);
        const int r = lane & 31, h = lane >> 5;
        int L, f, nch, ci_n;
        if (frag < kStemBlock) {
            L = 0, f = frag, nch = 2, ci_n = 18;
        } else {
            L = 1 + (frag - kStemBlock) / kConvBlock, f = (frag - kStemBlock) % kConvBlock, nch = 4, ci_n = 64;
        }
        const int nfrag = 9 * nch * 2;
        uint16_t out;
        if (f == nfrag) {   // bias fragment: 64 f32 (folded bias) then zeros, as bf16 pairs
            const int word = (int)(e % 512) / 2, half = (int)(e % 2);
            float v = 0.0f;
            if (word < 64) {
                const float sc = bn_scale(p, L, word, eps);
                const float b = p[6 * L + 1][word];
                // separate correctly rounded ops, as PyTorch's two elementwise kernels (no FMA)
                v = p[6 * L + 2] ? __fadd_rn(__fmul_rn(__fsub_rn(b, p[6 * L + 4][word]), sc), p[6 * L + 3][word]) : b;
            }
            out = (uint16_t)(__float_as_uint(v) >> (16 * half));
        } else {
            const int m = f & 1, sk = (f >> 1) % nch, t = (f >> 1) / nch;
            const int co = 32 * m + r;
            const int ci = nch == 2 ? 16 * sk + 8 * h + j : 16 * sk + 8 * (j >> 2) + 4 * h + (j & 3);
            float v = 0.0f;
            if (ci < ci_n)
                v = __fmul_rn(p[6 * L][((int64_t)co * ci_n + ci) * 9 + t], bn_scale(p, L, co, eps));
            const __bf16 bv = (__bf16)v;
            out = __builtin_bit_cast(uint16_t, bv);
        }
        blob[e] = out;
        return;
    }
    const int64_t k = e - kBlobElems;                                 // head weight element
    if (k < kHeadBf16) {
        const int cell = (int)(k / 256), hh = (int)(k / 128) % 2, a = (int)(k / 32) % 4, idx = (int)(k % 32);
        const int kk = idx >> 1, ee = idx & 1, sq = kk >> 2, q = kk & 3, m = sq >> 1;
        const int i = 8 * (sq & 1) + 2 * q + ee;
        const int ci = 32 * m + 8 * (i >> 2) + 4 * hh + (i & 3);
        const __bf16 bv = (__bf16)p[54][a * 1024 + cell * 64 + ci];
        head_w[k] = __builtin_bit_cast(uint16_t, bv);
        return;
    }
    if (k - kHeadBf16 < 4)
        head_b[k - kHeadBf16] = p[55][k - kHeadBf16];
}

int fail(int code, const char *msg)
{
    r48::set_last_error(msg);
    return code;
}

}  // namespace

extern "C" {

int r48_resnet_q_forward(const int8_t *boards, int64_t n, const void *wblob, const void *head_w, const float *head_b,
                         float *q, int8_t *actions, float eps, uint64_t seed, int64_t gid0, uint32_t ctr, void *stream)
{
    if (!boards || !wblob || !head_w || !head_b || n < 0 || gid0 < 0 || (!q && !actions))
        return fail(R48_EINVAL, "NULL argument, n/gid0 < 0, or neither q nor actions requested");
    if (((uintptr_t)wblob & 15u) || ((uintptr_t)head_w & 15u) || (q && ((uintptr_t)q & 15u)))
        return fail(R48_EINVAL, "wblob, head_w and q must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int64_t tiles = (n + kBoardsPerTile - 1) / kBoardsPerTile;
    const int grid = (int)(tiles < cus ? tiles : cus);
    const size_t lds = (size_t)(2 * kBufFrags * 64) * 16 + kHeadBf16 * 2;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_resnet_q),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_resnet_q, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, boards, n,
                       reinterpret_cast<const uint4 *>(wblob), reinterpret_cast<const uint4 *>(head_w), head_b, q,
                       actions, eps, (uint32_t)seed, (uint32_t)(seed >> 32), gid0, ctr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        r48::set_last_error(std::string("k_resnet_q: ") + hipGetErrorString(e));
        return R48_EHIP;
    }
    return R48_OK;
}

int64_t r48_resnet_q_blob_bytes(void) { return (int64_t)kBlobFrags * 1024; }

int r48_resnet_pack(const float *const *ptrs, float bn_eps, void *wblob, void *head_w, float *head_b, void *stream)
{
    if (!ptrs || !wblob || !head_w || !head_b || ((uintptr_t)wblob & 15u) || ((uintptr_t)head_w & 15u))
        return fail(R48_EINVAL, "r48_resnet_pack: NULL or misaligned argument");
    const int64_t total = (int64_t)kBlobFrags * 512 + kHeadBf16 + 4;
    hipLaunchKernelGGL(k_resnet_pack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ptrs,
                       bn_eps, (uint16_t *)wblob, (uint16_t *)head_w, head_b);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        r48::set_last_error(std::string("k_resnet_pack: ") + hipGetErrorString(e));
        return R48_EHIP;
    }
    return R48_OK;
}

}  // extern "C"
