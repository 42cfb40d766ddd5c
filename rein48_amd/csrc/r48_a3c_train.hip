// r48_a3c_train.hip -- fused A3C update for the CNN policy on gfx950 MFMA (BASELINE configs 3-4).
//
// One pass over T x n training states computes the gradient of the A3C loss of
// rein48_amd/a3c/losses.py (algorithm/a3c/a3c.py:99-123: textbook, or the reference's literal
// [B,B,4]-broadcast actor loss) w.r.t. every parameter of rein48_amd/a3c/nets.py:ActorCriticCNN,
// without writing a single activation to HBM. Per row: 16 board bytes + action + target + weight
// in, nothing out; per wave: one gradient record at the end.
//
// Every wave owns its 32-row tiles and the WHOLE weight gradient (173 accumulator registers in
// AGPRs), so waves never share rows: no workgroup barrier in the main loop, and LDS holds only
// the weights (shared, read-only) and each wave's own images.
//
// Two MFMA orientations. A layer's output computed as D = W . act^T has the rows (training
// states) on the lanes and the features in registers ("orientation 1": what the next layer's
// contraction over features needs). The same input registers used as the A operand instead give
// D = act . W^T, rows in registers and features on the lanes ("orientation 2": what a contraction
// over rows, i.e. a weight gradient, needs). Rows in registers come in the order
// rho(s, j, h) = 16s + 8(j >> 2) + 4h + (j & 3) of an accumulator packed for k-step s; every
// row-contracting operand below is built in that order, so any two of them pair up.
//
// Per 32-row tile and wave:
//   forward   x -> h1 (9 x 32) -> h2 (4 x 64) -> out (4 logits + value)          89 MFMAs
//             (h2 stored row-major into the wave's image as it is formed)
//   loss      per row: dout = dL/d(logits, value)  (softmax, entropy, td; lane-local)
//   dh2       = Wh^T dout . [h2 > 0]  (orientation 1)                              8 MFMAs
//   dWh, dbh  += h2^T dout            (h2^T read back transposed, ds_read_b64_tr_b16;
//                                      16x16x32 with a selector B operand: 10 of 16 columns)  16 x 16x16x32
//   dh2^T     dh2 stored over the image and read back transposed
//   db2       += sum over rows of dh2^T (16x16x32, selector B)                     16 x 16x16x32
//   per conv1 position R (9):
//     h1^T_R  = relu(x W1_R^T + b1)   (orientation 2, recomputed: no h1 image)      1 MFMA
//     dh1^T_R = sum over the (p, kk) of R: dh2_p W2_kk^T, . [h1^T_R > 0]  (orientation 2)  4 per pair
//     dW2     += dh2_p^T h1^T_R       (every (p, kk) of R, both output halves)      4 per pair
//     dW1,db1 += dh1^T_R x-patch_R    (16x16x32, selector B from the Xt image)     2 x 16x16x32
// = 234 v_mfma_f32_32x32x16_bf16 + 50 v_mfma_f32_16x16x32_bf16 per tile; LDS traffic ~150 KB
// (weights 122, two 16 KB transposes, small images) instead of the four transposes and the
// cross-wave sharing of a slice-per-wave design.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
// The weight-fragment fences (r48_cnn_common.h wfence) also let global memory instructions and LDS
// writes cross here (mask 0x616 instead of 0x406), and the kernel's own phase fences (the epilogue /
// transpose points of conv1 and the dh2 phase) use the same mask instead of a full barrier; the LDS
// fragment reads and the MFMAs keep their order. Bit-identical gradients. PERFORMANCE-NEUTRAL: the
// ~3 % gains first measured for each step were the A/B tool's first-position penalty (the base
// library was always timed first in its process); order-balanced runs put this build and the
// shared-mask one within 0.1 % (profiles/r05/a3c/train/fence_mask_vmem_ab.txt, last section).
#ifndef R48_WFENCE
#define R48_WFENCE 0x616
#endif
#include "r48_cnn_common.h"
#include "r48_host.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using namespace r48cnn;
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define R48_LDS __attribute__((address_space(3)))

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kFragWhT = 8, kFragW2T = 16;
constexpr int kFragsTrain = kFrags + kFragWhT + kFragW2T;    // 65: forward 41 | Wh^T 8 | W2^T 16
constexpr int kOffWhT = kFrags, kOffW2T = kFrags + kFragWhT;
constexpr int kBlock = 32 * 32;
// per-wave slot (bf16 elements):
//   [0, kImg)   image of h2, later of dh2: [32 rows][256 features] in blocks of 32 features,
//               64-byte rows, 8-byte chunk index XOR (row >> 1) & 7
//   kXt         board cells of the tile: [16 cells][32 rows in rho order], then 11 rows of ones
//               and 11 of zeros (the bias and empty columns of dW1's B operand; every lane reads
//               unconditionally and the lane's base address selects cell, ones or zeros)
//   kDt         dout: [5 outputs][32 rows in rho order]
constexpr int kImg = 8 * kBlock;
constexpr int kXt = kImg, kXtOnes = kXt + 16 * 32, kXtZeros = kXtOnes + 11 * 32;
constexpr int kDt = kXtZeros + 11 * 32;
constexpr int kSlot = kDt + 5 * 32;                           // 9568 elements = 19136 B
// gradient record per wave (floats): dW2 [64][128] | db2 [64] | dW1 [32][5] | dWh [5][257] | losses [2]
constexpr int kOffDb2 = 64 * 128, kOffDw1 = kOffDb2 + 64, kOffDwh = kOffDw1 + 32 * 5, kOffLoss = kOffDwh + 5 * 257;
constexpr int kPartial = kOffLoss + 2;                        // 9703
constexpr size_t kLdsWeights = (size_t)(kFragsTrain * 64 + 32) * 16;
constexpr size_t kLds = kLdsWeights + (size_t)kWaves * kSlot * 2;         // 143,520 B
constexpr float kEntropyEps = 1e-5f;                          // a3c.py:114
constexpr float kLn2 = 0.69314718055994531f;

// (conv2 output p, input block kk) pairs grouped by the conv1 position R = kP2[p][kk]
__device__ constexpr int kDh1P[16] = {0, 0, 1, 1, 0, 2, 0, 1, 2, 3, 1, 3, 2, 2, 3, 3};
__device__ constexpr int kDh1K[16] = {0, 1, 0, 1, 2, 0, 3, 2, 1, 0, 3, 1, 2, 3, 2, 3};
__device__ constexpr int kRFirst[10] = {0, 1, 3, 4, 6, 10, 12, 13, 15, 16};   // pairs of R: [kRFirst[R], kRFirst[R+1])

// conv1's 2x2 patch at position R: top-left cell, and tap t's offset from it
__host__ __device__ constexpr int cell_base(int R) { return (R / 3) * 4 + R % 3; }
__host__ __device__ constexpr int tap_off(int t) { return (t >> 1) * 4 + (t & 1); }

// position of row r in a rho-ordered image (the inverse of rho: r = 16s + 8a + 4h + e -> 16s + 8h + 4a + e)
__device__ __forceinline__ int rho_pos(int r) { return 16 * (r >> 4) + 8 * ((r >> 2) & 1) + 4 * ((r >> 3) & 1) + (r & 3); }

// element offset of image (row r, column c): block c >> 5, 64-byte rows, chunk XOR (r >> 1) & 7
__device__ __forceinline__ int img_at(int r, int c)
{
    return (c >> 5) * kBlock + r * 32 + ((((c >> 2) & 7) ^ ((r >> 1) & 7)) << 2) + (c & 3);
}

// Per-lane LDS bases; every access adds a compile-time offset that folds into the DS instruction
struct LaneAddr {
    int st[4];   // stores of image row `col`: chunk columns 8k + 4h
    int tr[2];   // rho-order transposed read (u = 0, 1): rows 8u + 4(g >> 1) + (i >> 2), columns 16(g & 1) + 4(i & 3)
    int xw;      // this lane's row in the rho-ordered images
    int xr;      // dW1 B operand (R = 0, s = 0): cell tap_off(t) of Xt, its ones or its zeros
    int dr;      // dWh B operand (s = 0): output n >> 1 of Dt, or zeros
};

__device__ __forceinline__ LaneAddr lane_addr(int lane)
{
    LaneAddr a;
    const int h = lane >> 5, col = lane & 31, g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; k++)
        a.st[k] = img_at(col, 4 * (2 * k + h));
#pragma unroll
    for (int u = 0; u < 2; u++)
        a.tr[u] = img_at(8 * u + 4 * (g >> 1) + (i >> 2), 16 * (g & 1) + 4 * (i & 3));
    a.xw = rho_pos(col);
    // 16x16x32 selector operands: column n = 2q + b takes lane group g's 16 rows when g & 1 == b
    // (the A fragment's lanes 16b..16b+15 of each half carry features 16b + m), else zeros
    const int n = i, q = n >> 1, b = n & 1, hh = g >> 1;
    const bool sel = (g & 1) == b;
    a.xr = (sel && q < 4 ? kXt + tap_off(q) * 32 : sel && q == 4 ? kXtOnes : kXtZeros) + 8 * hh;
    a.dr = (sel && q < 5 ? kDt + q * 32 : kXtZeros) + 8 * hh;
    return a;
}

__device__ __forceinline__ bf16x8 tr_pair(const uint16_t *p0, const uint16_t *p1)
{
    const i16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((R48_LDS i16x4 *)(p0));
    const i16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((R48_LDS i16x4 *)(p1));
    bf16x8 f;
    __builtin_memcpy(&f, &r0, 8);
    __builtin_memcpy(reinterpret_cast<char *>(&f) + 8, &r1, 8);
    return f;
}

// image block blk (features 32 blk .. +31) transposed: lane (f = lane & 31, h), element j = image
// row rho(s, j, h) -- a 32x32x16 A/B operand indexed by feature with k = rows in rho order
__device__ __forceinline__ bf16x8 trr(const uint16_t *slot, const LaneAddr &la, int blk, int s)
{
    const uint16_t *b = slot + blk * kBlock + 16 * s * 32;     // +16 rows: the swizzle repeats
    return tr_pair(b + la.tr[0], b + la.tr[1]);
}

// store an orientation-1 fragment (elements j = feature cbase + 8(j>>2) + 4h + (j&3), cbase a
// multiple of 16) as image row `col`: two packed 8-byte chunks
__device__ __forceinline__ void store_frag(uint16_t *slot, const LaneAddr &la, int cbase, const bf16x8 &f)
{
    uint4 v;
    __builtin_memcpy(&v, &f, 16);
    uint16_t *b = slot + (cbase >> 5) * kBlock;
    const int s = (cbase >> 4) & 1;
    *reinterpret_cast<uint2 *>(b + la.st[2 * s]) = make_uint2(v.x, v.y);
    *reinterpret_cast<uint2 *>(b + la.st[2 * s + 1]) = make_uint2(v.z, v.w);
}

// ReLU' on packed bf16: d where the (post-ReLU, >= 0) activation is nonzero, else +0, as
// d * min(act, 1) per 16-bit half: one v_pk_min_u16 + one v_pk_mul_lo_u16 per word (in asm: as
// plain code the compiler rewrites the 0/1 product as compares + selects)
__device__ __forceinline__ bf16x8 mask_pk(const bf16x8 &d, const bf16x8 &act)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    uint32_t dw[4], aw[4];
    __builtin_memcpy(dw, &d, 16);
    __builtin_memcpy(aw, &act, 16);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t m;
        asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(aw[q]), "s"(0x00010001u));
        dw[q] = __builtin_bit_cast(uint32_t, (u16x2)(__builtin_bit_cast(u16x2, dw[q]) * __builtin_bit_cast(u16x2, m)));
    }
    bf16x8 f;
    __builtin_memcpy(&f, dw, 16);
    return f;
}

// Gradient accumulation with the accumulator pinned in AGPRs ("+a"), while the activation MFMAs
// (builtins, VGPR form: Makefile FLAGS_r48_a3c_train) keep their results in VGPRs for the
// epilogues. hipcc pads nothing inside asm: the _v forms start with s_nop 1 (an operand may be a
// just-written VGPR); the others take operands that only LDS reads write (tools/
// check_asm_hazards.py verifies both on the compiled code). D -> the next MFMA of the same chain
// taking it whole as C needs no wait; D -> any other reader: the fence after the loop. Not
// volatile: a volatile asm is a scheduling barrier for the LDS reads that feed the next MFMAs.
__device__ __forceinline__ void acc32_v(f32x16 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// the same with the A operand held in AGPRs (dh2^T: only ever an MFMA operand, so it waits in
// the accumulator file and leaves the VGPRs to the in-flight accumulators of the position loop)
__device__ __forceinline__ void acc32_av(f32x16 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "a"(a), "v"(b));
}

__device__ __forceinline__ void acc32_a(f32x16 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "a"(a), "v"(b));
}

__device__ __forceinline__ void acc16_a(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "a"(a), "v"(b));
}

__device__ __forceinline__ void acc16_av(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "a"(a), "v"(b));
}

__device__ __forceinline__ void acc16_v(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ void acc16_lds(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ bf16x8 lds_frag(const uint16_t *p)
{
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

__device__ __forceinline__ bf16x8 splat_frag(uint32_t w)
{
    const uint4 v = make_uint4(w, w, w, w);
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// weight-fragment read-ahead depth of the forward and of the position loop's W2^T stream: 3 fragments
// (3 MFMAs, ~96 cycles) ahead of their MFMA, +4 VGPRs over 2; kernel 19.38-19.43 vs 19.59-19.69 ms per
// 1e8 rows for the round-5 kernel (depth 2), 19.54-19.66 at depth 4, four alternated process-per-library
// rounds, identical gradient digests (profiles/r06/a3c/train/read_ahead_depth_ab.txt)
#ifndef R48_WDEPTH
#define R48_WDEPTH 3
#endif
constexpr int kWDepth = R48_WDEPTH;
struct WStreamD {
    bf16x8 q[kWDepth];
    __device__ __forceinline__ void start(const uint4 *w, int lane)
    {
#pragma unroll
        for (int d = 0; d < kWDepth; d++)
            q[d] = frag_at(w, fwd_frag(d), lane);
    }
    __device__ __forceinline__ bf16x8 step(const uint4 *w, int ahead, int lane)
    {
        const bf16x8 cur = q[0];
#pragma unroll
        for (int d = 0; d + 1 < kWDepth; d++)
            q[d] = q[d + 1];
        q[kWDepth - 1] = frag_at(w, ahead, lane);
        return cur;
    }
};
__host__ __device__ constexpr int fwd_ahead(int i) { return i + kWDepth < kFwdMfmas ? fwd_frag(i + kWDepth) : 0; }

// conv1 as cnn_conv1 (same products, same bits), with the MFMA of position R + 1 issued before the
// epilogue of R (two accumulators in flight) so the pipe runs under the bf16 pack + ReLU
__device__ __forceinline__ void fwd_conv1(const uint4 *w, const float *b, int lane, int h, const bf16x8 &x,
                                          WStreamD &ws, bf16x8 (&h1)[9][2])
{
    const f32x16 b1 = load_bias(b, h);
    bf16x8 wa = ws.step(w, fwd_ahead(0), lane);
    wfence();
    f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, x, b1, 0, 0, 0);
#pragma unroll
    for (int R = 0; R < 9; R++) {
        f32x16 nxt = acc;
        if (R + 1 < 9) {
            wa = ws.step(w, fwd_ahead(R + 1), lane);
            wfence();
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, x, b1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(R48_WFENCE);
        h1[R][0] = acc_to_frag_relu(acc, 0);
        h1[R][1] = acc_to_frag_relu(acc, 1);
        acc = nxt;
    }
}

// conv2 + heads in chain order (as cnn_conv2_heads: chain c = 2p + g is output position p, half g,
// its 8 W2 fragments accumulated in one register set; the 2 head MFMAs of chain c issue after chain
// c + 1), so at most two conv2 accumulators are live and each chain's bf16 pack + ReLU + image store
// runs under the next chain's MFMAs. 89 fragment reads per tile (the grouped order reads 41 but
// needs four accumulators and all of h1 at once: no room for the epilogues to overlap).
__device__ __forceinline__ void fwd_conv2_heads_chain(const uint4 *w, const float *b, int lane, int h,
                                                      const bf16x8 (&h1)[9][2], WStreamD &ws, bf16x8 (&h2)[4][2][2],
                                                      f32x16 &out, uint16_t *img, const LaneAddr &la)
{
    const f32x16 b2[2] = {load_bias(b + 32, h), load_bias(b + 64, h)};
    out = f32x16{};
    f32x16 acc[2];
    int i = 9;
#pragma unroll
    for (int c = 0; c <= 8; c++) {
        if (c < 8) {
            const int p = c >> 1;
            f32x16 a = b2[c & 1];
#pragma unroll
            for (int u = 0; u < 8; u++, i++) {
                const bf16x8 wa = ws.step(w, fwd_ahead(i), lane);
                wfence();
                a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, h1[kP2[p][u >> 1]][u & 1], a, 0, 0, 0);
                wfence();
            }
            acc[c & 1] = a;
        }
        if (c >= 1) {
            const int cp = c - 1, p = cp >> 1, g = cp & 1;
#pragma unroll
            for (int s = 0; s < 2; s++, i++) {
                h2[p][g][s] = acc_to_frag_relu(acc[cp & 1], s);
                store_frag(img, la, 64 * p + 32 * g + 16 * s, h2[p][g][s]);
                const bf16x8 wa = ws.step(w, fwd_ahead(i), lane);
                wfence();
                out = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, h2[p][g][s], out, 0, 0, 0);
                wfence();
            }
        }
    }
}

// SEG: the row weights come per board (seg[b] = {w0, c0, L, 0} of r48_a3c_segments, row t * n_boards + b
// weighted iff t < L; reference loss iff counts != NULL) instead of per row (wn, cm)
template <int MODE, bool SEG>
__global__ __launch_bounds__(kThreads, 1) void k_cnn_train(
    const int8_t *__restrict__ boards, int64_t rows, int64_t n_boards, const int8_t *__restrict__ actions,
    const float *__restrict__ targets, const float *__restrict__ wn, const float *__restrict__ cm,
    const float4 *__restrict__ seg, const float *__restrict__ counts, float beta, const uint4 *__restrict__ wfrag,
    const float *__restrict__ bias, float *__restrict__ partials)
{
    extern __shared__ uint4 lds[];
    // LDS: the 4 wave slots first (small DS offsets), then the weight fragments and biases
    uint16_t *slots = reinterpret_cast<uint16_t *>(lds);
    uint4 *w_lds_base = lds + kWaves * kSlot / 8;                         // kFragsTrain x 1 KiB
    float *b_lds_base = reinterpret_cast<float *>(w_lds_base + kFragsTrain * 64);  // 104 floats
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint16_t *my = slots + wave * kSlot;
    const LaneAddr la = lane_addr(lane);
    stage_lds<kFragsTrain * 64, kThreads>(w_lds_base, wfrag);
    for (int i = threadIdx.x; i < 104; i += kThreads)
        b_lds_base[i] = bias[i];
    // the constant rows of Xt: 11 x 32 ones (bf16 1.0) and 11 x 32 zeros
    for (int i = lane; i < 11 * 32; i += 64) {
        my[kXtOnes + i] = 0x3F80;
        my[kXtZeros + i] = 0;
    }
    __syncthreads();   // the only barrier: waves never share rows

    const f32x16 zero = {};
    const f32x4 zero4 = {};
    // the whole weight gradient of this wave's rows (AGPRs)
    f32x16 dw2[2][4];                              // dW2[32 ot + row][32 kk + lane col]
#pragma unroll
    for (int ot = 0; ot < 2; ot++)
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
            dw2[ot][kk] = zero;
    f32x4 dwh[8];                                  // 16x16 D: [feature 32 ft + 16 b + m][column 2o + b]
#pragma unroll
    for (int ft = 0; ft < 8; ft++)
        dwh[ft] = zero4;
    f32x4 db2 = zero4;                             // [o 32 ot + 16 b + m][column 2 ot + b]
    f32x4 dw1 = zero4;                             // [c 16 b + m][column 2t + b], t = 4: conv1 bias
    float dbh[5] = {0.f, 0.f, 0.f, 0.f, 0.f};      // heads bias, per row lane (half 0)
    float loss_actor = 0.0f, loss_critic = 0.0f;
    // db2's selector B operands: column 2 ot + (g & 1) sums output tile ot's half (g & 1)
    const int g16 = lane >> 4, n16 = lane & 15;
    const uint32_t one2 = 0x3F803F80u;

    const int64_t n_tiles = (rows + 31) / 32;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    const int64_t first = (int64_t)blockIdx.x * kWaves + wave;
    // per-row inputs of the NEXT tile, loaded after the current tile's loss has consumed its own
    // (so the loads' latency hides behind the backward and no wait on them lands mid-tile); every
    // lane loads (no divergent branches around the loads), wt = 0 on padding rows
    struct RowIn {
        uint2 raw;
        float wt, tgt, c;
        int act;
        float4 cnt;
        uint32_t t, L;   // SEG: the row's step (UINT32_MAX when not live) and its segment length
    };
    // SEG: (step, board) of the lane's unclamped row tile * 32 + col, advanced by 32 stride rows per
    // fetch without a division (rows of a prefetch past the end are not live; their board index stays
    // in range)
    const uint32_t nb = (uint32_t)n_boards;
    uint32_t seg_t = 0, seg_b = 0, seg_dt = 0, seg_db = 0;
    if (SEG) {
        const uint32_t u0 = (uint32_t)(first * 32 + col), du = (uint32_t)(stride * 32);
        seg_t = u0 / nb, seg_b = u0 % nb, seg_dt = du / nb, seg_db = du % nb;
    }
    const bool ref = SEG ? counts != nullptr : cm != nullptr;   // wave-uniform
    auto fetch = [&](int64_t tile) {
        RowIn in;
        const int64_t r = std::min<int64_t>(tile, n_tiles - 1) * 32 + col;
        const bool live = r < rows && tile < n_tiles;
        const int64_t rr = r < rows ? r : rows - 1;     // padding lanes compute on a valid row, weight 0
        in.raw = *reinterpret_cast<const uint2 *>(boards + 16 * rr + 8 * h);
        in.tgt = targets[rr];
        in.act = actions[rr] & 3;
        in.c = 0.f, in.cnt = make_float4(0.f, 0.f, 0.f, 0.f);
        if (SEG) {   // raw per-board values: the step test waits for the load in the loss, not here
            const float4 sg = seg[seg_b];
            in.wt = sg.x;
            in.L = (uint32_t)__float_as_int(sg.z);
            in.t = live ? seg_t : 0xFFFFFFFFu;
            if (ref) {
                in.c = sg.y;
                in.cnt = *reinterpret_cast<const float4 *>(counts + 4 * (int64_t)seg_b);
            }
            seg_b += seg_db;
            seg_t += seg_dt;
            if (seg_b >= nb)
                seg_b -= nb, seg_t++;
        } else {
            const float wt = wn[rr];
            in.wt = live ? wt : 0.0f;
            if (ref) {
                const float c = cm[rr];
                in.c = live ? c : 0.0f;
                // row rr belongs to board rr % n_boards (rows are [T][n_boards]); 32-bit when it fits
                const int64_t bidx =
                    rows <= 0xFFFFFFFFll ? (int64_t)((uint32_t)rr % (uint32_t)n_boards) : rr % n_boards;
                in.cnt = *reinterpret_cast<const float4 *>(counts + 4 * bidx);
            }
        }
        return in;
    };
    RowIn next = fetch(first);
    for (int64_t tile = first; tile < n_tiles; tile += stride) {
        const RowIn in = next;
        // weights and biases are re-read from LDS every tile: an opaque zero offset keeps the
        // compiler from hoisting hundreds of registers of loop-invariant fragments out of the loop
        int wofs = 0;
        asm volatile("" : "+s"(wofs));
        const uint4 *w = w_lds_base + wofs;
        const float *bl = b_lds_base + wofs;
        // ---------------- forward (the math of r48_policy.hip k_cnn_forward; conv2 in chain order)
        uint32_t xp[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t wv = q < 2 ? in.raw.x : in.raw.y;
            const int sh = 16 * (q & 1);
            xp[q] = cell_bf16((wv >> sh) & 0xffu, MODE) | (cell_bf16((wv >> (sh + 8)) & 0xffu, MODE) << 16);
        }
        bf16x8 x;
        __builtin_memcpy(&x, xp, 16);
        // Xt: this row's cells 8h..8h+7 at its rho position (dW1's B operand)
#pragma unroll
        for (int j = 0; j < 8; j++)
            my[kXt + (8 * h + j) * 32 + la.xw] = (uint16_t)(xp[j >> 1] >> (16 * (j & 1)));
        bf16x8 h2[4][2][2];
        f32x16 out;
        {
            bf16x8 h1[9][2];
            WStreamD ws;
            ws.start(w, lane);
            fwd_conv1(w, bl, lane, h, x, ws, h1);
            fwd_conv2_heads_chain(w, bl, lane, h, h1, ws, h2, out, my, la);
        }
        // ---------------- loss gradient per row (lane half 0: logits rows 0..3; value in lane + 32)
        // the value (row 4 = lane half 1's first register) into lane half 0: v_permlane32_swap, no LDS
        const float v = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(out[0]),
                                                                          __float_as_uint(out[0]), false, false)[1]) +
                        bl[100];
        float dz[4] = {0.f, 0.f, 0.f, 0.f}, dv = 0.f;
        if (h == 0) {
            const bool on = !SEG || in.t < in.L;
            const float wt = on ? in.wt : 0.0f;
            float z[4], p[4], gr[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                z[k] = out[k] + bl[96 + k];
            const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
            float se = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                p[k] = __expf(z[k] - m);
                se += p[k];
            }
            // native v_log_f32 (log2): every argument is >= 1 (se) or >= 1e-5 (p + eps), no denormal path
            const float inv = __builtin_amdgcn_rcpf(se), lse = m + kLn2 * __builtin_amdgcn_logf(se);
            float H = 0.f, gbar = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                p[k] *= inv;
                const float lq = kLn2 * __builtin_amdgcn_logf(p[k] + kEntropyEps);
                H -= p[k] * lq;
                gr[k] = -(lq + p[k] * __builtin_amdgcn_rcpf(p[k] + kEntropyEps));     // dH/dp_k
                gbar += p[k] * gr[k];
            }
            const float td = in.tgt - v;
            const int a = in.act;
            if (ref) {   // reference: -beta wn H - cm sum_k c_k log p_k  (losses.py, a3c.py:110-116)
                const float c = on ? in.c : 0.0f;
                const float4 cnt = in.cnt;
                const float ck[4] = {cnt.x, cnt.y, cnt.z, cnt.w}, C = cnt.x + cnt.y + cnt.z + cnt.w;
                float sa = 0.f;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    dz[k] = -beta * wt * p[k] * (gr[k] - gbar) - c * (ck[k] - p[k] * C);
                    sa += ck[k] * (z[k] - lse);
                }
                loss_actor += -beta * wt * H - c * sa;
            } else {    // textbook: -wn (beta H + td log p[a]), td constant for the actor
#pragma unroll
                for (int k = 0; k < 4; k++)
                    dz[k] = -wt * (beta * p[k] * (gr[k] - gbar) + td * ((k == a ? 1.0f : 0.0f) - p[k]));
                loss_actor += -wt * (beta * H + td * (z[a] - lse));
            }
            dv = -2.0f * wt * td;                             // critic = wn td^2
            loss_critic += wt * td * td;
#pragma unroll
            for (int k = 0; k < 4; k++)
                dbh[k] += dz[k];
            dbh[4] += dv;
            // Dt: dout of this row at its rho position (dWh's B operand)
            const float dd[5] = {dz[0], dz[1], dz[2], dz[3], dv};
#pragma unroll
            for (int o = 0; o < 5; o++)
                my[kDt + o * 32 + la.xw] = __builtin_bit_cast(uint16_t, (__bf16)dd[o]);
        }
        next = fetch(tile + stride);      // the current tile's row inputs are consumed
        // dout as the B operand: k = 8h + j = output o (half 0: dz0..3, dv; half 1: 0)
        bf16x8 dout;
        {
            const uint32_t d0 = pack_bf16x2(dz[0], dz[1]), d1 = pack_bf16x2(dz[2], dz[3]), d2 = pack_bf16x2(dv, 0.f);
            uint32_t pk[4] = {h == 0 ? d0 : 0u, h == 0 ? d1 : 0u, h == 0 ? d2 : 0u, 0u};
            __builtin_memcpy(&dout, pk, 16);
        }
        // ---------------- dh2 = Wh^T dout . [h2 > 0] (orientation 1; h2 dies here), and under it:
        //   dWh[o][f] += sum over rows of h2^T[f] dout[o]  (A = h2^T read back transposed from the
        //     image, B = Dt with the column selector; 16x16x32, 8 feature tiles x 2 row steps)
        //   the dh2 image, block m written over h2 block m once its last dWh read is issued (one
        //     wave's LDS operations execute in order), then read back transposed: dh2^T (AGPRs)
        //   db2 += row sums of dh2^T (16x16x32 with a selector B), two blocks behind
        // Per step m (= 2p + g = feature block): dh2 MFMA m + 1, two dWh MFMAs (their h2^T operands
        // read two MFMAs ahead), two db2 MFMAs, then the epilogue of m (bf16 pack + ReLU') -- the
        // pipe runs under every epilogue.
        bf16x8 dh2[4][2][2];
        bf16x8 dh2t[4][2][2];
        {
            const bf16x8 sel0 = splat_frag(n16 == (g16 & 1) ? one2 : 0u);
            const bf16x8 sel1 = splat_frag(n16 == 2 + (g16 & 1) ? one2 : 0u);
            const bf16x8 bd0 = lds_frag(my + la.dr), bd1 = lds_frag(my + la.dr + 16);
            bf16x8 A = trr(my, la, 0, 0), A1 = trr(my, la, 0, 1);
            f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w, kOffWhT, lane), dout, zero, 0, 0, 0);
            bf16x8 q = frag_at(w, kOffWhT + 1, lane);
#pragma unroll
            for (int m = 0; m <= 9; m++) {              // m = 2p + g = the feature block
                f32x16 nxt = acc;
                if (m + 1 < 8) {
                    const bf16x8 wa = q;
                    if (m + 2 < 8)
                        q = frag_at(w, kOffWhT + m + 2, lane);
                    wfence();
                    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, dout, zero, 0, 0, 0);
                }
                if (m < 8) {
#pragma unroll
                    for (int k = 2 * m; k < 2 * m + 2; k++) {
                        const bf16x8 An = k + 2 < 16 ? trr(my, la, (k + 2) >> 1, (k + 2) & 1) : A;
                        acc16_lds(dwh[m], A, (k & 1) ? bd1 : bd0);
                        A = A1;
                        A1 = An;
                    }
                }
                if (m >= 2) {                           // db2 of block m - 2 (read at step m - 2)
                    const int b = m - 2;
#pragma unroll
                    for (int s = 0; s < 2; s++) {
                        if (b == 0 && s == 0)
                            acc16_av(db2, dh2t[b >> 1][b & 1][s], sel0);
                        else if (b == 1 && s == 0)
                            acc16_av(db2, dh2t[b >> 1][b & 1][s], sel1);
                        else
                            acc16_a(db2, dh2t[b >> 1][b & 1][s], (b & 1) ? sel1 : sel0);
                    }
                }
                __builtin_amdgcn_sched_barrier(R48_WFENCE);
                if (m < 8) {
                    const int p = m >> 1, g = m & 1;
                    dh2[p][g][0] = mask_pk(acc_to_frag(acc, 0), h2[p][g][0]);
                    dh2[p][g][1] = mask_pk(acc_to_frag(acc, 1), h2[p][g][1]);
                    store_frag(my, la, 64 * p + 32 * g, dh2[p][g][0]);
                    store_frag(my, la, 64 * p + 32 * g + 16, dh2[p][g][1]);
                    dh2t[p][g][0] = trr(my, la, m, 0);
                    dh2t[p][g][1] = trr(my, la, m, 1);
                    __builtin_amdgcn_sched_barrier(R48_WFENCE);
                }
                acc = nxt;
            }
        }
        // ---------------- per conv1 position R: h1^T_R, dh1^T_R, dW2, dW1. Software-pipelined: the
        // h1^T MFMA of R + 1 and the dh1^T epilogue + dW1 MFMAs of R - 1 are issued in the shadow of
        // R's first dh1 MFMA, so no MFMA waits on an epilogue at a position boundary; the dW2 MFMAs
        // of R alternate with the dh1 chain's, so no two consecutive MFMAs share an accumulator
        {
            const float b1c = bl[col];
            f32x16 b1s;
#pragma unroll
            for (int r = 0; r < 16; r++)
                b1s[r] = b1c;
            // W2^T fragments (B operands of dh1^T) stream kWDepth MFMAs ahead over the 64 (pair, g, s)
            auto w2t = [](int m) { return kOffW2T + (kDh1K[m >> 2] * 2 + ((m >> 1) & 1)) * 2 + (m & 1); };
            bf16x8 qw[kWDepth];
#pragma unroll
            for (int d = 0; d < kWDepth; d++)
                qw[d] = frag_at(w, w2t(d), lane);
            // h1^T_R: A = x (rows x cells), B = W1_R^T (the W1 fragment's registers), C = b1 per lane
            f32x16 a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, frag_at(w, 0, lane), b1s, 0, 0, 0);
            f32x16 dprev = zero;
            bf16x8 hprev[2], xprev[2];
#pragma unroll
            for (int R = 0; R < 9; R++) {
                const bf16x8 xb0 = lds_frag(my + la.xr + cell_base(R) * 32);
                const bf16x8 xb1 = lds_frag(my + la.xr + cell_base(R) * 32 + 16);
                const bf16x8 w1n = frag_at(w, R + 1 < 9 ? R + 1 : 0, lane);
                bf16x8 h1t[2], t0, t1;
                f32x16 d = zero, a1n = a1;
                // (1) the dh1^T chain of R (independent of h1^T_R), interleaved with (2); the h1^T
                // epilogue of R and the dh1^T epilogue of R - 1 run under it, the h1^T MFMA of R + 1
                // issues after its first
#pragma unroll
                for (int m = 4 * kRFirst[R]; m < 4 * kRFirst[R + 1]; m++) {
                    const int n = m >> 2, p = kDh1P[n], g = (m >> 1) & 1, s = m & 1;
                    const int first = 4 * kRFirst[R];
                    const bf16x8 wb = qw[0];
#pragma unroll
                    for (int d = 0; d + 1 < kWDepth; d++)
                        qw[d] = qw[d + 1];
                    if (m + kWDepth < 64)
                        qw[kWDepth - 1] = frag_at(w, w2t(m + kWDepth), lane);
                    wfence();
                    d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dh2[p][g][s], wb, d, 0, 0, 0);
                    if (m == first && R + 1 < 9)
                        a1n = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w1n, b1s, 0, 0, 0);
                    wfence();
                    if (m == first) {
                        h1t[0] = acc_to_frag_relu(a1, 0);
                        h1t[1] = acc_to_frag_relu(a1, 1);
                    }
                    if (m == first + 1 && R > 0) {
                        t0 = mask_pk(acc_to_frag(dprev, 0), hprev[0]);
                        t1 = mask_pk(acc_to_frag(dprev, 1), hprev[1]);
                    }
                    // (2) interleaved: dW2[ot = g'][kk'] += dh2_p'^T (o-tile g', row step s') x
                    // h1^T_R (row step s') for step m - 1 of R, between two MFMAs of the dh1 chain
                    if (m > first) {
                        const int mp = m - 1, np = mp >> 2, pp = kDh1P[np], kp = kDh1K[np];
                        const int gp = (mp >> 1) & 1, sp = mp & 1;
                        if (mp < first + 2)   // the first may follow the h1^T epilogue closely
                            acc32_av(dw2[gp][kp], dh2t[pp][gp][sp], h1t[sp]);
                        else
                            acc32_a(dw2[gp][kp], dh2t[pp][gp][sp], h1t[sp]);
                    }
                    wfence();
                }
                if (R > 0) {
                    acc16_v(dw1, t0, xprev[0]);
                    acc16_v(dw1, t1, xprev[1]);
                }
                {   // the last dW2 MFMA of R
                    const int mp = 4 * kRFirst[R + 1] - 1, np = mp >> 2, pp = kDh1P[np], kp = kDh1K[np];
                    const int gp = (mp >> 1) & 1, sp = mp & 1;
                    acc32_a(dw2[gp][kp], dh2t[pp][gp][sp], h1t[sp]);
                }
                dprev = d;
                hprev[0] = h1t[0], hprev[1] = h1t[1];
                xprev[0] = xb0, xprev[1] = xb1;
                a1 = a1n;
            }
            const bf16x8 t0 = mask_pk(acc_to_frag(dprev, 0), hprev[0]);
            const bf16x8 t1 = mask_pk(acc_to_frag(dprev, 1), hprev[1]);
            acc16_v(dw1, t0, xprev[0]);
            acc16_v(dw1, t1, xprev[1]);
        }
    }

    // ---------------- flush: this wave's gradient record straight to HBM. acc fence: 24 wait
    // states between the last accumulating MFMA and any other reader of its AGPRs
    asm volatile("s_nop 15\n\ts_nop 7"
                 : "+a"(dw2[0][0]), "+a"(dw2[0][1]), "+a"(dw2[0][2]), "+a"(dw2[0][3]), "+a"(dw2[1][0]),
                   "+a"(dw2[1][1]), "+a"(dw2[1][2]), "+a"(dw2[1][3]), "+a"(db2), "+a"(dw1), "+a"(dwh[0]),
                   "+a"(dwh[1]), "+a"(dwh[2]), "+a"(dwh[3]), "+a"(dwh[4]), "+a"(dwh[5]), "+a"(dwh[6]),
                   "+a"(dwh[7]));
    float *rec = partials + ((int64_t)blockIdx.x * kWaves + wave) * kPartial;
    // dW2: 32x32 D = [o (row 8(i>>2) + 4h + (i&3))][c = lane col]
#pragma unroll
    for (int ot = 0; ot < 2; ot++)
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
#pragma unroll
            for (int i = 0; i < 16; i++)
                rec[(32 * ot + 8 * (i >> 2) + 4 * h + (i & 3)) * 128 + 32 * kk + col] = dw2[ot][kk][i];
    // 16x16 D tiles: column n16, rows 4 g16 + i
    {
        const int q = n16 >> 1, b = n16 & 1;
        if (n16 < 4) {
#pragma unroll
            for (int i = 0; i < 4; i++)
                rec[kOffDb2 + 32 * q + 16 * b + 4 * g16 + i] = db2[i];
        }
        if (n16 < 10) {
#pragma unroll
            for (int i = 0; i < 4; i++)
                rec[kOffDw1 + (16 * b + 4 * g16 + i) * 5 + q] = dw1[i];
#pragma unroll
            for (int ft = 0; ft < 8; ft++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    rec[kOffDwh + q * 257 + 32 * ft + 16 * b + 4 * g16 + i] = dwh[ft][i];
        }
    }
    float red[7] = {dbh[0], dbh[1], dbh[2], dbh[3], dbh[4], loss_actor, loss_critic};
#pragma unroll
    for (int k = 0; k < 7; k++)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1)
            red[k] += __shfl_xor(red[k], off);
    if (lane == 0) {
#pragma unroll
        for (int o = 0; o < 5; o++)
            rec[kOffDwh + o * 257 + 256] = red[o];
        rec[kOffLoss] = red[5];
        rec[kOffLoss + 1] = red[6];
    }
}

// fixed-order sum of the per-wave records in two passes: pass 1 sums the records of group g
// (records g, g + kGroups, ...) per output (kGroups x 38 blocks instead of 38 reading all 1024
// records each), pass 2 sums the kGroups group sums in order -- deterministic
constexpr int kGroups = 32;

__global__ __launch_bounds__(256) void k_reduce_groups(const float *__restrict__ partials, int64_t n_rec,
                                                       float *__restrict__ group_sums)
{
    const int k = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
    if (k >= kPartial)
        return;
    float s = 0.f;
    for (int64_t w = g; w < n_rec; w += kGroups)
        s += partials[w * kPartial + k];
    group_sums[(int64_t)g * kPartial + k] = s;
}

__global__ __launch_bounds__(256) void k_reduce(const float *__restrict__ group_sums, float *__restrict__ out)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= kPartial)
        return;
    float s = 0.f;
    for (int g = 0; g < kGroups; g++)
        s += group_sums[(int64_t)g * kPartial + k];
    out[k] = s;
}

int fail(int code, const std::string &msg)
{
    r48::set_last_error(msg);
    return code;
}

// the persistent grid: one workgroup per CU of the stream's device, at most kMaxGrid (the MI355X's
// 256 CUs) -- the per-wave record workspace (r48_cnn_train_workspace_floats) is sized for kMaxGrid,
// so it covers any device (a compute partition with fewer CUs launches fewer workgroups, each
// walking more tiles; the reduction sums exactly the records the launch wrote)
constexpr int kMaxGrid = 256;
constexpr int grid_size() { return kMaxGrid; }

int cnn_train_launch(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions, const float *targets,
                     const float *wn, const float *cm, const float *seg, const float *counts, float beta, int32_t mode,
                     const void *wfrag, const float *bias, float *workspace, float *grad, void *stream)
{
    const int cus = r48::device_cus(r48::stream_device((hipStream_t)stream));
    const int grid = cus < kMaxGrid ? cus : kMaxGrid;
    const size_t lds = kLds;
    // one instantiation per input encoding (no per-cell branch); each needs the LDS opt-in once
    auto kern = seg ? (mode == R48_FEAT_VALUES ? k_cnn_train<R48_FEAT_VALUES, true> : k_cnn_train<R48_FEAT_EXPONENTS, true>)
                    : (mode == R48_FEAT_VALUES ? k_cnn_train<R48_FEAT_VALUES, false> : k_cnn_train<R48_FEAT_EXPONENTS, false>);
    if (!r48::ensure_dynamic_lds(reinterpret_cast<const void *>(kern), (int)lds, r48::stream_device((hipStream_t)stream)))
        return R48_EHIP;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, boards, rows, n_boards, actions,
                       targets, wn, cm, (const float4 *)seg, counts, beta, (const uint4 *)wfrag, bias, workspace);
    // the group sums go after the records in the workspace (r48_cnn_train_workspace_floats)
    float *group_sums = workspace + (int64_t)kMaxGrid * kWaves * kPartial;
    hipLaunchKernelGGL(k_reduce_groups, dim3((kPartial + 255) / 256, kGroups), dim3(256), 0, (hipStream_t)stream,
                       workspace, (int64_t)grid * kWaves, group_sums);
    hipLaunchKernelGGL(k_reduce, dim3((kPartial + 255) / 256), dim3(256), 0, (hipStream_t)stream, group_sums, grad);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string("k_cnn_train: ") + hipGetErrorString(e));
    return R48_OK;
}
}  // namespace

extern "C" {

// per-wave records + the reduction's kGroups group sums
int64_t r48_cnn_train_workspace_floats(void) { return ((int64_t)grid_size() * kWaves + kGroups) * kPartial; }

int64_t r48_cnn_train_grad_floats(void) { return kPartial; }

int r48_cnn_train_grad(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                       const float *targets, const float *wn, const float *cm, const float *counts, float beta,
                       int32_t mode, const void *wfrag, const float *bias, float *workspace, float *grad,
                       void *stream)
{
    if (!boards || !actions || !targets || !wn || !wfrag || !bias || !workspace || !grad || rows < 1 ||
        n_boards < 1 || (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS) || (cm && !counts))
        return fail(R48_EINVAL, "NULL argument, rows/n_boards < 1, bad mode, or cm without counts");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(wfrag) |
         reinterpret_cast<uintptr_t>(counts)) & 15u)
        return fail(R48_EINVAL, "boards, wfrag and counts must be 16-byte aligned");
    return cnn_train_launch(boards, rows, n_boards, actions, targets, wn, cm, nullptr, counts, beta, mode, wfrag, bias,
                            workspace, grad, stream);
}

int r48_cnn_train_grad_seg(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                           const float *targets, const float *seg, const float *counts, float beta, int32_t mode,
                           const void *wfrag, const float *bias, float *workspace, float *grad, void *stream)
{
    if (!boards || !actions || !targets || !seg || !wfrag || !bias || !workspace || !grad || rows < 1 ||
        n_boards < 1 || n_boards > 0x7FFFFFFF || (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS))
        return fail(R48_EINVAL, "NULL argument, rows/n_boards < 1, n_boards >= 2^31 or bad mode");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(wfrag) | reinterpret_cast<uintptr_t>(seg) |
         reinterpret_cast<uintptr_t>(counts)) & 15u)
        return fail(R48_EINVAL, "boards, wfrag, seg and counts must be 16-byte aligned");
    return cnn_train_launch(boards, rows, n_boards, actions, targets, nullptr, nullptr, seg, counts, beta, mode, wfrag,
                            bias, workspace, grad, stream);
}

}  // extern "C"
