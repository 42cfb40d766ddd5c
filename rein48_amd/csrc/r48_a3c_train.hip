// r48_a3c_train.hip -- fused A3C update for the CNN policy on gfx950 MFMA (BASELINE configs 3-4).
//
// One pass over T x n training states computes the gradient of the A3C loss of
// rein48_amd/a3c/losses.py (algorithm/a3c/a3c.py:99-123: textbook, or the reference's literal
// [B,B,4]-broadcast actor loss) w.r.t. every parameter of rein48_amd/a3c/nets.py:ActorCriticCNN,
// without writing a single activation to HBM (the PyTorch path streams ~115 GB of activations
// and their gradients per 10M states). Per row: 16 board bytes + action + target + weight in,
// nothing out; per wave: one partial-gradient record at the end.
//
// Per 32-row tile and wave (rows on the MFMA column, as in r48_policy.hip):
//   forward   x -> h1 (9 x 32) -> h2 (4 x 64) -> out (4 logits + value)        89 MFMAs
//             (bias preloaded as the MFMA accumulator, ReLU as an int16 max on the packed bf16)
//   loss      per row: d out = dL/d(logits, value)   (softmax, entropy, td; lane-local)
//   backward  dh2 = Wh^T dout . [h2 > 0]                                          8 MFMAs
//             dh1 = W2^T dh2 . [h1 > 0]      (conv2 transposed, shared over positions) 64 MFMAs
//             (ReLU' applied to the packed bf16 gradient: d * min(h, 1) per 16-bit half)
//   weights   dWh = dout h2^T, dW2 = dh2 h1^T, dW1 = dh1 x^T (+ biases by a ones operand):
//             these contract over ROWS, so rows move to the MFMA K dimension: every lane stores
//             its row's activations / gradients as packed 8-byte chunks into its wave's LDS slot,
//             a [row][feature] image read back transposed with ds_read_b64_tr_b16 (gfx950).
//
// The four waves of a workgroup SHARE their slots: after a barrier every wave contracts over all
// 4 x 32 rows, but only for its own slice of the weight gradient (wave w: dW2 input block kk = w,
// dWh features 64w..64w+63, one (patch, half) pair of db2), so each wave's accumulators are a
// quarter of the full gradient and fit in registers next to the activations. dW1 is contracted
// over the wave's own slot. Images are 32-row x 32-column blocks of 64-byte rows with the 8-byte
// chunk XOR-swizzled by (row >> 1) & 7: the 16-row column stores (ds_write_b64) and the 4-row
// transposed reads are both bank-conflict free. Each wave writes one partial record (staged in
// LDS); k_reduce sums the records in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_cnn_common.h"

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
// per-wave slot (bf16 elements): 10 image blocks of 32 rows x 32 columns
//   phase A: h2 (blocks 0-7: feature 32b + c) | dout [5][32 rows] at kDoutOff
//   phase B half ph: dh2 of patches 2ph, 2ph+1 (blocks 0-3) | h1 positions 3ph..3ph+5 (blocks 4-9)
//   phase C: dh1 (blocks 0-8: position R) | x [16 cells][32 rows] at kXOff
constexpr int kBlock = 32 * 32;
constexpr int kSlot = 10 * kBlock;
constexpr int kDoutOff = 8 * kBlock, kXOff = 9 * kBlock;
// partial record per wave (floats): dW2 [64][128] | db2 [64] | dW1 [32][5] | dWh [5][257] | losses [2]
constexpr int kOffDb2 = 64 * 128, kOffDw1 = kOffDb2 + 64, kOffDwh = kOffDw1 + 32 * 5, kOffLoss = kOffDwh + 5 * 257;
constexpr int kPartial = kOffLoss + 2;                        // 9703
constexpr size_t kLdsWeights = (size_t)(kFragsTrain * 64 + 32) * 16;
constexpr size_t kLdsLoop = kLdsWeights + (size_t)kWaves * kSlot * 2;     // 148992 B
constexpr size_t kLdsFlush = (size_t)kWaves * kPartial * 4;              // 155248 B (records staged)
constexpr size_t kLds = kLdsLoop > kLdsFlush ? kLdsLoop : kLdsFlush;
constexpr float kEntropyEps = 1e-5f;                          // a3c.py:114
// ablation knob for tools/exp_train_ablate.py (wrong gradients when nonzero; never in the product
// build): bit 0 drops phase A, bit 1 phase B, bit 2 dh1 + phase C (7 leaves forward + loss)
#ifndef R48_TRAIN_SKIP
#define R48_TRAIN_SKIP 0
#endif
constexpr int kSkip = R48_TRAIN_SKIP;
// ablation knob (timing only, wrong gradients): R48_TRAIN_NOBAR drops the per-tile workgroup
// barriers around the shared-slot contractions
#ifndef R48_TRAIN_NOBAR
#define R48_TRAIN_NOBAR 0
#endif
__device__ __forceinline__ void tile_barrier()
{
    if (!R48_TRAIN_NOBAR)
        __syncthreads();
}

// dh1's (conv2 output p, input block kk) pairs grouped by the conv1 position R = kP2[p][kk]
__device__ constexpr int kDh1P[16] = {0, 0, 1, 1, 0, 2, 0, 1, 2, 3, 1, 3, 2, 2, 3, 3};
__device__ constexpr int kDh1K[16] = {0, 1, 0, 1, 2, 0, 3, 2, 1, 0, 3, 1, 2, 3, 2, 3};
__device__ constexpr int kDh1R[16] = {0, 1, 1, 2, 3, 3, 4, 4, 4, 4, 5, 5, 6, 7, 7, 8};

// conv1's 2x2 patches over the 4x4 board: cell of tap t (row-major dr, dc) at output position R
__device__ __forceinline__ int cell_of(int R, int t) { return (R / 3 + (t >> 1)) * 4 + (R % 3) + (t & 1); }

// element offset of image (row r, column c) inside a slot: block c >> 5, 64-byte rows, the
// 8-byte chunk index XOR (r >> 1) & 7
__device__ __forceinline__ int img_at(int r, int c)
{
    return (c >> 5) * kBlock + r * 32 + ((((c >> 2) & 7) ^ ((r >> 1) & 7)) << 2) + (c & 3);
}

// The swizzle is not additive in the column, so every image access is written as a per-lane base
// (computed once, 10 VGPRs) plus a compile-time block / row offset that folds into the DS
// instruction's offset field; otherwise each call site gets its own hoisted address register.
struct LaneAddr {
    int st[4];       // stores of row `col`: chunk 2k + h of a block
    int t32[2];      // 32x32x16 transposed read, rows 8h + (i >> 2) + 4u, chunk 4(g & 1) + (i & 3)
    int t16[2][2];   // 16x16x32 transposed read, rows 8G + (i >> 2) + 4u, chunk 4v + (i & 3)
};

__device__ __forceinline__ LaneAddr lane_addr(int lane)
{
    LaneAddr a;
    const int h = lane >> 5, col = lane & 31, g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; k++)
        a.st[k] = img_at(col, 4 * (2 * k + h));
#pragma unroll
    for (int u = 0; u < 2; u++) {
        a.t32[u] = img_at(8 * (g >> 1) + (i >> 2) + 4 * u, 16 * (g & 1) + 4 * (i & 3));
#pragma unroll
        for (int v = 0; v < 2; v++)
            a.t16[v][u] = img_at(8 * g + (i >> 2) + 4 * u, 16 * v + 4 * (i & 3));
    }
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

// 32x32x16 operand: index 32 blk + (lane & 31), k = image row r0 + 8h + j (r0 = 0 or 16; the
// swizzle of row + 16 equals that of row). Per 16-lane group, lane 4q + p addresses row q of the
// group's 4-row block, columns 4p..4p+3.
__device__ __forceinline__ bf16x8 tr32(const uint16_t *slot, const LaneAddr &la, int blk, int r0)
{
    const uint16_t *b = slot + blk * kBlock + r0 * 32;
    return tr_pair(b + la.t32[0], b + la.t32[1]);
}

// 16x16x32 operand: index 32 blk + 16 v + (lane & 15), k = image row 8(lane >> 4) + j
__device__ __forceinline__ bf16x8 tr16(const uint16_t *slot, const LaneAddr &la, int blk, int v)
{
    const uint16_t *b = slot + blk * kBlock;
    return tr_pair(b + la.t16[v][0], b + la.t16[v][1]);
}

// store a B-layout fragment (elements j = feature cbase + 8(j>>2) + 4h + (j&3), cbase a multiple
// of 16) as image row `col`: two packed 8-byte chunks
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
// d * min(act, 1) per 16-bit half: one v_pk_min_u16 + one v_pk_mul_lo_u16 per word. The min is
// written in asm: as plain code its 0/1 range lets the compiler rewrite min and product as
// per-element compares + selects (4-5 instructions per word).
__device__ __forceinline__ bf16x8 mask_pk(const bf16x8 &d, const bf16x8 &act)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    uint32_t dw[4], aw[4];
    __builtin_memcpy(dw, &d, 16);
    __builtin_memcpy(aw, &act, 16);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t m;
        asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(aw[q]), "s"(0x00010001u));   // 1 in both halves
        dw[q] = __builtin_bit_cast(uint32_t, (u16x2)(__builtin_bit_cast(u16x2, dw[q]) * __builtin_bit_cast(u16x2, m)));
    }
    bf16x8 f;
    __builtin_memcpy(&f, dw, 16);
    return f;
}

// Gradient-slice accumulation: acc += A B with the accumulator pinned in AGPRs ("+a") while the
// activation MFMAs (builtins, VGPR form: FLAGS_r48_a3c_train) keep their results in VGPRs for the
// epilogues. Wait states, as hipcc pads nothing inside asm: s_nop 1 first (an operand may be a
// just-written VGPR, e.g. a rematerialised ones fragment); D -> the next MFMA of the same chain
// taking it whole as C needs none; D -> any other reader: the s_nop fence after the loop. Not
// volatile: a volatile asm is a scheduling barrier for the LDS reads that feed the next step.
__device__ __forceinline__ void mfma_acc32(f32x16 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// the same without the leading pad, for operands that come straight from LDS reads (the s_waitcnt
// orders those; only a VALU write needs the wait states). tools/check_asm_hazards.py verifies on
// the compiled code that no VALU write reaches these within 2 states.
__device__ __forceinline__ void mfma_acc32_lds(f32x16 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma_acc16_lds(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma_acc16(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ bf16x8 ones_frag()
{
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; j++)
        f[j] = (short)0x3F80;
    return f;
}

__device__ __forceinline__ bf16x8 lds_frag(const uint16_t *p)
{
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_cnn_train(
    const int8_t *__restrict__ boards, int64_t rows, int64_t n_boards, const int8_t *__restrict__ actions,
    const float *__restrict__ targets, const float *__restrict__ wn, const float *__restrict__ cm,
    const float *__restrict__ counts, float beta, const uint4 *__restrict__ wfrag,
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
    for (int i = threadIdx.x; i < kFragsTrain * 64; i += kThreads)
        w_lds_base[i] = wfrag[i];
    for (int i = threadIdx.x; i < 104; i += kThreads)
        b_lds_base[i] = bias[i];
    __syncthreads();

    const f32x16 zero = {};
    const f32x4 zero4 = {};
    const bf16x8 ones = ones_frag();
    // this wave's slice of the weight gradient
    f32x16 dw2[2] = {zero, zero};                  // dW2[32 (g_mine ^ u) + i][32 wave + j], u = 0, 1
    f32x16 db2 = zero;                             // db2[32 (wave & 1) + i], patches wave >> 1 and 2 + (wave >> 1)
    f32x4 dwh[4] = {zero4, zero4, zero4, zero4};   // dWh[o][64 wave + 16 ft + i]
    f32x4 dbh = zero4;                             // heads bias (wave 0)
    f32x4 dw1[2] = {zero4, zero4};                 // dW1[16 ct + i][t] (t = 4: conv1 bias), own rows
    float loss_actor = 0.0f, loss_critic = 0.0f;
    // conv1 input position of dW2 block kk = wave relative to the phase-B half:
    // kP2[2 ph + pl][kk] - 3 ph = pl + 3 (kk >> 1) + (kk & 1)
    const int pos_kk = 3 * (wave >> 1) + (wave & 1);
    // ones/zero operands that select this wave's bias-gradient work without a branch (a
    // conditional MFMA on a loop-carried accumulator makes the register allocator copy it)
    const bf16x8 nil = {};
    const bf16x8 ones_w0 = wave == 0 ? ones : nil;                    // heads bias: wave 0 only
    const bf16x8 ones_pl0 = (wave >> 1) == 0 ? ones : nil, ones_pl1 = (wave >> 1) == 1 ? ones : nil;
    const int g_mine = wave & 1;                                      // db2 half of this wave

    const int64_t n_tiles = (rows + 31) / 32;
    const int64_t per_round = (int64_t)gridDim.x * kWaves;
    const int64_t rounds = (n_tiles + per_round - 1) / per_round;   // every wave runs every round (barriers)
    // per-row inputs of tile `round`, loaded one tile ahead so their HBM latency hides behind the
    // previous tile's work (wt = 0 on padding rows; loss inputs only in lane half 0)
    struct RowIn {
        uint2 raw;
        float wt, tgt, c;
        int act;
        float4 cnt;
    };
    auto fetch = [&](int64_t round) {
        RowIn in;
        const int64_t r = (round * per_round + (int64_t)blockIdx.x * kWaves + wave) * 32 + col;
        const bool live = r < rows;
        const int64_t rr = live ? r : rows - 1;          // padding lanes compute on a valid row, weight 0
        in.raw = *reinterpret_cast<const uint2 *>(boards + 16 * rr + 8 * h);
        in.wt = 0.f, in.tgt = 0.f, in.c = 0.f, in.act = 0, in.cnt = make_float4(0.f, 0.f, 0.f, 0.f);
        if (h == 0) {
            in.wt = live ? wn[rr] : 0.0f;
            in.tgt = targets[rr];
            in.act = actions[rr] & 3;
            if (cm) {
                in.c = live ? cm[rr] : 0.0f;
                in.cnt = *reinterpret_cast<const float4 *>(counts + 4 * (rr % n_boards));
            }
        }
        return in;
    };
    RowIn next = fetch(0);
    for (int64_t round = 0; round < rounds; round++) {
        const RowIn in = next;
        if (round + 1 < rounds)
            next = fetch(round + 1);
        // weights and biases are re-read from LDS every tile: an opaque zero offset keeps the
        // compiler from hoisting ~300 registers of loop-invariant fragments out of the loop
        int wofs = 0;
        asm volatile("" : "+s"(wofs));
        const uint4 *w_lds = w_lds_base + wofs;
        const float *b_lds = b_lds_base + wofs;
        // ---------------- forward (r48_policy.hip k_cnn_forward)
        const uint2 raw = in.raw;
        uint32_t xp[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t w = q < 2 ? raw.x : raw.y;
            const int sh = 16 * (q & 1);
            xp[q] = cell_bf16((w >> sh) & 0xffu, MODE) | (cell_bf16((w >> (sh + 8)) & 0xffu, MODE) << 16);
        }
        bf16x8 x;
        __builtin_memcpy(&x, xp, 16);
        bf16x8 h1[9][2];
        bf16x8 h2[4][2][2];
        f32x16 out;
        {
            // h1 stays live until dh1 (the allocator parks it in AGPRs across the loss, dh2 and
            // phase A; measured 2 % faster than recomputing it before phase B)
            WStream ws;
            ws.start(w_lds, fwd_frag(0), fwd_frag(1), lane);
            cnn_conv1(w_lds, b_lds, lane, h, x, ws, h1);
            cnn_conv2_heads(w_lds, b_lds, lane, h, h1, ws, h2, out);
        }
        // ---------------- loss gradient per row (lane half 0: logits rows 0..3; value in lane + 32)
        const float v = __shfl(out[0], col + 32) + b_lds[100];
        float dz[4] = {0.f, 0.f, 0.f, 0.f}, dv = 0.f;
        if (h == 0) {
            const float wt = in.wt;
            float z[4], p[4], g[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                z[k] = out[k] + b_lds[96 + k];
            const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
            float se = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                p[k] = __expf(z[k] - m);
                se += p[k];
            }
            const float inv = __builtin_amdgcn_rcpf(se), lse = m + __logf(se);
            float H = 0.f, gbar = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                p[k] *= inv;
                const float lq = __logf(p[k] + kEntropyEps);
                H -= p[k] * lq;
                g[k] = -(lq + p[k] * __builtin_amdgcn_rcpf(p[k] + kEntropyEps));     // dH/dp_k
                gbar += p[k] * g[k];
            }
            const float td = in.tgt - v;
            const int a = in.act;
            if (cm) {   // reference: -beta wn H - cm sum_k c_k log p_k  (losses.py, a3c.py:110-116)
                const float c = in.c;
                const float4 cnt = in.cnt;
                const float ck[4] = {cnt.x, cnt.y, cnt.z, cnt.w}, C = cnt.x + cnt.y + cnt.z + cnt.w;
                float sa = 0.f;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    dz[k] = -beta * wt * p[k] * (g[k] - gbar) - c * (ck[k] - p[k] * C);
                    sa += ck[k] * (z[k] - lse);
                }
                loss_actor += -beta * wt * H - c * sa;
            } else {    // textbook: -wn (beta H + td log p[a]), td constant for the actor
#pragma unroll
                for (int k = 0; k < 4; k++)
                    dz[k] = -wt * (beta * p[k] * (g[k] - gbar) + td * ((k == a ? 1.0f : 0.0f) - p[k]));
                loss_actor += -wt * (beta * H + td * (z[a] - lse));
            }
            dv = -2.0f * wt * td;                             // critic = wn td^2
            loss_critic += wt * td * td;
        }
        // dout as the B operand: k = 8h + j = output o (half 0: dz0..3, dv; half 1: 0)
        bf16x8 dout;
        {
            const uint32_t d0 = pack_bf16x2(dz[0], dz[1]), d1 = pack_bf16x2(dz[2], dz[3]), d2 = pack_bf16x2(dv, 0.f);
            uint32_t pk[4] = {h == 0 ? d0 : 0u, h == 0 ? d1 : 0u, h == 0 ? d2 : 0u, 0u};
            __builtin_memcpy(&dout, pk, 16);
        }
        // ---------------- phase A stores: h2 and dout of the tile's 32 rows into the own slot
        if (!(kSkip & 1)) {
#pragma unroll
            for (int p = 0; p < 4; p++)
#pragma unroll
                for (int g = 0; g < 2; g++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        store_frag(my, la, 64 * p + 32 * g + 16 * s, h2[p][g][s]);
            if (h == 0) {
                const float dd[5] = {dz[0], dz[1], dz[2], dz[3], dv};
#pragma unroll
                for (int o = 0; o < 5; o++)
                    my[kDoutOff + o * 32 + col] = __builtin_bit_cast(uint16_t, (__bf16)dd[o]);
            }
        }
        // ---------------- dh2 = Wh^T dout . [h2 > 0]   (h2 dies here)
        bf16x8 dh2[4][2][2];
        {
            WStream ws;
            ws.start(w_lds, kOffWhT, kOffWhT + 1, lane);
#pragma unroll
            for (int m = 0; m < 8; m++) {               // m = 2p + g
                const bf16x8 wa = ws.step(w_lds, kOffWhT + (m + 2) % 8, lane);
                wfence();
                const f32x16 a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, dout, zero, 0, 0, 0);
                wfence();
                dh2[m >> 1][m & 1][0] = mask_pk(acc_to_frag(a, 0), h2[m >> 1][m & 1][0]);
                dh2[m >> 1][m & 1][1] = mask_pk(acc_to_frag(a, 1), h2[m >> 1][m & 1][1]);
            }
        }
        // ---------------- phase A: dWh[o][f] (f in the wave's 64 features) = sum over the 4 x 32 rows
        // of the workgroup of dout[o] h2[f]; 16x16x32 with A = h2^T (features x rows), B = dout
        if (!(kSkip & 1)) {
            tile_barrier();
            // the 4 dout operands up front, the h2^T operands one (slot, ft) step ahead
            const int o = lane & 15;
            bf16x8 bd[kWaves];
#pragma unroll
            for (int sl = 0; sl < kWaves; sl++) {
                bd[sl] = bf16x8{};
                if (o < 5)
                    bd[sl] = lds_frag(slots + sl * kSlot + kDoutOff + o * 32 + 8 * (lane >> 4));
            }
            bf16x8 A = tr16(slots, la, 2 * wave, 0);
#pragma unroll
            for (int k = 0; k < 4 * kWaves; k++) {
                const int sl = k >> 2, ft = k & 3, k1 = (k + 1) & 15;
                const bf16x8 An = tr16(slots + (k1 >> 2) * kSlot, la, 2 * wave + ((k1 & 3) >> 1), k1 & 1);
                wfence();
                mfma_acc16_lds(dwh[ft], A, bd[sl]);
                if (ft == 3)
                    mfma_acc16(dbh, ones_w0, bd[sl]);
                wfence();
                A = An;
            }
            tile_barrier();
        }
        // ---------------- phase B: dW2[:, 32 wave ..] = sum_p dh2[p] h1[kP2[p][wave]]^T, in two
        // halves of two patches each (the slot holds one half); dh1 is formed between the halves
        bf16x8 dh1[9][2];
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            if (!(kSkip & 2)) {
#pragma unroll
                for (int pl = 0; pl < 2; pl++)
#pragma unroll
                    for (int g = 0; g < 2; g++)
#pragma unroll
                        for (int s = 0; s < 2; s++)
                            store_frag(my, la, 64 * pl + 32 * g + 16 * s, dh2[2 * ph + pl][g][s]);
#pragma unroll
                for (int q = 0; q < 6; q++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        store_frag(my, la, 128 + 32 * q + 16 * s, h1[3 * ph + q][s]);
            }
            if (ph == 1 && !(kSkip & 4)) {
                // dh1 = W2^T dh2 . [h1 > 0]: each conv1 position R gathers the conv2 outputs (p, kk)
                // whose patch contains it (kDh1*: the 16 pairs in R order); one stream of 64
                // MFMAs, each A fragment read one MFMA ahead (h1 and dh2 die here)
                f32x16 a = zero;
                auto w2t = [](int m) { return kOffW2T + (kDh1K[(m & 63) >> 2] * 2 + ((m >> 1) & 1)) * 2 + (m & 1); };
                WStream ws;
                ws.start(w_lds, w2t(0), w2t(1), lane);
#pragma unroll
                for (int m = 0; m < 64; m++) {
                    const int n = m >> 2, g = (m >> 1) & 1, sk = m & 1;
                    const bf16x8 wa = ws.step(w_lds, w2t(m + 2), lane);
                    wfence();
                    a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, dh2[kDh1P[n]][g][sk], a, 0, 0, 0);
                    wfence();
                    if ((m & 3) == 3 && (n == 15 || kDh1R[n + 1] != kDh1R[n])) {
                        const int R = kDh1R[n];
                        dh1[R][0] = mask_pk(acc_to_frag(a, 0), h1[R][0]);
                        dh1[R][1] = mask_pk(acc_to_frag(a, 1), h1[R][1]);
                        a = zero;
                    }
                }
            }
            if (!(kSkip & 2)) {
                tile_barrier();
                // 16 K-steps (slot sl, patch pl of the half, 16-row block ks), software-pipelined:
                // the operands of step k + 1 are read before the MFMAs of step k issue
                // (dw2[0] holds output half g_mine, dw2[1] the other one)
                auto ld = [&](int st, bf16x8 *op) {
                    const uint16_t *slot = slots + (st >> 2) * kSlot;
                    const int pl = (st >> 1) & 1, ks = st & 1;
                    op[0] = tr32(slot, la, 4 + pl + pos_kk, 16 * ks);
                    op[1] = tr32(slot, la, 2 * pl + g_mine, 16 * ks);
                    op[2] = tr32(slot, la, 2 * pl + (g_mine ^ 1), 16 * ks);
                };
                bf16x8 cur[3], nxt[3];
                ld(0, cur);
#pragma unroll
                for (int st = 0; st < 16; st++) {
                    if (st + 1 < 16)
                        ld(st + 1, nxt);
                    __builtin_amdgcn_sched_barrier(0);
                    mfma_acc32_lds(dw2[0], cur[1], cur[0]);
                    mfma_acc32_lds(dw2[1], cur[2], cur[0]);
                    mfma_acc32(db2, cur[1], ((st >> 1) & 1) == 0 ? ones_pl0 : ones_pl1);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = 0; k < 3; k++)
                        cur[k] = nxt[k];
                }
                tile_barrier();
            }
        }
        // ---------------- phase C: dW1[co][t] (+ bias t = 4) = sum over the own 32 rows of
        // dh1[R][co] x[cell(R, t)]; 16x16x32 with A = dh1^T (channels x rows), B = x patch
        if (!(kSkip & 4)) {
#pragma unroll
            for (int R = 0; R < 9; R++)
#pragma unroll
                for (int s = 0; s < 2; s++)
                    store_frag(my, la, 32 * R + 16 * s, dh1[R][s]);
#pragma unroll
            for (int j = 0; j < 8; j++)
                my[kXOff + (8 * h + j) * 32 + col] = (uint16_t)x[j];
            const int t = lane & 15;
            // B[row][t]: t < 4 -> x[cell(R, t)], t == 4 -> 1 (conv1 bias), else 0
            auto patch = [&](int R) {
                bf16x8 b = {};
                if (t < 4)
                    b = lds_frag(my + kXOff + cell_of(R, t) * 32 + 8 * (lane >> 4));
                else if (t == 4)
                    b = ones;
                return b;
            };
            // operands one (R, ct) step ahead
            bf16x8 B = patch(0), A = tr16(my, la, 0, 0);
#pragma unroll
            for (int k = 0; k < 18; k++) {
                const int R = k >> 1, ct = k & 1, k1 = (k + 1) % 18;
                const bf16x8 An = tr16(my, la, k1 >> 1, k1 & 1);
                bf16x8 Bn = B;
                if (ct == 1)
                    Bn = patch(k1 >> 1);
                wfence();
                mfma_acc16(dw1[ct], A, B);
                wfence();
                A = An;
                B = Bn;
                (void)R;
            }
        }
    }

    // ---------------- flush: stage this wave's partial record in LDS (zeros outside its slice),
    // then one coalesced copy to HBM. acc fence: 24 wait states between the last accumulating MFMA
    // and any other reader of its AGPRs (16-pass XDL write -> read)
    asm volatile("s_nop 15\n\ts_nop 7"
                 : "+a"(dw2[0]), "+a"(dw2[1]), "+a"(db2), "+a"(dwh[0]), "+a"(dwh[1]), "+a"(dwh[2]), "+a"(dwh[3]),
                   "+a"(dbh), "+a"(dw1[0]), "+a"(dw1[1]));
    __syncthreads();
    float *rec = reinterpret_cast<float *>(lds) + wave * kPartial;
    for (int i = lane; i < kPartial; i += 64)
        rec[i] = 0.0f;
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 2; g++)
#pragma unroll
        for (int i = 0; i < 16; i++)
            rec[(32 * (g ^ (wave & 1)) + 8 * (i >> 2) + 4 * h + (i & 3)) * 128 + 32 * wave + col] = dw2[g][i];
    if (col == 0) {
#pragma unroll
        for (int i = 0; i < 16; i++)
            rec[kOffDb2 + 32 * (wave & 1) + 8 * (i >> 2) + 4 * h + (i & 3)] = db2[i];
    }
    {
        const int j = lane & 15, G = lane >> 4;            // 16x16 D: column j, rows 4G + reg
        if (j < 5) {
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    rec[kOffDw1 + (16 * ct + 4 * G + i) * 5 + j] = dw1[ct][i];
#pragma unroll
            for (int ft = 0; ft < 4; ft++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    rec[kOffDwh + j * 257 + 64 * wave + 16 * ft + 4 * G + i] = dwh[ft][i];
            if (wave == 0 && G == 0)
                rec[kOffDwh + j * 257 + 256] = dbh[0];     // every row of D is the same column sum
        }
    }
    float lsa = loss_actor, lsc = loss_critic;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        lsa += __shfl_xor(lsa, off);
        lsc += __shfl_xor(lsc, off);
    }
    if (lane == 0) {
        rec[kOffLoss] = lsa;
        rec[kOffLoss + 1] = lsc;
    }
    __syncthreads();
    float *dst = partials + ((int64_t)blockIdx.x * kWaves + wave) * kPartial;
    for (int i = lane; i < kPartial; i += 64)
        dst[i] = rec[i];
}

// deterministic sum of the per-wave records: out[k] = sum_w partials[w][k]
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

int grid_size()
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
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
    const int grid = grid_size();
    const size_t lds = kLds;
    // one instantiation per input encoding (no per-cell branch); each needs the LDS opt-in once
    auto kern = mode == R48_FEAT_VALUES ? k_cnn_train<R48_FEAT_VALUES> : k_cnn_train<R48_FEAT_EXPONENTS>;
    static bool attr_set[2] = {false, false};
    if (!attr_set[mode == R48_FEAT_VALUES]) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr_set[mode == R48_FEAT_VALUES] = true;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, boards, rows, n_boards, actions,
                       targets, wn, cm, counts, beta, (const uint4 *)wfrag, bias, workspace);
    // the group sums go after the records in the workspace (r48_cnn_train_workspace_floats)
    float *group_sums = workspace + (int64_t)grid * kWaves * kPartial;
    hipLaunchKernelGGL(k_reduce_groups, dim3((kPartial + 255) / 256, kGroups), dim3(256), 0, (hipStream_t)stream,
                       workspace, (int64_t)grid * kWaves, group_sums);
    hipLaunchKernelGGL(k_reduce, dim3((kPartial + 255) / 256), dim3(256), 0, (hipStream_t)stream, group_sums, grad);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string("k_cnn_train: ") + hipGetErrorString(e));
    return R48_OK;
}

}  // extern "C"
