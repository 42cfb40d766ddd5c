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

constexpr int kWaves = 8, kPairs = kWaves / 2;
constexpr int kThreads = 64 * kWaves;
// waves 2k and 2k + 1 form pair k (R48_PAIR_MAP 1: waves k and k + 4)
#ifndef R48_PAIR_MAP
#define R48_PAIR_MAP 0
#endif
#ifndef R48_PAIR_STAGGER
#define R48_PAIR_STAGGER 0
#endif
#ifndef R48_PAIR_PRIO
#define R48_PAIR_PRIO 0
#endif
__device__ __forceinline__ int kPairOf(int wave) { return R48_PAIR_MAP ? (wave & 3) : (wave >> 1); }
__device__ __forceinline__ int kHalfOf(int wave) { return R48_PAIR_MAP ? (wave >> 2) : (wave & 1); }
constexpr int kFragWhT = 8, kFragW2T = 16;
constexpr int kFragsTrain = kFrags + kFragWhT + kFragW2T;    // 65: forward 41 | Wh^T 8 | W2^T 16
constexpr int kOffWhT = kFrags, kOffW2T = kFrags + kFragWhT;
constexpr int kBlock = 32 * 32;
// per-pair slot (bf16 elements):
//   [0, kImg)   image of h2, later of dh2: [32 rows][256 features] in blocks of 32 features,
//               64-byte rows, 8-byte chunk index XOR (row >> 1) & 7; wave Q owns blocks 4Q..4Q+3
//   kXt         board cells of the tile: [16 cells][32 rows in rho order], then 11 rows of ones
//               and 11 of zeros (the bias and empty columns of dW1's B operand; every lane reads
//               unconditionally and the lane's base address selects cell, ones or zeros)
//   kDt         dout, one copy per wave: [2][5 outputs][32 rows in rho order]
//   kXo         head partial sums: [2 waves][5 outputs][32 rows] floats
//   kFlags      the pair's two sync words
constexpr int kImg = 8 * kBlock;
constexpr int kXt = kImg, kXtOnes = kXt + 16 * 32, kXtZeros = kXtOnes + 11 * 32;
constexpr int kDt = kXtZeros + 11 * 32;
constexpr int kXo = kDt + 2 * 5 * 32;
constexpr int kFlags = kXo + 2 * 2 * 5 * 32;
constexpr int kSlot = kFlags + 8;                             // 10376 elements = 20752 B
// gradient record per wave (floats): dW2 [64][128] | db2 [64] | dW1 [32][5] | dWh [5][257] | losses [2]
constexpr int kOffDb2 = 64 * 128, kOffDw1 = kOffDb2 + 64, kOffDwh = kOffDw1 + 32 * 5, kOffLoss = kOffDwh + 5 * 257;
constexpr int kPartial = kOffLoss + 2;                        // 9703
constexpr size_t kLdsWeights = (size_t)(kFragsTrain * 64 + 32) * 16;
constexpr size_t kLds = kLdsWeights + (size_t)kPairs * kSlot * 2;         // 150,080 B
static_assert(kSlot % 8 == 0 && kLds <= 160 * 1024, "LDS layout");
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
    int dr;      // dWh B operand (s = 0): output n >> 1 of the wave's Dt (at dt), or zeros
};

__device__ __forceinline__ LaneAddr lane_addr(int lane, int dt)
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
    a.dr = (sel && q < 5 ? dt + q * 32 : kXtZeros) + 8 * hh;
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

// conv1 as cnn_conv1 (same products, same bits), with the MFMA of position R + 1 issued before the
// epilogue of R (two accumulators in flight) so the pipe runs under the bf16 pack + ReLU
__device__ __forceinline__ void fwd_conv1(const uint4 *w, const float *b, int lane, int h, const bf16x8 &x,
                                          WStream &ws, bf16x8 (&h1)[9][2], int after0, int after1)
{
    const f32x16 b1 = load_bias(b, h);
    bf16x8 wa = ws.step(w, 2, lane);
    wfence();
    f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, x, b1, 0, 0, 0);
#pragma unroll
    for (int R = 0; R < 9; R++) {
        f32x16 nxt = acc;
        if (R + 1 < 9) {
            wa = ws.step(w, R + 3 < 9 ? R + 3 : (R + 3 == 9 ? after0 : after1), lane);
            wfence();
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, x, b1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
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
                                                      const bf16x8 (&h1)[9][2], WStream &ws, bf16x8 (&h2)[4][2][2],
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
                const bf16x8 wa = ws.step(w, fwd_frag(i + 2 < kFwdMfmas ? i + 2 : 0), lane);
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
                const bf16x8 wa = ws.step(w, fwd_frag(i + 2 < kFwdMfmas ? i + 2 : 0), lane);
                wfence();
                out = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, h2[p][g][s], out, 0, 0, 0);
                wfence();
            }
        }
    }
}

// Pair synchronisation through two LDS words (one per wave of the pair, the last epoch it
// reached): wait for this wave's LDS writes, publish the epoch, spin (s_sleep) until the partner
// has published it too. Both waves of a pair run the same tiles and the same three syncs per tile;
// the spin is still bounded, so a broken pairing ends the kernel (NaN loss) instead of hanging it.
constexpr int kSpinLimit = 1 << 20;

__device__ __forceinline__ void pair_sync(volatile int *flags, int q, int epoch, bool &bad)
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0)
        flags[q] = epoch;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!bad) {
        int spins = 0;
#pragma clang loop unroll(disable)
        while (flags[q ^ 1] < epoch) {
            if (++spins > kSpinLimit) {
                bad = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    asm volatile("" ::: "memory");
}

// orientation-1 fragment of image row `col` (the inverse of store_frag)
__device__ __forceinline__ bf16x8 load_frag(const uint16_t *slot, const LaneAddr &la, int cbase)
{
    const uint16_t *b = slot + (cbase >> 5) * kBlock;
    const int s = (cbase >> 4) & 1;
    const uint2 lo = *reinterpret_cast<const uint2 *>(b + la.st[2 * s]);
    const uint2 hi = *reinterpret_cast<const uint2 *>(b + la.st[2 * s + 1]);
    const uint4 v = make_uint4(lo.x, lo.y, hi.x, hi.y);
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// conv1 positions R whose dh1 wave Q computes (8 (p, kk) pairs each side)
__host__ __device__ constexpr bool dh1_mine(int Q, int R) { return Q == 0 ? (R <= 3 || R == 5) : (R == 4 || R >= 6); }

struct TrainArgs {
    const int8_t *boards;
    int64_t rows, n_boards;
    const int8_t *actions;
    const float *targets, *wn, *cm, *counts;
    float beta;
};

// One wave of a pair: half Q of every tile of the pair (see the file header). Runs the pair's
// whole persistent loop and writes this wave's gradient record.
template <int MODE, int Q>
__device__ __forceinline__ void pair_wave(const TrainArgs &A, uint16_t *my, volatile int *flags, int64_t first,
                                          int64_t stride, const uint4 *w_lds_base, const float *b_lds_base,
                                          float *rec)
{
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const LaneAddr la = lane_addr(lane, kDt + Q * 5 * 32);
    float *xo = reinterpret_cast<float *>(my + kXo);           // [2 waves][5 outputs][32 rows]
    const f32x16 zero = {};
    const f32x4 zero4 = {};
    // this wave's share of the weight gradient (AGPRs)
    f32x16 dw2[2][2];                              // dW2[32 g + row][32 (2Q + kl) + lane col]
#pragma unroll
    for (int g = 0; g < 2; g++)
#pragma unroll
        for (int kl = 0; kl < 2; kl++)
            dw2[g][kl] = zero;
    f32x4 dwh[4];                                  // feature blocks 4Q + mb
#pragma unroll
    for (int mb = 0; mb < 4; mb++)
        dwh[mb] = zero4;
    f32x4 db2 = zero4, dw1 = zero4;
    float dbh[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float loss_actor = 0.0f, loss_critic = 0.0f;
    const int g16 = lane >> 4, n16 = lane & 15;
    const uint32_t one2 = 0x3F803F80u;
    bool bad = false;
    int epoch = 0;

    const int64_t rows = A.rows, n_tiles = (rows + 31) / 32;
    struct RowIn {
        uint2 raw;
        float wt, tgt, c;
        int act;
        float4 cnt;
    };
    auto fetch = [&](int64_t tile) {
        RowIn in;
        const int64_t r = std::min<int64_t>(tile, n_tiles - 1) * 32 + col;
        const bool live = r < rows && tile < n_tiles;
        const int64_t rr = r < rows ? r : rows - 1;     // padding lanes compute on a valid row, weight 0
        in.raw = *reinterpret_cast<const uint2 *>(A.boards + 16 * rr + 8 * h);
        const float wt = A.wn[rr];
        in.wt = live ? wt : 0.0f;
        in.tgt = A.targets[rr];
        in.act = A.actions[rr] & 3;
        in.c = 0.f, in.cnt = make_float4(0.f, 0.f, 0.f, 0.f);
        if (A.cm) {   // wave-uniform
            const float c = A.cm[rr];
            in.c = live ? c : 0.0f;
            // row rr belongs to board rr % n_boards (rows are [T][n_boards]); 32-bit when it fits
            const int64_t bidx =
                rows <= 0xFFFFFFFFll ? (int64_t)((uint32_t)rr % (uint32_t)A.n_boards) : rr % A.n_boards;
            in.cnt = *reinterpret_cast<const float4 *>(A.counts + 4 * bidx);
        }
        return in;
    };
    RowIn next = fetch(first);
    for (int64_t tile = first; tile < n_tiles; tile += stride) {
        const RowIn in = next;
        // weights and biases are re-read from LDS every tile (an opaque zero offset keeps the
        // compiler from hoisting loop-invariant fragments out of the loop)
        int wofs = 0;
        asm volatile("" : "+s"(wofs));
        const uint4 *w = w_lds_base + wofs;
        const float *bl = b_lds_base + wofs;
        // ---------------- forward: conv1 at R = 3Q .. 3Q + 5, conv2 + heads of positions 2Q, 2Q + 1
        uint32_t xp[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t wv = q < 2 ? in.raw.x : in.raw.y;
            const int sh = 16 * (q & 1);
            xp[q] = cell_bf16((wv >> sh) & 0xffu, MODE) | (cell_bf16((wv >> (sh + 8)) & 0xffu, MODE) << 16);
        }
        bf16x8 x;
        __builtin_memcpy(&x, xp, 16);
        if (Q == 0) {   // Xt (dW1's B operand, both waves): the partner reads it after sync B
#pragma unroll
            for (int j = 0; j < 8; j++)
                my[kXt + (8 * h + j) * 32 + la.xw] = (uint16_t)(xp[j >> 1] >> (16 * (j & 1)));
        }
        f32x16 outp = zero;
        {
            // conv1 of the local positions i (R = 3Q + i) each chain pair needs, just before it:
            // position 2Q uses i = 0, 1, 3, 4 and position 2Q + 1 uses i = 1, 2, 4, 5
            bf16x8 h1[6][2];
            auto conv1 = [&](int i) {
                const f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w, 3 * Q + i, lane), x,
                                                                           load_bias(bl, h), 0, 0, 0);
                h1[i][0] = acc_to_frag_relu(acc, 0);
                h1[i][1] = acc_to_frag_relu(acc, 1);
            };
#pragma unroll
            for (int pl = 0; pl < 2; pl++) {
                const int p = 2 * Q + pl;
                if (pl == 0) {
                    conv1(0), conv1(1), conv1(3), conv1(4);
                } else {
                    conv1(2), conv1(5);
                }
#pragma unroll
                for (int g = 0; g < 2; g++) {
                    f32x16 a = load_bias(bl + 32 + 32 * g, h);
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w, kFragW1 + (g * 4 + (u >> 1)) * 2 + (u & 1), lane),
                                                                    h1[kP2[p][u >> 1] - 3 * Q][u & 1], a, 0, 0, 0);
#pragma unroll
                    for (int s = 0; s < 2; s++) {
                        const bf16x8 hf = acc_to_frag_relu(a, s);
                        store_frag(my, la, 64 * p + 32 * g + 16 * s, hf);
                        outp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                            frag_at(w, kFragW1 + kFragW2 + (2 * p + g) * 2 + s, lane), hf, outp, 0, 0, 0);
                    }
                }
            }
        }
        // ---------------- exchange the head partial sums (rows 0..3 logits in half 0, row 4 the
        // value in half 1), both waves add them in the same order
        {
            float *xw = xo + Q * 160;
            if (h == 0) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    xw[k * 32 + col] = outp[k];
            } else {
                xw[4 * 32 + col] = outp[0];
            }
        }
        pair_sync(flags, Q, ++epoch, bad);                          // sync A
        float dz[4] = {0.f, 0.f, 0.f, 0.f}, dv = 0.f;
        if (h == 0) {
            const float wt = in.wt;
            float z[4], p[4], gr[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                z[k] = (xo[k * 32 + col] + xo[160 + k * 32 + col]) + bl[96 + k];
            const float v = (xo[128 + col] + xo[160 + 128 + col]) + bl[100];
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
            float la_ = 0.f;
            if (A.cm) {   // reference: -beta wn H - cm sum_k c_k log p_k  (losses.py, a3c.py:110-116)
                const float c = in.c;
                const float4 cnt = in.cnt;
                const float ck[4] = {cnt.x, cnt.y, cnt.z, cnt.w}, C = cnt.x + cnt.y + cnt.z + cnt.w;
                float sa = 0.f;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    dz[k] = -A.beta * wt * p[k] * (gr[k] - gbar) - c * (ck[k] - p[k] * C);
                    sa += ck[k] * (z[k] - lse);
                }
                la_ = -A.beta * wt * H - c * sa;
            } else {    // textbook: -wn (beta H + td log p[a]), td constant for the actor
#pragma unroll
                for (int k = 0; k < 4; k++)
                    dz[k] = -wt * (A.beta * p[k] * (gr[k] - gbar) + td * ((k == a ? 1.0f : 0.0f) - p[k]));
                la_ = -wt * (A.beta * H + td * (z[a] - lse));
            }
            dv = -2.0f * wt * td;                             // critic = wn td^2
            if (Q == 0) {   // the loss is computed by both waves and counted once
                loss_actor += la_;
                loss_critic += wt * td * td;
#pragma unroll
                for (int k = 0; k < 4; k++)
                    dbh[k] += dz[k];
                dbh[4] += dv;
            }
            // Dt (this wave's copy): dout of this row at its rho position (dWh's B operand)
            const float dd[5] = {dz[0], dz[1], dz[2], dz[3], dv};
#pragma unroll
            for (int o = 0; o < 5; o++)
                my[kDt + Q * 160 + o * 32 + la.xw] = __builtin_bit_cast(uint16_t, (__bf16)dd[o]);
        }
        next = fetch(tile + stride);      // the current tile's row inputs are consumed
        bf16x8 dout;
        {
            const uint32_t d0 = pack_bf16x2(dz[0], dz[1]), d1 = pack_bf16x2(dz[2], dz[3]), d2 = pack_bf16x2(dv, 0.f);
            uint32_t pk[4] = {h == 0 ? d0 : 0u, h == 0 ? d1 : 0u, h == 0 ? d2 : 0u, 0u};
            __builtin_memcpy(&dout, pk, 16);
        }
        // ---------------- dh2 of this wave's blocks m = 4Q + mb (positions 2Q, 2Q + 1):
        //   dWh += h2^T dout (h2^T read back transposed before the overwrite), dh2 = Wh^T dout .
        //   [h2 > 0] (h2 read back in orientation 1) written over the block, dh2^T read back (AGPRs),
        //   db2 += row sums of dh2^T
        bf16x8 dh2t[4][2];
        {
            const bf16x8 sel0 = splat_frag(n16 == (g16 & 1) ? one2 : 0u);
            const bf16x8 sel1 = splat_frag(n16 == 2 + (g16 & 1) ? one2 : 0u);
            const bf16x8 bd0 = lds_frag(my + la.dr), bd1 = lds_frag(my + la.dr + 16);
#pragma unroll
            for (int mb = 0; mb < 4; mb++) {
                const int m = 4 * Q + mb;
                const f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w, kOffWhT + m, lane), dout, zero, 0, 0, 0);
                acc16_lds(dwh[mb], trr(my, la, m, 0), bd0);
                acc16_lds(dwh[mb], trr(my, la, m, 1), bd1);
                const bf16x8 hm0 = load_frag(my, la, 32 * m), hm1 = load_frag(my, la, 32 * m + 16);
                const bf16x8 d0 = mask_pk(acc_to_frag(acc, 0), hm0);
                const bf16x8 d1 = mask_pk(acc_to_frag(acc, 1), hm1);
                store_frag(my, la, 32 * m, d0);
                store_frag(my, la, 32 * m + 16, d1);
                dh2t[mb][0] = trr(my, la, m, 0);
                dh2t[mb][1] = trr(my, la, m, 1);
                acc16_av(db2, dh2t[mb][0], (m & 1) ? sel1 : sel0);
                acc16_av(db2, dh2t[mb][1], (m & 1) ? sel1 : sel0);
            }
        }
        pair_sync(flags, Q, ++epoch, bad);                          // sync B: the whole dh2 image
        // ---------------- conv1 positions R = 3Q .. 3Q + 5: h1^T_R; dW2 columns kk = 2Q, 2Q + 1 of
        // every (p, kk) of R; dh1^T_R and dW1 for this wave's R
        {
            const float b1c = bl[col];
#pragma unroll
            for (int i = 0; i < 6; i++) {
                const int R = 3 * Q + i;
                // bias added in the epilogue: a splat C operand would hold 16 registers all loop long
                f32x16 a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, frag_at(w, R, lane), zero, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 16; r++)
                    a1[r] += b1c;
                bf16x8 h1t[2];
                h1t[0] = acc_to_frag_relu(a1, 0);
                h1t[1] = acc_to_frag_relu(a1, 1);
#pragma unroll
                for (int n = kRFirst[R]; n < kRFirst[R + 1]; n++) {
                    const int p = kDh1P[n], kk = kDh1K[n];
                    if ((kk >> 1) != Q)
                        continue;
#pragma unroll
                    for (int g = 0; g < 2; g++)
#pragma unroll
                        for (int s = 0; s < 2; s++) {
                            if ((p >> 1) == Q)
                                acc32_av(dw2[g][kk & 1], dh2t[2 * (p & 1) + g][s], h1t[s]);
                            else
                                acc32_v(dw2[g][kk & 1], trr(my, la, 2 * p + g, s), h1t[s]);
                        }
                }
                if (dh1_mine(Q, R)) {
                    f32x16 d = zero;
#pragma unroll
                    for (int n = kRFirst[R]; n < kRFirst[R + 1]; n++) {
                        const int p = kDh1P[n], kk = kDh1K[n];
#pragma unroll
                        for (int g = 0; g < 2; g++)
#pragma unroll
                            for (int s = 0; s < 2; s++)
                                d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    load_frag(my, la, 64 * p + 32 * g + 16 * s),
                                    frag_at(w, kOffW2T + (kk * 2 + g) * 2 + s, lane), d, 0, 0, 0);
                    }
                    const bf16x8 t0 = mask_pk(acc_to_frag(d, 0), h1t[0]);
                    const bf16x8 t1 = mask_pk(acc_to_frag(d, 1), h1t[1]);
                    acc16_v(dw1, t0, lds_frag(my + la.xr + cell_base(R) * 32));
                    acc16_v(dw1, t1, lds_frag(my + la.xr + cell_base(R) * 32 + 16));
                }
            }
        }
        pair_sync(flags, Q, ++epoch, bad);                          // sync C: both waves done with the tile
    }

    // ---------------- flush: this wave's gradient record (zeros where the partner owns the entry).
    // acc fence: 24 wait states between the last accumulating MFMA and any other reader of its AGPRs
    asm volatile("s_nop 15\n\ts_nop 7"
                 : "+a"(dw2[0][0]), "+a"(dw2[0][1]), "+a"(dw2[1][0]), "+a"(dw2[1][1]), "+a"(db2), "+a"(dw1),
                   "+a"(dwh[0]), "+a"(dwh[1]), "+a"(dwh[2]), "+a"(dwh[3]));
    // dW2: 32x32 D = [o (row 8(i>>2) + 4h + (i&3))][c = lane col]
#pragma unroll
    for (int g = 0; g < 2; g++)
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
#pragma unroll
            for (int i = 0; i < 16; i++)
                rec[(32 * g + 8 * (i >> 2) + 4 * h + (i & 3)) * 128 + 32 * kk + col] =
                    (kk >> 1) == Q ? dw2[g][kk & 1][i] : 0.0f;
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
                    rec[kOffDwh + q * 257 + 32 * ft + 16 * b + 4 * g16 + i] =
                        (ft >> 2) == Q ? dwh[ft & 3][i] : 0.0f;
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
        rec[kOffLoss] = bad ? __builtin_nanf("") : red[5];
        rec[kOffLoss + 1] = red[6];
    }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_cnn_train(
    const int8_t *__restrict__ boards, int64_t rows, int64_t n_boards, const int8_t *__restrict__ actions,
    const float *__restrict__ targets, const float *__restrict__ wn, const float *__restrict__ cm,
    const float *__restrict__ counts, float beta, const uint4 *__restrict__ wfrag,
    const float *__restrict__ bias, float *__restrict__ partials)
{
    extern __shared__ uint4 lds[];
    // LDS: the 4 pair slots first (small DS offsets), then the weight fragments and biases
    uint16_t *slots = reinterpret_cast<uint16_t *>(lds);
    uint4 *w_lds_base = lds + kPairs * kSlot / 8;                         // kFragsTrain x 1 KiB
    float *b_lds_base = reinterpret_cast<float *>(w_lds_base + kFragsTrain * 64);  // 104 floats
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pair = kPairOf(wave), q = kHalfOf(wave);
    uint16_t *my = slots + pair * kSlot;
    stage_lds<kFragsTrain * 64, kThreads>(w_lds_base, wfrag);
    for (int i = threadIdx.x; i < 104; i += kThreads)
        b_lds_base[i] = bias[i];
    // the constant rows of each pair's Xt (11 x 32 ones, 11 x 32 zeros) and the sync words
    if (q == 0) {
        for (int i = threadIdx.x & 63; i < 11 * 32; i += 64) {
            my[kXtOnes + i] = 0x3F80;
            my[kXtZeros + i] = 0;
        }
        if ((threadIdx.x & 63) < 2)
            reinterpret_cast<int *>(my + kFlags)[threadIdx.x & 63] = 0;
    }
    __syncthreads();   // the only workgroup barrier; pairs synchronise through their sync words

#if R48_PAIR_STAGGER
    // the second half of the pairs starts about half a tile later, so the two waves sharing a
    // SIMD are not in the same phase (MFMA-heavy forward vs VALU-heavy loss) at the same time
    if (pair >= kPairs / 2) {
        for (int i = 0; i < R48_PAIR_STAGGER; i++)
            __builtin_amdgcn_s_sleep(127);
    }
#endif
#if R48_PAIR_PRIO
    if (pair >= kPairs / 2)
        __builtin_amdgcn_s_setprio(1);
#endif
    const TrainArgs args = {boards, rows, n_boards, actions, targets, wn, cm, counts, beta};
    const int64_t first = (int64_t)blockIdx.x * kPairs + pair, stride = (int64_t)gridDim.x * kPairs;
    volatile int *flags = reinterpret_cast<volatile int *>(my + kFlags);
    float *rec = partials + ((int64_t)blockIdx.x * kWaves + wave) * kPartial;
    if (q == 0)
        pair_wave<MODE, 0>(args, my, flags, first, stride, w_lds_base, b_lds_base, rec);
    else
        pair_wave<MODE, 1>(args, my, flags, first, stride, w_lds_base, b_lds_base, rec);
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

// one fixed persistent grid (the MI355X's 256 CUs), not a query of the current device, so the
// per-wave record workspace (r48_cnn_train_workspace_floats) and the launch always agree
constexpr int grid_size() { return 256; }

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
    r48::ensure_dynamic_lds(reinterpret_cast<const void *>(kern), (int)lds, r48::stream_device((hipStream_t)stream));
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
