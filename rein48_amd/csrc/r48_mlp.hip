// r48_mlp.hip -- the reference's own A3C network (algorithm/a3c/a3c.py:136-169, fp32) fused on gfx950.
//
// ActorCriticMLP (rein48_amd/a3c/nets.py): actor 16 -> 64 ReLU6 -> 4 ReLU (-> softmax), critic
// 16 -> 64 ReLU6 -> 1, on the 16 raw tile values (a3c.py:37-39,139) or exponents. The network is
// tiny (2,501 parameters, ~2.4 k FMAs per board) and fp32 like the reference, so it runs on the
// VALU with ONE BOARD PER LANE: the weights are wave-uniform and come through the scalar cache into
// SGPRs (s_load), the activations never leave the lane, and every FMA is a v_pk_fma_f32 over two
// hidden units. No MFMA: an fp32 16x64 layer has no bf16 form that keeps the reference's fp32
// numbers, and at one board per lane no data moves between lanes.
//
// k_mlp_forward   logits (post-ReLU, a3c.py:153), value, and the choose_action draw (a3c.py:89-93:
//                 softmax + Philox inverse CDF, the r48_sample_actions contract) of every board
// k_mlp_rollout   the whole A3C rollout (a3c.py:194-212 batched) in ONE launch: each lane keeps its
//                 board in registers for all T steps -- policy, draw, env step (Game.step,
//                 GameClient.py:40-51, the r48_env_step Philox contract) -- and writes only the
//                 trajectory rows; bit-identical to T x (k_mlp_forward + r48_env_step)
//
// Weight blob (rein48_amd/a3c/fused.py pack_mlp, 2,504 floats), grouped by hidden-unit PAIR p
// (units 2p, 2p + 1): a1 [32 p][16 in][2] | a1.b [64] | a2 [32 p][4 out][2] | a2.b [4] |
// c1 [32 p][16 in][2] | c1.b [64] | c2 [64] | c2.b [1] | pad -- one pair's weights are contiguous
// (s_load_dwordx16 twice for its 32 layer-1 weights) and every SGPR pair feeds one packed FMA. The
// pair loop is NOT unrolled: the scalar loads then stay next to their use instead of being
// scheduled together (2,500 weights do not fit the SGPRs; they spilled into VGPR lanes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;
constexpr uint32_t kSampleTag = 0xA3Cu;   // r48_a3c.hip k_sample's draw tag
constexpr int kA1W = 0, kA1B = 1024, kA2W = 1088, kA2B = 1344, kC1W = 1348, kC1B = 2372, kC2W = 2436, kC2B = 2500;

// cell exponent -> network input: the raw tile value 2^e (0 for an empty cell), exact in fp32, or e
template <int MODE>
__device__ __forceinline__ float cell_input(uint32_t e)
{
    if (MODE == R48_FEAT_EXPONENTS)
        return (float)e;
    return __uint_as_float(e ? (127u + e) << 23 : 0u);
}

template <int MODE>
__device__ __forceinline__ void board_inputs(const r48::Board &b, float (&x)[16])
{
    const uint32_t w[4] = {b.w0, b.w1, b.w2, b.w3};
#pragma unroll
    for (int c = 0; c < 16; c++)
        x[c] = cell_input<MODE>((w[c >> 2] >> (8 * (c & 3))) & 0xFFu);
}

__device__ __forceinline__ f32x2 pair_at(const float *__restrict__ w, int off)
{
    return *reinterpret_cast<const f32x2 *>(w + off);
}

__device__ __forceinline__ float relu6(float a) { return fminf(fmaxf(a, 0.0f), 6.0f); }

// One 16 -> 64 ReLU6 layer folded straight into its consumer: hidden units are formed two at a time
// (one packed FMA chain per pair, inputs in order 0..15 after the bias) and immediately contracted
// into the NO outputs as per-parity partial sums acc[k] = (sum over even units, sum over odd units).
template <int NO>
__device__ __forceinline__ void hidden_into(const float *__restrict__ w, int w1, int b1, int w2, const float (&x)[16],
                                            f32x2 (&acc)[NO])
{
#pragma unroll
    for (int k = 0; k < NO; k++)
        acc[k] = f32x2{0.0f, 0.0f};
#pragma unroll 1
    for (int p = 0; p < 32; p++) {
        // four independent FMA chains over inputs f = q mod 4 (the bias starts chain 0), summed in a
        // fixed order: a 16-long dependent chain per pair left the VALU waiting on its latency
        f32x2 c4[4] = {pair_at(w, b1 + 2 * p), f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}};
#pragma unroll
        for (int f = 0; f < 16; f++)
            c4[f & 3] = __builtin_elementwise_fma(pair_at(w, w1 + 32 * p + 2 * f), f32x2{x[f], x[f]}, c4[f & 3]);
        const f32x2 a = (c4[0] + c4[1]) + (c4[2] + c4[3]);
        const f32x2 h = f32x2{relu6(a.x), relu6(a.y)};
#pragma unroll
        for (int k = 0; k < NO; k++)
            acc[k] = __builtin_elementwise_fma(pair_at(w, w2 + (NO == 1 ? 2 * p : 8 * p + 2 * k)), h, acc[k]);
    }
}

// hidden_into for the actor (4 outputs) and the critic (1 output) in ONE pair loop: two independent
// FMA chains per trip under one round of scalar loads (the update's forward, where the latency of the
// loads is exposed at two waves per SIMD)
__device__ __forceinline__ void hidden_both(const float *__restrict__ w, const float (&x)[16], f32x2 (&acc)[4], f32x2 &cv)
{
#pragma unroll
    for (int k = 0; k < 4; k++)
        acc[k] = f32x2{0.0f, 0.0f};
    cv = f32x2{0.0f, 0.0f};
#pragma unroll 1
    for (int p = 0; p < 32; p++) {
        f32x2 ca[4] = {pair_at(w, kA1B + 2 * p), f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}};
        f32x2 cc[4] = {pair_at(w, kC1B + 2 * p), f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}};
#pragma unroll
        for (int f = 0; f < 16; f++) {
            ca[f & 3] = __builtin_elementwise_fma(pair_at(w, kA1W + 32 * p + 2 * f), f32x2{x[f], x[f]}, ca[f & 3]);
            cc[f & 3] = __builtin_elementwise_fma(pair_at(w, kC1W + 32 * p + 2 * f), f32x2{x[f], x[f]}, cc[f & 3]);
        }
        const f32x2 a = (ca[0] + ca[1]) + (ca[2] + ca[3]), c = (cc[0] + cc[1]) + (cc[2] + cc[3]);
        const f32x2 h = f32x2{relu6(a.x), relu6(a.y)}, hc = f32x2{relu6(c.x), relu6(c.y)};
#pragma unroll
        for (int k = 0; k < 4; k++)
            acc[k] = __builtin_elementwise_fma(pair_at(w, kA2W + 8 * p + 2 * k), h, acc[k]);
        cv = __builtin_elementwise_fma(pair_at(w, kC2W + 2 * p), hc, cv);
    }
}

// logits z (post-ReLU) and, when VALUE, the critic's value of one board's inputs
template <bool VALUE>
__device__ __forceinline__ void mlp_forward(const float *__restrict__ w, const float (&x)[16], float (&z)[4], float &v)
{
    f32x2 acc[4];
    hidden_into<4>(w, kA1W, kA1B, kA2W, x, acc);
#pragma unroll
    for (int k = 0; k < 4; k++)
        z[k] = fmaxf(w[kA2B + k] + (acc[k].x + acc[k].y), 0.0f);
    v = 0.0f;
    if (VALUE) {
        f32x2 c[1];
        hidden_into<1>(w, kC1W, kC1B, kC2W, x, c);
        v = w[kC2B] + (c[0].x + c[0].y);
    }
}

// softmax + Philox inverse CDF, exactly k_sample's (r48_a3c.hip) and k_cnn_forward's epilogue
__device__ __forceinline__ uint32_t sample_action(const float (&z)[4], uint64_t gid, uint32_t ctr, uint32_t pk0,
                                                  uint32_t pk1)
{
    const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
    const float e0 = __expf(z[0] - m), e1 = __expf(z[1] - m), e2 = __expf(z[2] - m), e3 = __expf(z[3] - m);
    const float inv = 1.0f / (e0 + e1 + e2 + e3);
    const float p0 = e0 * inv, c1 = p0 + e1 * inv, c2 = c1 + e2 * inv;
    uint32_t q[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), ctr, kSampleTag};
    r48::philox4x32_10(q, pk0, pk1);
    const float u = (float)(q[0] >> 8) * (1.0f / 16777216.0f);
    return (p0 > u) ? 0u : (c1 > u) ? 1u : (c2 > u) ? 2u : 3u;
}

__device__ __forceinline__ r48::Board load_board(const int8_t *boards, int64_t i)
{
    const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    return r48::Board{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void store_board(int8_t *boards, int64_t i, const r48::Board &b)
{
    *reinterpret_cast<uint4 *>(boards + 16 * i) = make_uint4(b.w0, b.w1, b.w2, b.w3);
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_mlp_forward(const int8_t *__restrict__ boards, int64_t n,
                                                        const float *__restrict__ w, float *__restrict__ logits,
                                                        float *__restrict__ value, int8_t *__restrict__ actions,
                                                        int64_t gid0, uint32_t pk0, uint32_t pk1, uint32_t ctr)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    float x[16], z[4], v;
    board_inputs<MODE>(load_board(boards, i), x);
    if (value)
        mlp_forward<true>(w, x, z, v);
    else
        mlp_forward<false>(w, x, z, v);
    if (logits)
        *reinterpret_cast<float4 *>(logits + 4 * i) = make_float4(z[0], z[1], z[2], z[3]);
    if (value)
        value[i] = v;
    if (actions)
        actions[i] = (int8_t)sample_action(z, (uint64_t)(gid0 + i), ctr, pk0, pk1);
}

// VALUES: also V(boards[t]) of every step (the reference loss's td sums need V of the training
// states before the gradient pass; rollout_values in trainer.py)
template <int MODE, bool REWARD, bool VALUES>
__global__ __launch_bounds__(kBlock) void k_mlp_rollout(int8_t *__restrict__ boards, int64_t n, int32_t T,
                                                        const float *__restrict__ w, int8_t *__restrict__ traj,
                                                        int8_t *__restrict__ actions, uint8_t *__restrict__ done,
                                                        float *__restrict__ reward, int32_t *__restrict__ lengths,
                                                        float *__restrict__ values, int64_t gid0, uint32_t pk0,
                                                        uint32_t pk1, uint32_t ctr0, uint32_t ek0, uint32_t ek1,
                                                        uint32_t step0)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t gid = (uint64_t)(gid0 + i);
    r48::Board b = load_board(boards, i);
    int32_t len = T;
    for (int32_t t = 0; t < T; t++) {
        const int64_t at = (int64_t)t * n + i;
        store_board(traj, at, b);
        float x[16], z[4], v;
        board_inputs<MODE>(b, x);
        mlp_forward<VALUES>(w, x, z, v);
        if (VALUES)
            values[at] = v;
        const uint32_t act = sample_action(z, gid, ctr0 + (uint32_t)t, pk0, pk1);
        uint32_t dx, dy;
        r48::step_draw(gid, step0 + (uint32_t)t, ek0, ek1, dx, dy);
        const r48::StepOut o = r48::step_board<REWARD, false, true>(b, act, dy, (dx & 0x3FFFFFFFu) < r48::kFourThresh30);
        actions[at] = (int8_t)act;
        done[at] = (uint8_t)o.done;
        if (reward)   // merge reward as fp32 (exact: < 2^24)
            reward[at] = REWARD ? (float)o.reward : 0.0f;
        if (o.done && len == T)
            len = t + 1;   // through the first done step (a3c.py:201)
    }
    store_board(traj, (int64_t)T * n + i, b);
    store_board(boards, i, b);
    if (lengths)
        lengths[i] = len;
}

// ---------------------------------------------------------------- fused update
// k_mlp_train: the gradient of the A3C loss (rein48_amd/a3c/losses.py restating a3c.py:99-123,
// textbook or the reference's broadcast actor loss; the per-row formulas of r48_a3c_train.hip's
// k_cnn_train) w.r.t. all 2,501 parameters, fp32, in ONE pass over the training states.
// A wave takes 64 rows per tile in two phases:
//   phase 1, lane = row: the forward of mlp_forward (SGPR weights, packed FMAs), softmax / entropy
//     / td, the row's output gradient dz (through the logits' ReLU) and dv; the row's inputs x and
//     (dz, dv) go to the wave's LDS stash (24 floats per row)
//   phase 2, lane = hidden unit l (actor unit l and critic unit l): for each of the 64 rows (LDS
//     broadcast reads) recompute a_l, c_l (the same FMA sequence as phase 1, so the same values),
//     then dh_l = [0 < a_l < 6] sum_k W2[k][l] dz_k, dhc_l = [0 < c_l < 6] wc2[l] dv, and
//     accumulate the unit's gradient row in registers: dW1[l][:] += dh_l x, db1, dW2[:][l] += dz h_l,
//     dWc1[l][:], dbc1, dwc2[l]
// so the weight gradients (contractions over rows) never cross lanes. Per wave one record of the
// flat gradient in FlatParams order (a1.w [64][16] | a1.b | a2.w [4][64] | a2.b | c1.w | c1.b |
// c2.w | c2.b) + the two losses; k_mlp_reduce sums the records in a fixed order (deterministic).
// The ReLU derivatives of the update are decisions at 0 (and 6, ReLU6): an fp32 pre-activation within
// its rounding error of the boundary may land on the other side than the exact value, and with raw
// tile values as inputs (up to 2^17) a flipped hidden-unit mask moves a weight-gradient entry by a
// whole row's term (dh x). So the update decides them on exact-enough values: a hidden pre-activation
// (phase 2) or a logit (phase 1) whose fp32 value lies within the fp32 error bound of its boundary is
// recomputed in fp64 (rare: a divergent branch taken by ~1e-5 of the units / logits).
constexpr int kTrainWaves = 4;
constexpr int kStash = 28;                 // x[16] | dz[4] | dv | max x | dz before the logits' ReLU [4] | pad
constexpr int kRec = 2504;                 // 2,501 gradient floats + actor loss + critic loss + pad
constexpr int kRecLossA = 2501, kRecLossC = 2502;
// (the record's section offsets equal the blob's, kA1W .. kC2B; inside a1 / a2 / c1 the record has
// the parameters' own [out][in] order)
constexpr float kEntropyEps = 1e-5f;       // a3c.py:114
constexpr float kLn2 = 0.69314718055994531f;

// the wave's LDS stash is written by one phase and read by the other: every outstanding LDS
// operation completes (s_waitcnt lgkmcnt(0)) before the next phase's first access, and the
// compiler moves no LDS access across the point
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float uniform(float v)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
        v += __shfl_xor(v, m);
    return v;
}

// phase 2's (a_l, c_l) of one stashed row (its inputs returned as pairs (x_2i, x_2i+1)), in the
// four-chain FMA order of phase 1 (hidden_into: chain q takes the inputs f = q mod 4 in order, the
// bias starts chain 0), so the same values: chains (0, 1) are the pair p*, chains (2, 3) the pair q*
__device__ __forceinline__ f32x2 unit_preacts(const float (&row)[kStash], const f32x2 (&wa)[8], const f32x2 (&wc)[8],
                                              f32x2 bl, f32x2 (&xp)[8])
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const float4 t4 = *reinterpret_cast<const float4 *>(&row[4 * q]);
        xp[2 * q] = f32x2{t4.x, t4.y};
        xp[2 * q + 1] = f32x2{t4.z, t4.w};
    }
    f32x2 pa = f32x2{bl.x, 0.f}, qa = f32x2{0.f, 0.f}, pc = f32x2{bl.y, 0.f}, qc = f32x2{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        pa = __builtin_elementwise_fma(wa[i], xp[i], pa);
        pc = __builtin_elementwise_fma(wc[i], xp[i], pc);
        qa = __builtin_elementwise_fma(wa[i + 1], xp[i + 1], qa);
        qc = __builtin_elementwise_fma(wc[i + 1], xp[i + 1], qc);
    }
    return f32x2{(pa.x + pa.y) + (qa.x + qa.y), (pc.x + pc.y) + (qc.x + qc.y)};
}

template <int MODE, bool REF>
__global__ __launch_bounds__(64 * kTrainWaves) __attribute__((amdgpu_waves_per_eu(2))) void k_mlp_train(
    const int8_t *__restrict__ boards, int64_t rows, int64_t n_boards, const int8_t *__restrict__ actions,
    const float *__restrict__ targets, const float *__restrict__ wn, const float *__restrict__ cm,
    const float *__restrict__ counts, float beta, const float *__restrict__ w, float *__restrict__ partials)
{
    __shared__ float stash[kTrainWaves][64][kStash];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float(*st)[kStash] = stash[wave];
    // phase-2 weights of unit l = lane in input pairs (2i, 2i + 1) -- every phase-2 FMA is a
    // v_pk_fma_f32 over two inputs, whose values the LDS reads deliver as aligned pairs -- and its
    // gradient accumulators
    f32x2 wa[8], wc[8], w2l[2];
    const int pl = 32 * (lane >> 1) + (lane & 1);      // unit l's place in its pair's layer-1 block
#pragma unroll
    for (int i = 0; i < 8; i++) {
        wa[i] = f32x2{w[kA1W + pl + 4 * i], w[kA1W + pl + 4 * i + 2]};
        wc[i] = f32x2{w[kC1W + pl + 4 * i], w[kC1W + pl + 4 * i + 2]};
    }
#pragma unroll
    for (int k = 0; k < 2; k++)
        w2l[k] = f32x2{w[kA2W + 8 * (lane >> 1) + 4 * k + (lane & 1)], w[kA2W + 8 * (lane >> 1) + 4 * k + 2 + (lane & 1)]};
    const float wc2l = w[kC2W + lane];
    const f32x2 bl = f32x2{w[kA1B + lane], w[kC1B + lane]};
    // fp32 error bound of the unit's pre-activation: 16 roundings of partial sums below
    // |b| + sum |w| max x, i.e. < 2^-20 (|b| + sum |w| max x); 2x margin, + 2^-21 for the rounding
    // of the decision's own al - 3 (phase 2)
    f32x2 sl = f32x2{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; i++)
        sl += f32x2{fabsf(wa[i].x) + fabsf(wa[i].y), fabsf(wc[i].x) + fabsf(wc[i].y)};
    sl *= 0x1p-19f;
    const f32x2 el = f32x2{fmaf(fabsf(bl.x), 0x1p-19f, 0x1p-21f), fmaf(fabsf(bl.y), 0x1p-19f, 0x1p-21f)};
    f32x2 ga[8], gc[8], gbl = f32x2{0.f, 0.f}, g2l[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < 8; i++)
        ga[i] = gc[i] = f32x2{0.f, 0.f};
    float gc2 = 0.f;
    // per-row-lane sums (reduced over the wave at the end)
    float gb2[4] = {0.f, 0.f, 0.f, 0.f}, gbc2 = 0.f, loss_a = 0.f, loss_c = 0.f;
    // fp32 error bound of a pre-ReLU logit: its own sum (64 products of |h| <= 6 in parity halves:
    // < 2^-18 (|b2| + 6 sum |W2[k][:]|)) plus the hidden units' errors carried through W2 (each
    // < 2^-20 (|b1| + sum |W1[j][:]| max x), see sl above); 2x-4x margins
    // (wave-uniform: kept in SGPRs)
    float zedge[4], zcarry[4], hb = 0.f, hw = 0.f;
    for (int j = 0; j < 64; j++) {
        float sw = 0.f;
        for (int f = 0; f < 16; f++)
            sw += fabsf(w[kA1W + 32 * (j >> 1) + 2 * f + (j & 1)]);
        hw = fmaxf(hw, sw);
        hb = fmaxf(hb, fabsf(w[kA1B + j]));
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        float sa = 0.f;
        for (int j = 0; j < 64; j++)
            sa += fabsf(w[kA2W + 8 * (j >> 1) + 2 * k + (j & 1)]);
        zedge[k] = uniform((fabsf(w[kA2B + k]) + 6.0f * sa) * 0x1p-16f);
        zcarry[k] = uniform(sa * 0x1p-19f);
    }
    hb = uniform(hb);
    hw = uniform(hw);

    const int64_t n_tiles = (rows + 63) / 64;
    const int64_t stride = (int64_t)gridDim.x * kTrainWaves;
    for (int64_t tile = (int64_t)blockIdx.x * kTrainWaves + wave; tile < n_tiles; tile += stride) {
        // ---------------- phase 1: lane = row
        const int64_t r = tile * 64 + lane;
        const bool live = r < rows;
        const int64_t rr = live ? r : rows - 1;      // padding lanes: a valid row with weight 0
        float x[16], zr[4], v;
        board_inputs<MODE>(load_board(boards, rr), x);
        const float xmax = fmaxf(fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])), fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7]))),
                                 fmaxf(fmaxf(fmaxf(x[8], x[9]), fmaxf(x[10], x[11])), fmaxf(fmaxf(x[12], x[13]), fmaxf(x[14], x[15]))));
        // the row's inputs go to the stash at once (they are dead after the forward)
        wave_lds_sync();   // the previous tile's phase 2 has read the stash
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<float4 *>(&st[lane][4 * q]) = make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
        st[lane][21] = xmax;
        {
            const float *wp = w;
            f32x2 acc[4], c;
            hidden_both(wp, x, acc, c);
#pragma unroll
            for (int k = 0; k < 4; k++)
                zr[k] = wp[kA2B + k] + (acc[k].x + acc[k].y);      // pre-ReLU
            v = wp[kC2B] + (c.x + c.y);
        }
        const float wt = live ? wn[rr] : 0.0f;
        const float tgt = targets[rr];
        const int a = actions[rr] & 3;
        float z[4], p[4], gr[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            z[k] = fmaxf(zr[k], 0.0f);                            // the logits' ReLU (a3c.py:153)
        const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
        float se = 0.f;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            p[k] = __expf(z[k] - m);
            se += p[k];
        }
        const float inv = __builtin_amdgcn_rcpf(se), lse = m + kLn2 * __builtin_amdgcn_logf(se);
        float H = 0.f, gbar = 0.f;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            p[k] *= inv;
            const float lq = kLn2 * __builtin_amdgcn_logf(p[k] + kEntropyEps);
            H -= p[k] * lq;
            gr[k] = -(lq + p[k] * __builtin_amdgcn_rcpf(p[k] + kEntropyEps));   // dH/dp_k
            gbar += p[k] * gr[k];
        }
        const float td = tgt - v;
        float dz[4];
        if (REF) {   // reference: -beta wn H - cm sum_k c_k log p_k  (losses.py, a3c.py:110-116)
            const float c = live ? cm[rr] : 0.0f;
            const int64_t bidx = rows <= 0xFFFFFFFFll ? (int64_t)((uint32_t)rr % (uint32_t)n_boards) : rr % n_boards;
            const float4 cnt = *reinterpret_cast<const float4 *>(counts + 4 * bidx);
            const float ck[4] = {cnt.x, cnt.y, cnt.z, cnt.w}, C = cnt.x + cnt.y + cnt.z + cnt.w;
            float sa = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                dz[k] = -beta * wt * p[k] * (gr[k] - gbar) - c * (ck[k] - p[k] * C);
                sa += ck[k] * (z[k] - lse);
            }
            loss_a += -beta * wt * H - c * sa;
        } else {     // textbook: -wn (beta H + td log p[a]), td constant for the actor
#pragma unroll
            for (int k = 0; k < 4; k++)
                dz[k] = -wt * (beta * p[k] * (gr[k] - gbar) + td * ((k == a ? 1.0f : 0.0f) - p[k]));
            loss_a += -wt * (beta * H + td * (z[a] - lse));
        }
        const float dv = -2.0f * wt * td;                          // critic = wn td^2
        loss_c += wt * td * td;
        // through the logits' ReLU; a logit within its fp32 error bound of 0 is decided on its exact
        // value by the whole wave at the start of phase 2 (rows flagged in `near_rows`)
        bool near = false;
        float dzm[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            near |= fabsf(zr[k]) < zedge[k] + zcarry[k] * (hb + hw * xmax);
            dzm[k] = zr[k] > 0.0f ? dz[k] : 0.0f;
        }
        if (!near) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                gb2[k] += dzm[k];
        }
        const uint64_t near_rows = __ballot(near);
        gbc2 += dv;
        *reinterpret_cast<float4 *>(&st[lane][16]) = make_float4(dzm[0], dzm[1], dzm[2], dzm[3]);
        st[lane][20] = dv;
        if (near_rows)
            *reinterpret_cast<float4 *>(&st[lane][24]) = make_float4(dz[0], dz[1], dz[2], dz[3]);
        wave_lds_sync();
        // exact logits of the flagged rows, lane = hidden unit: its fp64 pre-activation, times W2,
        // summed over the wave; lane 0 writes the row's dz through the exact ReLU decision
        for (uint64_t m = near_rows; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            double ad = bl.x;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                ad = __builtin_fma((double)wa[i].x, (double)st[j][2 * i], ad);
                ad = __builtin_fma((double)wa[i].y, (double)st[j][2 * i + 1], ad);
            }
            const double hd = ad < 0.0 ? 0.0 : (ad > 6.0 ? 6.0 : ad);
            const double w2d[4] = {w2l[0].x, w2l[0].y, w2l[1].x, w2l[1].y};
            double t[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                t[k] = w2d[k] * hd;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1)
                    t[k] += __shfl_xor(t[k], o);
            }
            if (lane == 0) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float d = (double)w[kA2B + k] + t[k] > 0.0 ? st[j][24 + k] : 0.0f;
                    st[j][16 + k] = d;
                    gb2[k] += d;
                }
            }
        }
        if (near_rows)
            wave_lds_sync();
        // ---------------- phase 2: lane = hidden unit
        // the ReLU6 decisions 0 < a < 6, i.e. |a - 3| < 3, are taken on the fp32 values; a row whose
        // pre-activation lies within the fp32 error bound of 0 or 6 (min(|a|, |a - 6|) = ||a - 3| - 3|)
        // is flagged, and after the row loop its decision is redone in fp64 and, where it differs,
        // the row's term is moved (no branch in the row loop)
        uint32_t flagged[2] = {0u, 0u};
#pragma unroll 1
        for (int half = 0; half < 2; half++) {
            uint32_t fl = 0u;
#pragma unroll 2
            for (int jj = 0; jj < 32; jj++) {
                const int j = 32 * half + jj;
                f32x2 xp[8];
                const f32x2 ac = unit_preacts(st[j], wa, wc, bl, xp);
                const float4 dz4 = *reinterpret_cast<const float4 *>(&st[j][16]);
                const f32x2 dvm = *reinterpret_cast<const f32x2 *>(&st[j][20]);   // dv | max x
                const f32x2 d = ac - f32x2{3.0f, 3.0f};
                const f32x2 bound = __builtin_elementwise_fma(sl, f32x2{dvm.y, dvm.y}, el);
                const int edge = (int)(fabsf(fabsf(d.x) - 3.0f) < bound.x) | (int)(fabsf(fabsf(d.y) - 3.0f) < bound.y);
                fl = edge ? fl | (1u << jj) : fl;
                const float hl = __builtin_amdgcn_fmed3f(ac.x, 0.0f, 6.0f), hcl = __builtin_amdgcn_fmed3f(ac.y, 0.0f, 6.0f);
                const f32x2 sdh = w2l[0] * f32x2{dz4.x, dz4.y} + w2l[1] * f32x2{dz4.z, dz4.w};
                const float dha = fabsf(d.x) < 3.0f ? sdh.x + sdh.y : 0.0f;
                const float dhc = fabsf(d.y) < 3.0f ? wc2l * dvm.x : 0.0f;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    ga[i] = __builtin_elementwise_fma(f32x2{dha, dha}, xp[i], ga[i]);
                    gc[i] = __builtin_elementwise_fma(f32x2{dhc, dhc}, xp[i], gc[i]);
                }
                gbl += f32x2{dha, dhc};
                g2l[0] = __builtin_elementwise_fma(f32x2{dz4.x, dz4.y}, f32x2{hl, hl}, g2l[0]);
                g2l[1] = __builtin_elementwise_fma(f32x2{dz4.z, dz4.w}, f32x2{hl, hl}, g2l[1]);
                gc2 = __builtin_fmaf(dvm.x, hcl, gc2);
            }
            flagged[half] = fl;
        }
        // the flagged rows of this lane's unit (~1e-5 of the decisions; lanes diverge here)
        for (uint64_t m = ((uint64_t)flagged[1] << 32) | flagged[0]; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            f32x2 xp[8];
            const f32x2 ac = unit_preacts(st[j], wa, wc, bl, xp);
            const float4 dz4 = *reinterpret_cast<const float4 *>(&st[j][16]);
            const float dvr = st[j][20];
            double ad = bl.x, cd = bl.y;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                ad = __builtin_fma((double)wa[i].x, (double)xp[i].x, ad);
                ad = __builtin_fma((double)wa[i].y, (double)xp[i].y, ad);
                cd = __builtin_fma((double)wc[i].x, (double)xp[i].x, cd);
                cd = __builtin_fma((double)wc[i].y, (double)xp[i].y, cd);
            }
            const bool ma = ad > 0.0 && ad < 6.0, mc = cd > 0.0 && cd < 6.0;
            const bool ma32 = fabsf(ac.x - 3.0f) < 3.0f, mc32 = fabsf(ac.y - 3.0f) < 3.0f;
            const f32x2 sdh = w2l[0] * f32x2{dz4.x, dz4.y} + w2l[1] * f32x2{dz4.z, dz4.w};
            // + the row's term where the exact decision is "on", - where the fp32 one was
            const float dha = ma == ma32 ? 0.0f : (ma ? sdh.x + sdh.y : -(sdh.x + sdh.y));
            const float dhc = mc == mc32 ? 0.0f : (mc ? wc2l * dvr : -(wc2l * dvr));
#pragma unroll
            for (int i = 0; i < 8; i++) {
                ga[i] = __builtin_elementwise_fma(f32x2{dha, dha}, xp[i], ga[i]);
                gc[i] = __builtin_elementwise_fma(f32x2{dhc, dhc}, xp[i], gc[i]);
            }
            gbl += f32x2{dha, dhc};
        }
    }
    // ---------------- this wave's record (FlatParams order)
    float *rec = partials + ((int64_t)blockIdx.x * kTrainWaves + wave) * kRec;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        *reinterpret_cast<float4 *>(rec + kA1W + 16 * lane + 4 * q) =
            make_float4(ga[2 * q].x, ga[2 * q].y, ga[2 * q + 1].x, ga[2 * q + 1].y);
        *reinterpret_cast<float4 *>(rec + kC1W + 16 * lane + 4 * q) =
            make_float4(gc[2 * q].x, gc[2 * q].y, gc[2 * q + 1].x, gc[2 * q + 1].y);
    }
    rec[kA1B + lane] = gbl.x;
    rec[kC1B + lane] = gbl.y;
    rec[kA2W + lane] = g2l[0].x;
    rec[kA2W + 64 + lane] = g2l[0].y;
    rec[kA2W + 128 + lane] = g2l[1].x;
    rec[kA2W + 192 + lane] = g2l[1].y;
    rec[kC2W + lane] = gc2;
    const float s0 = wave_sum(gb2[0]), s1 = wave_sum(gb2[1]), s2 = wave_sum(gb2[2]), s3 = wave_sum(gb2[3]);
    const float sc = wave_sum(gbc2), la = wave_sum(loss_a), lc = wave_sum(loss_c);
    if (lane == 0) {
        *reinterpret_cast<float4 *>(rec + kA2B) = make_float4(s0, s1, s2, s3);
        rec[kC2B] = sc;
        rec[kRecLossA] = la;
        rec[kRecLossC] = lc;
        rec[kRec - 1] = 0.0f;
    }
}

// fixed-order sum of `n_rec` records of kRec floats into out[kRec]: pass 1 sums groups of kRedGroup
// records (one thread per (group, float4)), pass 2 the group sums
constexpr int kRedGroup = 64;

__global__ __launch_bounds__(256) void k_mlp_reduce1(const float4 *__restrict__ rec, int n_rec, float4 *__restrict__ groups)
{
    constexpr int q = kRec / 4;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n_grp = (n_rec + kRedGroup - 1) / kRedGroup;
    if (i >= q * n_grp)
        return;
    const int g = i / q, e = i % q;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = g * kRedGroup; r < n_rec && r < (g + 1) * kRedGroup; r++) {
        const float4 v = rec[(int64_t)r * q + e];
        s.x += v.x, s.y += v.y, s.z += v.z, s.w += v.w;
    }
    groups[(int64_t)g * q + e] = s;
}

__global__ __launch_bounds__(256) void k_mlp_reduce2(const float4 *__restrict__ groups, int n_grp, float4 *__restrict__ out)
{
    constexpr int q = kRec / 4;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= q)
        return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int g = 0; g < n_grp; g++) {
        const float4 v = groups[(int64_t)g * q + e];
        s.x += v.x, s.y += v.y, s.z += v.z, s.w += v.w;
    }
    out[e] = s;
}

constexpr int kTrainGroups = 1024;   // persistent grid: 4 workgroups of 4 waves per CU on 256 CUs

int fail(int code, const std::string &msg)
{
    r48::set_last_error(msg);
    return code;
}

int launched(const char *what)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return R48_OK;
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

}  // namespace

extern "C" {

int32_t r48_mlp_weight_floats(void) { return 2504; }

int r48_mlp_policy_forward(const int8_t *boards, int64_t n, const float *w, int32_t mode, float *logits, float *value,
                           int8_t *actions, uint64_t seed, int64_t gid0, uint32_t ctr, void *stream)
{
    if (!boards || !w || n < 0 || gid0 < 0 || (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS))
        return fail(R48_EINVAL, "r48_mlp_policy_forward: NULL argument, n/gid0 < 0 or bad mode");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(logits)) & 15u)
        return fail(R48_EINVAL, "r48_mlp_policy_forward: boards, w and logits must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    auto kern = mode == R48_FEAT_VALUES ? k_mlp_forward<R48_FEAT_VALUES> : k_mlp_forward<R48_FEAT_EXPONENTS>;
    hipLaunchKernelGGL(kern, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, boards, n, w, logits, value, actions,
                       gid0, (uint32_t)seed, (uint32_t)(seed >> 32), ctr);
    return launched("k_mlp_forward");
}

int r48_mlp_rollout(int8_t *boards, int64_t n, int32_t n_steps, const float *w, int32_t mode, int8_t *traj_boards,
                    int8_t *actions, uint8_t *done, float *reward, int32_t *lengths, float *values, uint64_t policy_seed,
                    int64_t gid0, uint32_t sample_ctr, uint64_t env_seed, uint32_t env_step, uint32_t flags,
                    void *stream)
{
    if (!boards || !w || !traj_boards || !actions || !done || n < 0 || gid0 < 0 || n_steps < 1 ||
        (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS) || (flags & ~R48_MERGE_REWARD))
        return fail(R48_EINVAL, "r48_mlp_rollout: NULL argument, n/gid0 < 0, n_steps < 1, bad mode or flags");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(traj_boards)) &
        15u)
        return fail(R48_EINVAL, "r48_mlp_rollout: boards, traj_boards and w must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const bool rw = flags & R48_MERGE_REWARD, vals = values != nullptr;
    const uint32_t pk0 = (uint32_t)policy_seed, pk1 = (uint32_t)(policy_seed >> 32);
    const uint32_t ek0 = (uint32_t)env_seed, ek1 = (uint32_t)(env_seed >> 32);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, boards, n, n_steps, w, traj_boards,
                           actions, done, reward, lengths, values, gid0, pk0, pk1, sample_ctr, ek0, ek1, env_step);
    };
#define R48_MLP_GO(M) \
    (rw ? (vals ? go(k_mlp_rollout<M, true, true>) : go(k_mlp_rollout<M, true, false>)) \
        : (vals ? go(k_mlp_rollout<M, false, true>) : go(k_mlp_rollout<M, false, false>)))
    if (mode == R48_FEAT_VALUES)
        R48_MLP_GO(R48_FEAT_VALUES);
    else
        R48_MLP_GO(R48_FEAT_EXPONENTS);
#undef R48_MLP_GO
    return launched("k_mlp_rollout");
}

/* workspace floats of r48_mlp_train_grad: the per-wave records + the first reduction pass's groups */
int64_t r48_mlp_train_workspace_floats(void)
{
    const int64_t recs = (int64_t)kTrainGroups * kTrainWaves;
    return (recs + (recs + kRedGroup - 1) / kRedGroup) * kRec;
}

int r48_mlp_train_grad(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                       const float *targets, const float *wn, const float *cm, const float *counts, float beta,
                       int32_t mode, const float *w, float *workspace, float *grad, void *stream)
{
    if (!boards || !actions || !targets || !wn || !w || !workspace || !grad || rows < 1 || n_boards < 1 ||
        (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS) || (cm && !counts))
        return fail(R48_EINVAL, "r48_mlp_train_grad: NULL argument, rows/n_boards < 1, bad mode, or cm without counts");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(counts) |
         reinterpret_cast<uintptr_t>(workspace) | reinterpret_cast<uintptr_t>(grad)) & 15u)
        return fail(R48_EINVAL, "r48_mlp_train_grad: boards, w, counts, workspace and grad must be 16-byte aligned");
    const int n_rec = kTrainGroups * kTrainWaves, n_grp = (n_rec + kRedGroup - 1) / kRedGroup;
    hipStream_t s = (hipStream_t)stream;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(kTrainGroups), dim3(64 * kTrainWaves), 0, s, boards, rows, n_boards, actions,
                           targets, wn, cm, counts, beta, w, workspace);
    };
    if (mode == R48_FEAT_VALUES)
        cm ? go(k_mlp_train<R48_FEAT_VALUES, true>) : go(k_mlp_train<R48_FEAT_VALUES, false>);
    else
        cm ? go(k_mlp_train<R48_FEAT_EXPONENTS, true>) : go(k_mlp_train<R48_FEAT_EXPONENTS, false>);
    float4 *groups = reinterpret_cast<float4 *>(workspace + (int64_t)n_rec * kRec);
    constexpr int q = kRec / 4;
    hipLaunchKernelGGL(k_mlp_reduce1, dim3((q * n_grp + 255) / 256), dim3(256), 0, s, (const float4 *)workspace, n_rec,
                       groups);
    hipLaunchKernelGGL(k_mlp_reduce2, dim3((q + 255) / 256), dim3(256), 0, s, (const float4 *)groups, n_grp,
                       (float4 *)grad);
    return launched("k_mlp_train");
}

}  // extern "C"
