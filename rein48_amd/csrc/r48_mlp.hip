// r48_mlp.hip -- the reference's own A3C network (algorithm/a3c/a3c.py:136-169, fp32) fused on gfx950.
//
// ActorCriticMLP (rein48_amd/a3c/nets.py): actor 16 -> 64 ReLU6 -> 4 ReLU (-> softmax), critic
// 16 -> 64 ReLU6 -> 1, on the 16 raw tile values (a3c.py:37-39,139) or exponents, fp32 like the
// reference. ONE BOARD PER LANE, 64 boards per wave: both 16 -> 64 layers (86 % of the FMAs) run on the
// f32 MFMA (v_mfma_f32_32x32x2_f32: exact f32, bit for bit the k-ordered fmaf chain, at twice the rate
// a packed-f32 VALU kernel reaches, and beside the VALU), the 64 -> 4 / 64 -> 1 layers, the draw and the
// env step on the VALU (mlp_forward below). Round 4 ran everything as v_pk_fma_f32 chains with the
// weights in SGPRs: rollout 6.68 -> 5.90 ms (reference loss, with V(s_t)), 3.92 -> 3.39 ms (textbook)
// per 100 steps of 2^20 boards (profiles/r05/a3c/mlp_policy_f32_mfma_ab.txt). (The fused update, which
// has row contractions to do, is in r48_mlp_train.hip.)
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
// c1 [32 p][16 in][2] | c1.b [64] | c2 [64] | c2.b [1] | pad; each kernel gathers the layer-1 A
// operands of its lanes from it once (32 VGPRs) and stages the layer-1 biases and layer-2 weights in
// LDS by lane half.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"
#include "r48_mlp_common.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBlock = 256;
constexpr uint32_t kSampleTag = 0xA3Cu;   // r48_a3c.hip k_sample's draw tag
using namespace r48mlp;

template <int MODE>
__device__ __forceinline__ void board_inputs(const r48::Board &b, float (&x)[16])
{
    const uint32_t w[4] = {b.w0, b.w1, b.w2, b.w3};
#pragma unroll
    for (int c = 0; c < 16; c++)
        x[c] = cell_input<MODE>((w[c >> 2] >> (8 * (c & 3))) & 0xFFu);
}

// ReLU6 as one v_med3_f32: fminf(fmaxf(a, 0), 6) on an MFMA result also costs a v_max_f32 a, a, a (the
// IEEE-mode quieting of a possible signalling NaN) per value -- 128 extra VALU per rollout step
__device__ __forceinline__ float relu6(float a) { return __builtin_amdgcn_fmed3f(a, 0.0f, 6.0f); }

// ---- the policy of a wave's 64 boards (lane l holds board l) ----
// Layer 1 (16 -> 64 actor, 16 -> 64 critic) on the f32 MFMA: D[unit][board] = W1 . x + b1 per unit block
// m (0, 1: actor units 32m..32m+31; 2, 3: critic) and board block nb (boards 32nb..32nb+31 of the wave),
// eight v_mfma_f32_32x32x2_f32 K-steps (inputs 2s + h) from C = the bias (LDS). An f32 MFMA is bit for
// bit the k-ordered fmaf chain, so every hidden unit is fma(w15, x15, ... fma(w0, x0, b1)) -- one chain
// in input order. Layer 2 (64 -> 4 actor, 64 -> 1
// critic) on the VALU: a lane holds 16 units of each block for one board (D rows 8(r >> 2) + 4h +
// (r & 3)), contracts them with its half's layer-2 weights (LDS), and one v_permlane32_swap + add per
// output sums the two halves into the lane that owns the board.

// A operands: a[m][s] = W1[unit 32(m & 1) + (lane & 31) of net m >> 1][input 2s + h] -- loaded once per
// kernel (32 VGPRs)
__device__ __forceinline__ void load_layer1(const float *__restrict__ w, int lane, float (&a)[4][8])
{
    const int h = lane >> 5;
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int u = 32 * (m & 1) + (lane & 31), w1 = m < 2 ? kA1W : kC1W;
#pragma unroll
        for (int s = 0; s < 8; s++)
            a[m][s] = w[w1 + 32 * (u >> 1) + 2 * (2 * s + h) + (u & 1)];
    }
}

// layer-2 weights by lane half h, actor block mm and D register r (unit u = 32 mm + 8(r >> 2) + 4h + (r & 3)):
// a2l[(2h + mm) 16 + r] = a2[0..3][u], c2l[(2h + mm) 16 + r] = c2[u]; and the layer-1 biases as the MFMA's
// C operand, b1l[(2m + h) 16 + r] = bias of D register r's unit in block m; filled by the whole block
__device__ __forceinline__ void stage_layer2(const float *__restrict__ w, float4 *a2l, float *c2l, float *b1l)
{
    const int t = threadIdx.x;
    if (t < 128) {
        const int m = t >> 5, h = (t >> 4) & 1, r = t & 15;
        b1l[t] = w[(m < 2 ? kA1B : kC1B) + 32 * (m & 1) + 8 * (r >> 2) + 4 * h + (r & 3)];
    }
    if (t < 64) {
        const int h = t >> 5, mm = (t >> 4) & 1, r = t & 15;
        const int u = 32 * mm + 8 * (r >> 2) + 4 * h + (r & 3), p = u >> 1, e = u & 1;
        a2l[t] = make_float4(w[kA2W + 8 * p + e], w[kA2W + 8 * p + 2 + e], w[kA2W + 8 * p + 4 + e],
                             w[kA2W + 8 * p + 6 + e]);
        c2l[t] = w[kC2W + u];
    }
}

__device__ __forceinline__ float2 swap32(float lo, float hi)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    return make_float2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// logits z (post-ReLU, a3c.py:153) and, when VALUE, the critic's value of the lane's board; every lane of
// the wave must be active (padding lanes run on a valid duplicate board)
template <bool VALUE>
__device__ __forceinline__ void mlp_forward(const float *__restrict__ w, const float (&a)[4][8], const float4 *a2l,
                                            const float *c2l, const float *b1l, int h, const float (&x)[16],
                                            float (&z)[4], float &v)
{
    // B operands of board block 0 / 1: one swap per K-step turns the lanes' own inputs (2s, 2s + 1)
    // into [own x_2s | partner's x_2s+1] and [partner's x_2s | own x_2s+1]
    float b0[8], b1[8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const float2 q = swap32(x[2 * s], x[2 * s + 1]);
        b0[s] = q.x;
        b1[s] = q.y;
    }
    float zp[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, vp[2] = {0.f, 0.f};
    constexpr int kM = VALUE ? 4 : 2;
    // Software pipeline over the 32-unit blocks: block m + 1's MFMA chains are issued before block m's
    // ReLU6 + layer-2 VALU (two D register pairs)...
    f32x16 D0[2], D1[2];
    auto issue = [&](int m, f32x16 &d0, f32x16 &d1) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float4 bq = reinterpret_cast<const float4 *>(b1l + (2 * m + h) * 16)[q];
            d0[4 * q] = bq.x, d0[4 * q + 1] = bq.y, d0[4 * q + 2] = bq.z, d0[4 * q + 3] = bq.w;
        }
        d1 = d0;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m][s], b0[s], d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m][s], b1[s], d1, 0, 0, 0);
        }
    };
    issue(0, D0[0], D1[0]);
#pragma unroll
    for (int m = 0; m < kM; m++) {
        if (m + 1 < kM)
            issue(m + 1, D0[(m + 1) & 1], D1[(m + 1) & 1]);
        const f32x16 &d0 = D0[m & 1], &d1 = D1[m & 1];
        const int base = (2 * h + (m & 1)) * 16;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const float h0 = relu6(d0[r]), h1 = relu6(d1[r]);
            if (m < 2) {
                const float4 wk = a2l[base + r];
                zp[0][0] = fmaf(wk.x, h0, zp[0][0]), zp[1][0] = fmaf(wk.x, h1, zp[1][0]);
                zp[0][1] = fmaf(wk.y, h0, zp[0][1]), zp[1][1] = fmaf(wk.y, h1, zp[1][1]);
                zp[0][2] = fmaf(wk.z, h0, zp[0][2]), zp[1][2] = fmaf(wk.z, h1, zp[1][2]);
                zp[0][3] = fmaf(wk.w, h0, zp[0][3]), zp[1][3] = fmaf(wk.w, h1, zp[1][3]);
            } else {
                const float wc = c2l[base + r];
                vp[0] = fmaf(wc, h0, vp[0]), vp[1] = fmaf(wc, h1, vp[1]);
            }
        }
        // ...and the scheduler is told to interleave them: one MFMA of block m + 1, then that many VALU of
        // block m (its 160 / 64 instructions over the next block's 16 MFMAs). Left alone it issues all
        // MFMAs first and the ReLU6 / layer-2 VALU after them.
        if (m + 1 < kM) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                if (m < 2)
                    __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);   // VALU
                else
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            }
        }
    }
    // the board's two halves: lanes 0-31 own block 0's boards, lanes 32-63 block 1's; half 0's part first
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float2 q = swap32(zp[0][k], zp[1][k]);
        z[k] = fmaxf(w[kA2B + k] + (q.x + q.y), 0.0f);
    }
    v = 0.0f;
    if (VALUE) {
        const float2 q = swap32(vp[0], vp[1]);
        v = w[kC2B] + (q.x + q.y);
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
    __shared__ float4 a2l[64];
    __shared__ float c2l[64];
    __shared__ __attribute__((aligned(16))) float b1l[128];
    stage_layer2(w, a2l, c2l, b1l);
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((i0 & ~63ll) >= n)
        return;   // a whole wave past the end (wave-uniform)
    const bool live = i0 < n;
    const int64_t i = live ? i0 : n - 1;   // padding lanes: a valid duplicate, nothing stored
    float a[4][8];
    load_layer1(w, lane, a);
    float x[16], z[4], v;
    board_inputs<MODE>(load_board(boards, i), x);
    if (value)   // wave-uniform
        mlp_forward<true>(w, a, a2l, c2l, b1l, h, x, z, v);
    else
        mlp_forward<false>(w, a, a2l, c2l, b1l, h, x, z, v);
    if (!live)
        return;
    if (logits)
        *reinterpret_cast<float4 *>(logits + 4 * i) = make_float4(z[0], z[1], z[2], z[3]);
    if (value)
        value[i] = v;
    if (actions)
        actions[i] = (int8_t)sample_action(z, (uint64_t)(gid0 + i), ctr, pk0, pk1);
}

// VALUES: also V(boards[t]) of every step (the reference loss's td sums need V of the training
// states before the gradient pass; rollout_values in trainer.py)
// The two waves of a SIMD run identical step loops from the same start: odd hardware wave slots issue at
// raised priority, so one wave runs ahead and the other fills its gaps instead of both reaching the
// MFMA-heavy layer 1 together (with the bias as the C operand: rollout 5.96 -> 5.78 ms, reference loss,
// n = 6, bit-identical; profiles/r05/a3c/mlp_policy_bias_c_desync_ab.txt)
__device__ __forceinline__ void desync_waves()
{
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (hw & 1)
        __builtin_amdgcn_s_setprio(1);
}

template <int MODE, bool REWARD, bool VALUES>
__global__ __launch_bounds__(kBlock) void k_mlp_rollout(int8_t *__restrict__ boards, int64_t n, int32_t T,
                                                        const float *__restrict__ w, int8_t *__restrict__ traj,
                                                        int8_t *__restrict__ actions, uint8_t *__restrict__ done,
                                                        float *__restrict__ reward, int32_t *__restrict__ lengths,
                                                        float *__restrict__ values, int64_t gid0, uint32_t pk0,
                                                        uint32_t pk1, uint32_t ctr0, uint32_t ek0, uint32_t ek1,
                                                        uint32_t step0)
{
    __shared__ float4 a2l[64];
    __shared__ float c2l[64];
    __shared__ __attribute__((aligned(16))) float b1l[128];
    stage_layer2(w, a2l, c2l, b1l);
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((i0 & ~63ll) >= n)
        return;   // a whole wave past the end (wave-uniform)
    const bool live = i0 < n;
    const int64_t i = live ? i0 : n - 1;   // padding lanes step a valid duplicate and store nothing
    float a[4][8];
    load_layer1(w, lane, a);
    desync_waves();
    const uint64_t gid = (uint64_t)(gid0 + i);
    r48::Board b = load_board(boards, i);
    int32_t len = T;
    for (int32_t t = 0; t < T; t++) {
        const int64_t at = (int64_t)t * n + i;
        if (live)
            store_board(traj, at, b);
        float x[16], z[4], v;
        board_inputs<MODE>(b, x);
        mlp_forward<VALUES>(w, a, a2l, c2l, b1l, h, x, z, v);
        const uint32_t act = sample_action(z, gid, ctr0 + (uint32_t)t, pk0, pk1);
        uint32_t dx, dy;
        r48::step_draw(gid, step0 + (uint32_t)t, ek0, ek1, dx, dy);
        const r48::StepOut o = r48::step_board<REWARD, false, true>(b, act, dy, (dx & 0x3FFFFFFFu) < r48::kFourThresh30);
        if (live) {
            if (VALUES)
                values[at] = v;
            actions[at] = (int8_t)act;
            done[at] = (uint8_t)o.done;
            if (reward)   // merge reward as fp32 (exact: < 2^24)
                reward[at] = REWARD ? (float)o.reward : 0.0f;
        }
        if (o.done && len == T)
            len = t + 1;   // through the first done step (a3c.py:201)
    }
    if (live) {
        store_board(traj, (int64_t)T * n + i, b);
        store_board(boards, i, b);
        if (lengths)
            lengths[i] = len;
    }
}


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

int32_t r48_mlp_weight_floats(void) { return kBlobFloats; }

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

}  // extern "C"
