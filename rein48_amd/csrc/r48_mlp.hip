// r48_mlp.hip -- the reference's own A3C network (algorithm/a3c/a3c.py:136-169, fp32) fused on gfx950.
//
// ActorCriticMLP (rein48_amd/a3c/nets.py): actor 16 -> 64 ReLU6 -> 4 ReLU (-> softmax), critic
// 16 -> 64 ReLU6 -> 1, on the 16 raw tile values (a3c.py:37-39,139) or exponents. The network is
// tiny (2,501 parameters, ~2.4 k FMAs per board) and fp32 like the reference, so it runs on the
// VALU with ONE BOARD PER LANE: the weights are wave-uniform and come through the scalar cache into
// SGPRs (s_load), the activations never leave the lane, and every FMA is a v_pk_fma_f32 over two
// hidden units. No MFMA: an fp32 16x64 layer has no bf16 form that keeps the reference's fp32
// numbers, and at one board per lane no data moves between lanes. (The fused update, which has
// row contractions to do, is in r48_mlp_train.hip.)
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
#include "r48_mlp_common.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

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
