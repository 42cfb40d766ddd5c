// r48_policy.hip -- fused CNN policy inference on gfx950 MFMA (BASELINE config 3).
//
// The 2-layer CNN of rein48_amd/a3c/nets.py:ActorCriticCNN (trunk of nevertiree/Rein48
// algorithm/ddpg/actor.py:51-85 + actor/critic heads), forward only, for the A3C rollout:
//   x[16] (board cells as bf16: raw tile value 2^e or the exponent e)
//   h1 = relu(conv2x2(x) + b1)      9 positions x 32 filters   (16 -> 288)
//   h2 = relu(conv2x2(h1) + b2)     4 positions x 64 filters   (288 -> 256, weights shared)
//   out = Wh h2 + bh                4 logits + 1 value
// and, optionally, the A3C action draw (softmax + Philox inverse CDF, identical to k_sample).
//
// Orientation: boards are the MFMA N dimension (one board per lane column, 32 boards per wave
// tile); features are rows. A 32x32 f32 accumulator of v_mfma_f32_32x32x16_bf16 then holds a
// board's features in the lane's registers, so each layer's output becomes the next layer's B
// operand in registers (v_cvt_pk_bf16_f32, no LDS, no lane movement). The k order inside such a
// fragment is permuted (element j of lane half h = row 16s + 8(j>>2) + 4h + (j&3)); the host
// packs the weight (A) fragments in exactly that order, once per parameter update
// (rein48_amd/a3c/fused.py). Per 32 boards: 9 + 64 32x32x16 MFMAs and, for the 5 head outputs,
// 16 v_mfma_f32_16x16x32_bf16 (half the cycles of 32x32 ones with 27 of 32 rows padding;
// r48_cnn_common.h cnn_conv2_heads16), ~70 kFLOP per board.
// Weights (33 fragments x 1 KiB) are staged in LDS once per workgroup; waves loop over tiles.
// Biases enter as the MFMA accumulator, ReLU is an int16 max on the packed bf16 pairs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"
#include "r48_cnn_common.h"
#include "r48_host.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using namespace r48cnn;

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
#ifndef R48_POLICY_OCC
#define R48_POLICY_OCC 2
#endif
constexpr int kOcc = R48_POLICY_OCC;   // workgroups (= waves per SIMD) per CU the forward is built for
#ifndef R48_ROLLOUT_OCC
#define R48_ROLLOUT_OCC 2
#endif
constexpr int kOccRoll = R48_ROLLOUT_OCC;
constexpr uint32_t kSampleTag = 0xA3Cu;
#ifndef R48_STAGE_PLAIN
#define R48_STAGE_PLAIN 0   // 1: the weight image staged by a plain load / store loop (A/B builds)
#endif

// conv1 + conv2 + heads of one 32-board tile: the fragment-grouped conv2 (r48_cnn_common.h) and the
// heads on 16x16x32 MFMAs (cnn_conv2_heads16): 33 LDS fragment reads and 9 + 64 32x32 + 16 16x16
// MFMAs per tile. Shared by k_cnn_forward and k_cnn_rollout, so both sum identically.
__device__ __forceinline__ void policy_logits(const uint4 *w_lds, const float *b_lds, int lane, int h, const bf16x8 &x,
                                              f32x16 &out)
{
    bf16x8 h1[9][2];
    PolicyWStream ws;
    ws.start(w_lds, lane);
    policy_conv1(w_lds, b_lds, lane, h, x, ws, h1);
    cnn_conv2_heads16(w_lds, b_lds, lane, h, h1, ws, out);
}

// The two waves of a SIMD run identical tile loops and start together, so their MFMA-free phases
// (conv1 epilogues, the dependent head chain, softmax + draw) can coincide. R48_POLICY_DESYNC: 1 =
// odd wave slots sleep ~2.5k cycles at entry, 2 (default) = odd wave slots issue at higher
// priority, so one wave runs ahead and the other fills its gaps (forward 0.0748 -> 0.0713 ms per
// 2^20 boards, 0.518 -> 0.503 ms per 2^23; rollout unchanged: profiles/r02/a3c/policy_grouped.txt).
#ifndef R48_POLICY_DESYNC
#define R48_POLICY_DESYNC 2
#endif
__device__ __forceinline__ void desync_waves()
{
    if (R48_POLICY_DESYNC) {
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        if (hw & 1) {
            if (R48_POLICY_DESYNC == 1)
                __builtin_amdgcn_s_sleep(40);
            else
                __builtin_amdgcn_s_setprio(1);
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, kOcc) void k_cnn_forward(const int8_t *__restrict__ boards, int64_t n,
                                                             const uint4 *__restrict__ wfrag,
                                                             const float *__restrict__ bias,
                                                             float *__restrict__ logits, float *__restrict__ value,
                                                             int8_t *__restrict__ actions,
                                                             int8_t *__restrict__ boards_out, int64_t gid0,
                                                             uint32_t k0, uint32_t k1, uint32_t ctr)
{
    __shared__ uint4 w_lds[kFragsPolicy * 64];
    __shared__ __attribute__((aligned(16))) float b_lds[32 + 64 + 8];   // float4 reads (load_bias)
#if R48_STAGE_PLAIN
    for (int i = threadIdx.x; i < kFragsPolicy * 64; i += kThreads)
        w_lds[i] = wfrag[i];
#else
    stage_lds<kFragsPolicy * 64, kThreads>(w_lds, wfrag);
#endif
    for (int i = threadIdx.x; i < 32 + 64 + 8; i += kThreads)
        b_lds[i] = bias[i];
    __syncthreads();
    desync_waves();

    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const int64_t n_tiles = (n + 31) / 32;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t tile = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    // board bytes are prefetched one tile ahead (clamped index: always a valid address)
    auto fetch = [&](int64_t t) {
        const int64_t bb = std::min<int64_t>(t * 32 + col, n - 1);
        return *reinterpret_cast<const uint2 *>(boards + 16 * bb + 8 * h);
    };
    uint2 next = fetch(std::min<int64_t>(tile, n_tiles - 1));
    for (; tile < n_tiles; tile += stride) {
        const int64_t b = tile * 32 + col;
        const bool live = b < n;
        // B operand of layer 1: cells 8h..8h+7 of this lane's board (k = 8h + j, natural order)
        const uint2 raw = next;
        next = fetch(std::min<int64_t>(tile + stride, n_tiles - 1));
        uint32_t xp[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t w = q < 2 ? raw.x : raw.y;
            const int sh = 16 * (q & 1);
            xp[q] = cell_bf16((w >> sh) & 0xffu, MODE) | (cell_bf16((w >> (sh + 8)) & 0xffu, MODE) << 16);
        }
        bf16x8 x;
        __builtin_memcpy(&x, xp, 16);
        // layer 1 (9 row tiles: one per conv1 output position, rows = 32 filters), then layer 2
        // (conv2: weights shared by the 4 output positions) fused with the heads; weight
        // fragments stream from LDS two MFMAs ahead (r48_cnn_common.h)
        f32x16 out;
        policy_logits(w_lds, b_lds, lane, h, x, out);
        if (!live)
            continue;  // padding lanes of the last tile computed on a clamped duplicate board
        if (boards_out)  // the rollout's trajectory snapshot of the input board (no separate copy)
            *reinterpret_cast<uint2 *>(boards_out + 16 * b + 8 * h) = raw;
        // head rows: lane half 0 registers 0..3 = logits 0..3, lane half 1 register 0 = value
        if (h == 0) {
            const float z0 = out[0] + b_lds[96], z1 = out[1] + b_lds[97], z2 = out[2] + b_lds[98],
                        z3 = out[3] + b_lds[99];
            if (logits)
                *reinterpret_cast<float4 *>(logits + 4 * b) = make_float4(z0, z1, z2, z3);
            if (actions) {
                const float m = fmaxf(fmaxf(z0, z1), fmaxf(z2, z3));
                const float e0 = __expf(z0 - m), e1 = __expf(z1 - m), e2 = __expf(z2 - m), e3 = __expf(z3 - m);
                const float inv = 1.0f / (e0 + e1 + e2 + e3);
                const float p0 = e0 * inv, c1 = p0 + e1 * inv, c2 = c1 + e2 * inv;
                uint32_t w[4] = {(uint32_t)(gid0 + b), (uint32_t)((uint64_t)(gid0 + b) >> 32), ctr, kSampleTag};
                r48::philox4x32_10(w, k0, k1);
                const float u = (float)(w[0] >> 8) * (1.0f / 16777216.0f);
                actions[b] = (int8_t)((p0 > u) ? 0 : (c1 > u) ? 1 : (c2 > u) ? 2 : 3);
            }
        } else if (value) {
            value[b] = out[0] + b_lds[100];
        }
    }
}

// ---------------------------------------------------------------- rollout megakernel
// The whole A3C rollout (a3c.py:194-212 batched, trainer.A3CTrainer.rollout) in one launch: every
// board is independent, so a wave keeps its boards in registers for all T steps and writes only
// the trajectory rows (pre-step board, action, done, merge reward) -- no per-step launches and no
// board round trip through HBM. A wave owns a PAIR of 32-board tiles (A, B). Lane (col, h) holds
// bytes 8h..8h+7 (rows 2h, 2h+1) of board col of both tiles. Per step: the policy of
// k_cnn_forward on A, then on B (boards on the MFMA columns), ONE softmax + draw pass for both
// (lane half 0 samples A's board, half 1 B's), then ONE env step pass (Game.step, GameClient.py:40-51, r48_board.h, the k_step draw contract) in which
// lane half 0 steps tile A's board and lane half 1 tile B's: one cross-half shuffle assembles the
// whole board, one more returns the halves -- every lane does useful env work. Per board the first
// step that ends done gives the segment length (a3c.py:201). Results are bit-identical to
// T x (r48_cnn_policy_forward + r48_env_step) (tests/test_a3c_gpu.py).

// logits rows of one 32-board tile (lane half 0: registers 0..3, without the head bias)
template <int MODE>
__device__ __forceinline__ f32x16 policy_out(const uint4 *w_lds, const float *b_lds, int lane, int h, uint2 raw)
{
    uint32_t xp[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t w = q < 2 ? raw.x : raw.y;
        const int sh = 16 * (q & 1);
        xp[q] = cell_bf16((w >> sh) & 0xffu, MODE) | (cell_bf16((w >> (sh + 8)) & 0xffu, MODE) << 16);
    }
    bf16x8 x;
    __builtin_memcpy(&x, xp, 16);
    f32x16 out;
    policy_logits(w_lds, b_lds, lane, h, x, out);
    return out;
}

// the action draw's uniform (Philox4x32-10 keyed by board and sample counter, the k_sample contract):
// it depends on neither the board nor the logits, so the rollout computes it before the step's
// policy MFMAs, where it fills their issue gaps
__device__ __forceinline__ float sample_uniform(uint64_t gid, uint32_t ctr, uint32_t pk0, uint32_t pk1)
{
    uint32_t w[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), ctr, kSampleTag};
    r48::philox4x32_10(w, pk0, pk1);
    return (float)(w[0] >> 8) * (1.0f / 16777216.0f);
}

// softmax + inverse CDF of one board's logits z at uniform u, exactly as k_cnn_forward's epilogue
__device__ __forceinline__ uint32_t sample_action(const float (&z)[4], float u)
{
    const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
    const float e0 = __expf(z[0] - m), e1 = __expf(z[1] - m), e2 = __expf(z[2] - m), e3 = __expf(z[3] - m);
    const float inv = 1.0f / (e0 + e1 + e2 + e3);
    const float p0 = e0 * inv, c1 = p0 + e1 * inv, c2 = c1 + e2 * inv;
    return (p0 > u) ? 0u : (c1 > u) ? 1u : (c2 > u) ? 2u : 3u;
}

// The env step's draws (the k_step contract, r48_board.h step_draw) of a lane PAIR holding boards
// 2q and 2q + 1 of one Philox call per pair-step: instead of both lanes computing the same call every
// step, each computes one call every OTHER step -- the even lane the call for step s, the odd lane
// the call for step s + 1 -- and the two words its partner needs cross the pair in one DPP swap.
// m = 0 on the even board, ~0 on the odd one; every lane of the wave must be active. Returns this
// board's (x, y) for steps s (d0) and s + 1 (d1), bit-identical to step_draw.
__device__ __forceinline__ void pair_block_draws(uint64_t q, uint32_t step, uint32_t m, uint32_t k0, uint32_t k1,
                                                 uint2 &d0, uint2 &d1)
{
    uint32_t w[4] = {(uint32_t)q, (uint32_t)(q >> 32), step + (m & 1u), r48::kStepTag};
    r48::philox4x32_r<r48::kStepRounds>(w, k0, k1);
    auto swap = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); };
    // the even lane holds call(step) and gives words 2, 3 (its partner's step draws); the odd lane
    // holds call(step + 1) and gives words 0, 1 (its partner's step + 1 draws)
    const uint32_t rx = swap(r48::bsel(m, w[0], w[2])), ry = swap(r48::bsel(m, w[1], w[3]));
    d0 = make_uint2(r48::bsel(m, rx, w[0]), r48::bsel(m, ry, w[1]));
    d1 = make_uint2(r48::bsel(m, w[2], rx), r48::bsel(m, w[3], ry));
}

template <int MODE, bool REWARD>
__global__ __launch_bounds__(kThreads, kOccRoll) void k_cnn_rollout(int8_t *__restrict__ boards, int64_t n, int32_t T,
                                                             const uint4 *__restrict__ wfrag,
                                                             const float *__restrict__ bias,
                                                             int8_t *__restrict__ traj, int8_t *__restrict__ actions,
                                                             uint8_t *__restrict__ done, float *__restrict__ reward,
                                                             int32_t *__restrict__ lengths, float *__restrict__ values,
                                                             int64_t gid0, uint32_t pk0,
                                                             uint32_t pk1, uint32_t ctr0, uint32_t ek0, uint32_t ek1,
                                                             uint32_t step0)
{
    __shared__ uint4 w_lds[kFragsPolicy * 64];
    __shared__ __attribute__((aligned(16))) float b_lds[32 + 64 + 8];
#if R48_STAGE_PLAIN
    for (int i = threadIdx.x; i < kFragsPolicy * 64; i += kThreads)
        w_lds[i] = wfrag[i];
#else
    stage_lds<kFragsPolicy * 64, kThreads>(w_lds, wfrag);
#endif
    for (int i = threadIdx.x; i < 32 + 64 + 8; i += kThreads)
        b_lds[i] = bias[i];
    __syncthreads();
    desync_waves();

    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const int64_t n_pairs = (n + 63) / 64;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    for (int64_t pair = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); pair < n_pairs; pair += stride) {
        const int64_t bA = pair * 64 + col, bB = bA + 32;
        const bool liveA = bA < n, liveB = bB < n;
        const int64_t cA = liveA ? bA : n - 1, cB = liveB ? bB : n - 1;   // padding lanes: a valid duplicate
        uint2 rawA = *reinterpret_cast<const uint2 *>(boards + 16 * cA + 8 * h);
        uint2 rawB = *reinterpret_cast<const uint2 *>(boards + 16 * cB + 8 * h);
        const uint64_t gA = (uint64_t)(gid0 + cA), gB = (uint64_t)(gid0 + cB);
        // the board this lane steps in the env pass: tile A in half 0, tile B in half 1
        const int64_t bE = h == 0 ? bA : bB;
        const bool liveE = h == 0 ? liveA : liveB;
        const uint64_t gE = h == 0 ? gA : gB;
        int32_t len = T;
        // lanes col, col ^ 1 of a half hold boards 2q, 2q + 1 when gid0 is even (wave-uniform): they
        // share the env draws (pair_block_draws); otherwise every lane draws for itself
        const bool paired = (gid0 & 1) == 0;
        const uint32_t pm = 0u - (uint32_t)(col & 1);
        uint2 draw0 = make_uint2(0u, 0u), draw1 = draw0;
        for (int32_t t = 0; t < T; t++) {
            const int64_t row0 = (int64_t)t * n;
            if (paired && (t & 1) == 0)
                pair_block_draws(gE >> 1, step0 + (uint32_t)t, pm, ek0, ek1, draw0, draw1);
            if (liveA)
                *reinterpret_cast<uint2 *>(traj + 16 * (row0 + bA) + 8 * h) = rawA;
            if (liveB)
                *reinterpret_cast<uint2 *>(traj + 16 * (row0 + bB) + 8 * h) = rawB;
            const float u = sample_uniform(gE, ctr0 + (uint32_t)t, pk0, pk1);
            const f32x16 oA = policy_out<MODE>(w_lds, b_lds, lane, h, rawA);
            const f32x16 oB = policy_out<MODE>(w_lds, b_lds, lane, h, rawB);
            // V(pre-step board): the value head sits in register 0 of lane half 1 (as in
            // k_cnn_forward, same bias add), so the reference loss needs no separate value pass
            if (values && h == 1) {
                if (liveA)
                    values[row0 + bA] = oA[0] + b_lds[100];
                if (liveB)
                    values[row0 + bB] = oB[0] + b_lds[100];
            }
            // one draw pass for both tiles: half 0 samples A's board col, half 1 B's (whose logits
            // sit in half 0 of oB) -- the lane's action is the one its env step below needs
            float z[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float zb = __shfl_xor(oB[k], 32);
                z[k] = (h == 0 ? oA[k] : zb) + b_lds[96 + k];
            }
            const uint32_t act = sample_action(z, u);
            // assemble the env board: half 0 gets A's rows 2-3 from its partner, half 1 B's rows 0-1
            const uint2 send = h == 0 ? rawB : rawA;
            const uint2 recv = make_uint2((uint32_t)__shfl_xor((int)send.x, 32), (uint32_t)__shfl_xor((int)send.y, 32));
            r48::Board bd = h == 0 ? r48::Board{rawA.x, rawA.y, recv.x, recv.y} : r48::Board{recv.x, recv.y, rawB.x, rawB.y};
            uint32_t dx, dy;
            if (paired) {
                dx = (t & 1) ? draw1.x : draw0.x;
                dy = (t & 1) ? draw1.y : draw0.y;
            } else {
                r48::step_draw(gE, step0 + (uint32_t)t, ek0, ek1, dx, dy);
            }
            const r48::StepOut o =
                r48::step_board<REWARD, false, true>(bd, act, dy, (dx & 0x3FFFFFFFu) < r48::kFourThresh30);
            // return the halves: half 0 keeps A's rows 0-1, half 1 keeps B's rows 2-3, and each sends
            // the other half of its board to its partner
            const uint2 back = h == 0 ? make_uint2(bd.w2, bd.w3) : make_uint2(bd.w0, bd.w1);
            const uint2 got = make_uint2((uint32_t)__shfl_xor((int)back.x, 32), (uint32_t)__shfl_xor((int)back.y, 32));
            if (h == 0) {
                rawA = make_uint2(bd.w0, bd.w1);
                rawB = got;
            } else {
                rawA = got;
                rawB = make_uint2(bd.w2, bd.w3);
            }
            if (o.done && len == T)
                len = t + 1;                                   // through the first done step
            if (liveE) {
                actions[row0 + bE] = (int8_t)act;
                done[row0 + bE] = (uint8_t)o.done;
                if (reward)   // merge reward as fp32 (exact: < 2^24), the update's input as is
                    reward[row0 + bE] = REWARD ? (float)o.reward : 0.0f;
            }
        }
        const int64_t rowT = (int64_t)T * n;
        if (liveA) {
            *reinterpret_cast<uint2 *>(traj + 16 * (rowT + bA) + 8 * h) = rawA;
            *reinterpret_cast<uint2 *>(boards + 16 * bA + 8 * h) = rawA;
        }
        if (liveB) {
            *reinterpret_cast<uint2 *>(traj + 16 * (rowT + bB) + 8 * h) = rawB;
            *reinterpret_cast<uint2 *>(boards + 16 * bB + 8 * h) = rawB;
        }
        if (lengths && liveE)
            lengths[bE] = len;
    }
}

int fail(int code, const std::string &msg)
{
    r48::set_last_error(msg);
    return code;
}

}  // namespace

extern "C" {

int r48_cnn_policy_forward(const int8_t *boards, int64_t n, const void *wfrag, const float *bias, int32_t mode,
                           float *logits, float *value, int8_t *actions, int8_t *boards_out, uint64_t seed,
                           int64_t gid0, uint32_t ctr, void *stream)
{
    if (!boards || !wfrag || !bias || n < 0 || gid0 < 0 || (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS))
        return fail(R48_EINVAL, "NULL argument, n/gid0 < 0 or bad mode");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(wfrag) |
         reinterpret_cast<uintptr_t>(boards_out)) & 15u ||
        (logits && (reinterpret_cast<uintptr_t>(logits) & 15u)))
        return fail(R48_EINVAL, "boards, boards_out, wfrag and logits must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const int cus = r48::device_cus(r48::stream_device((hipStream_t)stream));
    const int64_t tiles = (n + 31) / 32;
    const int64_t blocks = std::min<int64_t>((tiles + kWaves - 1) / kWaves, (int64_t)cus * kOcc);
    // one instantiation per input encoding (no per-cell branch)
    auto kern = mode == R48_FEAT_VALUES ? k_cnn_forward<R48_FEAT_VALUES> : k_cnn_forward<R48_FEAT_EXPONENTS>;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, boards, n,
                       (const uint4 *)wfrag, bias, logits, value, actions, boards_out, gid0, (uint32_t)seed,
                       (uint32_t)(seed >> 32), ctr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string("k_cnn_forward: ") + hipGetErrorString(e));
    return R48_OK;
}

int r48_cnn_rollout(int8_t *boards, int64_t n, int32_t n_steps, const void *wfrag, const float *bias, int32_t mode,
                    int8_t *traj_boards, int8_t *actions, uint8_t *done, float *reward, int32_t *lengths,
                    float *values, uint64_t policy_seed, int64_t gid0, uint32_t sample_ctr, uint64_t env_seed, uint32_t env_step,
                    uint32_t flags, void *stream)
{
    if (!boards || !wfrag || !bias || !traj_boards || !actions || !done || n < 0 || gid0 < 0 || n_steps < 1 ||
        (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS) || (flags & ~R48_MERGE_REWARD))
        return fail(R48_EINVAL, "r48_cnn_rollout: NULL argument, n/gid0 < 0, n_steps < 1, bad mode or flags");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(wfrag) |
         reinterpret_cast<uintptr_t>(traj_boards)) & 15u)
        return fail(R48_EINVAL, "boards, traj_boards and wfrag must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const int cus = r48::device_cus(r48::stream_device((hipStream_t)stream));
    const int64_t pairs = (n + 63) / 64;
    const int64_t blocks = std::min<int64_t>((pairs + kWaves - 1) / kWaves, (int64_t)cus * kOccRoll);
    const bool rw = flags & R48_MERGE_REWARD;
    auto kern = mode == R48_FEAT_VALUES ? (rw ? k_cnn_rollout<R48_FEAT_VALUES, true> : k_cnn_rollout<R48_FEAT_VALUES, false>)
                                        : (rw ? k_cnn_rollout<R48_FEAT_EXPONENTS, true>
                                              : k_cnn_rollout<R48_FEAT_EXPONENTS, false>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)stream, boards, n, n_steps,
                       (const uint4 *)wfrag, bias, traj_boards, actions, done, reward, lengths, values, gid0, (uint32_t)policy_seed,
                       (uint32_t)(policy_seed >> 32), sample_ctr, (uint32_t)env_seed, (uint32_t)(env_seed >> 32),
                       env_step);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string("k_cnn_rollout: ") + hipGetErrorString(e));
    return R48_OK;
}

}  // extern "C"
