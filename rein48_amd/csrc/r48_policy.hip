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
// (rein48_amd/a3c/fused.py). Per 32 boards: 9 + 64 + 16 = 89 MFMAs (~70 kFLOP per board).
// Weights (41 fragments x 1 KiB) are staged in LDS once per workgroup; waves loop over tiles.
// Biases enter as the MFMA accumulator, ReLU is an int16 max on the packed bf16 pairs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"
#include "r48_cnn_common.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using namespace r48cnn;

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr uint32_t kSampleTag = 0xA3Cu;

template <int MODE>
__global__ __launch_bounds__(kThreads, 2) void k_cnn_forward(const int8_t *__restrict__ boards, int64_t n,
                                                             const uint4 *__restrict__ wfrag,
                                                             const float *__restrict__ bias,
                                                             float *__restrict__ logits, float *__restrict__ value,
                                                             int8_t *__restrict__ actions,
                                                             int8_t *__restrict__ boards_out, int64_t gid0,
                                                             uint32_t k0, uint32_t k1, uint32_t ctr)
{
    __shared__ uint4 w_lds[kFrags * 64];
    __shared__ __attribute__((aligned(16))) float b_lds[32 + 64 + 8];   // float4 reads (load_bias)
    for (int i = threadIdx.x; i < kFrags * 64; i += kThreads)
        w_lds[i] = wfrag[i];
    for (int i = threadIdx.x; i < 32 + 64 + 8; i += kThreads)
        b_lds[i] = bias[i];
    __syncthreads();

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
        bf16x8 h1[9][2], h2[4][2][2];
        f32x16 out;
        WStream ws;
        ws.start(w_lds, fwd_frag(0), fwd_frag(1), lane);
        cnn_conv1(w_lds, b_lds, lane, h, x, ws, h1);
        cnn_conv2_heads(w_lds, b_lds, lane, h, h1, ws, h2, out);
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
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t tiles = (n + 31) / 32;
    const int64_t blocks = std::min<int64_t>((tiles + kWaves - 1) / kWaves, (int64_t)cus * 2);
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

}  // extern "C"
