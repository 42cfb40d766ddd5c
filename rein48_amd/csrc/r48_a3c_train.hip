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
//   loss      per row: d out = dL/d(logits, value)   (softmax, entropy, td; lane-local)
//   backward  dh2 = Wh^T dout . [h2 > 0]                                          8 MFMAs
//             dh1 = W2^T dh2 . [h1 > 0]      (conv2 transposed, shared over positions) 64 MFMAs
//   weights   dWh = dout h2^T, dW2 = dh2 h1^T, dW1 = dh1 x^T (+ biases by a ones row/column):
//             these contract over ROWS, so rows move to the MFMA K dimension: the lanes of one
//             16-row half-tile store their activations / gradients as packed 8-byte chunks into a
//             per-wave [row][feature] LDS image and the operands are read back transposed with
//             ds_read_b64_tr_b16 (gfx950).                                       ~100 MFMAs
// dW2 (+ its bias) and dW1 (+ bias) accumulate in AGPRs for the whole kernel; dWh (+ bias) in a
// per-wave LDS block. Every wave owns its LDS images and accumulators, so after the weights are
// staged no workgroup barrier is needed. Each wave writes one partial record; k_reduce sums
// the records in a fixed order (deterministic).
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
#define R48_LDS __attribute__((address_space(3)))

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kFragWhT = 8, kFragW2T = 16;
constexpr int kFragsTrain = kFrags + kFragWhT + kFragW2T;    // 65: forward 41 | Wh^T 8 | W2^T 16
constexpr int kOffWhT = kFrags, kOffW2T = kFrags + kFragWhT;
// per-wave LDS image region (bf16 elements), one 16-row half-tile at a time:
//   phase A: img_h2 [16][288] (256 features + ones column) + img_dout [8][16]
//   phase B: img_dh2 [16][256] + img_h1 [16][288]
//   phase C: img_dh1 [16][288] + img_x [16 cells][16 rows]
constexpr int kStrideH2 = 288, kStrideDh2 = 256, kStrideH1 = 288;
constexpr int kImgElems = 16 * kStrideDh2 + 16 * kStrideH1;  // 8704 bf16 = 17 KiB (phase B, the largest)
constexpr int kAccWhCols = 288;                               // dWh accumulator [5][288] f32 (col 256 = bias)
// partial record per wave (floats): dW2 [64][128] | db2 [64] | dW1 [32][5] | dWh [5][257] | losses [2]
constexpr int kOffDb2 = 64 * 128, kOffDw1 = kOffDb2 + 64, kOffDwh = kOffDw1 + 32 * 5, kOffLoss = kOffDwh + 5 * 257;
constexpr int kPartial = kOffLoss + 2;                        // 9703
constexpr float kEntropyEps = 1e-5f;                          // a3c.py:114
// ablation knob for tools/exp_train_ablate.py (wrong gradients when nonzero; never in the product
// build): bit 0 drops phase A, bit 1 phase B, bit 2 dh1 + phase C (7 leaves forward + loss)
#ifndef R48_TRAIN_SKIP
#define R48_TRAIN_SKIP 0
#endif
constexpr int kSkip = R48_TRAIN_SKIP;

// conv1's 2x2 patches over the 4x4 board: cell of tap t (row-major dr, dc) at output position R
__device__ __forceinline__ int cell_of(int R, int t) { return (R / 3 + (t >> 1)) * 4 + (R % 3) + (t & 1); }

// 32x32x16 operand with k = row of a 16-row half-tile (k = 8h + j) and the operand's row/column
// index = image column c0 + (lane & 31), from a [row][column] bf16 image: two transposed reads
// (lane 4q + p of each 16-lane group addresses image row q, columns 4p..4p+3 of its block).
__device__ __forceinline__ bf16x8 tr_operand(const uint16_t *img, int stride, int c0, int lane)
{
    const int g = lane >> 4, i = lane & 15, h = g >> 1;
    const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
    const uint16_t *a0 = img + (8 * h + (i >> 2)) * stride + col;
    const uint16_t *a1 = a0 + 4 * stride;
    const i16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((R48_LDS i16x4 *)(a0));
    const i16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((R48_LDS i16x4 *)(a1));
    bf16x8 f;
    __builtin_memcpy(&f, &r0, 8);
    __builtin_memcpy(reinterpret_cast<char *>(&f) + 8, &r1, 8);
    return f;
}

// store a B-layout fragment (elements j = channel cbase + 8(j>>2) + 4h + (j&3)) of image row
// `row` as two packed 8-byte chunks
__device__ __forceinline__ void store_frag(uint16_t *img, int stride, int row, int cbase, int h, const bf16x8 &f)
{
    uint4 v;
    __builtin_memcpy(&v, &f, 16);
    *reinterpret_cast<uint2 *>(img + row * stride + cbase + 4 * h) = make_uint2(v.x, v.y);
    *reinterpret_cast<uint2 *>(img + row * stride + cbase + 8 + 4 * h) = make_uint2(v.z, v.w);
}

// ReLU'(activation) of one 32-row accumulator tile as 16 bits: bit i <-> accumulator register i =
// element i & 7 of fragment i >> 3 (activations are >= 0 post-ReLU bf16, so "> 0" as int16).
// Keeping the masks as bits lets the activations themselves die early (register pressure).
__device__ __forceinline__ uint32_t relu_bits(const bf16x8 &a0, const bf16x8 &a1)
{
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 16; i++)
        m |= ((i < 8 ? a0[i] : a1[i - 8]) > 0 ? 1u : 0u) << i;
    return m;
}

__device__ __forceinline__ f32x16 relu_mask(f32x16 acc, uint32_t bits)
{
#pragma unroll
    for (int i = 0; i < 16; i++)
        acc[i] = ((bits >> i) & 1u) ? acc[i] : 0.0f;
    return acc;
}

__device__ __forceinline__ bf16x8 ones_frag()
{
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; j++)
        f[j] = (short)0x3F80;
    return f;
}

__global__ __launch_bounds__(kThreads, 1) void k_cnn_train(
    const int8_t *__restrict__ boards, int64_t rows, int64_t n_boards, const int8_t *__restrict__ actions,
    const float *__restrict__ targets, const float *__restrict__ wn, const float *__restrict__ cm,
    const float *__restrict__ counts, float beta, int32_t mode, const uint4 *__restrict__ wfrag,
    const float *__restrict__ bias, float *__restrict__ partials)
{
    extern __shared__ uint4 lds[];
    uint4 *w_lds = lds;                                                   // kFragsTrain x 1 KiB
    float *b_lds = reinterpret_cast<float *>(lds + kFragsTrain * 64);     // 104 floats in 32 x 16 B
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, col = lane & 31;
    uint16_t *img = reinterpret_cast<uint16_t *>(lds + kFragsTrain * 64 + 32) + wave * kImgElems;
    float *acc_wh = reinterpret_cast<float *>(reinterpret_cast<uint16_t *>(lds + kFragsTrain * 64 + 32) +
                                              kWaves * kImgElems) + wave * 5 * kAccWhCols;
    for (int i = threadIdx.x; i < kFragsTrain * 64; i += kThreads)
        w_lds[i] = wfrag[i];
    for (int i = threadIdx.x; i < 104; i += kThreads)
        b_lds[i] = bias[i];
    for (int i = lane; i < 5 * kAccWhCols; i += 64)
        acc_wh[i] = 0.0f;
    __syncthreads();

    const f32x16 zero = {};
    const bf16x8 ones = ones_frag();
    f32x16 dw2[2][4], db2[2], dw1;
#pragma unroll
    for (int g = 0; g < 2; g++) {
        db2[g] = zero;
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
            dw2[g][kk] = zero;
    }
    dw1 = zero;
    float loss_actor = 0.0f, loss_critic = 0.0f;

    const int64_t n_tiles = (rows + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < n_tiles; tile += (int64_t)gridDim.x * kWaves) {
        const int64_t r = tile * 32 + col;
        const bool live = r < rows;
        const int64_t rr = live ? r : rows - 1;          // padding lanes compute on a valid row, weight 0
        // ---------------- forward (r48_policy.hip k_cnn_forward)
        const uint2 raw = *reinterpret_cast<const uint2 *>(boards + 16 * rr + 8 * h);
        uint32_t xp[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t w = q < 2 ? raw.x : raw.y;
            const int sh = 16 * (q & 1);
            xp[q] = cell_bf16((w >> sh) & 0xffu, mode) | (cell_bf16((w >> (sh + 8)) & 0xffu, mode) << 16);
        }
        bf16x8 x;
        __builtin_memcpy(&x, xp, 16);
        bf16x8 h1[9][2];
#pragma unroll
        for (int R = 0; R < 9; R++) {
            f32x16 a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w_lds, R, lane), x, zero, 0, 0, 0);
            a = bias_relu(a, load_bias(b_lds, h));
            h1[R][0] = acc_to_frag(a, 0);
            h1[R][1] = acc_to_frag(a, 1);
        }
        bf16x8 h2[4][2][2];
        f32x16 out = zero;
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int g = 0; g < 2; g++) {
                f32x16 a = zero;
#pragma unroll
                for (int kk = 0; kk < 4; kk++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w_lds, kFragW1 + (g * 4 + kk) * 2 + s, lane),
                                                                    h1[kP2[p][kk]][s], a, 0, 0, 0);
                a = bias_relu(a, load_bias(b_lds + 32 + 32 * g, h));
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    h2[p][g][s] = acc_to_frag(a, s);
                    out = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        frag_at(w_lds, kFragW1 + kFragW2 + (p * 2 + g) * 2 + s, lane), h2[p][g][s], out, 0, 0, 0);
                }
            }
        uint32_t m1[9], m2[8];
#pragma unroll
        for (int R = 0; R < 9; R++)
            m1[R] = relu_bits(h1[R][0], h1[R][1]);
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int g = 0; g < 2; g++)
                m2[2 * p + g] = relu_bits(h2[p][g][0], h2[p][g][1]);
        // ---------------- loss gradient per row (lane half 0: logits rows 0..3; value in lane + 32)
        const float v = __shfl(out[0], col + 32) + b_lds[100];
        float dz[4] = {0.f, 0.f, 0.f, 0.f}, dv = 0.f;
        if (h == 0) {
            const float wt = live ? wn[rr] : 0.0f;
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
            const float inv = 1.0f / se, lse = m + __logf(se);
            float H = 0.f, gbar = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                p[k] *= inv;
                const float lq = __logf(p[k] + kEntropyEps);
                H -= p[k] * lq;
                g[k] = -(lq + p[k] / (p[k] + kEntropyEps));     // dH/dp_k
                gbar += p[k] * g[k];
            }
            const float td = targets[rr] - v;
            const int a = actions[rr] & 3;
            if (cm) {   // reference: -beta wn H - cm sum_k c_k log p_k  (losses.py, a3c.py:110-116)
                const float c = live ? cm[rr] : 0.0f;
                const float4 cnt = *reinterpret_cast<const float4 *>(counts + 4 * (rr % n_boards));
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
        // ---------------- phase A: dWh (+ bias) = dout h2^T over the tile's rows
#pragma unroll
        for (int u = 0; u < ((kSkip & 1) ? 0 : 2); u++) {
            if ((col >> 4) == u) {
                const int rowi = col & 15;
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int g = 0; g < 2; g++)
#pragma unroll
                        for (int s = 0; s < 2; s++)
                            store_frag(img, kStrideH2, rowi, 64 * p + 32 * g + 16 * s, h, h2[p][g][s]);
                if (h == 0) {
                    *reinterpret_cast<uint2 *>(img + rowi * kStrideH2 + 256) = make_uint2(0x3F80u, 0u);   // ones column
                    uint16_t *dimg = img + 16 * kStrideH2;                                              // [o][16 rows]
                    const float dd[5] = {dz[0], dz[1], dz[2], dz[3], dv};
#pragma unroll
                    for (int o = 0; o < 5; o++)
                        dimg[o * 16 + rowi] = __builtin_bit_cast(uint16_t, (__bf16)dd[o]);
                }
            }
            // A[row o][k = row]: lanes with o < 5 read their 8 rows of img_dout
            bf16x8 aout = {};
            if (col < 5) {
                const uint4 v4 = *reinterpret_cast<const uint4 *>(img + 16 * kStrideH2 + col * 16 + 8 * h);
                __builtin_memcpy(&aout, &v4, 16);
            }
#pragma unroll
            for (int T = 0; T < 9; T++) {
                const f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aout, tr_operand(img, kStrideH2, 32 * T, lane),
                                                                         zero, 0, 0, 0);
                // D rows o: half 0 registers 0..3 = o 0..3, half 1 register 0 = o 4
                if (h == 0) {
#pragma unroll
                    for (int o = 0; o < 4; o++)
                        acc_wh[o * kAccWhCols + 32 * T + col] += d[o];
                } else {
                    acc_wh[4 * kAccWhCols + 32 * T + col] += d[0];
                }
            }
        }
        // ---------------- dh2 = Wh^T dout . [h2 > 0]
        bf16x8 dh2[4][2][2];
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int g = 0; g < 2; g++) {
                f32x16 a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_at(w_lds, kOffWhT + p * 2 + g, lane), dout,
                                                                   zero, 0, 0, 0);
                a = relu_mask(a, m2[2 * p + g]);
                dh2[p][g][0] = acc_to_frag(a, 0);
                dh2[p][g][1] = acc_to_frag(a, 1);
            }
        // ---------------- phase B: dW2 = sum_p dh2[p] h1[patch p]^T, db2 = sum_p dh2[p] 1^T
#pragma unroll
        for (int u = 0; u < ((kSkip & 2) ? 0 : 2); u++) {
            uint16_t *img_dh2 = img, *img_h1 = img + 16 * kStrideDh2;
            if ((col >> 4) == u) {
                const int rowi = col & 15;
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int g = 0; g < 2; g++)
#pragma unroll
                        for (int s = 0; s < 2; s++)
                            store_frag(img_dh2, kStrideDh2, rowi, 64 * p + 32 * g + 16 * s, h, dh2[p][g][s]);
#pragma unroll
                for (int R = 0; R < 9; R++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        store_frag(img_h1, kStrideH1, rowi, 32 * R + 16 * s, h, h1[R][s]);
            }
#pragma unroll
            for (int p = 0; p < 4; p++) {
                bf16x8 B[4];
#pragma unroll
                for (int kk = 0; kk < 4; kk++)
                    B[kk] = tr_operand(img_h1, kStrideH1, 32 * kP2[p][kk], lane);
#pragma unroll
                for (int g = 0; g < 2; g++) {
                    const bf16x8 A = tr_operand(img_dh2, kStrideDh2, 64 * p + 32 * g, lane);
#pragma unroll
                    for (int kk = 0; kk < 4; kk++)
                        dw2[g][kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B[kk], dw2[g][kk], 0, 0, 0);
                    db2[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, ones, db2[g], 0, 0, 0);
                }
            }
        }
        // ---------------- dh1 = W2^T dh2 . [h1 > 0] (each conv1 position gathers the conv2 outputs
        // whose patch contains it)
        bf16x8 dh1[9][2];
#pragma unroll
        for (int R = 0; R < ((kSkip & 4) ? 0 : 9); R++) {
            f32x16 a = zero;
#pragma unroll
            for (int p = 0; p < 4; p++)
#pragma unroll
                for (int kk = 0; kk < 4; kk++)
                    if (kP2[p][kk] == R) {
#pragma unroll
                        for (int g = 0; g < 2; g++)
#pragma unroll
                            for (int s = 0; s < 2; s++)
                                a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    frag_at(w_lds, kOffW2T + (kk * 2 + g) * 2 + s, lane), dh2[p][g][s], a, 0, 0, 0);
                    }
            a = relu_mask(a, m1[R]);
            dh1[R][0] = acc_to_frag(a, 0);
            dh1[R][1] = acc_to_frag(a, 1);
        }
        // ---------------- phase C: dW1 (+ bias) = sum_R dh1[R] x[patch R]^T
#pragma unroll
        for (int u = 0; u < 2; u++) {
            if (kSkip & 4)
                break;
            uint16_t *img_dh1 = img, *img_x = img + 16 * kStrideH1;              // img_x: [16 cells][16 rows]
            if ((col >> 4) == u) {
                const int rowi = col & 15;
#pragma unroll
                for (int R = 0; R < 9; R++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        store_frag(img_dh1, kStrideH1, rowi, 32 * R + 16 * s, h, dh1[R][s]);
                // cells 8h..8h+7 of this row (the x fragment: element j = cell 8h + j)
#pragma unroll
                for (int j = 0; j < 8; j++)
                    img_x[(8 * h + j) * 16 + rowi] = (uint16_t)x[j];
            }
#pragma unroll
            for (int R = 0; R < 9; R++) {
                // B[k = row][col t]: t < 4 -> x[cell(R, t)], t == 4 -> 1 (bias), else 0
                bf16x8 b = {};
                if (col < 4) {
                    const uint4 v4 = *reinterpret_cast<const uint4 *>(img_x + cell_of(R, col) * 16 + 8 * h);
                    __builtin_memcpy(&b, &v4, 16);
                } else if (col == 4) {
                    b = ones;
                }
                dw1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_operand(img_dh1, kStrideH1, 32 * R, lane), b, dw1,
                                                              0, 0, 0);
            }
        }
    }

    // ---------------- flush this wave's partial record
    float *rec = partials + ((int64_t)blockIdx.x * kWaves + wave) * kPartial;
#pragma unroll
    for (int g = 0; g < 2; g++)
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int row = 32 * g + 8 * (i >> 2) + 4 * h + (i & 3);
#pragma unroll
            for (int kk = 0; kk < 4; kk++)
                rec[row * 128 + 32 * kk + col] = dw2[g][kk][i];
            if (col == 0)
                rec[kOffDb2 + row] = db2[g][i];
        }
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int row = 8 * (i >> 2) + 4 * h + (i & 3);
        if (col < 5)
            rec[kOffDw1 + row * 5 + col] = dw1[i];
    }
    for (int i = lane; i < 5 * 257; i += 64)
        rec[kOffDwh + i] = acc_wh[(i / 257) * kAccWhCols + (i % 257)];
    // losses: sum over the wave's half-0 lanes
    float la = loss_actor, lc = loss_critic;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        la += __shfl_xor(la, off);
        lc += __shfl_xor(lc, off);
    }
    if (lane == 0) {
        rec[kOffLoss] = la;
        rec[kOffLoss + 1] = lc;
    }
}

// deterministic sum of the per-wave records: out[k] = sum_w partials[w][k]
__global__ __launch_bounds__(256) void k_reduce(const float *__restrict__ partials, int64_t n_rec,
                                                float *__restrict__ out)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= kPartial)
        return;
    float s = 0.f;
    for (int64_t w = 0; w < n_rec; w++)
        s += partials[w * kPartial + k];
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

int64_t r48_cnn_train_workspace_floats(void) { return (int64_t)grid_size() * kWaves * kPartial; }

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
    const size_t lds = (size_t)(kFragsTrain * 64 + 32) * 16 + (size_t)kWaves * kImgElems * 2 +
                       (size_t)kWaves * 5 * kAccWhCols * 4;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_cnn_train),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_cnn_train, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, boards, rows, n_boards,
                       actions, targets, wn, cm, counts, beta, mode, (const uint4 *)wfrag, bias, workspace);
    hipLaunchKernelGGL(k_reduce, dim3((kPartial + 255) / 256), dim3(256), 0, (hipStream_t)stream, workspace,
                       (int64_t)grid * kWaves, grad);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string("k_cnn_train: ") + hipGetErrorString(e));
    return R48_OK;
}

}  // extern "C"
