// r48_conv.hip -- the 3x3 (pad 1) convolutions of the ResNet-10 Q-network's UPDATE on the 4x4 grid
// (BASELINE config 5; rein48_amd/dqn/nets.py), hand-written for gfx950 MFMA, behind include/rein48.h.
//
// Activations are channels-last bf16 [boards][16 cells][C]. Only the 100 in-grid (cell, tap) pairs
// of the 144 are computed (the dense structured GEMM of the PyTorch path does 1.44x their work at
// 64 channels and reads/writes the same bytes through hipBLASLt).
//
// k_conv3x3 (forward, and the data gradient: the same kernel with the flipped, transposed taps)
//   v_mfma_f32_16x16x32_bf16, rows = 16 output channels (row tile O of 4), columns = 16 BOARDS at
//   the same cell (the layout of the inference kernel r48_resnet.hip): a wave loads all 16 cells of
//   its 16 boards (16-byte chunks, lane = board l & 15, channel group g = l >> 4) and the 3x3 tap
//   (dr, dc) of output cell p is just the input cell p + 4dr + dc of the same lane -- no lane
//   movement; one LDS weight fragment (tap, O, k-chunk) feeds every cell that has the tap (9, 12
//   or 16 MFMAs). Accumulators start at the bias; finished output rows are staged through a per-wave
//   LDS row and stored in 16-byte pieces. Weights: 9 x 4 x NC fragments of 1 KiB in LDS (72 KiB at
//   64 input channels), one workgroup of 8 waves per CU. Epilogue options: + a residual gradient,
//   the BN forward statistics of the output, the BN backward reduction of the layer below.
// k_conv_wgrad (weight gradient, summed over boards and cells)
//   dW[t][co][ci] = sum over (board, cell p in grid for t) of dy[b][p][co] x[b][p + off(t)][ci]:
//   a contraction over rows, so rows go to the MFMA K dimension through LDS images read back with
//   ds_read_b64_tr_b16. Per step a workgroup stages kStepRows rows of dy and x by LDS-DMA into a
//   ring of kRing buffers; the x operand of tap t is the same image read with per-lane row addresses
//   shifted by the tap (rows outside the grid point at a zero row). 8 waves, each owning one
//   input-channel tile and its share of the output tiles, accumulate in AGPRs. Each workgroup writes
//   one fp32 record; k_conv_wgrad_reduce sums the records in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_bn_finish.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x4 = __attribute__((ext_vector_type(4))) float;
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
#define R48_LDS __attribute__((address_space(3)))

constexpr int kCout = 64;

// tap t = 3 (dr + 1) + (dc + 1); centre first (all 16 cells: it starts every accumulator)
__device__ constexpr int kTapOrder[9] = {4, 0, 1, 2, 3, 5, 6, 7, 8};

__host__ __device__ constexpr bool in_grid(int p, int t)
{
    const int r = (p >> 2) + t / 3 - 1, c = (p & 3) + t % 3 - 1;
    return r >= 0 && r < 4 && c >= 0 && c < 4;
}
__host__ __device__ constexpr int tap_off(int t) { return 4 * (t / 3 - 1) + (t % 3 - 1); }

__device__ __forceinline__ bf16x8 as_frag(const uint4 &v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint32_t pack2(float lo, float hi)
{
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{lo, hi}), bf16x2_t));
}

int fail(int code, const std::string &msg)
{
    r48::set_last_error(msg);
    return code;
}

int launched(const char *what)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        r48::set_last_error(std::string(what) + ": " + hipGetErrorString(e));
        return R48_EHIP;
    }
    return R48_OK;
}

// Persistent grids and their per-workgroup record buffers use ONE fixed workgroup count -- the
// MI355X's 256 CUs -- not a query of the current device: the statistics / workspace sizes
// (r48_conv_stats_floats, r48_conv_wgrad_workspace_floats, r48_q_head_workspace_floats) and the
// launch grids then agree whatever device is current at allocation or call time, and a device with
// fewer CUs (a compute partition) just runs the extra workgroups in a second wave.
constexpr int kPersistentGroups = 256;

constexpr int cu_count() { return kPersistentGroups; }

// ---------------------------------------------------------------------------------- forward
// x bf16 [boards][16][32 NC], wfrag (tap, O, c) fragments: lane l element j = W[16 O + (l & 15)]
// [32 c + 8 (l >> 4) + j][tap] (rein48_amd/dqn/conv.py pack_conv), bias fp32 [64] or null,
// y bf16 [boards][16][64].
//
// One workgroup of 8 waves per CU shares one LDS copy of the weights; each wave walks its tiles of
// 16 boards one grid row at a time. Output row r needs input rows r - 1 .. r + 1, so the row
// registers of a tile are refilled while it is still being computed: input rows 2 and 3 load under
// output rows 0 and 1, and the NEXT tile's rows 0 and 1 load under output rows 2 and 3 (their
// registers are free by then). A wave keeps 1-2 rows (8-16 KB) in flight behind its MFMAs. Finished
// output rows go through a per-wave LDS staging row so that they are stored in full 16-byte pieces.
constexpr int kConvWaves = 8;
constexpr int kOutPitch = 4 * 64 + 8;      // bf16 per board in the output-row staging (+16 B: banks)

// ADD: y += add[b][p][co] (bf16, the same layout as y) before the bf16 rounding -- the data
// gradient of a basic block's first conv plus the gradient of the identity path. ADD = 2: the
// identity path's gradient is add . [add_mask bit] (add = the gradient reaching the block's output
// ReLU, add_mask its forward mask, one byte per 8 channels): the masked copy the BN backward would
// otherwise write out and this conv read back is formed here from the mask byte instead.
// STATS: the per-channel sums S1 = sum y, S2 = sum y^2 of the bf16 outputs (the statistics of the
// training-mode BN that follows), accumulated from the staged 16-byte pieces (a lane's pieces are
// always the same 8 channels), one record [S1 64][S2 64] per workgroup (the grid is then exactly
// one workgroup per CU, idle ones write zeros). SM = 1.
// SM = 2 (a data-gradient conv whose output y is the gradient reaching a training-mode BN + ReLU):
// the BN backward's reduction fused the same way -- g = y . [relu mask], records [sum g 64]
// [sum g (bn_x - mean) 64] with bn_x the BN's input (the forward conv output) and mean from its
// save (r48_bn_backward's k_bn_bwd_reduce, without its second pass over y and bn_x).
// Passes of PO row tiles: 2, or 1 with statistics to make room for their 16 accumulators.
// IN (the forward's input is the PREVIOUS layer's training-mode BN + ReLU, folded into this conv's
// operand load instead of a separate apply pass): x is that BN's input (the previous conv's output),
// and each input row, once loaded, becomes z = relu(a x + b (+ res)) with the BN's per-channel
// coefficients (coef: a[64] | b[64], r48_bn_finish) -- IN = 2 adds the block's identity input res.
// z is what the MFMAs consume, and it is also written out (z_out, with its ReLU mask byte per 8
// channels in m_out) for the backward: the weight gradient's input, the residual path, BN's
// backward. Same arithmetic and bf16 rounding as k_bn_apply, so z equals the apply pass's output.
// A row is transformed just before its first use (output row r - 1), one row-load after it was
// issued, so the loads stay ahead of the MFMAs.
template <int NC, int ADD, int SM, int IN = 0>
__global__ __launch_bounds__(64 * kConvWaves, 1) void k_conv3x3(const uint16_t *__restrict__ x, int64_t boards,
                                                               const uint4 *__restrict__ wfrag,
                                                               const float *__restrict__ bias,
                                                               const uint16_t *__restrict__ add,
                                                               uint16_t *__restrict__ y, float *__restrict__ stats,
                                                               const uint16_t *__restrict__ bn_x,
                                                               const uint8_t *__restrict__ bn_mask,
                                                               const float *__restrict__ bn_save,
                                                               const float *__restrict__ coef = nullptr,
                                                               const uint16_t *__restrict__ res = nullptr,
                                                               uint16_t *__restrict__ z_out = nullptr,
                                                               uint8_t *__restrict__ m_out = nullptr,
                                                               const uint8_t *__restrict__ add_mask = nullptr,
                                                               const r48_bn_finish_args fin = r48_bn_finish_args{})
{
    constexpr bool STATS = SM != 0;
    constexpr int PO = STATS ? 1 : 2;
    constexpr int kFrags = 9 * 4 * NC;
    constexpr int kCin = 32 * NC;
    __shared__ uint4 w_lds[kFrags * 64];
    __shared__ __attribute__((aligned(16))) float b_lds[kCout];
    __shared__ __attribute__((aligned(16))) uint16_t o_lds[kConvWaves][16 * kOutPitch];
    __shared__ float st_lds[STATS ? kConvWaves : 1][8][16];
    __shared__ __attribute__((aligned(16))) float mean_lds[SM == 2 ? kCout : 4];
    __shared__ __attribute__((aligned(16))) float cf_lds[IN ? 2 * kCout : 4];
    for (int i = threadIdx.x; i < kFrags * 64; i += 64 * kConvWaves)
        w_lds[i] = wfrag[i];
    if (threadIdx.x < kCout)
        b_lds[threadIdx.x] = bias ? bias[threadIdx.x] : 0.0f;
    if (SM == 2 && threadIdx.x < kCout)
        mean_lds[threadIdx.x] = bn_save[threadIdx.x];
    if (IN && threadIdx.x < 2 * kCout)
        cf_lds[threadIdx.x] = coef[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
    const int wave = threadIdx.x >> 6;
    const int64_t n_tiles = (boards + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * kConvWaves;
    int64_t tile = (int64_t)blockIdx.x * kConvWaves + wave;
    if (!STATS && tile >= n_tiles)
        return;
    uint16_t *orow = o_lds[wave];          // this wave's output row: 16 boards x 4 cells x 64 channels
    float s1[8] = {}, s2[8] = {};          // statistics of channels 8 (lane & 7) .. + 7
    // xr[R][col][c]: input cell 4 R + col of this lane's board, channels 32 c + 8 g .. + 7
    uint4 xr[4][4][NC];
    auto load_row = [&](int64_t t, int R, const uint16_t *base) {
        const int64_t b = t * 16 + n;
        const uint16_t *src = base + ((b < boards ? b : boards - 1) * 16 + 4 * R) * kCin + 8 * g;
#pragma unroll
        for (int col = 0; col < 4; col++)
#pragma unroll
            for (int c = 0; c < NC; c++)
                xr[R][col][c] = *reinterpret_cast<const uint4 *>(src + col * kCin + 32 * c);
    };
    // IN: the loaded row R of tile t becomes z = relu(a x + b (+ res)) in place; z and its mask go out
    auto transform_row = [&](int64_t t, int R) {
        const int64_t bz = t * 16 + n;
        const int64_t bc = bz < boards ? bz : boards - 1;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int ch = 32 * c + 8 * g;
            const float4 a0 = *reinterpret_cast<const float4 *>(cf_lds + ch), a1 = *reinterpret_cast<const float4 *>(cf_lds + ch + 4);
            const float4 b0 = *reinterpret_cast<const float4 *>(cf_lds + kCout + ch),
                         b1 = *reinterpret_cast<const float4 *>(cf_lds + kCout + ch + 4);
            const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
            for (int col = 0; col < 4; col++) {
                const int64_t o = (bc * 16 + 4 * R + col) * kCin + ch;
                uint4 q = make_uint4(0u, 0u, 0u, 0u);
                if (IN == 2)
                    q = *reinterpret_cast<const uint4 *>(res + o);
                const uint4 v = xr[R][col][c];
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, q4[4] = {q.x, q.y, q.z, q.w};
                uint32_t pk[4], m = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float lo = __builtin_fmaf(av[2 * k], __uint_as_float(w4[k] << 16), bv[2 * k]);
                    float hi = __builtin_fmaf(av[2 * k + 1], __uint_as_float(w4[k] & 0xFFFF0000u), bv[2 * k + 1]);
                    if (IN == 2) {
                        lo += __uint_as_float(q4[k] << 16);
                        hi += __uint_as_float(q4[k] & 0xFFFF0000u);
                    }
                    pk[k] = pack2(fmaxf(lo, 0.f), fmaxf(hi, 0.f));
                    m |= ((pk[k] & 0x7FFFu) != 0 && !(pk[k] & 0x8000u) ? 1u : 0u) << (2 * k) |
                         ((pk[k] & 0x7FFF0000u) != 0 && !(pk[k] & 0x80000000u) ? 1u : 0u) << (2 * k + 1);
                }
                const uint4 zv = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                xr[R][col][c] = zv;
                if (bz < boards) {
                    *reinterpret_cast<uint4 *>(z_out + o) = zv;
                    m_out[o >> 3] = (uint8_t)m;
                }
            }
        }
    };
    if (tile < n_tiles) {
        load_row(tile, 0, x);
        load_row(tile, 1, x);
    }
    for (; tile < n_tiles; tile += stride) {
        const int64_t next = tile + stride;
        const int64_t b = tile * 16 + n;
        const bool live = b < boards;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            // rows r - 2 of this tile were last read by output row r - 1. Unconditional: a load under
            // a branch makes hipcc's counted waits at the join drain everything in flight. After the
            // wave's last tile the two loads of a next tile read the weight fragments instead (first
            // 33 KiB, resident in L2 since the workgroup's start; the values are never used): a reload
            // of the tile itself went back to HBM, 1.25x the input bytes at two tiles per wave
            // (profiles/r06/dqn/conv_tail_reload.txt)
            if (r < 2)
                load_row(tile, r + 2, x);
            else
                load_row(next < n_tiles ? next : 0, r - 2,
                         next < n_tiles ? x : reinterpret_cast<const uint16_t *>(wfrag));
            __builtin_amdgcn_sched_barrier(0);   // issue the row loads here, ahead of this row's MFMAs
            if (IN) {   // rows first used by this output row: 0 and 1 at r = 0, then r + 1
                if (r == 0)
                    transform_row(tile, 0);
                if (r < 3)
                    transform_row(tile, r + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int oh = 0; oh < 4 / PO; oh++) {   // passes of PO row tiles
                f32x4 acc[4][PO];                    // [output column][row tile PO oh + o]
                uint2 ad[4][PO];
                uint32_t am[4][PO];   // ADD = 2: the mask byte of the lane's 4 channels (bits 4 (g & 1) ..)
                if (ADD) {
                    const int64_t bb = live ? b : 0;
                    const uint16_t *ar = add + bb * 16 * kCout + 4 * g;
#pragma unroll
                    for (int col = 0; col < 4; col++)
#pragma unroll
                        for (int o = 0; o < PO; o++) {
                            ad[col][o] = *reinterpret_cast<const uint2 *>(ar + (4 * r + col) * kCout + 16 * (PO * oh + o));
                            if (ADD == 2)
                                am[col][o] = add_mask[(bb * 16 + 4 * r + col) * (kCout / 8) + 2 * (PO * oh + o) + (g >> 1)];
                        }
                }
#pragma unroll
                for (int k = 0; k < 9 * NC; k++) {
                    const int t = kTapOrder[k / NC], c = k % NC;
                    const int dr = t / 3 - 1, dc = t % 3 - 1;
                    if (r + dr < 0 || r + dr > 3)
                        continue;
                    bf16x8 A[PO];
#pragma unroll
                    for (int o = 0; o < PO; o++)
                        A[o] = as_frag(w_lds[((t * 4 + PO * oh + o) * NC + c) * 64 + lane]);
#pragma unroll
                    for (int col = 0; col < 4; col++) {
                        if (col + dc < 0 || col + dc > 3)
                            continue;
#pragma unroll
                        for (int o = 0; o < PO; o++)
                            acc[col][o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                A[o], as_frag(xr[r + dr][col + dc][c]),
                                k == 0 ? *reinterpret_cast<const f32x4 *>(b_lds + 16 * (PO * oh + o) + 4 * g)
                                       : acc[col][o],
                                0, 0, 0);
                    }
                }
                if (ADD) {
#pragma unroll
                    for (int col = 0; col < 4; col++)
#pragma unroll
                        for (int o = 0; o < PO; o++) {
                            if (ADD == 2) {   // masked-off channels add +0, as the written-out copy did
                                const uint32_t mb = am[col][o] >> (4 * (g & 1));
                                ad[col][o].x &= (mb & 1u ? 0xFFFFu : 0u) | (mb & 2u ? 0xFFFF0000u : 0u);
                                ad[col][o].y &= (mb & 4u ? 0xFFFFu : 0u) | (mb & 8u ? 0xFFFF0000u : 0u);
                            }
                            acc[col][o][0] += __uint_as_float(ad[col][o].x << 16);
                            acc[col][o][1] += __uint_as_float(ad[col][o].x & 0xFFFF0000u);
                            acc[col][o][2] += __uint_as_float(ad[col][o].y << 16);
                            acc[col][o][3] += __uint_as_float(ad[col][o].y & 0xFFFF0000u);
                        }
                }
#pragma unroll
                for (int col = 0; col < 4; col++)
#pragma unroll
                    for (int o = 0; o < PO; o++)
                        *reinterpret_cast<uint2 *>(orow + n * kOutPitch + col * kCout + 16 * (PO * oh + o) + 4 * g) =
                            make_uint2(pack2(acc[col][o][0], acc[col][o][1]), pack2(acc[col][o][2], acc[col][o][3]));
            }
            // the row leaves in 16-byte pieces, 1 KiB (two boards' 512-byte rows) per store
            // instruction: 8-byte stores straight from the accumulator layout (16 boards x 32 bytes
            // each) write at about 0.6 of the rate
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (SM == 2 && k == 4)
                    __builtin_amdgcn_sched_barrier(0);   // two batches of BN-input loads: registers
                const int m = 64 * k + lane, bl = m >> 5, e = 8 * (m & 31);
                const uint4 v = *reinterpret_cast<const uint4 *>(orow + bl * kOutPitch + e);
                const int64_t bg = tile * 16 + bl;
                if (bg < boards) {
                    const int64_t o = (bg * 16 + 4 * r) * kCout + e;
                    *reinterpret_cast<uint4 *>(y + o) = v;
                    if (SM == 2) {
                        const uint4 xb = *reinterpret_cast<const uint4 *>(bn_x + o);
                        const uint32_t mk = bn_mask[o >> 3];
                        const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, x4[4] = {xb.x, xb.y, xb.z, xb.w};
                        const float4 m0 = *reinterpret_cast<const float4 *>(mean_lds + (e & 63));
                        const float4 m1 = *reinterpret_cast<const float4 *>(mean_lds + (e & 63) + 4);
                        const float mn[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            const uint32_t wv = (q & 1) ? (w4[q >> 1] & 0xFFFF0000u) : (w4[q >> 1] << 16);
                            const uint32_t xv = (q & 1) ? (x4[q >> 1] & 0xFFFF0000u) : (x4[q >> 1] << 16);
                            const float gq = (mk >> q) & 1u ? __uint_as_float(wv) : 0.f;
                            s1[q] += gq;
                            s2[q] = __builtin_fmaf(gq, __uint_as_float(xv) - mn[q], s2[q]);
                        }
                    }
                    if (SM == 1) {
                        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const float lo = __uint_as_float(w4[q] << 16), hi = __uint_as_float(w4[q] & 0xFFFF0000u);
                            s1[2 * q] += lo;
                            s2[2 * q] = __builtin_fmaf(lo, lo, s2[2 * q]);
                            s1[2 * q + 1] += hi;
                            s2[2 * q + 1] = __builtin_fmaf(hi, hi, s2[2 * q + 1]);
                        }
                    }
                }
            }
        }
    }
    if (STATS) {
        // lanes l, l ^ 8, l ^ 16, l ^ 32 ... share channels 8 (l & 7) .. + 7: fixed-order butterfly,
        // then the 8 waves in wave order
#pragma unroll
        for (int m = 8; m < 64; m <<= 1)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                s1[k] += __shfl_xor(s1[k], m);
                s2[k] += __shfl_xor(s2[k], m);
            }
        if (lane < 8)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                st_lds[wave][lane][k] = s1[k];
                st_lds[wave][lane][8 + k] = s2[k];
            }
        __syncthreads();
        if (threadIdx.x < 2 * kCout) {
            const int v = threadIdx.x >> 6, c = threadIdx.x & 63;
            float t = 0.f;
#pragma unroll
            for (int w = 0; w < kConvWaves; w++)
                t += st_lds[w][c >> 3][8 * v + (c & 7)];
            // device-coherent stores (agent scope: no L2 write-back fence needed before the ticket)
            __hip_atomic_store(stats + (int64_t)blockIdx.x * 2 * kCout + threadIdx.x, t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (fin.save) {
            // the BN's finish in the workgroup whose record arrives last (r48_bn_finish_args): every
            // record store is acknowledged at the device's coherence point before this workgroup
            // takes a ticket, and the last one reads every record with device-coherent loads
            __shared__ unsigned int ticket;
            __shared__ double fin_lds[8 * kCout];
            unsigned int *counter = reinterpret_cast<unsigned int *>(stats + (int64_t)kPersistentGroups * 2 * kCout);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0)
                ticket = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (ticket == kPersistentGroups - 1) {
                r48bn::finish_records<kCout, kPersistentGroups, SM == 2>(stats, fin, fin_lds);
                if (threadIdx.x == 0)   // ready for the next launch on this buffer
                    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// --------------------------------------------------------------------------------- wgrad
// Per step a workgroup stages kStepRows rows (kStepRows / 16 boards) of dy [rows][64] and x
// [rows][CIN] into LDS images by LDS-DMA (global_load_lds_dwordx4: no staging registers): row-major,
// the 16-byte chunk index XOR-ed with swz(row) (applied to the per-lane SOURCE address, the LDS side
// of one DMA is lane-linear). A ring of kRing buffers keeps steps s + 1, s + 2 in flight while
// step s computes (32-64 KB per CU), waited for with a counted vmcnt and a raw barrier. The x image
// has a zero band: rows kStepRows + 32 ks, one per k-step, so that every transposed-read address of
// k-step ks is the k-step-0 address plus the constant 32 ks rows (an immediate offset) -- also for
// the out-of-grid taps, which read the zero row.
constexpr int kStepRows = 128;
constexpr int kKSteps = kStepRows / 32;
constexpr int kZeroRow = kStepRows;                              // zero band: kZeroRow + 32 ks
constexpr int kXRows = kStepRows + 32 * (kKSteps - 1) + 1;
constexpr int kRing = 3;                                          // LDS buffers: 2 steps ahead
constexpr int kRedGroup = 16;                                     // records per group of records_sum16

// chunk swizzle of image row `row`: XOR with row & 7 spreads a transposed read's 4 consecutive rows
// over the bank row; XOR with 4 when row & 8 keeps the rows 8 apart (the lane groups g = 0, 1 of
// one 32-lane half) off each other's banks
__host__ __device__ constexpr int swz(int row) { return (row & 7) ^ ((row & 8) >> 1); }

template <int COLS>
__device__ __forceinline__ int wimg(int row, int col)
{
    constexpr int kChunks = COLS / 8;
    return row * COLS + ((((col >> 3) ^ swz(row)) & (kChunks - 1)) << 3) + (col & 7);
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

// gradient accumulation (36 accumulators = 144 registers: more than the 128 AGPRs a wave gets at
// two waves per SIMD, so the builtin, whose hazards hipcc pads, with the accumulators where it
// places them)
__device__ __forceinline__ void acc16(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

// One DMA of 64 x 16 bytes: rows [row0, row0 + 512 / COLS) of a [rows][COLS] bf16 tensor into the
// LDS image rows starting at img_row (wave-uniform), swizzled; source rows clamped to `last`.
template <int COLS>
__device__ __forceinline__ void dma_rows(const uint16_t *src, int64_t row0, int64_t last, uint16_t *img,
                                         int img_row, int lane)
{
    constexpr int kChunks = COLS / 8, kRows = 64 / kChunks;
    const int r = lane / kChunks, phys = lane % kChunks;
    const int chunk = (phys ^ swz(img_row + r)) & (kChunks - 1);
    const int64_t gr = row0 + r < last ? row0 + r : last;
    // inline asm: the builtin makes hipcc wait vmcnt(0) before every later ds_read of the array
    // (it cannot tell the ring buffers apart), which would drain the ring each step
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (uint32_t)reinterpret_cast<uintptr_t>((R48_LDS void *)(img + img_row * COLS)));   // wave-uniform
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src + gr * COLS + 8 * chunk), "s"(dst)
                 : "memory");
    static_assert(kRows * kChunks == 64, "one DMA = 64 chunks");
}

// partial record per workgroup: [9 taps][64 co][CIN ci] fp32. Eight waves, two per SIMD (one wave's
// DMA issue and barrier waits run under the other's MFMAs). Wave w owns input-channel tile w % NCT
// and ALL four output tiles, for every tap, over its share of each step's k-steps: k-steps
// kPer (w / NCT) .. kPer (w / NCT + 1) - 1 (split K). Its dy^T fragments then feed 9 MFMAs each and its
// x^T fragments 4: 13 transposed fragment pairs per 36 MFMAs (the former split by output tile read
// 11 per 18, and the CU's LDS read port, not the MFMA pipe, set the step time). The kSplit waves of
// one channel tile add their accumulators in wave order through LDS at the end (deterministic).
constexpr int kWgWaves = 8;

template <int CIN>
__global__ __launch_bounds__(64 * kWgWaves, 1) void k_conv_wgrad(const uint16_t *__restrict__ dy,
                                                           const uint16_t *__restrict__ x, int64_t boards,
                                                           float *__restrict__ partials)
{
    constexpr int kThr = 64 * kWgWaves;
    constexpr int NCT = CIN / 16;                                // input-channel tiles of 16
    constexpr int kSplit = kWgWaves / NCT;                       // waves per channel tile (2 or 4)
    constexpr int kPer = kKSteps / kSplit;                       // k-steps per wave and step (2 or 1)
    static_assert(kSplit * NCT == kWgWaves && kPer * kSplit == kKSteps, "wave split");
    constexpr int kDyImg = kStepRows * kCout, kXImg = kXRows * CIN;
    constexpr int kBuf = kDyImg + kXImg;
    constexpr int kDyRowsPerDma = 512 / kCout, kXRowsPerDma = 512 / CIN;
    constexpr int kDyDmas = kStepRows / kDyRowsPerDma, kXDmas = kStepRows / kXRowsPerDma;   // per step
    constexpr int kDmas = kDyDmas + kXDmas;
    constexpr int kMyDmas = kDmas / kWgWaves;                    // per wave and step (4 or 3)
    static_assert(kDyDmas * kDyRowsPerDma == kStepRows && kXDmas * kXRowsPerDma == kStepRows, "staging split");
    static_assert(kMyDmas * kWgWaves == kDmas && kDyDmas % kWgWaves == 0, "the same DMA count for every wave");
    // the end's partial sums (one tap at a time) reuse the ring
    static_assert((kSplit - 1) * NCT * 4 * 64 * 8 <= kRing * kBuf, "partial sums fit the ring");
    __shared__ __attribute__((aligned(16))) uint16_t lds[kRing * kBuf];   // the only LDS object
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, g = lane >> 4;
    const int ct = wave % NCT, kh = wave / NCT;                  // channel tile, k share of this wave
    for (int i = threadIdx.x; i < kRing * kKSteps * CIN; i += kThr) {   // zero bands (never overwritten)
        const int buf = i / (kKSteps * CIN), k = i % (kKSteps * CIN);
        lds[buf * kBuf + kDyImg + (kZeroRow + 32 * (k / CIN)) * CIN + k % CIN] = 0;
    }
    // transposed-read addresses of this wave's first k-step (its k-step kk adds 32 kk rows). A (dy^T,
    // lanes = co): rows 8g + 4u + q, columns 16 o + 4p (lane 4q + p of a 16-lane group addresses row q
    // of the group's 4-row block). B (x^T shifted by tap t, lanes = ci): row + off(t) when that cell is
    // in the grid, else the zero row (the zero band keeps both 32-row periodic, swz has period 16).
    const int q = i16 >> 2, p4 = i16 & 3;
    int a_off[4][2], b_off[9][2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int row = 8 * g + 4 * u + q;
#pragma unroll
        for (int o = 0; o < 4; o++)
            a_off[o][u] = wimg<kCout>(row + 32 * kPer * kh, 16 * o + 4 * p4);
#pragma unroll
        for (int t = 0; t < 9; t++) {
            const int src = in_grid(row & 15, t) ? row + tap_off(t) : kZeroRow;
            b_off[t][u] = kDyImg + wimg<CIN>(src + 32 * kPer * kh, 16 * ct + 4 * p4);
        }
    }
    f32x4 acc[9][4];
#pragma unroll
    for (int t = 0; t < 9; t++)
#pragma unroll
        for (int o = 0; o < 4; o++)
            acc[t][o] = f32x4{0.f, 0.f, 0.f, 0.f};
    // this workgroup's steps: blockIdx.x + i * gridDim.x (the grid sweeps the tensors in order)
    const int64_t rows_total = boards * 16, last = rows_total - 1;
    const int64_t steps_total = (rows_total + kStepRows - 1) / kStepRows;
    const int64_t n_my = blockIdx.x < steps_total ? (steps_total - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
    // one DMA of this wave (its k-th of the step) for step i into ring buffer `buf`. Steps past the
    // end are staged too (clamped rows, a buffer nobody reads), so every step issues the same count
    // and the counted wait below stays exact.
    auto stage_one = [&](int64_t i, int buf, int k) {
        uint16_t *dimg = lds + buf * kBuf, *ximg = dimg + kDyImg;
        const int64_t row0 = ((int64_t)blockIdx.x + i * gridDim.x) * kStepRows;
        const int d = wave + k * kWgWaves;                       // dy pieces first: d < kDyDmas iff k < 2
        if (k < kDyDmas / kWgWaves)
            dma_rows<kCout>(dy, row0 + d * kDyRowsPerDma, last, dimg, d * kDyRowsPerDma, lane);
        else
            dma_rows<CIN>(x, row0 + (d - kDyDmas) * kXRowsPerDma, last, ximg, (d - kDyDmas) * kXRowsPerDma, lane);
    };
    __syncthreads();                                              // zero bands written
#pragma unroll
    for (int i = 0; i < kRing - 1; i++)
#pragma unroll
        for (int k = 0; k < kMyDmas; k++)
            stage_one(i, i, k);
    for (int64_t i = 0; i < n_my; i++) {
        const int64_t s = (int64_t)blockIdx.x + i * gridDim.x;
        const int buf = (int)(i % kRing);
        // this wave's DMAs of step s done (step s + 1's may stay in flight), then the barrier that
        // orders them for every reader -- and that every wave passes only after its reads of step
        // s - 1, whose buffer is restaged below
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kRing - 2) * kMyDmas) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (s == steps_total - 1 && rows_total - s * kStepRows < kStepRows) {
            // the ragged last step: its rows past the end were staged from the clamped last row
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int real = (int)(rows_total - s * kStepRows);
            uint16_t *dimg = lds + buf * kBuf, *ximg = dimg + kDyImg;
            for (int i = threadIdx.x; i < (kStepRows - real) * kCout; i += kThr)
                dimg[real * kCout + i] = 0;
            for (int i = threadIdx.x; i < (kStepRows - real) * CIN; i += kThr)
                ximg[real * CIN + i] = 0;
            __syncthreads();
        }
        const uint16_t *img = lds + buf * kBuf;
        const int nbuf = (buf + kRing - 1) % kRing;
        // this wave's DMAs of step i + kRing - 1 (into the buffer of step i - 1) spread over its
        // (k-step, tap) items, so that the CU's DMAs issue in bursts of 8 under the MFMAs
        constexpr int kItems = kPer * 9;
#pragma unroll
        for (int kk = 0; kk < kPer; kk++) {
            bf16x8 A[4];
#pragma unroll
            for (int o = 0; o < 4; o++)
                A[o] = tr_pair(img + a_off[o][0] + 32 * kk * kCout, img + a_off[o][1] + 32 * kk * kCout);
#pragma unroll
            for (int t = 0; t < 9; t++) {
#pragma unroll
                for (int k = 0; k < kMyDmas; k++)
                    if ((k * kItems) / kMyDmas == kk * 9 + t)
                        stage_one(i + kRing - 1, nbuf, k);
                const bf16x8 B = tr_pair(img + b_off[t][0] + 32 * kk * CIN, img + b_off[t][1] + 32 * kk * CIN);
#pragma unroll
                for (int o = 0; o < 4; o++)
                    acc16(acc[t][o], A[o], B);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // no DMA outlives the kernel
    __syncthreads();                                              // every read of the ring done
    // record: D[m = co 16][n = ci 16], lane l: column i16 (ci), rows 4g + i (co) of output tile o.
    // Waves kh > 0 park a tap's accumulators in the ring, wave kh = 0 of the tile adds them in order.
    f32x4 *part = reinterpret_cast<f32x4 *>(lds);
    float *rec = partials + (int64_t)blockIdx.x * 9 * kCout * CIN;
#pragma unroll
    for (int t = 0; t < 9; t++) {
        if (kh > 0)
#pragma unroll
            for (int o = 0; o < 4; o++)
                part[(((kh - 1) * NCT + ct) * 4 + o) * 64 + lane] = acc[t][o];
        __syncthreads();
        if (kh == 0) {
#pragma unroll
            for (int o = 0; o < 4; o++) {
                f32x4 v = acc[t][o];
#pragma unroll
                for (int h = 1; h < kSplit; h++)
                    v += part[(((h - 1) * NCT + ct) * 4 + o) * 64 + lane];
#pragma unroll
                for (int i = 0; i < 4; i++)
                    rec[(t * kCout + 16 * o + 4 * g + i) * CIN + 16 * ct + i16] = v[i];
            }
        }
        __syncthreads();
    }
}

// Fixed-order sum of n_rec <= kRedGroup^2 records of len4 float4 entries in ONE pass: a block of
// 256 threads takes 16 entries; thread (entry e, group q) sums records 16 q .. 16 q + 15 of its entry
// in record order (beyond n_rec: + 0, as a shorter group), then the first group's threads add the
// other groups' sums in group order through LDS -- the arithmetic of the former two-pass form
// (groups, then the groups in order), so bit-identical to it, without the second launch and the
// group round trip through memory.
__device__ __forceinline__ bool records_sum16(const float4 *__restrict__ recs, int n_rec, int len4, float4 &out)
{
    __shared__ float4 part[kRedGroup][16];
    const int el = threadIdx.x & 15, q = threadIdx.x >> 4;
    const int k = blockIdx.x * 16 + el;
    const int n_grp = (n_rec + kRedGroup - 1) / kRedGroup;
    if (k < len4 && q < n_grp) {
        const int r0 = q * kRedGroup;
        float4 v[kRedGroup];
#pragma unroll
        for (int r = 0; r < kRedGroup; r++)
            v[r] = r0 + r < n_rec ? recs[(int64_t)(r0 + r) * len4 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 t = v[0];
#pragma unroll
        for (int r = 1; r < kRedGroup; r++) {
            t.x += v[r].x;
            t.y += v[r].y;
            t.z += v[r].z;
            t.w += v[r].w;
        }
        part[q][el] = t;
    }
    __syncthreads();
    if (q != 0 || k >= len4)
        return false;
    float4 t = part[0][el];
    for (int g = 1; g < n_grp; g++) {
        const float4 v = part[g][el];
        t.x += v.x;
        t.y += v.y;
        t.z += v.z;
        t.w += v.w;
    }
    out = t;
    return true;
}

// the weight gradient's records [t][co][ci] summed, written in torch's [co][ci][3][3] layout
template <int CIN>
__global__ __launch_bounds__(256) void k_conv_wgrad_reduce(const float4 *__restrict__ partials, int n_rec,
                                                          float *__restrict__ out)
{
    constexpr int kQ = 9 * kCout * CIN / 4;                       // float4 entries per record
    float4 s;
    if (!records_sum16(partials, n_rec, kQ, s))
        return;
    const int e = 4 * (blockIdx.x * 16 + (threadIdx.x & 15)), t = e / (kCout * CIN), co = (e / CIN) % kCout,
              ci = e % CIN;
    float *o = out + (co * CIN + ci) * 9 + t;
    o[0] = s.x;
    o[9] = s.y;
    o[18] = s.z;
    o[27] = s.w;
}

// --------------------------------------------------------------------------------- Q head
// q[b][a] = bf16(sum_k h[b][k] W[a][k] + bias[a]) for the 4 actions, k < 1024 = 16 cells x 64
// channels (nets.py: linear(h, head.weight, head.bias, bf16).float()). A wave takes one board at a
// time, lane l its k = 16 l .. 16 l + 15 (one 32-byte piece of the 2 KiB row: the wave reads the
// row in full lines); W stays in 32 registers; the 4 dot products are summed across the wave.
// kHeadUnroll boards per iteration keep 8 KiB per wave in flight. HBM-bound: 2 KiB per board.
constexpr int kHeadK = 1024, kHeadWaves = 8, kHeadUnroll = 4;

__device__ __forceinline__ void unpack16(const uint4 (&v)[2], float (&f)[16])
{
    const uint32_t w[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
    for (int i = 0; i < 8; i++) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}

__device__ __forceinline__ float bf16_round(float v)   // round to nearest even, as a float
{
    return (float)(__bf16)v;
}

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        v += __shfl_xor(v, m);
    return v;
}

__global__ __launch_bounds__(64 * kHeadWaves) void k_q_head_fwd(const uint16_t *__restrict__ h, int64_t boards,
                                                             const uint16_t *__restrict__ w,
                                                             const float *__restrict__ bias, float *__restrict__ q)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * kHeadWaves + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * kHeadWaves;
    float wf[4][16];
#pragma unroll
    for (int a = 0; a < 4; a++) {
        uint4 v[2];
        v[0] = *reinterpret_cast<const uint4 *>(w + a * kHeadK + 16 * lane);
        v[1] = *reinterpret_cast<const uint4 *>(w + a * kHeadK + 16 * lane + 8);
        unpack16(v, wf[a]);
    }
    float b4[4];
#pragma unroll
    for (int a = 0; a < 4; a++)
        b4[a] = bf16_round(bias[a]);
    for (int64_t b0 = wave * kHeadUnroll; b0 < boards; b0 += n_waves * kHeadUnroll) {
        uint4 v[kHeadUnroll][2];
#pragma unroll
        for (int u = 0; u < kHeadUnroll; u++) {
            const int64_t b = b0 + u < boards ? b0 + u : boards - 1;
            v[u][0] = *reinterpret_cast<const uint4 *>(h + b * kHeadK + 16 * lane);
            v[u][1] = *reinterpret_cast<const uint4 *>(h + b * kHeadK + 16 * lane + 8);
        }
#pragma unroll
        for (int u = 0; u < kHeadUnroll; u++) {
            float f[16];
            unpack16(v[u], f);
            float s[4];
#pragma unroll
            for (int a = 0; a < 4; a++) {
                s[a] = 0.f;
#pragma unroll
                for (int i = 0; i < 16; i++)
                    s[a] = __builtin_fmaf(f[i], wf[a][i], s[a]);
                s[a] = wave_sum(s[a]);
            }
            if (lane == 0 && b0 + u < boards)
                *reinterpret_cast<float4 *>(q + 4 * (b0 + u)) =
                    make_float4(bf16_round(s[0] + b4[0]), bf16_round(s[1] + b4[1]), bf16_round(s[2] + b4[2]),
                                bf16_round(s[3] + b4[3]));
        }
    }
}

// Backward of the head for one board per wave step: g = bf16(dq[b]) (the bf16 output's gradient);
// dh[b][k] = bf16(sum_a g[a] W[a][k]); the weight gradient sum_b g[a] h[b][k] and the bias gradient
// sum_b g[a] accumulate per lane in fp32 (lane l owns k = 16 l .. + 15 of all 4 rows), the waves of a
// workgroup are summed through LDS in a fixed order, and each workgroup writes one record of
// kHeadK * 4 + 4 floats (summed by k_records_reduce: deterministic).
constexpr int kHeadRec = 4 * kHeadK + 4;

__global__ __launch_bounds__(64 * kHeadWaves) void k_q_head_bwd(const float *__restrict__ dq,
                                                             const uint16_t *__restrict__ h, int64_t boards,
                                                             const uint16_t *__restrict__ w,
                                                             uint16_t *__restrict__ dh, float *__restrict__ records)
{
    __shared__ float red[kHeadWaves][kHeadRec];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t wave = (int64_t)blockIdx.x * kHeadWaves + wv;
    const int64_t n_waves = (int64_t)gridDim.x * kHeadWaves;
    float wf[4][16];
#pragma unroll
    for (int a = 0; a < 4; a++) {
        uint4 v[2];
        v[0] = *reinterpret_cast<const uint4 *>(w + a * kHeadK + 16 * lane);
        v[1] = *reinterpret_cast<const uint4 *>(w + a * kHeadK + 16 * lane + 8);
        unpack16(v, wf[a]);
    }
    float gw[4][16], gb[4];
#pragma unroll
    for (int a = 0; a < 4; a++) {
        gb[a] = 0.f;
#pragma unroll
        for (int i = 0; i < 16; i++)
            gw[a][i] = 0.f;
    }
    for (int64_t b0 = wave * kHeadUnroll; b0 < boards; b0 += n_waves * kHeadUnroll) {
        uint4 v[kHeadUnroll][2];
        float4 g4[kHeadUnroll];
#pragma unroll
        for (int u = 0; u < kHeadUnroll; u++) {
            const int64_t b = b0 + u < boards ? b0 + u : boards - 1;
            v[u][0] = *reinterpret_cast<const uint4 *>(h + b * kHeadK + 16 * lane);
            v[u][1] = *reinterpret_cast<const uint4 *>(h + b * kHeadK + 16 * lane + 8);
            g4[u] = *reinterpret_cast<const float4 *>(dq + 4 * b);
        }
#pragma unroll
        for (int u = 0; u < kHeadUnroll; u++) {
            const bool live = b0 + u < boards;
            const float g[4] = {live ? bf16_round(g4[u].x) : 0.f, live ? bf16_round(g4[u].y) : 0.f,
                                live ? bf16_round(g4[u].z) : 0.f, live ? bf16_round(g4[u].w) : 0.f};
            float f[16];
            unpack16(v[u], f);
            uint32_t o[8];
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                float d0 = 0.f, d1 = 0.f;
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    d0 = __builtin_fmaf(g[a], wf[a][i], d0);
                    d1 = __builtin_fmaf(g[a], wf[a][i + 1], d1);
                }
                o[i / 2] = pack2(d0, d1);
            }
#pragma unroll
            for (int a = 0; a < 4; a++) {
                gb[a] += g[a];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    gw[a][i] = __builtin_fmaf(g[a], f[i], gw[a][i]);
            }
            if (live) {
                uint16_t *dst = dh + (b0 + u) * kHeadK + 16 * lane;
                *reinterpret_cast<uint4 *>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
                *reinterpret_cast<uint4 *>(dst + 8) = make_uint4(o[4], o[5], o[6], o[7]);
            }
        }
    }
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int i = 0; i < 16; i++)
            red[wv][a * kHeadK + 16 * lane + i] = gw[a][i];
    if (lane < 4)
        red[wv][4 * kHeadK + lane] = gb[lane];
    __syncthreads();
    float *rec = records + (int64_t)blockIdx.x * kHeadRec;
    for (int i = threadIdx.x; i < kHeadRec; i += 64 * kHeadWaves) {
        float t = red[0][i];
#pragma unroll
        for (int k = 1; k < kHeadWaves; k++)
            t += red[k][i];
        rec[i] = t;
    }
}

// fixed-order sum of n_rec records of `len` floats (len % 4 == 0, records_sum16's order), the
// result rounded through bf16 when round_bf16 (the bf16 parameter-gradient contract of nets.py's linear)
__global__ __launch_bounds__(256) void k_records_reduce(const float4 *__restrict__ recs, int n_rec, int len4,
                                                       int round_bf16, float4 *__restrict__ out)
{
    float4 s;
    if (!records_sum16(recs, n_rec, len4, s))
        return;
    if (round_bf16)
        s = make_float4(bf16_round(s.x), bf16_round(s.y), bf16_round(s.z), bf16_round(s.w));
    out[blockIdx.x * 16 + (threadIdx.x & 15)] = s;
}

// ------------------------------------------------------------------- weight fragments
// The A fragments of every conv of the ResNet-10 update in one launch: part 0 = stem forward
// (18 input channels padded to one 32-channel k-chunk: 36 fragments), parts 1..8 = conv1..8
// forward (72 each), parts 9..16 = conv1..8 data gradient (W'[ci][co][t] = W[co][ci][8 - t]). One
// thread per bf16 element: fragment (t, O, c), lane l, element j holds
// W[16 O + (l & 15)][32 c + 8 (l >> 4) + j][t] of the (possibly flipped) weight -- the layout of
// rein48_amd/dqn/conv.py pack_conv / pack_conv_dgrad.
constexpr int kPackParts = 17;

__global__ __launch_bounds__(256) void k_conv_pack(const float *const *__restrict__ w, uint16_t *__restrict__ fwd,
                                                  uint16_t *__restrict__ dgrad)
{
    const int part = blockIdx.y;
    const int nc = part == 0 ? 1 : 2;
    const int n = 9 * 4 * nc * 512;                              // elements of this part
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n)
        return;
    const int frag = e >> 9, lane = (e >> 3) & 63, j = e & 7;
    const int c = frag % nc, O = (frag / nc) % 4, t = frag / (4 * nc);
    const int m = 16 * O + (lane & 15), k = 32 * c + 8 * (lane >> 4) + j;   // A row (output), k (input)
    float v;
    uint16_t *out;
    if (part == 0) {                                             // stem [64][18][9]
        v = k < 18 ? w[0][(m * 18 + k) * 9 + t] : 0.f;
        out = fwd;
    } else if (part <= 8) {                                      // conv `part` forward [64][64][9]
        v = w[part][(m * 64 + k) * 9 + t];
        out = fwd + 36 * 512 + (part - 1) * 72 * 512;
    } else {                                                     // conv part - 8, data gradient
        v = w[part - 8][(k * 64 + m) * 9 + (8 - t)];
        out = dgrad + (part - 9) * 72 * 512;
    }
    out[e] = (uint16_t)(__builtin_bit_cast(uint32_t, (float)(__bf16)v) >> 16);
}

// one lane per (board, cell): the one-hot of the exponent over 32 bf16 planes (e = 0..17, planes
// 18..31 zero: the stem's input channels padded to one 32-channel k-chunk), four 16-byte stores
__global__ __launch_bounds__(256) void k_onehot32(const int8_t *__restrict__ boards, int64_t n_cells,
                                                 uint4 *__restrict__ out)
{
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= n_cells)
        return;
    const uint32_t e = (uint32_t)(uint8_t)boards[c];
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        w[k] = (e == 2u * k ? 0x3F80u : 0u) | (e == 2u * k + 1u ? 0x3F800000u : 0u);
#pragma unroll
    for (int k = 0; k < 4; k++)
        out[4 * c + k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

}  // namespace

extern "C" {

int r48_board_onehot32(const int8_t *boards, int64_t n, void *out, void *stream)
{
    if (!boards || !out || n < 0 || (reinterpret_cast<uintptr_t>(out) & 15u))
        return fail(R48_EINVAL, "r48_board_onehot32: NULL argument, n < 0 or out not 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const int64_t cells = 16 * n;
    hipLaunchKernelGGL(k_onehot32, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, (hipStream_t)stream, boards,
                       cells, (uint4 *)out);
    return launched("k_onehot32");
}

// the records, then one float holding the finishing forms' arrival counter (+ 3 to keep 16 B)
int64_t r48_conv_stats_floats(void) { return (int64_t)cu_count() * 2 * kCout + 4; }

int r48_conv3x3_stats_finish(const void *x, int64_t boards, int32_t cin, const void *wfrag, const float *bias, void *y,
                             float *stats, const r48_bn_finish_args *fin, void *stream)
{
    if (!x || !wfrag || !y || !stats || !fin || !fin->gamma || !fin->beta || !fin->save || !fin->coef || boards < 1 ||
        (cin != 32 && cin != 64) || fin->rows < 1)
        return fail(R48_EINVAL, "r48_conv3x3_stats_finish: NULL argument, boards < 1, rows < 1 or cin not 32/64");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wfrag) | reinterpret_cast<uintptr_t>(y) |
         reinterpret_cast<uintptr_t>(bias)) & 15u)
        return fail(R48_EINVAL, "r48_conv3x3_stats_finish: x, wfrag, bias and y must be 16-byte aligned");
    if ((fin->running_mean == nullptr) != (fin->running_var == nullptr))
        return fail(R48_EINVAL, "r48_conv3x3_stats_finish: running_mean and running_var go together");
    const dim3 g(cu_count()), blk(64 * kConvWaves);
    hipStream_t s = (hipStream_t)stream;
    const uint16_t *xs = (const uint16_t *)x;
    const uint4 *wf = (const uint4 *)wfrag;
    if (cin == 64)
        hipLaunchKernelGGL((k_conv3x3<2, 0, 1>), g, blk, 0, s, xs, boards, wf, bias, nullptr, (uint16_t *)y, stats,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, *fin);
    else
        hipLaunchKernelGGL((k_conv3x3<1, 0, 1>), g, blk, 0, s, xs, boards, wf, bias, nullptr, (uint16_t *)y, stats,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, *fin);
    return launched("k_conv3x3 (stats + BN finish)");
}

int r48_conv3x3(const void *x, int64_t boards, int32_t cin, const void *wfrag, const float *bias, const void *add,
                void *y, float *stats, void *stream)
{
    if (!x || !wfrag || !y || boards < 1 || (cin != 32 && cin != 64))
        return fail(R48_EINVAL, "r48_conv3x3: NULL argument, boards < 1 or cin not 32/64");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wfrag) | reinterpret_cast<uintptr_t>(y) |
         reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(add)) & 15u)
        return fail(R48_EINVAL, "r48_conv3x3: x, wfrag, bias, add and y must be 16-byte aligned");
    if (add && (cin != 64 || stats))
        return fail(R48_EINVAL, "r48_conv3x3: add needs 64 input channels and no stats");
    const int64_t tiles = (boards + 15) / 16;
    const int64_t want = (tiles + kConvWaves - 1) / kConvWaves;
    const int grid = stats ? cu_count() : (int)(want < cu_count() ? want : cu_count());
    const uint16_t *xs = (const uint16_t *)x, *a = (const uint16_t *)add;
    const uint4 *wf = (const uint4 *)wfrag;
    uint16_t *ys = (uint16_t *)y;
    const dim3 g(grid), blk(64 * kConvWaves);
    hipStream_t s = (hipStream_t)stream;
    const uint16_t *nx = nullptr;
    const uint8_t *nm = nullptr;
    const float *ns = nullptr;
    if (cin == 64 && add)
        hipLaunchKernelGGL((k_conv3x3<2, 1, 0>), g, blk, 0, s, xs, boards, wf, bias, a, ys, stats, nx, nm, ns);
    else if (cin == 64 && stats)
        hipLaunchKernelGGL((k_conv3x3<2, 0, 1>), g, blk, 0, s, xs, boards, wf, bias, a, ys, stats, nx, nm, ns);
    else if (cin == 64)
        hipLaunchKernelGGL((k_conv3x3<2, 0, 0>), g, blk, 0, s, xs, boards, wf, bias, a, ys, stats, nx, nm, ns);
    else if (stats)
        hipLaunchKernelGGL((k_conv3x3<1, 0, 1>), g, blk, 0, s, xs, boards, wf, bias, a, ys, stats, nx, nm, ns);
    else
        hipLaunchKernelGGL((k_conv3x3<1, 0, 0>), g, blk, 0, s, xs, boards, wf, bias, a, ys, stats, nx, nm, ns);
    return launched("k_conv3x3");
}

int r48_conv3x3_bn_in(const void *x, int64_t boards, const void *wfrag, const float *bias, const float *coef,
                      const void *residual, void *z_out, uint8_t *mask_out, void *y, float *stats,
                      const r48_bn_finish_args *fin, void *stream)
{
    if (fin && (!fin->gamma || !fin->beta || !fin->save || !fin->coef || fin->rows < 1 ||
                (fin->running_mean == nullptr) != (fin->running_var == nullptr)))
        return fail(R48_EINVAL, "r48_conv3x3_bn_in: incomplete BN finish arguments");
    const r48_bn_finish_args f = fin ? *fin : r48_bn_finish_args{};
    if (!x || !wfrag || !coef || !z_out || !mask_out || !y || !stats || boards < 1)
        return fail(R48_EINVAL, "r48_conv3x3_bn_in: NULL argument or boards < 1");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wfrag) | reinterpret_cast<uintptr_t>(y) |
         reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(coef) | reinterpret_cast<uintptr_t>(residual) |
         reinterpret_cast<uintptr_t>(z_out)) & 15u)
        return fail(R48_EINVAL, "r48_conv3x3_bn_in: x, wfrag, bias, coef, residual, z_out and y must be 16-byte aligned");
    const dim3 g(cu_count()), blk(64 * kConvWaves);
    hipStream_t s = (hipStream_t)stream;
    const uint16_t *xs = (const uint16_t *)x, *rs = (const uint16_t *)residual;
    const uint4 *wf = (const uint4 *)wfrag;
    if (residual)
        hipLaunchKernelGGL((k_conv3x3<2, 0, 1, 2>), g, blk, 0, s, xs, boards, wf, bias, nullptr, (uint16_t *)y, stats,
                           nullptr, nullptr, nullptr, coef, rs, (uint16_t *)z_out, mask_out, nullptr, f);
    else
        hipLaunchKernelGGL((k_conv3x3<2, 0, 1, 1>), g, blk, 0, s, xs, boards, wf, bias, nullptr, (uint16_t *)y, stats,
                           nullptr, nullptr, nullptr, coef, rs, (uint16_t *)z_out, mask_out, nullptr, f);
    return launched("k_conv3x3 (bn in)");
}

int r48_conv3x3_bn_grad(const void *dy, int64_t boards, const void *wfrag, const void *add, const uint8_t *add_mask,
                        void *dx, const void *bn_x, const uint8_t *bn_mask, const float *bn_save, float *bn_part,
                        const r48_bn_finish_args *fin, void *stream)
{
    if (fin && (!fin->gamma || !fin->coef || fin->save != bn_save || fin->rows < 1))
        return fail(R48_EINVAL, "r48_conv3x3_bn_grad: incomplete BN finish arguments (fin->save must be bn_save)");
    const r48_bn_finish_args f = fin ? *fin : r48_bn_finish_args{};
    if (add_mask && !add)
        return fail(R48_EINVAL, "r48_conv3x3_bn_grad: add_mask without add");
    if (!dy || !wfrag || !dx || !bn_x || !bn_mask || !bn_save || !bn_part || boards < 1)
        return fail(R48_EINVAL, "r48_conv3x3_bn_grad: NULL argument or boards < 1");
    if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(wfrag) | reinterpret_cast<uintptr_t>(dx) |
         reinterpret_cast<uintptr_t>(add) | reinterpret_cast<uintptr_t>(bn_x) | reinterpret_cast<uintptr_t>(bn_save)) &
        15u)
        return fail(R48_EINVAL, "r48_conv3x3_bn_grad: dy, wfrag, add, dx, bn_x and bn_save must be 16-byte aligned");
    const dim3 g(cu_count()), blk(64 * kConvWaves);
    hipStream_t s = (hipStream_t)stream;
    const uint16_t *xs = (const uint16_t *)dy, *a = (const uint16_t *)add, *bx = (const uint16_t *)bn_x;
    const uint4 *wf = (const uint4 *)wfrag;
    if (add_mask)
        hipLaunchKernelGGL((k_conv3x3<2, 2, 2>), g, blk, 0, s, xs, boards, wf, nullptr, a, (uint16_t *)dx, bn_part,
                           bx, bn_mask, bn_save, nullptr, nullptr, nullptr, nullptr, add_mask, f);
    else if (add)
        hipLaunchKernelGGL((k_conv3x3<2, 1, 2>), g, blk, 0, s, xs, boards, wf, nullptr, a, (uint16_t *)dx, bn_part,
                           bx, bn_mask, bn_save, nullptr, nullptr, nullptr, nullptr, nullptr, f);
    else
        hipLaunchKernelGGL((k_conv3x3<2, 0, 2>), g, blk, 0, s, xs, boards, wf, nullptr, a, (uint16_t *)dx,
                           bn_part, bx, bn_mask, bn_save, nullptr, nullptr, nullptr, nullptr, nullptr, f);
    return launched("k_conv3x3 (bn grad)");
}

int64_t r48_conv_wgrad_workspace_floats(int32_t cin)
{
    const int64_t recs = cu_count();
    return (recs + (recs + kRedGroup - 1) / kRedGroup) * 9 * kCout * (cin == 32 ? 32 : 64);
}

int r48_conv3x3_wgrad(const void *dy, const void *x, int64_t boards, int32_t cin, float *workspace, float *dw,
                      void *stream)
{
    if (!dy || !x || !workspace || !dw || boards < 1 || (cin != 32 && cin != 64))
        return fail(R48_EINVAL, "r48_conv3x3_wgrad: NULL argument, boards < 1 or cin not 32/64");
    if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(workspace)) &
        15u)
        return fail(R48_EINVAL, "r48_conv3x3_wgrad: dy, x and workspace must be 16-byte aligned");
    const int grid = cu_count();
    static_assert(kPersistentGroups <= kRedGroup * kRedGroup, "records_sum16 sums at most 256 records");
    const int q = 9 * kCout * cin / 4;
    hipStream_t s = (hipStream_t)stream;
    if (cin == 64) {
        hipLaunchKernelGGL(k_conv_wgrad<64>, dim3(grid), dim3(64 * kWgWaves), 0, s, (const uint16_t *)dy,
                           (const uint16_t *)x, boards, workspace);
        hipLaunchKernelGGL(k_conv_wgrad_reduce<64>, dim3((q + 15) / 16), dim3(256), 0, s, (const float4 *)workspace,
                           grid, dw);
    } else {
        hipLaunchKernelGGL(k_conv_wgrad<32>, dim3(grid), dim3(64 * kWgWaves), 0, s, (const uint16_t *)dy,
                           (const uint16_t *)x, boards, workspace);
        hipLaunchKernelGGL(k_conv_wgrad_reduce<32>, dim3((q + 15) / 16), dim3(256), 0, s, (const float4 *)workspace,
                           grid, dw);
    }
    return launched("k_conv_wgrad");
}

int64_t r48_q_head_workspace_floats(void)
{
    const int64_t recs = cu_count();
    return (recs + (recs + kRedGroup - 1) / kRedGroup) * kHeadRec;
}

int r48_q_head_forward(const void *h, int64_t boards, const void *w, const float *bias, float *q, void *stream)
{
    if (!h || !w || !bias || !q || boards < 1)
        return fail(R48_EINVAL, "r48_q_head_forward: NULL argument or boards < 1");
    if ((reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(q)) & 15u)
        return fail(R48_EINVAL, "r48_q_head_forward: h, w and q must be 16-byte aligned");
    const int64_t want = (boards + kHeadWaves * kHeadUnroll - 1) / (kHeadWaves * kHeadUnroll);
    const int grid = (int)(want < 2 * cu_count() ? want : 2 * cu_count());
    hipLaunchKernelGGL(k_q_head_fwd, dim3(grid), dim3(64 * kHeadWaves), 0, (hipStream_t)stream, (const uint16_t *)h,
                       boards, (const uint16_t *)w, bias, q);
    return launched("k_q_head_fwd");
}

int r48_q_head_backward(const float *dq, const void *h, int64_t boards, const void *w, void *dh, float *workspace,
                        float *dw, void *stream)
{
    if (!dq || !h || !w || !dh || !workspace || !dw || boards < 1)
        return fail(R48_EINVAL, "r48_q_head_backward: NULL argument or boards < 1");
    if ((reinterpret_cast<uintptr_t>(dq) | reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(w) |
         reinterpret_cast<uintptr_t>(dh) | reinterpret_cast<uintptr_t>(workspace) |
         reinterpret_cast<uintptr_t>(dw)) & 15u)
        return fail(R48_EINVAL, "r48_q_head_backward: all pointers must be 16-byte aligned");
    const int grid = cu_count();
    const int len4 = kHeadRec / 4;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_q_head_bwd, dim3(grid), dim3(64 * kHeadWaves), 0, s, dq, (const uint16_t *)h, boards,
                       (const uint16_t *)w, (uint16_t *)dh, workspace);
    hipLaunchKernelGGL(k_records_reduce, dim3((len4 + 15) / 16), dim3(256), 0, s, (const float4 *)workspace, grid,
                       len4, 1, (float4 *)dw);
    return launched("k_q_head_bwd");
}

int r48_conv_pack_resnet(const float *const *weights, void *fwd, void *dgrad, void *stream)
{
    if (!weights || !fwd || !dgrad || ((reinterpret_cast<uintptr_t>(fwd) | reinterpret_cast<uintptr_t>(dgrad)) & 15u))
        return fail(R48_EINVAL, "r48_conv_pack_resnet: NULL or misaligned argument");
    hipLaunchKernelGGL(k_conv_pack, dim3(9 * 4 * 2 * 512 / 256, kPackParts), dim3(256), 0, (hipStream_t)stream, weights,
                       (uint16_t *)fwd, (uint16_t *)dgrad);
    return launched("k_conv_pack");
}

}  // extern "C"
