// r48_mlp_train.hip -- the fused A3C update of the reference's own network (algorithm/a3c/a3c.py:99-169,
// fp32) on gfx950: r48_mlp_train_grad (include/rein48.h). The forward / rollout kernels are in
// r48_mlp.hip; this file is built on its own because its scalar f32 VALU code must not be SLP-packed
// (packed f32 VALU issues at half rate; Makefile FLAGS_r48_mlp_train).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_mlp_common.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using namespace r48mlp;

// ---------------------------------------------------------------- fused update
// k_mlp_train: the gradient of the A3C loss (rein48_amd/a3c/losses.py restating a3c.py:99-123,
// textbook or the reference's broadcast actor loss; the per-row formulas of r48_a3c_train.hip's
// k_cnn_train) w.r.t. all 2,501 parameters, fp32, in ONE pass over the training states.
// The two 16 -> 64 layers are the bulk of the work (4,096 of ~5,000 FMAs per row: the forward and the
// dW1 contraction of both networks) and run on the fp32 MFMA (v_mfma_f32_16x16x4_f32: bit-for-bit
// a k-ordered fmaf chain, 1,024 FMAs per 32-cycle issue); the rest is VALU. The f32 MFMA runs at the
// f32 VALU rate and did not co-execute with the VALU here (SQ_VALU_MFMA_COEXEC_CYCLES 0): what it
// buys is instruction count -- 4 MFMAs per row for the 4,096 FMAs -- not overlap. A wave takes 16 rows
// per tile in ONE orientation, rows in registers and hidden units on the lanes:
//   layer 1   pre-activation P[r][u] = b1[u] + sum_f x[r][f] W1[u][f] (one fmaf chain over f = 0..15):
//             A = x (16 rows x 4 inputs per k-step, lane j + 16g holds x[r0 + j][4s + g]), B = W1^T
//             (lane j + 16g: W1[16ub + j][4s + g], constant); D lane j + 16g, register i = row
//             4g + i, unit 16ub + j.  2 nets x 4 unit blocks x 4 k-steps = 32 MFMAs per tile
//   ReLU6     mask / h elementwise in that layout (exact decisions near 0 and 6, below)
//   layer 2   logits and value of the group's rows: each lane sums its 4 units per row, then one
//             transposing DPP reduction over the 16 lanes per output leaves row 4g + lrow in lane j
//             (lrow = 2 bit3(j) + bit2(j); the row's four lanes hold the bitwise same sums)
//   loss      lane 4r + k on logit k of tile row r (sums / max over k within the DPP quad):
//             softmax, entropy, td -> dz (through the logits' ReLU), dv; via the wave's LDS tile area
//   dh        [mask] W2^T dz / [mask] wc2 dv, elementwise; db1, dW2, dwc2 in per-lane LDS partials
//   dW1       += x^T dh on the MFMA: A = x^T (lane j + 16g, k-step i: x[r0 + 4g + i][j]), B = dh (the
//             layer-1 layout IS the B layout of a k = rows contraction), C = dW1^T (f x units, 4
//             accumulators per net and unit block, in AGPRs).  32 MFMAs per tile
// Per wave one record of the flat gradient in FlatParams order (a1.w [64][16] | a1.b | a2.w [4][64] |
// a2.b | c1.w | c1.b | c2.w | c2.b) + the two losses; k_mlp_reduce sums the records in a fixed order
// (deterministic).
// The ReLU derivatives are decisions at 0 (and 6, ReLU6): an fp32 pre-activation within its rounding
// error of the boundary may land on the other side than the exact value, and with raw tile values as
// inputs (up to 2^17) a flipped hidden-unit mask moves a weight-gradient entry by a whole row's term
// (dh x). So the update decides them on exact-enough values: a hidden pre-activation or a logit whose
// fp32 value lies within its fp32 error bound of the boundary is recomputed in fp64. Two passes:
//   FIX = false  the hot path: fp32 decisions everywhere; a tile with any decision inside its bound
//                (6.6-6.9 % of the config-3 tiles) only goes on the wave's list (no fix-up code in
//                this kernel: its registers stay free for the hot loop)
//   FIX = true   one wave per hot wave walks that wave's list in order: the same forward (the same
//                instructions, so the same bits), the exact decisions of the flagged units and rows,
//                and -- only where a decision changes (~1e-3 of them) -- the loss and the row's backward
//                on the difference (exact decisions minus the hot path's), into its own record.
// The records of both passes are summed in one fixed order (deterministic).
constexpr int kTrainWaves = 4;
constexpr int kRec = 2504;                 // 2,501 gradient floats + actor loss + critic loss + pad
constexpr int kRecLossA = 2501, kRecLossC = 2502;
// (the record's section offsets equal the blob's, kA1W .. kC2B; inside a1 / a2 / c1 the record has
// the parameters' own [out][in] order)
constexpr float kEntropyEps = 1e-5f;       // a3c.py:114
constexpr float kLn2 = 0.69314718055994531f;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// the wave's LDS board area is written and read by different lanes: every outstanding LDS
// operation completes (s_waitcnt lgkmcnt(0)) before the next access, and the compiler moves no LDS
// access across the point
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

// DPP moves within a 16-lane row. (A row rotation or mirror and a quad permutation read no lane
// outside the row, so bound_ctrl is moot; set, it lets the compiler fold each move into its add as a
// DPP operand.)
template <int N>
__device__ __forceinline__ float row_ror(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + N, 0xF, 0xF, true));
}
// max / sum over the 4 lanes of a DPP quad (quad_perm [1,0,3,2] then [2,3,0,1]): all four lanes get
// the bitwise same result ((a + b) + (c + d) in every lane, by commutativity)
template <int CTRL>
__device__ __forceinline__ float quad_perm(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float quad_sum(float v)
{
    v += quad_perm<0xB1>(v);
    return v + quad_perm<0x4E>(v);
}
__device__ __forceinline__ float quad_max(float v)
{
    v = fmaxf(v, quad_perm<0xB1>(v));
    return fmaxf(v, quad_perm<0x4E>(v));
}
// four 16-lane sums at once, transposed: v0..v3 are a lane's terms of rows 0..3, and lane j ends with
// the sum over the 16 lanes of its DPP row of row 2 bit3(j) + bit2(j). Lanes j, j ^ 8 split the rows
// in halves (row_ror:8 is the exchange j ^ 8), lanes j, j ^ 7 (row_half_mirror) halve again, then
// the quad adds the rest (^1, ^2): 6 selects + 5 DPP adds instead of 4 x 4 adds. The four lanes of a
// row get the bitwise same sum.
__device__ __forceinline__ float row_sum4x16(float v0, float v1, float v2, float v3, bool hi8, bool hi4)
{
    const float a0 = hi8 ? v2 : v0, a1 = hi8 ? v3 : v1, s0 = hi8 ? v0 : v2, s1 = hi8 ? v1 : v3;
    const float r0 = a0 + row_ror<8>(s0), r1 = a1 + row_ror<8>(s1);
    const float c = hi4 ? r1 : r0, s = hi4 ? r0 : r1;
    float t = c + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x141, 0xF, 0xF, true));
    t += quad_perm<0xB1>(t);
    return t + quad_perm<0x4E>(t);
}
// fp64 all-reduce over the 16 lanes of a DPP row by rotations 8, 4, 2, 1: at every level a lane adds
// the same two operands as its partner (IEEE addition commutes), so all 16 lanes get the bitwise
// same sum
template <int N>
__device__ __forceinline__ double row_ror_d(double v)
{
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, 0x120 + N, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), 0x120 + N, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double row_sum16_d(double v)
{
    v += row_ror_d<8>(v);
    v += row_ror_d<4>(v);
    v += row_ror_d<2>(v);
    v += row_ror_d<1>(v);
    return v;
}

// blob accessors (pack_mlp layout: layer-1 and W2 grouped by hidden-unit pair)
__device__ __forceinline__ float w1_at(const float *w, int base, int u, int f) { return w[base + 32 * (u >> 1) + 2 * f + (u & 1)]; }
__device__ __forceinline__ float w2_at(const float *w, int u, int k) { return w[kA2W + 8 * (u >> 1) + 2 * k + (u & 1)]; }

// fp64 pre-activation of one hidden unit on the row whose 16 cell bytes are `cells`; `unit` = the
// unit's 16 weights and bias in the workgroup's LDS copy (unit-major, 17 floats: conflict-free)
template <int MODE>
__device__ __forceinline__ double preact64(const float *unit, const uint8_t *cells)
{
    double a = unit[16];
    for (int f = 0; f < 16; f++)
        a = __builtin_fma((double)unit[f], (double)cell_input<MODE>(cells[f]), a);
    return a;
}

// per-wave LDS area of a 16-row tile (32-bit words): boards [16][4] | max input | row weight |
// target | action | cm | counts [16][4] | pre-ReLU logits [16][4] | value | dz through the logits'
// ReLU [16][4] | dv | dz before it [16][4]
constexpr int kTB = 0, kTXm = 64, kTWt = 80, kTTg = 96, kTAc = 112, kTCm = 128, kTCn = 144, kTZr = 208, kTV = 272,
              kTDz = 288, kTDv = 352, kTDu = 368, kTileWords = 432;

// the inputs of one training row, loaded a tile ahead by lane j of every lane group
struct RowIn {
    uint4 b;
    float wt, tgt, c;
    int a;
    float4 cnt;
    int32_t t, L;   // SEG: the row's step (INT32_MAX when not live) and its segment length
};

// SEG: the row weights per board (seg[bidx] = {w0, c0, L, 0} of r48_a3c_segments; the row is weighted
// iff its step tidx < L) instead of per row (wn, cm)
template <bool REF, bool SEG>
__device__ __forceinline__ RowIn fetch_row(int64_t r, int64_t rows, int64_t bidx, int64_t tidx, const int8_t *boards,
                                           const int8_t *actions, const float *targets, const float *wn,
                                           const float *cm, const float4 *seg, const float *counts)
{
    const bool live = r < rows;
    const int64_t rr = live ? r : rows - 1;   // padding rows: a valid row with weight 0
    RowIn x;
    x.b = *reinterpret_cast<const uint4 *>(boards + 16 * rr);
    x.tgt = targets[rr];
    x.a = actions[rr] & 3;
    x.c = 0.0f;
    x.cnt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (SEG) {   // raw per-board values: the step test waits for the load where the row is used
        const float4 sg = seg[bidx];
        x.wt = sg.x;
        x.c = sg.y;
        x.L = __float_as_int(sg.z);
        x.t = live ? (int32_t)tidx : 0x7FFFFFFF;
    } else {
        x.wt = live ? wn[rr] : 0.0f;
        if (REF)
            x.c = live ? cm[rr] : 0.0f;
    }
    if (REF)
        x.cnt = *reinterpret_cast<const float4 *>(counts + 4 * bidx);
    return x;
}

// flag list of hot wave q: int2 entries (tile, any logit near its boundary) at list[2 q cap ..], its
// length in list_len[q]; cap >= the wave's tile count
template <int MODE, bool REF, bool FIX, bool SEG>
__global__ __launch_bounds__(64 * kTrainWaves) __attribute__((amdgpu_waves_per_eu(2))) void k_mlp_train(
    const int8_t *__restrict__ boards, int64_t rows, int64_t n_boards, const int8_t *__restrict__ actions,
    const float *__restrict__ targets, const float *__restrict__ wn, const float *__restrict__ cm,
    const float4 *__restrict__ seg, const float *__restrict__ counts, float beta, const float *__restrict__ w,
    float *__restrict__ partials,
    int32_t *__restrict__ list, int32_t *__restrict__ list_len, int64_t cap)
{
    // per wave: the tile's 16 boards (64 words) and each row's largest input; per workgroup: the
    // layer-1 B operands and biases of every lane (read back each tile: 40 registers the rest of
    // the tile needs)
    __shared__ __attribute__((aligned(16))) uint32_t tiles_lds[kTrainWaves][kTileWords];
    __shared__ __attribute__((aligned(16))) float w1_lds[64][100];   // 100: conflict-free b128 reads
    // both networks' layer 1 for the fix-up's fp64 recompute: [net][unit][16 weights | bias]
    __shared__ float w1x_lds[2][64][17];
    // per lane: the db1 / dW2 / dwc2 partials, per unit block [dW2[k] x 4 | dwc2 | db1 | dbc1 | pad]
    // (read-modified-written by the backward one unit block at a time: registers for two waves per
    // SIMD)
    __shared__ __attribute__((aligned(16))) float acc_lds[kTrainWaves][64][36];   // 36: conflict-free b128 reads and writes
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t qw = (int64_t)blockIdx.x * kTrainWaves + wave;   // this wave's record / list
    const int n_waves = (int)gridDim.x * kTrainWaves;
    // FIX: the entries of all lists in one order (hot wave, position) -- deterministic -- split evenly:
    // this wave takes entries [e_lo, e_hi); (fw, fo) = list and position of entry e_lo
    int64_t e_lo = 0, e_hi = 0;
    int fw = 0, fo = 0;
    if (FIX) {
        // lane l sums the lengths of lists [l * per, (l + 1) * per); an inclusive scan over the lanes
        const int per = (n_waves + 63) / 64;
        int64_t part = 0;
        for (int k = 0; k < per; k++) {
            const int w = lane * per + k;
            part += w < n_waves ? list_len[w] : 0;
        }
        int64_t incl = part;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(incl, d);
            incl += lane >= d ? o : 0;
        }
        const int64_t total = __shfl(incl, 63);
        e_lo = total * qw / n_waves;
        e_hi = total * (qw + 1) / n_waves;
        // the lane whose lists hold entry e_lo, then the list within them (scalar walk over <= per lists)
        const uint64_t past = __builtin_amdgcn_ballot_w64(incl <= e_lo);
        const int l0 = __builtin_popcountll(past);   // first lane with incl > e_lo (64 if none)
        if (e_lo < e_hi) {
            int64_t before = l0 > 0 ? __shfl(incl, l0 - 1) : 0;
            before = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(before >> 32)) << 32) |
                               (uint32_t)__builtin_amdgcn_readfirstlane((int)before));
            int w = l0 * per;
            while (before + list_len[w] <= e_lo) {
                before += list_len[w];
                w++;
            }
            fw = w;
            fo = (int)(e_lo - before);
        }
    }
    uint32_t *bw = tiles_lds[wave];
    const uint8_t *cells = reinterpret_cast<const uint8_t *>(bw);
    constexpr int kW1[2] = {kA1W, kC1W}, kB1[2] = {kA1B, kC1B};

    // constants of lane (j, g)'s units 16ub + j: layer-1 B operands (inputs 4s + g) and biases in
    // LDS (w1_lds[lane][4 (4 net + ub) + s], [32 + 4 net + ub], W2 [40 + 4 ub + k], wc2 [56 + ub], the
    // bias broadcast [60 + 4 (4 net + ub) + q])
    if (threadIdx.x < 64) {
#pragma unroll
        for (int net = 0; net < 2; net++)
#pragma unroll
            for (int ub = 0; ub < 4; ub++) {
                const int u = 16 * ub + j;
#pragma unroll
                for (int s4 = 0; s4 < 4; s4++)
                    w1_lds[lane][4 * (4 * net + ub) + s4] = w1_at(w, kW1[net], u, 4 * s4 + g);
                w1_lds[lane][32 + 4 * net + ub] = w[kB1[net] + u];
#pragma unroll
                for (int q = 0; q < 4; q++)   // the bias again, broadcast: layer 1's C operand as one read
                    w1_lds[lane][60 + 4 * (4 * net + ub) + q] = w[kB1[net] + u];
            }
#pragma unroll
        for (int ub = 0; ub < 4; ub++) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                w1_lds[lane][40 + 4 * ub + k] = w2_at(w, 16 * ub + j, k);
            w1_lds[lane][56 + ub] = w[kC2W + 16 * ub + j];
            w1_lds[lane][92 + ub] = w2_at(w, 16 * ub + j, g);   // the dh MFMA's B operand: W2[g][16ub + j]
        }
    }
    float *acc = acc_lds[wave][lane];
#pragma unroll
    for (int q = 0; q < 8; q++)
        reinterpret_cast<float4 *>(acc)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = threadIdx.x; q < 2 * 64 * 17; q += 64 * kTrainWaves) {
        const int net = q / (64 * 17), u = (q / 17) % 64, f = q % 17;
        w1x_lds[net][u][f] = f < 16 ? w1_at(w, kW1[net], u, f) : w[kB1[net] + u];
    }
    __syncthreads();
    const float4 *wl = reinterpret_cast<const float4 *>(w1_lds[lane]);   // this lane's constants
    // fp32 error bound of a hidden pre-activation: the MFMA's k-ordered chain of 16 fmaf from b is
    // within gamma_16 (|b| + sum |w x|) of the exact value (gamma_n = n u / (1 - n u), u = 2^-24:
    // 2^-20 (1 + 2^-20)); bounded by 1.0625 * 2^-20 (|b| + sum |w| max x) (the 1/16 covers gamma's
    // excess and the bound's own fp32 roundings), + 2^-21 for the rounding of the decision's a - 3;
    // with the largest |b| and sum |w| of the network's 64 units (wave-uniform, SGPRs)
    float s1[2], e1[2];
#pragma unroll
    for (int net = 0; net < 2; net++) {
        float sm = 0.f, bm = 0.f;
        for (int u = 0; u < 64; u++) {
            float sa = 0.f;
            for (int f = 0; f < 16; f++)
                sa += fabsf(w1_at(w, kW1[net], u, f));
            sm = fmaxf(sm, sa);
            bm = fmaxf(bm, fabsf(w[kB1[net] + u]));
        }
        s1[net] = uniform(sm * 0x1.1p-20f);
        e1[net] = uniform(fmaf(bm, 0x1.1p-20f, 0x1p-21f));
    }
    // fp32 error bound of a pre-ReLU logit: its own sum (64 products of |h| <= 6, b2 added last; every
    // term passes 9 roundings -- a 4-fmaf chain per lane, the 4 levels of the 16-lane reduction, the
    // bias: < 9 u (|b2| + 6 sum |W2[k][:]|), bounded by 2^-19 (...)) plus the hidden units' errors
    // carried through W2 (each < 1.0625 * 2^-20 (|b1| + sum |W1[u][:]| max x), see above; the clamp
    // is 1-Lipschitz) (wave-uniform: kept in SGPRs)
    float zedge[4], zcarry[4], hb = 0.f, hw = 0.f;
    for (int u = 0; u < 64; u++) {
        float sw = 0.f;
        for (int f = 0; f < 16; f++)
            sw += fabsf(w1_at(w, kA1W, u, f));
        hw = fmaxf(hw, sw);
        hb = fmaxf(hb, fabsf(w[kA1B + u]));
    }
    float b2[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        float sa = 0.f;
        for (int u = 0; u < 64; u++)
            sa += fabsf(w2_at(w, u, k));
        zedge[k] = uniform((fabsf(w[kA2B + k]) + 6.0f * sa) * 0x1p-19f);
        zcarry[k] = uniform(sa * 0x1.1p-20f);
        b2[k] = uniform(w[kA2B + k]);
    }
    hb = uniform(hb);
    hw = uniform(hw);
    const float bc2 = uniform(w[kC2B]);

    // accumulators: dW1^T per net and unit block (MFMA C: f = 4g + i, unit 16ub + j), per-lane
    // partials of db1, dW2, dwc2 (summed over the lane's rows; the four lane groups are added at the
    // end), per-row sums (counted in the lanes j == 0)
    f32x4 gw1[2][4];
#pragma unroll
    for (int ub = 0; ub < 4; ub++)
        gw1[0][ub] = gw1[1][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
    // per-lane sums of the loss phase (lane 4r + k works on logit k = lk): db2[k], and the rows'
    // dbc2 and losses; the fix-up's db2 changes go to the LDS partials (slot a1.w of unit block k)
    float gb2l = 0.f, gbc2 = 0.f, loss_a = 0.f, loss_c = 0.f;
    const int lk = lane & 3;
    // layer 2's reduction: lane j of a row group ends with row lrow = 2 bit3(j) + bit2(j)
    const bool hi8 = (j & 8) != 0, hi4 = (j & 4) != 0;
    const int lrow = (hi8 ? 2 : 0) + (hi4 ? 1 : 0);
    const float zedge_l = lk == 0 ? zedge[0] : lk == 1 ? zedge[1] : lk == 2 ? zedge[2] : zedge[3];
    const float zcarry_l = lk == 0 ? zcarry[0] : lk == 1 ? zcarry[1] : lk == 2 ? zcarry[2] : zcarry[3];
    const float once = j == 0 ? 1.0f : 0.0f;   // the fix-up's per-row sums: one lane of the row group

    const int64_t n_tiles = (rows + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * kTrainWaves;
    int32_t *my_list = list + 2 * qw * cap;   // entries (tile, any logit near its boundary)
    int n_flag = 0;                       // hot pass: tiles put on the list (wave-uniform)
    // fix pass: the entry being processed (cur_near) and the next one's position (fw, fo)
    auto fix_entry = [&]() -> int2 {
        const int2 v = *reinterpret_cast<const int2 *>(list + 2 * ((int64_t)fw * cap + fo));
        if (++fo >= list_len[fw]) {
            fo = 0;
            do
                fw++;
            while (fw < n_waves && list_len[fw] == 0);
        }
        return v;
    };
    int cur_near = 0, nxt_near = 0;
    int64_t tile = qw;
    if (FIX) {
        const int2 v = e_lo < e_hi ? fix_entry() : make_int2((int)(n_tiles - 1), 0);
        tile = v.x;
        nxt_near = v.y;
    }
    // one wave per SIMD hides no load latency: row r0 + j's inputs arrive a tile ahead
    // the counts row of training row r is r mod n_boards (rows are step-major, t * n_boards + board):
    // kept incrementally as the lane's row advances by 16 * stride (a prefetch past the end, clamped
    // to the last tile, reads a valid counts row it never uses); the fix pass computes it per tile
    // SEG: the step of the row as well (tnext_t, with bnext: the row's (step, board)), both advanced
    // without a division in the hot pass
    const int64_t r0 = (SEG ? tile : std::min<int64_t>(tile, n_tiles - 1)) * 16 + j;
    int64_t bnext = REF || SEG ? r0 % n_boards : 0;
    int64_t tnext_t = SEG ? r0 / n_boards : 0;   // < 2^31: rows / n_boards steps
    const int64_t bstep = REF || SEG ? (stride * 16) % n_boards : 0;
    const int64_t tstep = SEG ? (stride * 16) / n_boards : 0;
    RowIn next = fetch_row<REF, SEG>(std::min<int64_t>(tile, n_tiles - 1) * 16 + j, rows, bnext, tnext_t, boards, actions,
                                     targets, wn, cm, seg, counts);
    for (int64_t e = e_lo; FIX ? e < e_hi : tile < n_tiles; e++) {
        // ---------------- inputs: row r0 + j in the four lanes j + 16g
        const RowIn in = next;
        int64_t tnext;
        if (FIX) {
            cur_near = nxt_near;
            tnext = tile;
            if (e + 1 < e_hi) {
                const int2 v = fix_entry();
                tnext = v.x;
                nxt_near = v.y;
            }
            if (REF || SEG)
                bnext = (tnext * 16 + j) % n_boards;
            if (SEG)
                tnext_t = (tnext * 16 + j) / n_boards;
        } else {
            tnext = std::min<int64_t>(tile + stride, n_tiles - 1);
            if (REF || SEG) {
                bnext += bstep;
                tnext_t += tstep;
                if (bnext >= n_boards)
                    bnext -= n_boards, tnext_t++;
            }
        }
        next = fetch_row<REF, SEG>(tnext * 16 + j, rows, bnext, tnext_t, boards, actions, targets, wn, cm, seg, counts);
        const uint4 bv = in.b;
        const uint32_t bwd[4] = {bv.x, bv.y, bv.z, bv.w};
        float xa[4];   // A operands of layer 1: x[r0 + j][4s + g]
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++)
            xa[s4] = cell_input<MODE>((bwd[s4] >> (8 * g)) & 0xFFu);
        uint32_t mb = 0;   // largest cell byte of the row (inputs grow with it)
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                mb = std::max(mb, (bwd[s4] >> (8 * q)) & 0xFFu);
        wave_lds_sync();   // the previous tile's reads of the board area are done
        if (g == 0) {
            *reinterpret_cast<uint4 *>(bw + kTB + 4 * j) = bv;
            bw[kTXm + j] = __float_as_uint(cell_input<MODE>(mb));
            const bool on = !SEG || in.t < in.L;
            bw[kTWt + j] = __float_as_uint(on ? in.wt : 0.0f);
            bw[kTTg + j] = __float_as_uint(in.tgt);
            bw[kTAc + j] = (uint32_t)in.a;
            if (REF) {
                bw[kTCm + j] = __float_as_uint(on ? in.c : 0.0f);
                *reinterpret_cast<float4 *>(bw + kTCn + 4 * j) = in.cnt;
            }
        }
        wave_lds_sync();
        float xt[4], xm[4];   // A operands of dW1: x[r0 + 4g + i][j]; max input of row 4g + i
#pragma unroll
        for (int i = 0; i < 4; i++) {
            xt[i] = cell_input<MODE>(cells[16 * (4 * g + i) + j]);
            xm[i] = __uint_as_float(bw[kTXm + 4 * g + i]);
        }

        // ---------------- layer 1 on the MFMA: register i = row 4g + i, lane j = unit 16ub + j
        f32x4 pre[2][4];
#pragma unroll
        for (int net = 0; net < 2; net++)
#pragma unroll
            for (int ub = 0; ub < 4; ub++) {
                const float4 wb = wl[4 * net + ub];
                const float4 b4 = wl[15 + 4 * net + ub];
                f32x4 acc = f32x4{b4.x, b4.y, b4.z, b4.w};
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[0], wb.x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[1], wb.y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[2], wb.z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[3], wb.w, acc, 0, 0, 0);
                pre[net][ub] = acc;
            }
        bool edge_any = false;
        // ---------------- ReLU6 decisions 0 < a < 6, i.e. |a - 3| < 3; within the fp32 error bound
        // of 0 or 6 (min(|a|, |a - 6|) = ||a - 3| - 3|) the pre-activation is redone in fp64
        // (the hot path takes the fp32 decision where it uses a mask and only asks whether any of
        // the tile's 512 pre-activations is near a boundary; the fix-up below finds which)
        if (!FIX) {   // (the fix pass tests each unit itself)
        float bound[2][4];
#pragma unroll
        for (int net = 0; net < 2; net++)
#pragma unroll
            for (int i = 0; i < 4; i++)
                bound[net][i] = fmaf(s1[net], xm[i], e1[net]);
        // (per row and net: the nearest of the lane's 4 units against the row's bound)
#pragma unroll
        for (int net = 0; net < 2; net++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                float dn[4];
#pragma unroll
                for (int ub = 0; ub < 4; ub++)
                    dn[ub] = fabsf(fabsf(pre[net][ub][i] - 3.0f) - 3.0f);
                edge_any |= fminf(fminf(dn[0], dn[1]), fminf(dn[2], dn[3])) < bound[net][i];
            }
        }
        // ---------------- per row i of the lane group (rows 4g + i): layer 2 (the group's 16 lanes
        // add up), the loss (every lane of the group computes it; counted once) -- the same code on
        // the hot path and in the exact-decision fix-up below, so the same values
        // layer 2: each lane's partial sums over its 4 units for the group's 4 rows, then one
        // transposing reduction over the 16 lanes per output (row_sum4x16): lane j ends with row
        // 4g + lrow's logits (pre-ReLU) and value
        auto layer2 = [&](float (&zr)[4], float &v) {
            float pk[4][4], pv[4];   // [i][k]
            const float4 c2 = wl[14];   // wc2 of the lane's 4 units
            const float wc2[4] = {c2.x, c2.y, c2.z, c2.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                pk[i][0] = pk[i][1] = pk[i][2] = pk[i][3] = pv[i] = 0.0f;
#pragma unroll
                for (int ub = 0; ub < 4; ub++) {
                    const float4 w4 = wl[10 + ub];   // W2[k][16ub + j]
                    const float ha = __builtin_amdgcn_fmed3f(pre[0][ub][i], 0.0f, 6.0f);
                    pk[i][0] = fmaf(w4.x, ha, pk[i][0]);
                    pk[i][1] = fmaf(w4.y, ha, pk[i][1]);
                    pk[i][2] = fmaf(w4.z, ha, pk[i][2]);
                    pk[i][3] = fmaf(w4.w, ha, pk[i][3]);
                    pv[i] = fmaf(wc2[ub], __builtin_amdgcn_fmed3f(pre[1][ub][i], 0.0f, 6.0f), pv[i]);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++)
                zr[k] = b2[k] + row_sum4x16(pk[0][k], pk[1][k], pk[2][k], pk[3][k], hi8, hi4);   // pre-ReLU
            v = bc2 + row_sum4x16(pv[0], pv[1], pv[2], pv[3], hi8, hi4);
        };
        // the backward of the lane group's 4 rows with output gradients dz (through the logits' ReLU)
        // and dv, and hidden masks (the fp32 decisions, or the given bits in the fix-up): the per-lane
        // partials (in LDS, one unit block at a time) and the rows' k-steps of dW1 on the MFMA
        // (register i = row, lane = unit); `sel` picks the rows (bit i). The fix-up runs it on
        // differences (`fix`): dv does not depend on any decision, so only its mask terms move there,
        // and the db2 change goes to the unit block's spare slot (slot k = ub, once per row group)
        f32x4 sdhm[4];   // the hot path's W2^T dz (MFMA, below)
        auto rows_backward = [&](const float (&dz)[4][4], const float (&dv)[4], uint32_t sel, bool bits, uint32_t mk,
                                 bool fix) {
            const float4 c2 = wl[14];
            const float wc2[4] = {c2.x, c2.y, c2.z, c2.w};
#pragma unroll
            for (int ub = 0; ub < 4; ub++) {
                const float4 w4 = wl[10 + ub];
                float4 a2 = reinterpret_cast<float4 *>(acc)[2 * ub];        // dW2[k][16ub + j] partials
                float4 a1 = reinterpret_cast<float4 *>(acc)[2 * ub + 1];    // dwc2 | db1 | dbc1 | db2 fix-ups
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    if (!((sel >> i) & 1u))
                        continue;
                    const float ha = __builtin_amdgcn_fmed3f(pre[0][ub][i], 0.0f, 6.0f);
                    const float hc = __builtin_amdgcn_fmed3f(pre[1][ub][i], 0.0f, 6.0f);
                    const float sdh = fix ? fmaf(w4.w, dz[i][3], fmaf(w4.z, dz[i][2], fmaf(w4.y, dz[i][1], w4.x * dz[i][0])))
                                          : sdhm[ub][i];
                    // the masks: the given bits (fix-up) or the fp32 decisions 0 < a < 6, i.e. |a - 3| < 3
                    const bool ma = bits ? ((mk >> (4 * ub + i)) & 1u) != 0 : fabsf(pre[0][ub][i] - 3.0f) < 3.0f;
                    const bool mc = bits ? ((mk >> (16 + 4 * ub + i)) & 1u) != 0 : fabsf(pre[1][ub][i] - 3.0f) < 3.0f;
                    const float dha = ma ? sdh : 0.0f;
                    const float dhc = mc ? wc2[ub] * dv[i] : 0.0f;
                    a2.x = fmaf(dz[i][0], ha, a2.x);
                    a2.y = fmaf(dz[i][1], ha, a2.y);
                    a2.z = fmaf(dz[i][2], ha, a2.z);
                    a2.w = fmaf(dz[i][3], ha, a2.w);
                    if (fix) {
                        a1.w = fmaf(once, dz[i][ub], a1.w);
                    } else {
                        a1.x = fmaf(dv[i], hc, a1.x);
                    }
                    a1.y += dha;
                    a1.z += dhc;
                    gw1[0][ub] = __builtin_amdgcn_mfma_f32_16x16x4f32(xt[i], dha, gw1[0][ub], 0, 0, 0);
                    gw1[1][ub] = __builtin_amdgcn_mfma_f32_16x16x4f32(xt[i], dhc, gw1[1][ub], 0, 0, 0);
                }
                reinterpret_cast<float4 *>(acc)[2 * ub] = a2;
                reinterpret_cast<float4 *>(acc)[2 * ub + 1] = a1;
            }
        };
        // layer 2 of the lane group's rows into the tile area: pre-ReLU logits (kTZr) and value (kTV)
        auto layer2_lds = [&]() {
            float zq[4], vq;
            layer2(zq, vq);
            if ((j & 3) == 0) {   // the four lanes of a row hold the bitwise same sums
                *reinterpret_cast<float4 *>(bw + kTZr + 4 * (4 * g + lrow)) = make_float4(zq[0], zq[1], zq[2], zq[3]);
                bw[kTV + 4 * g + lrow] = __float_as_uint(vq);
            }
            wave_lds_sync();
        };
        // lane 4r + k: is logit k of tile row r within its fp32 error bound of the logits' ReLU
        // boundary (bit 4r + k of the ballot); from the tile area after layer2_lds
        auto near_ballot = [&]() -> uint64_t {
            const int r = lane >> 2;
            const float zr = __uint_as_float(bw[kTZr + lane]);
            const float xml = __uint_as_float(bw[kTXm + r]);
            return __builtin_amdgcn_ballot_w64(fabsf(zr) < zedge_l + zcarry_l * (hb + hw * xml));
        };
        // this lane group's rows 4g + i with a logit near the boundary (bit i)
        auto group_rows = [&](uint64_t near_rows) {
            const uint32_t near_q = (uint32_t)(near_rows >> (16 * g)) & 0xFFFFu;
            uint32_t near = 0;
#pragma unroll
            for (int i = 0; i < 4; i++)
                near |= ((near_q >> (4 * i)) & 0xFu) != 0 ? 1u << i : 0u;
            return near;
        };
        // the loss with lane 4r + k on logit k of tile row r (the row's DPP quad does the sums over k):
        // dz through the logits' ReLU (kTDz), before it (kTDu), dv (kTDv) into the tile area; the hot
        // pass also sums db2, dbc2 and the losses
        auto loss_lds = [&]() {
            {
                const int r = lane >> 2;
                const float zr = __uint_as_float(bw[kTZr + lane]);
                const float v = __uint_as_float(bw[kTV + r]);
                const float wt = __uint_as_float(bw[kTWt + r]);
                const float tgt = __uint_as_float(bw[kTTg + r]);
                const float z = fmaxf(zr, 0.0f);                               // the logits' ReLU (a3c.py:153)
                const float mz = quad_max(z);
                float p = __expf(z - mz);
                const float se = quad_sum(p);
                const float inv = __builtin_amdgcn_rcpf(se), lse = mz + kLn2 * __builtin_amdgcn_logf(se);
                p *= inv;
                const float lq = kLn2 * __builtin_amdgcn_logf(p + kEntropyEps);
                const float hk = -p * lq;                                       // logit k's term of the entropy
                const float gr = -(lq + p * __builtin_amdgcn_rcpf(p + kEntropyEps));   // dH/dp_k
                const float gbar = quad_sum(p * gr);
                const float td = tgt - v;
                float dz, la;
                if (REF) {   // reference: -beta wn H - cm sum_k c_k log p_k  (losses.py, a3c.py:110-116)
                    const float c = __uint_as_float(bw[kTCm + r]);
                    const float ck = __uint_as_float(bw[kTCn + lane]);
                    const float C = quad_sum(ck);
                    dz = -beta * wt * p * (gr - gbar) - c * (ck - p * C);
                    la = -beta * wt * hk - c * (ck * (z - lse));
                } else {     // textbook: -wn (beta H + td log p[a]), td constant for the actor
                    const bool act = lk == (int)bw[kTAc + r];
                    dz = -wt * (beta * p * (gr - gbar) + td * ((act ? 1.0f : 0.0f) - p));
                    la = -wt * (beta * hk + (act ? td * (z - lse) : 0.0f));
                }
                const float dv = -2.0f * wt * td;                               // critic = wn td^2
                const float dzm = zr > 0.0f ? dz : 0.0f;
                if (!FIX) {      // the fix pass adds only differences
                    gb2l += dzm;
                    loss_a += la;
                }
                if (lk == 0) {   // the row's terms once
                    if (!FIX) {
                        gbc2 += dv;
                        loss_c += wt * td * td;
                    }
                    bw[kTDv + r] = __float_as_uint(dv);
                }
                bw[kTDz + lane] = __float_as_uint(dzm);
                bw[kTDu + lane] = __float_as_uint(dz);
            }
            wave_lds_sync();
        };
        if (!FIX) {
            // ---------------- hot pass: fp32 decisions everywhere
            layer2_lds();
            const uint64_t near_rows = near_ballot();
            loss_lds();
            const uint32_t near = group_rows(near_rows);
            float dz[4][4], dv[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float4 d4 = *reinterpret_cast<const float4 *>(bw + kTDz + 4 * (4 * g + i));
                dz[i][0] = d4.x, dz[i][1] = d4.y, dz[i][2] = d4.z, dz[i][3] = d4.w;
                dv[i] = __uint_as_float(bw[kTDv + 4 * g + i]);
            }
            // W2^T dz on the MFMA: A = dz (lane j + 16g: row j, logit g), B = W2[g][16ub + j], D = [row
            // 4g + i][unit 16ub + j] -- the same k-ordered fmaf chain as the fix pass's VALU form
            const float adz = __uint_as_float(bw[kTDz + 4 * j + g]);
            const float4 w2g = wl[23];
            const float w2b[4] = {w2g.x, w2g.y, w2g.z, w2g.w};
#pragma unroll
            for (int ub = 0; ub < 4; ub++)
                sdhm[ub] = __builtin_amdgcn_mfma_f32_16x16x4f32(adz, w2b[ub], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            rows_backward(dz, dv, 0xFu, false, 0u, false);
            // a tile with any decision within its bound goes on the list: (tile, any logit near)
            if (__builtin_amdgcn_ballot_w64(edge_any || near != 0)) {
                if (lane == 0)
                    *reinterpret_cast<int2 *>(my_list + 2 * n_flag) = make_int2((int)tile, near_rows != 0 ? 1 : 0);
                n_flag++;
            }
        } else {
            // ---------------- fix pass (the whole wave; lanes pick their own rows): the exact hidden
            // masks of the units within their bound (fp64), the exact logits' ReLU of the rows near
            // it (fp64, when the hot pass saw any), and only where a decision differs from the hot
            // path's: the loss (the hot path's dz) and the row's backward on the differences
            uint32_t mask = 0, edge = 0;   // fp32 decisions and flags, bit 16 net + 4 ub + i
#pragma unroll
            for (int net = 0; net < 2; net++)
#pragma unroll
                for (int ub = 0; ub < 4; ub++)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const float d = fabsf(pre[net][ub][i] - 3.0f);
                        const uint32_t bit = 1u << (16 * net + 4 * ub + i);
                        mask |= d < 3.0f ? bit : 0u;
                        edge |= fabsf(d - 3.0f) < fmaf(s1[net], xm[i], e1[net]) ? bit : 0u;
                    }
            uint32_t mx = mask;   // exact hidden masks
            for (uint32_t m = edge; m; m &= m - 1) {
                const int bit = __builtin_ctz(m), net = bit >> 4, ub = (bit >> 2) & 3, i = bit & 3;
                const double ad = preact64<MODE>(&w1x_lds[net][16 * ub + j][0], cells + 16 * (4 * g + i));
                mx = (ad > 0.0 && ad < 6.0) ? (mx | (1u << bit)) : (mx & ~(1u << bit));
            }
            uint32_t near = 0, posb = 0, chg = 0;   // per row i: near / exact logit decisions (bit 4i + k) / changed
            const bool have_z = cur_near != 0;      // wave-uniform: the hot pass saw a logit near its boundary
            if (have_z) {
                layer2_lds();
                near = group_rows(near_ballot());
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                bool changed = (((mx ^ mask) >> i) & 0x11111111u) != 0;
                if (__builtin_amdgcn_ballot_w64((near >> i) & 1u)) {   // the group's lanes together (DPP sums)
                    const int ri = 4 * g + i;
                    const float4 z4 = *reinterpret_cast<const float4 *>(bw + kTZr + 4 * ri);
                    const float zr[4] = {z4.x, z4.y, z4.z, z4.w};
                    const uint8_t *rc = cells + 16 * ri;
                    double pk[4] = {0.0, 0.0, 0.0, 0.0};
                    for (int ub = 0; ub < 4; ub++) {
                        const double ad = preact64<MODE>(&w1x_lds[0][16 * ub + j][0], rc);
                        const double h = ad < 0.0 ? 0.0 : (ad > 6.0 ? 6.0 : ad);
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            pk[k] = __builtin_fma((double)w1_lds[lane][40 + 4 * ub + k], h, pk[k]);
                    }
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const bool pos = (double)b2[k] + row_sum16_d(pk[k]) > 0.0;
                        posb |= pos ? 1u << (4 * i + k) : 0u;
                        changed |= ((near >> i) & 1u) && pos != (zr[k] > 0.0f);
                    }
                }
                chg |= changed ? 1u << i : 0u;
            }
            // nothing to correct where every exact decision equals the hot path's (nearly always:
            // the bounds flag ~7 % of the tiles, ~1e-3 of the flagged decisions flip)
            if (__builtin_amdgcn_ballot_w64(chg != 0)) {
                if (!have_z)
                    layer2_lds();
                loss_lds();
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    if (!__builtin_amdgcn_ballot_w64((chg >> i) & 1u))
                        continue;
                    const bool changed = (chg >> i) & 1u;
                    const int ri = 4 * g + i;
                    const float4 z4 = *reinterpret_cast<const float4 *>(bw + kTZr + 4 * ri);
                    const float4 m4 = *reinterpret_cast<const float4 *>(bw + kTDz + 4 * ri);
                    const float4 u4 = *reinterpret_cast<const float4 *>(bw + kTDu + 4 * ri);
                    const float zr[4] = {z4.x, z4.y, z4.z, z4.w}, dzm[4] = {m4.x, m4.y, m4.z, m4.w},
                                dzu[4] = {u4.x, u4.y, u4.z, u4.w};
                    const float dv = __uint_as_float(bw[kTDv + ri]);
                    // the hot path's terms with its decisions, then the exact ones: backward(exact) -
                    // backward(hot) is linear in dz and dv, so run the difference on each mask set. A
                    // lane whose row and units kept every decision adds exact zeros (its two terms
                    // would cancel only up to rounding)
                    float ndz[4][4] = {}, pdz[4][4] = {}, dv4[4] = {}, ndv4[4] = {};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const bool pos = (near >> i) & 1u ? ((posb >> (4 * i + k)) & 1u) != 0 : zr[k] > 0.0f;
                        ndz[i][k] = changed ? -dzm[k] : 0.0f;
                        pdz[i][k] = changed && pos ? dzu[k] : 0.0f;
                    }
                    dv4[i] = changed ? dv : 0.0f;
                    ndv4[i] = changed ? -dv : 0.0f;
                    rows_backward(ndz, ndv4, 1u << i, true, mask, true);
                    rows_backward(pdz, dv4, 1u << i, true, mx, true);
                }
            }
        }
        tile = FIX ? tnext : tile + stride;
    }
    if (!FIX && lane == 0)
        list_len[qw] = n_flag;
    // ---------------- this wave's record (FlatParams order)
    float *rec = partials + qw * kRec;
#pragma unroll
    for (int ub = 0; ub < 4; ub++) {
        const int u = 16 * ub + j;
        *reinterpret_cast<float4 *>(rec + kA1W + 16 * u + 4 * g) = make_float4(gw1[0][ub][0], gw1[0][ub][1], gw1[0][ub][2], gw1[0][ub][3]);
        *reinterpret_cast<float4 *>(rec + kC1W + 16 * u + 4 * g) = make_float4(gw1[1][ub][0], gw1[1][ub][1], gw1[1][ub][2], gw1[1][ub][3]);
    }
    // per-lane partials over the four lane groups (fixed order: (g0 + g1) + (g2 + g3) in every lane)
    auto groups = [](float x) {
        x += __shfl_xor(x, 16);
        return x + __shfl_xor(x, 32);
    };
#pragma unroll
    for (int ub = 0; ub < 4; ub++) {
        const int u = 16 * ub + j;
        const float4 a2 = reinterpret_cast<const float4 *>(acc)[2 * ub], a1 = reinterpret_cast<const float4 *>(acc)[2 * ub + 1];
        const float a1b = groups(a1.y), c1b = groups(a1.z), c2w = groups(a1.x);
        const float a2w[4] = {groups(a2.x), groups(a2.y), groups(a2.z), groups(a2.w)};
        if (g == 0) {
            rec[kA1B + u] = a1b;
            rec[kC1B + u] = c1b;
            rec[kC2W + u] = c2w;
#pragma unroll
            for (int k = 0; k < 4; k++)
                rec[kA2W + 64 * k + u] = a2w[k];
        }
    }
    float gk[4];   // db2[k]: the loss lanes of logit k + every lane's fix-up slot
#pragma unroll
    for (int k = 0; k < 4; k++)
        gk[k] = (lk == k ? gb2l : 0.0f) + reinterpret_cast<const float4 *>(acc)[2 * k + 1].w;
    const float s0 = wave_sum(gk[0]), s1s = wave_sum(gk[1]), s2 = wave_sum(gk[2]), s3 = wave_sum(gk[3]);
    const float sc = wave_sum(gbc2), la = wave_sum(loss_a), lc = wave_sum(loss_c);
    if (lane == 0) {
        *reinterpret_cast<float4 *>(rec + kA2B) = make_float4(s0, s1s, s2, s3);
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

constexpr int kTrainGroups = 512;    // persistent grid: two workgroups of 4 waves per CU (two waves per SIMD) on 256 CUs

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

}  // namespace

extern "C" {

/* workspace of r48_mlp_train_grad over `rows` training rows (4-byte words): the per-wave records of
 * both passes, the first reduction pass's groups, then the flag lists (one slot per tile of a wave)
 * and their lengths */
constexpr int64_t kTrainRecs = (int64_t)kTrainGroups * kTrainWaves;
constexpr int64_t kRecFloats = (2 * kTrainRecs + (2 * kTrainRecs + kRedGroup - 1) / kRedGroup) * kRec;
static int64_t list_cap(int64_t rows) { return std::max<int64_t>(1, ((rows + 15) / 16 + kTrainRecs - 1) / kTrainRecs); }

int64_t r48_mlp_train_workspace_floats(int64_t rows)
{
    if (rows < 1)
        return fail(R48_EINVAL, "r48_mlp_train_workspace_floats: rows < 1");
    return kRecFloats + 2 * kTrainRecs * list_cap(rows) + kTrainRecs;
}

static int mlp_train_launch(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                            const float *targets, const float *wn, const float *cm, const float *seg, const float *counts,
                            float beta, int32_t mode, const float *w, float *workspace, float *grad, void *stream)
{
    const int n_rec = 2 * kTrainRecs, n_grp = (n_rec + kRedGroup - 1) / kRedGroup;
    const int64_t cap = list_cap(rows);
    int32_t *list = reinterpret_cast<int32_t *>(workspace + kRecFloats);
    int32_t *list_len = list + 2 * kTrainRecs * cap;
    hipStream_t s = (hipStream_t)stream;
    const float4 *sg = reinterpret_cast<const float4 *>(seg);
    // hot pass (records 0 .. kTrainRecs - 1, the flag lists), then the fix pass over the lists (records
    // kTrainRecs ..): one stream, so the fix pass sees the hot pass's lists
    auto go = [&](auto hot, auto fix) {
        hipLaunchKernelGGL(hot, dim3(kTrainGroups), dim3(64 * kTrainWaves), 0, s, boards, rows, n_boards, actions,
                           targets, wn, cm, sg, counts, beta, w, workspace, list, list_len, cap);
        hipLaunchKernelGGL(fix, dim3(kTrainGroups), dim3(64 * kTrainWaves), 0, s, boards, rows, n_boards, actions,
                           targets, wn, cm, sg, counts, beta, w, workspace + kTrainRecs * kRec, list, list_len, cap);
    };
    // the reference loss: cm (per row) or counts with seg (per board)
    const bool ref = seg ? counts != nullptr : cm != nullptr;
    constexpr int V = R48_FEAT_VALUES, E = R48_FEAT_EXPONENTS;
    if (seg) {
        if (mode == V)
            ref ? go(k_mlp_train<V, true, false, true>, k_mlp_train<V, true, true, true>)
                : go(k_mlp_train<V, false, false, true>, k_mlp_train<V, false, true, true>);
        else
            ref ? go(k_mlp_train<E, true, false, true>, k_mlp_train<E, true, true, true>)
                : go(k_mlp_train<E, false, false, true>, k_mlp_train<E, false, true, true>);
    } else {
        if (mode == V)
            ref ? go(k_mlp_train<V, true, false, false>, k_mlp_train<V, true, true, false>)
                : go(k_mlp_train<V, false, false, false>, k_mlp_train<V, false, true, false>);
        else
            ref ? go(k_mlp_train<E, true, false, false>, k_mlp_train<E, true, true, false>)
                : go(k_mlp_train<E, false, false, false>, k_mlp_train<E, false, true, false>);
    }
    float4 *groups = reinterpret_cast<float4 *>(workspace + (int64_t)n_rec * kRec);
    constexpr int q = kRec / 4;
    hipLaunchKernelGGL(k_mlp_reduce1, dim3((q * n_grp + 255) / 256), dim3(256), 0, s, (const float4 *)workspace, n_rec,
                       groups);
    hipLaunchKernelGGL(k_mlp_reduce2, dim3((q + 255) / 256), dim3(256), 0, s, (const float4 *)groups, n_grp,
                       (float4 *)grad);
    return launched("k_mlp_train");
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
    return mlp_train_launch(boards, rows, n_boards, actions, targets, wn, cm, nullptr, counts, beta, mode, w, workspace,
                            grad, stream);
}

int r48_mlp_train_grad_seg(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                           const float *targets, const float *seg, const float *counts, float beta, int32_t mode,
                           const float *w, float *workspace, float *grad, void *stream)
{
    if (!boards || !actions || !targets || !seg || !w || !workspace || !grad || rows < 1 || n_boards < 1 ||
        (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS))
        return fail(R48_EINVAL, "r48_mlp_train_grad_seg: NULL argument, rows/n_boards < 1 or bad mode");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(seg) |
         reinterpret_cast<uintptr_t>(counts) | reinterpret_cast<uintptr_t>(workspace) |
         reinterpret_cast<uintptr_t>(grad)) & 15u)
        return fail(R48_EINVAL, "r48_mlp_train_grad_seg: boards, w, seg, counts, workspace and grad must be 16-byte "
                                "aligned");
    return mlp_train_launch(boards, rows, n_boards, actions, targets, nullptr, nullptr, seg, counts, beta, mode, w,
                            workspace, grad, stream);
}

}  // extern "C"
