// r48_cnn_common.h -- MFMA building blocks shared by the fused CNN kernels (inference:
// r48_policy.hip; training: r48_a3c_train.hip) for rein48_amd/a3c/nets.py:ActorCriticCNN.
//
// v_mfma_f32_32x32x16_bf16 lane maps: lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h + j]
// and B[k = 8h + j][col r] in element j = 0..7 of its fragment; C/D register i holds
// D[row 8(i>>2) + 4h + (i&3)][col r]. With boards on the column, a 32x32 accumulator feeds the
// next layer as its B operand after acc_to_frag, in the permuted k order
// f(s, j, h) = 16s + 8(j>>2) + 4h + (j&3) (host packing: rein48_amd/a3c/fused.py).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rein48.h"

namespace r48cnn {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x16 = __attribute__((ext_vector_type(16))) float;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

constexpr int kFragW1 = 9, kFragW2 = 16, kFragWh = 16, kFrags = kFragW1 + kFragW2 + kFragWh;
// conv2's 2x2 patches over the 3x3 conv1 grid: input positions of output position p
__device__ constexpr int kP2[4][4] = {{0, 1, 3, 4}, {1, 2, 4, 5}, {3, 4, 6, 7}, {4, 5, 7, 8}};

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi)
{
    // plain casts: hipcc emits one v_cvt_pk_bf16_f32 (round to nearest even)
    const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

// accumulator registers 8s..8s+7 -> the B fragment of k-step s: four v_cvt_pk_bf16_f32 (round to
// nearest even). Converted as 2-vectors: a wider conversion is split into single converts + perm.
__device__ __forceinline__ bf16x8 acc_to_frag(const f32x16 &acc, int s)
{
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    uint32_t p[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
        p[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                                                (f32x2{acc[8 * s + 2 * q], acc[8 * s + 2 * q + 1]}), bf16x2_t));
    bf16x8 f;
    __builtin_memcpy(&f, p, 16);
    return f;
}

// the same with ReLU: as int16 a negative bf16 (sign bit set) is below 0, so a packed int16
// max(v, 0) maps it (and -0) to +0 and keeps every positive value; = bf16(max(a, 0)) bit for bit
__device__ __forceinline__ bf16x8 acc_to_frag_relu(const f32x16 &acc, int s)
{
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef short i16x2 __attribute__((ext_vector_type(2)));
    uint32_t p[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const i16x2 v = __builtin_bit_cast(
            i16x2, __builtin_convertvector((f32x2{acc[8 * s + 2 * q], acc[8 * s + 2 * q + 1]}), bf16x2_t));
        p[q] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, i16x2{0, 0}));
    }
    bf16x8 f;
    __builtin_memcpy(&f, p, 16);
    return f;
}

// per-lane bias registers: C/D row of register r for lane half h is (r&3) + 8(r>>2) + 4h, so
// registers 4u..4u+3 are the 4 contiguous floats at 8u + 4h (four 16-byte LDS reads)
__device__ __forceinline__ f32x16 load_bias(const float *bias_lds, int h)
{
    f32x16 b;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const float4 v = *reinterpret_cast<const float4 *>(bias_lds + 8 * u + 4 * h);
        b[4 * u] = v.x;
        b[4 * u + 1] = v.y;
        b[4 * u + 2] = v.z;
        b[4 * u + 3] = v.w;
    }
    return b;
}

__device__ __forceinline__ f32x16 bias_relu(f32x16 acc, const f32x16 &b)
{
#pragma unroll
    for (int r = 0; r < 16; r++)
        acc[r] = fmaxf(acc[r] + b[r], 0.0f);
    return acc;
}

// exponent e -> bf16 bits of the network input (raw value 2^e, or e itself)
__device__ __forceinline__ uint32_t cell_bf16(uint32_t e, int mode)
{
    if (mode == R48_FEAT_VALUES)
        return e ? ((e + 127u) << 7) : 0u;                     // 2^e is exact in bf16
    return __float_as_uint((float)e) >> 16;                    // small integers are exact
}

// copy N16 16-byte words global -> LDS with every load of a thread in flight at once (the plain
// loop load / wait / store pays one global latency per iteration, ~11 for the 41 KB policy image)
template <int N16, int THREADS>
__device__ __forceinline__ void stage_lds(uint4 *dst, const uint4 *__restrict__ src)
{
    constexpr int kFull = N16 / THREADS, kTail = N16 - kFull * THREADS;
    const int t = (int)threadIdx.x;
    uint4 v[kFull];
#pragma unroll
    for (int j = 0; j < kFull; j++)
        v[j] = src[t + j * THREADS];
    uint4 tail = {};
    if (kTail && t < kTail)
        tail = src[t + kFull * THREADS];
#pragma unroll
    for (int j = 0; j < kFull; j++)
        dst[t + j * THREADS] = v[j];
    if (kTail && t < kTail)
        dst[t + kFull * THREADS] = tail;
}

__device__ __forceinline__ bf16x8 frag_at(const uint4 *w, int frag, int lane)
{
    const uint4 v = w[frag * 64 + lane];
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// ---- weight-fragment pipelining: with one wave per SIMD an MFMA that waits on its own A-fragment
// LDS read exposes the read's latency, so the fragment of the next MFMA is read before the current
// one issues. wfence() keeps that order (DS reads and MFMAs may not cross it; VALU, SALU and
// transcendental work may, so epilogues still interleave with the MFMA stream).
#ifndef R48_WFENCE
#define R48_WFENCE 0x406
#endif
__device__ __forceinline__ void wfence()
{
    if (R48_WFENCE >= 0)
        __builtin_amdgcn_sched_barrier(R48_WFENCE);
}

// A fragment of forward MFMA i (0..88) in issue order: conv1 positions R = 0..8, then the 8 conv2
// chains c = 2p + g (8 W2 fragments (kk, s) each) with the 2 head MFMAs of chain c issued after
// chain c + 1, so the head MFMAs never wait on their chain's epilogue (bf16 pack + ReLU)
constexpr int kFwdMfmas = 9 + 8 * 10;
__host__ __device__ constexpr int fwd_frag(int i)
{
    if (i < 9)
        return i;
    const int t = i - 9;
    if (t < 8)                                                       // chain 0
        return kFragW1 + (t >> 1) * 2 + (t & 1);
    const int t2 = t - 8;
    if (t2 >= 70)                                                    // heads of chain 7
        return kFragW1 + kFragW2 + 7 * 2 + (t2 - 70);
    const int b = t2 / 10, u = t2 % 10;
    return u < 8 ? kFragW1 + (((b + 1) & 1) * 4 + (u >> 1)) * 2 + (u & 1)   // chain b + 1
                 : kFragW1 + kFragW2 + b * 2 + (u - 8);                     // heads of chain b
}

// ---- policy form with the heads on v_mfma_f32_16x16x32_bf16 (r48_policy.hip). The heads have 5
// outputs: as 32x32x16 MFMAs they fill 5 of 32 rows (16 MFMAs, 512 cycles per tile); as 16x16x32 ones
// 5 of 16 (16 MFMAs of 16 cycles, 256). One head fragment H16(p, g) (16 outputs x the 32 features of
// conv2 block (p, g), lane l: output l & 15, features 8 (l >> 4) + j in the order below) feeds two
// MFMAs, one per 16-board group. A 16x16x32 B operand wants board l & 15 in every lane quarter, so
// the two 32x32-layout fragments s = 0, 1 of a block are exchanged in one v_permlane16_swap per
// dword: after it, fragment 0 holds boards 0-15 and fragment 1 boards 16-31, lane quarter q carrying
// features 16 (q & 1) + 4 (q >> 1) + 8 (j >> 2) + (j & 3) (rein48_amd/a3c/fused.py packs H16 so).
// Policy blob: conv1 (9) | conv2 (16) | H16 (p, g) at 25 + 2p + g (8) = 33 fragments.
constexpr int kFragWh16 = 8, kFragsPolicy = kFragW1 + kFragW2 + kFragWh16;
// read order: conv1 R (9), W2(0, u) (8), then per output position p: W2(1, 2p), H16(p, 0),
// W2(1, 2p + 1) (12), then H16(p, 1) (4)
constexpr int kPolicyReads = 9 + 8 + 12 + 4;
__host__ __device__ constexpr int policy_frag(int i)
{
    if (i < 9)
        return i;
    i -= 9;
    if (i < 8)
        return kFragW1 + i;                                             // W2(0, u = i)
    i -= 8;
    if (i < 12) {
        const int p = i / 3, r = i % 3;
        return r == 1 ? kFragW1 + kFragW2 + 2 * p : kFragW1 + 8 + 2 * p + (r >> 1);   // H16(p, 0) | W2(1, u)
    }
    i -= 12;
    if (i < 4)
        return kFragW1 + kFragW2 + 2 * i + 1;                           // H16(p = i, 1)
    return 0;
}

using f32x4 = __attribute__((ext_vector_type(4))) float;

// fragments x, y (s = 0, 1 of one 32x32 block) -> the 16x16x32 B operands of board groups 0 and 1
__device__ __forceinline__ void swap16(bf16x8 &x, bf16x8 &y)
{
    uint32_t a[4], b[4];
    __builtin_memcpy(a, &x, 16);
    __builtin_memcpy(b, &y, 16);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const auto r = __builtin_amdgcn_permlane16_swap(a[q], b[q], false, false);
        a[q] = r[0];
        b[q] = r[1];
    }
    __builtin_memcpy(&x, a, 16);
    __builtin_memcpy(&y, b, 16);
}

// out (lane half 0 registers 0..3: logits of board lane & 31, lane half 1 register 0: its value,
// without the head bias) from the 9 conv1 fragments h1; the stream continues at read 9. conv2 grouped
// by weight fragment: each of its 16 fragments W2(g, u) is read ONCE per tile and feeds the 4 output
// positions' accumulators of half g (no MFMA waits on the previous one); the heads on 16x16x32: half
// 0's 8 head MFMAs interleave with half 1's conv2 MFMAs, half 1's follow its epilogue.
// A-fragment stream D fragments deep over policy_frag (the policy kernels' read-ahead)
#ifndef R48_POLICY_WDEPTH
#define R48_POLICY_WDEPTH 2
#endif
template <int D>
struct PolicyStream {
    bf16x8 q[D];
    __device__ __forceinline__ void start(const uint4 *w, int lane)
    {
#pragma unroll
        for (int d = 0; d < D; d++)
            q[d] = frag_at(w, policy_frag(d), lane);
    }
    // the fragment of read i; issues the read of i + D
    __device__ __forceinline__ bf16x8 next(const uint4 *w, int i, int lane)
    {
        const bf16x8 cur = q[0];
#pragma unroll
        for (int d = 0; d + 1 < D; d++)
            q[d] = q[d + 1];
        q[D - 1] = frag_at(w, policy_frag(i + D < kPolicyReads ? i + D : 0), lane);
        return cur;
    }
};
using PolicyWStream = PolicyStream<R48_POLICY_WDEPTH>;

// ReLU(conv1 x + b1) for the 9 positions from the policy stream (reads 0..8)
__device__ __forceinline__ void policy_conv1(const uint4 *w, const float *b, int lane, int h, const bf16x8 &x,
                                             PolicyWStream &ws, bf16x8 (&h1)[9][2])
{
    const f32x16 b1 = load_bias(b, h);
#pragma unroll
    for (int R = 0; R < 9; R++) {
        const bf16x8 wa = ws.next(w, R, lane);
        wfence();
        const f32x16 a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, x, b1, 0, 0, 0);
        wfence();
        h1[R][0] = acc_to_frag_relu(a, 0);
        h1[R][1] = acc_to_frag_relu(a, 1);
    }
}

__device__ __forceinline__ void cnn_conv2_heads16(const uint4 *w, const float *b, int lane, int h,
                                                  const bf16x8 (&h1)[9][2], PolicyWStream &ws, f32x16 &out)
{
    auto next = [&](int i) { return ws.next(w, i, lane); };
    f32x16 acc[4];
    int i = 9;
    {
        const f32x16 b2 = load_bias(b + 32, h);
#pragma unroll
        for (int u = 0; u < 8; u++, i++) {
            const bf16x8 wa = next(i);
            wfence();
#pragma unroll
            for (int p = 0; p < 4; p++)
                acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, h1[kP2[p][u >> 1]][u & 1], u ? acc[p] : b2, 0, 0,
                                                                 0);
            wfence();
        }
    }
    bf16x8 h2[4][2];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        h2[p][0] = acc_to_frag_relu(acc[p], 0);
        h2[p][1] = acc_to_frag_relu(acc[p], 1);
    }
    f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0;     // board groups 0 (boards 0-15), 1 (16-31)
    {
        const f32x16 b2 = load_bias(b + 64, h);
        bf16x8 wh;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const bf16x8 wa = next(i++);
            wfence();
#pragma unroll
            for (int p = 0; p < 4; p++)
                acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, h1[kP2[p][u >> 1]][u & 1], u ? acc[p] : b2, 0, 0,
                                                                 0);
            wfence();
            const int p = u >> 1;
            if ((u & 1) == 0) {
                swap16(h2[p][0], h2[p][1]);
                wh = next(i++);
                wfence();
                o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, h2[p][0], o0, 0, 0, 0);
            } else {
                o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, h2[p][1], o1, 0, 0, 0);
            }
            wfence();
        }
    }
#pragma unroll
    for (int p = 0; p < 4; p++) {
        bf16x8 x = acc_to_frag_relu(acc[p], 0), y = acc_to_frag_relu(acc[p], 1);
        swap16(x, y);
        const bf16x8 wh = next(i++);
        wfence();
        o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, x, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, y, o1, 0, 0, 0);
        wfence();
    }
    // D of group g: lane l, register r = output 4 (l >> 4) + r of board 16 g + (l & 15): logits in
    // lanes 0-15, the value in register 0 of lanes 16-31. One permlane16 swap per register puts
    // group 1's logits into lanes 16-31 of o0 and group 0's values into lanes 0-15 of o1; one
    // permlane32 swap then moves the values to lane half 1 of o0's register 0.
    uint32_t a[4], c[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(o0[r]), __float_as_uint(o1[r]), false, false);
        a[r] = t[0];
        c[r] = t[1];
    }
    a[0] = __builtin_amdgcn_permlane32_swap(a[0], c[0], false, false)[0];
    out = f32x16{};
#pragma unroll
    for (int r = 0; r < 4; r++)
        out[r] = __uint_as_float(a[r]);
}

}  // namespace r48cnn
