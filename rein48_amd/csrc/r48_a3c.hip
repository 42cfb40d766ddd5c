// r48_a3c.hip -- gfx950 kernels for the A3C pieces on either side of the env step
// (nevertiree/Rein48 algorithm/a3c/a3c.py), behind the same C-ABI (include/rein48.h).
//
//   k_features   board int8[16] -> network input float/bf16[16]: raw tile values 2^e
//                (a3c.py:37-39,139 feed the raw state_matrix) or the exponent e
//   k_sample     fused softmax + Philox inverse-CDF draw over 4 actions (choose_action,
//                a3c.py:89-93: np.random.choice(range(4), p=softmax)); also log p[a] and the
//                entropy term -sum p log(p+1e-5) of a3c.py:114
//   k_returns    reverse discounted scan over a [T][n] reward slab (Worker._get_target_value_list,
//                a3c.py:246-256, gamma 0.9, last reward dropped) or the textbook n-step return
// All memory-bound elementwise/scan work: one row per lane, 16-B vector loads where the row
// allows, time-major [T][n] slabs so every step of the scan is a coalesced row.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kSampleTag = 0xA3Cu;

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

template <int MODE>
__device__ __forceinline__ float cell_feature(uint32_t e)
{
    if (MODE == 0)
        return e ? (float)(1u << (e & 31u)) : 0.0f;  // raw tile value
    return (float)e;                                 // exponent
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_features_f32(const int8_t *__restrict__ boards, int64_t n,
                                                         float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float4 *o = reinterpret_cast<float4 *>(out + 16 * i);
#pragma unroll
    for (int r = 0; r < 4; r++)
        o[r] = make_float4(cell_feature<MODE>(w[r] & 0xffu), cell_feature<MODE>((w[r] >> 8) & 0xffu),
                           cell_feature<MODE>((w[r] >> 16) & 0xffu), cell_feature<MODE>(w[r] >> 24));
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_features_bf16(const int8_t *__restrict__ boards, int64_t n,
                                                          uint16_t *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const uint4 v = *reinterpret_cast<const uint4 *>(boards + 16 * i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t packed[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t lo = (w[k >> 1] >> (16 * (k & 1))) & 0xffu, hi = (w[k >> 1] >> (16 * (k & 1) + 8)) & 0xffu;
        // 2^e and small integers are exact in bf16; plain casts keep NaN handling standard
        const __hip_bfloat16 a = __float2bfloat16(cell_feature<MODE>(lo));
        const __hip_bfloat16 b = __float2bfloat16(cell_feature<MODE>(hi));
        packed[k] = (uint32_t)__bfloat16_as_ushort(a) | ((uint32_t)__bfloat16_as_ushort(b) << 16);
    }
    uint4 *o = reinterpret_cast<uint4 *>(out + 16 * i);
    o[0] = make_uint4(packed[0], packed[1], packed[2], packed[3]);
    o[1] = make_uint4(packed[4], packed[5], packed[6], packed[7]);
}

// softmax over 4 logits + inverse-CDF draw with a Philox uniform (24-bit, [0,1))
__global__ __launch_bounds__(kBlock) void k_sample(const float *__restrict__ logits, int64_t n, int64_t gid0,
                                                   uint32_t k0, uint32_t k1, uint32_t ctr,
                                                   int8_t *__restrict__ actions, float *__restrict__ logp,
                                                   float *__restrict__ entropy)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const float4 z = *reinterpret_cast<const float4 *>(logits + 4 * i);
    const float m = fmaxf(fmaxf(z.x, z.y), fmaxf(z.z, z.w));
    const float e0 = __expf(z.x - m), e1 = __expf(z.y - m), e2 = __expf(z.z - m), e3 = __expf(z.w - m);
    const float s = e0 + e1 + e2 + e3, inv = 1.0f / s;
    const float p0 = e0 * inv, p1 = e1 * inv, p2 = e2 * inv, p3 = e3 * inv;
    uint32_t w[4] = {(uint32_t)(gid0 + i), (uint32_t)((uint64_t)(gid0 + i) >> 32), ctr, kSampleTag};
    r48::philox4x32_10(w, k0, k1);
    const float u = (float)(w[0] >> 8) * (1.0f / 16777216.0f);
    // first k with cdf(k) > u (np.random.choice's searchsorted(..., side='right'))
    const float c0 = p0, c1 = c0 + p1, c2 = c1 + p2;
    const int a = (c0 > u) ? 0 : (c1 > u) ? 1 : (c2 > u) ? 2 : 3;
    actions[i] = (int8_t)a;
    if (logp) {
        const float za = a == 0 ? z.x : a == 1 ? z.y : a == 2 ? z.z : z.w;
        logp[i] = za - m - __logf(s);
    }
    if (entropy)
        entropy[i] = -(p0 * __logf(p0 + 1e-5f) + p1 * __logf(p1 + 1e-5f) + p2 * __logf(p2 + 1e-5f) +
                       p3 * __logf(p3 + 1e-5f));
}

// targets[t][i] for t < len[i]; 0 for t >= len[i]. DROP_LAST: the reference's scan
// (targets[len-1] = bootstrap), else the textbook return (targets[len-1] = r + gamma*bootstrap).
template <bool DROP_LAST>
__global__ __launch_bounds__(kBlock) void k_returns(const float *__restrict__ rewards, const int32_t *__restrict__ len,
                                                    const float *__restrict__ bootstrap, int32_t T, int64_t n,
                                                    float gamma, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const int32_t L = min(max(len[i], 0), T);
    for (int32_t t = T - 1; t >= L; t--)
        out[(int64_t)t * n + i] = 0.0f;
    float g = bootstrap[i];
    int32_t t = L - 1;
    if (DROP_LAST && t >= 0) {
        out[(int64_t)t * n + i] = g;
        t--;
    }
    // the scan is serial in g, the loads are not: 8 rewards are in flight per chunk, so each
    // step no longer waits a full memory latency (same arithmetic, same order)
    constexpr int kAhead = 8;
    for (; t >= kAhead - 1; t -= kAhead) {
        float r[kAhead];
#pragma unroll
        for (int k = 0; k < kAhead; k++)
            r[k] = rewards[(int64_t)(t - k) * n + i];
#pragma unroll
        for (int k = 0; k < kAhead; k++) {
            g = r[k] + gamma * g;
            out[(int64_t)(t - k) * n + i] = g;
        }
    }
    for (; t >= 0; t--) {
        g = rewards[(int64_t)t * n + i] + gamma * g;
        out[(int64_t)t * n + i] = g;
    }
}

// k_returns for n % 4 == 0 and 16-byte aligned slabs: a lane owns 4 consecutive boards and walks
// every row t = T-1..0 with one 16-byte load and store (a wave moves 1 KiB per row, no divergence
// on the per-board lengths); per board the same values and the same arithmetic as k_returns.
template <bool DROP_LAST>
__global__ __launch_bounds__(kBlock) void k_returns4(const float4 *__restrict__ rewards, const int4 *__restrict__ len,
                                                     const float4 *__restrict__ bootstrap, int32_t T, int64_t n4,
                                                     float gamma, float4 *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n4)
        return;
    const int4 l4 = len[i];
    const int32_t L[4] = {min(max(l4.x, 0), T), min(max(l4.y, 0), T), min(max(l4.z, 0), T), min(max(l4.w, 0), T)};
    const float4 b4 = bootstrap[i];
    float g[4] = {b4.x, b4.y, b4.z, b4.w};
    constexpr int kAhead = 4;
    for (int32_t t0 = T - 1; t0 >= 0; t0 -= kAhead) {
        float4 r[kAhead];
#pragma unroll
        for (int k = 0; k < kAhead; k++)
            r[k] = t0 - k >= 0 ? rewards[(int64_t)(t0 - k) * n4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < kAhead; k++) {
            const int32_t t = t0 - k;
            if (t < 0)
                break;
            const float rr[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (t >= L[j]) {
                    o[j] = 0.0f;
                } else if (DROP_LAST && t == L[j] - 1) {
                    o[j] = g[j];
                } else {
                    g[j] = rr[j] + gamma * g[j];
                    o[j] = g[j];
                }
            }
            out[(int64_t)t * n4 + i] = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

// tf.train.RMSPropOptimizer (TF1) ApplyRMSProp over one flat parameter buffer:
//   ms  <- decay*ms + (1-decay)*g^2          (ms slot initialised to ONES by the caller)
//   mom <- momentum*mom + lr*g/sqrt(ms + eps)
//   var <- var - mom
__global__ __launch_bounds__(kBlock) void k_rmsprop_tf1(float *__restrict__ var, const float *__restrict__ grad,
                                                        float *__restrict__ ms, float *__restrict__ mom, int64_t n,
                                                        float lr, float decay, float momentum, float eps)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const float g = grad[i];
    const float m = decay * ms[i] + (1.0f - decay) * g * g;
    const float u = momentum * mom[i] + lr * g / sqrtf(m + eps);
    ms[i] = m;
    mom[i] = u;
    var[i] -= u;
}

int fail(int code, const char *msg)
{
    r48::set_last_error(msg);  // the thread-local message behind r48_last_error (r48_env.hip)
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

// Per-segment constants of the A3C loss (losses.segment_stats, a3c.py:99-123) for segments of
// length len[i] (mask = t < len[i]): B[i] = max(len[i], 1); td_sum[i] = sum over t < len[i] of
// targets[t][i] - values[t][i]; counts[i][k] = #{t < len[i] : actions[t][i] == k}. One lane per
// segment (summed from t = len[i] - 1 down); the T rows are coalesced across lanes, 8 rows of loads
// in flight.
template <bool TD>
__global__ __launch_bounds__(kBlock) void k_segment_stats(const float *__restrict__ values,
                                                          const float *__restrict__ targets,
                                                          const int8_t *__restrict__ actions,
                                                          const int32_t *__restrict__ len, int32_t T, int64_t n,
                                                          float *__restrict__ B, float *__restrict__ td_sum,
                                                          float4 *__restrict__ counts)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const int32_t L = min(max(len[i], 0), T);
    float td = 0.0f, c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    // summed from t = L - 1 down to 0: k_segments' order, so the fused update's c0 and this td_sum
    // are bit-identical
    constexpr int kAhead = 8;
    int32_t t = L - 1;
    for (; t + 1 >= kAhead; t -= kAhead) {
        float d[kAhead];
        int a[kAhead];
#pragma unroll
        for (int k = 0; k < kAhead; k++) {
            const int64_t o = (int64_t)(t - k) * n + i;
            d[k] = TD ? targets[o] - values[o] : 0.0f;
            a[k] = actions[o] & 3;
        }
#pragma unroll
        for (int k = 0; k < kAhead; k++) {
            td += d[k];
#pragma unroll
            for (int q = 0; q < 4; q++)
                c[q] += a[k] == q ? 1.0f : 0.0f;
        }
    }
    for (; t >= 0; t--) {
        const int64_t o = (int64_t)t * n + i;
        if (TD)
            td += targets[o] - values[o];
        const int a = actions[o] & 3;
#pragma unroll
        for (int q = 0; q < 4; q++)
            c[q] += a == q ? 1.0f : 0.0f;
    }
    B[i] = (float)max(L, 1);
    if (TD)
        td_sum[i] = td;
    counts[i] = make_float4(c[0], c[1], c[2], c[3]);
}

// The fused update's per-row weights (trainer._fused_gradient) over the [T][n] rows, in
// PyTorch's operation order so both are bit-identical to the tensor form (a tensor divided by a
// scalar is multiplied by the fp32 reciprocal there): m = t < len[i]; wn = (m / B[i]) (1 / n);
// reference loss: cm = ((td_sum[i] / ((4 B[i]) B[i])) m) (1 / n).
__global__ __launch_bounds__(kBlock) void k_row_weights(const int32_t *__restrict__ len, const float *__restrict__ B,
                                                        const float *__restrict__ td_sum, int32_t T, int64_t n,
                                                        float *__restrict__ wn, float *__restrict__ cm)
{
    // grid (ceil(n / kBlock), T): row t = blockIdx.y, no 64-bit division per element
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const int32_t t = (int32_t)blockIdx.y;
    const int64_t r = (int64_t)t * n + i;
    const float m = t < len[i] ? 1.0f : 0.0f, inv_n = 1.0f / (float)n, b = B[i];
    wn[r] = (m / b) * inv_n;
    if (cm)
        cm[r] = ((td_sum[i] / ((4.0f * b) * b)) * m) * inv_n;
}

// The update's per-board pass in one launch (trainer.A3CTrainer.update with the fused gradient):
// the discounted returns of k_returns (same recurrence, same instruction per step: identical
// targets), and per board seg = {w0, c0, L, 0} -- the per-row weights of k_row_weights at every row
// t < L (w0 = (1 / B) (1 / n), c0 = (td_sum / ((4 B) B)) (1 / n), B = max(L, 1), L as int bits),
// which the train kernels expand themselves -- plus, with TD (the reference loss), td_sum over
// t < L of targets - values (summed from t = L - 1 down: the scan's order, which k_segment_stats
// follows) and the action counts. One lane per board, the T rows coalesced across lanes, 8 rows of loads in
// flight.
template <bool DROP_LAST, bool TD>
__global__ __launch_bounds__(kBlock) void k_segments(const float *__restrict__ rewards, const float *__restrict__ values,
                                                     const int8_t *__restrict__ actions, const int32_t *__restrict__ len,
                                                     const float *__restrict__ bootstrap, int32_t T, int64_t n, float gamma,
                                                     float *__restrict__ out, float4 *__restrict__ seg,
                                                     float4 *__restrict__ counts)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const int32_t L = min(max(len[i], 0), T);
    float g = bootstrap[i], td = 0.0f, c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int kAhead = 8;
    for (int32_t t0 = T - 1; t0 >= 0; t0 -= kAhead) {
        float r[kAhead], v[kAhead];
        int a[kAhead];
#pragma unroll
        for (int k = 0; k < kAhead; k++) {
            const int32_t t = t0 - k;
            const int64_t o = (int64_t)max(t, 0) * n + i;
            r[k] = rewards[o];
            v[k] = TD ? values[o] : 0.0f;
            a[k] = TD ? actions[o] & 3 : 0;
        }
#pragma unroll
        for (int k = 0; k < kAhead; k++) {
            const int32_t t = t0 - k;
            if (t < 0)
                break;
            float o;
            if (t >= L) {
                o = 0.0f;
            } else if (DROP_LAST && t == L - 1) {
                o = g;
            } else {
                g = r[k] + gamma * g;
                o = g;
            }
            out[(int64_t)t * n + i] = o;
            if (TD && t < L) {
                td += o - v[k];
#pragma unroll
                for (int q = 0; q < 4; q++)
                    c[q] += a[k] == q ? 1.0f : 0.0f;
            }
        }
    }
    const float b = (float)max(L, 1), inv_n = 1.0f / (float)n;
    seg[i] = make_float4((1.0f / b) * inv_n, TD ? ((td / ((4.0f * b) * b)) * 1.0f) * inv_n : 0.0f, __int_as_float(L), 0.0f);
    if (TD)
        counts[i] = make_float4(c[0], c[1], c[2], c[3]);
}

}  // namespace

extern "C" {

int r48_board_features(const int8_t *boards, int64_t n, int32_t mode, int32_t out_dtype, void *out, void *stream)
{
    if (!boards || !out || n < 0 || (mode != R48_FEAT_VALUES && mode != R48_FEAT_EXPONENTS) ||
        (out_dtype != R48_F32 && out_dtype != R48_BF16))
        return fail(R48_EINVAL, "boards/out NULL, n < 0, or bad mode/dtype");
    if ((reinterpret_cast<uintptr_t>(boards) | reinterpret_cast<uintptr_t>(out)) & 15u)
        return fail(R48_EINVAL, "boards and out must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const hipStream_t s = (hipStream_t)stream;
    if (out_dtype == R48_F32) {
        if (mode == R48_FEAT_VALUES)
            hipLaunchKernelGGL(k_features_f32<0>, grid_for(n), dim3(kBlock), 0, s, boards, n, (float *)out);
        else
            hipLaunchKernelGGL(k_features_f32<1>, grid_for(n), dim3(kBlock), 0, s, boards, n, (float *)out);
    } else {
        if (mode == R48_FEAT_VALUES)
            hipLaunchKernelGGL(k_features_bf16<0>, grid_for(n), dim3(kBlock), 0, s, boards, n, (uint16_t *)out);
        else
            hipLaunchKernelGGL(k_features_bf16<1>, grid_for(n), dim3(kBlock), 0, s, boards, n, (uint16_t *)out);
    }
    return launched("k_features");
}

int r48_sample_actions(const float *logits, int64_t n, uint64_t seed, int64_t gid0, uint32_t ctr, int8_t *actions,
                       float *logp, float *entropy, void *stream)
{
    if (!logits || !actions || n < 0 || gid0 < 0)
        return fail(R48_EINVAL, "logits/actions NULL or n/gid0 < 0");
    if (reinterpret_cast<uintptr_t>(logits) & 15u)
        return fail(R48_EINVAL, "logits must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    hipLaunchKernelGGL(k_sample, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, logits, n, gid0, (uint32_t)seed,
                       (uint32_t)(seed >> 32), ctr, actions, logp, entropy);
    return launched("k_sample");
}

int r48_rmsprop_tf1(float *var, const float *grad, float *ms, float *mom, int64_t n, float lr, float decay,
                    float momentum, float eps, void *stream)
{
    if (!var || !grad || !ms || !mom || n < 0)
        return fail(R48_EINVAL, "NULL argument or n < 0");
    if (n == 0)
        return R48_OK;
    hipLaunchKernelGGL(k_rmsprop_tf1, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, var, grad, ms, mom, n, lr,
                       decay, momentum, eps);
    return launched("k_rmsprop_tf1");
}

int r48_discounted_returns(const float *rewards, const int32_t *lengths, const float *bootstrap, int32_t T, int64_t n,
                           float gamma, int32_t drop_last, float *out, void *stream)
{
    if (!rewards || !lengths || !bootstrap || !out || T < 1 || n < 0)
        return fail(R48_EINVAL, "NULL argument, T < 1 or n < 0");
    if (n == 0)
        return R48_OK;
    if ((n & 3) == 0 && ((reinterpret_cast<uintptr_t>(rewards) | reinterpret_cast<uintptr_t>(lengths) |
                          reinterpret_cast<uintptr_t>(bootstrap) | reinterpret_cast<uintptr_t>(out)) & 15u) == 0) {
        auto k4 = drop_last ? k_returns4<true> : k_returns4<false>;
        hipLaunchKernelGGL(k4, grid_for(n / 4), dim3(kBlock), 0, (hipStream_t)stream, (const float4 *)rewards,
                           (const int4 *)lengths, (const float4 *)bootstrap, T, n / 4, gamma, (float4 *)out);
    } else if (drop_last)
        hipLaunchKernelGGL(k_returns<true>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, rewards, lengths,
                           bootstrap, T, n, gamma, out);
    else
        hipLaunchKernelGGL(k_returns<false>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, rewards, lengths,
                           bootstrap, T, n, gamma, out);
    return launched("k_returns");
}

int r48_a3c_segment_stats(const float *values, const float *targets, const int8_t *actions, const int32_t *lengths,
                          int32_t T, int64_t n, float *B, float *td_sum, float *counts, void *stream)
{
    const bool td = td_sum != nullptr;
    if (!actions || !lengths || !B || !counts || T < 1 || n < 0 || (td && (!values || !targets)) ||
        (reinterpret_cast<uintptr_t>(counts) & 15))
        return fail(R48_EINVAL, "r48_a3c_segment_stats: NULL argument (values/targets needed with td_sum), T < 1, "
                                "n < 0 or counts not 16-byte aligned");
    if (n == 0)
        return R48_OK;
    if (td)
        hipLaunchKernelGGL(k_segment_stats<true>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, values, targets,
                           actions, lengths, T, n, B, td_sum, reinterpret_cast<float4 *>(counts));
    else
        hipLaunchKernelGGL(k_segment_stats<false>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, values, targets,
                           actions, lengths, T, n, B, td_sum, reinterpret_cast<float4 *>(counts));
    return launched("k_segment_stats");
}

int r48_a3c_row_weights(const int32_t *lengths, const float *B, const float *td_sum, int32_t T, int64_t n, float *wn,
                        float *cm, void *stream)
{
    if (!lengths || !B || !wn || T < 1 || n < 0 || (cm && !td_sum))
        return fail(R48_EINVAL, "r48_a3c_row_weights: NULL argument (td_sum needed with cm), T < 1 or n < 0");
    if (n == 0)
        return R48_OK;
    if (T > 65535)
        return fail(R48_EINVAL, "T > 65535");
    hipLaunchKernelGGL(k_row_weights, dim3((unsigned)((n + kBlock - 1) / kBlock), (unsigned)T), dim3(kBlock), 0,
                       (hipStream_t)stream, lengths, B,
                       td_sum, T, n, wn, cm);
    return launched("k_row_weights");
}

int r48_a3c_segments(const float *rewards, const float *values, const int8_t *actions, const int32_t *lengths,
                     const float *bootstrap, int32_t T, int64_t n, float gamma, int32_t drop_last, float *targets,
                     float *seg, float *counts, void *stream)
{
    const bool td = counts != nullptr;
    if (!rewards || !lengths || !bootstrap || !targets || !seg || T < 1 || n < 0 || (td && (!values || !actions)) ||
        ((reinterpret_cast<uintptr_t>(seg) | reinterpret_cast<uintptr_t>(counts)) & 15))
        return fail(R48_EINVAL, "r48_a3c_segments: NULL argument (values/actions needed with counts), T < 1, n < 0 "
                                "or seg/counts not 16-byte aligned");
    if (n == 0)
        return R48_OK;
    auto kern = drop_last ? (td ? k_segments<true, true> : k_segments<true, false>)
                          : (td ? k_segments<false, true> : k_segments<false, false>);
    hipLaunchKernelGGL(kern, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, rewards, values, actions, lengths,
                       bootstrap, T, n, gamma, targets, reinterpret_cast<float4 *>(seg), reinterpret_cast<float4 *>(counts));
    return launched("k_segments");
}

}  // extern "C"
